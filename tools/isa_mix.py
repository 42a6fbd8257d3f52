"""Instruction mix of the aligner's column loop from its ISA, for the issue-cost ceiling in bench.py.

Usage: python tools/isa_mix.py <kernel.s> <mangled kernel name> [out.json]
The ISA comes from `hipcc -O3 --offload-arch=gfx950 --cuda-device-only -S -DALIGN_PART=1 csrc/align_inst.hip`.
The column loop is the innermost loop with the most vector instructions.  Classes: VOP2/VOP1 (4-byte `_e32`
encodings), packed VOP3P (`v_pk_*`) and other VOP3 (8-byte encodings); their issue costs come from
tools/valu_rate.hip (profiles/r05/valu_rate.jsonl).
"""
import json
import re
import sys


def loops(lines):
    """(start, end) line ranges of every `.LBB` block run that a backward branch closes."""
    labels = {}
    for i, l in enumerate(lines):
        m = re.match(r"^(\.LBB\d+_\d+):", l)
        if m:
            labels[m.group(1)] = i
    out = []
    for i, l in enumerate(lines):
        m = re.search(r"s_cbranch_\w+\s+(\.LBB\d+_\d+)|s_branch\s+(\.LBB\d+_\d+)", l)
        if m:
            tgt = m.group(1) or m.group(2)
            if tgt in labels and labels[tgt] < i:
                out.append((labels[tgt], i))
    return out


def mix(lines):
    c = dict(vop2=0, vop3p=0, vop3=0, lds=0, vmem=0, salu=0)
    for l in lines:
        t = l.strip().split()
        if not t or t[0].startswith((";", ".")):
            continue
        op = t[0]
        if op.startswith("v_pk_"):
            c["vop3p"] += 1
        elif op.startswith("v_"):
            c["vop2" if op.endswith("_e32") or op in ("v_mov_b32",) else "vop3"] += 1
        elif op.startswith("ds_"):
            c["lds"] += 1
        elif op.startswith(("global_", "buffer_")):
            c["vmem"] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
    return c


def main():
    src, name = sys.argv[1], sys.argv[2]
    text = open(src).read().splitlines()
    s = next(i for i, l in enumerate(text) if l.startswith(name + ":"))
    e = next(i for i in range(s, len(text)) if text[i].startswith(".Lfunc_end"))
    body = text[s:e]
    ls = loops(body)
    inner = [r for r in ls if not any(o != r and r[0] <= o[0] and o[1] <= r[1] for o in ls)]
    # the main column loop: the innermost loop with the most vector instructions (the two LAST steps run in
    # a second, shorter loop)
    best = max(inner, key=lambda r: sum(mix(body[r[0]:r[1] + 1])[k] for k in ("vop2", "vop3p", "vop3")))
    # per-step instructions: drop the blocks that run once per pair -- the j == 0 boundary restore
    # (pk_init_rows, recognisable by its inline `v_mov_b32 %0, 0`)
    loop = body[best[0]:best[1] + 1]
    blocks, cur = [], []
    for l in loop:
        if re.match(r"^\.LBB\d+_\d+:", l) and cur:
            blocks.append(cur)
            cur = []
        cur.append(l)
    blocks.append(cur)
    kept = [b for b in blocks if not any(re.match(r"\s*v_mov_b32 v\d+, 0$", x) for x in b)]
    m = mix([l for b in kept for l in b])
    m["blocks_dropped"] = len(blocks) - len(kept)
    m.update(kernel=name, loop_lines=[best[0], best[1]])
    out = json.dumps(m, indent=1)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(out + "\n")
    print(out)


if __name__ == "__main__":
    main()
