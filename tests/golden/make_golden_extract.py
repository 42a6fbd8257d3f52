"""Generate tests/golden/extract/*.json from the REFERENCE itself (run here, not on the GPU box): inputs and
outputs of extract_umis (/root/reference/ont_tcr_consensus/extract_umis.py:189-267).

This pins the reference's glue around the pattern search: the strand split (:133-137) and read-name rule
(:129-130), the adapter windows including Python's `seq[-0:]` (:110-126), the `if not umi` skips (:246-247),
the header and combined-UMI format of write_fasta (:140-186), the output-path rule (:201-205), the records
written before a `Read strand not annotated!` exception, and the `None` return (:264-267).

`ray`, `pysam` and `edlib` are not installed (ordinary ModuleNotFoundError).  Stand-ins that
execute nothing from the data: ray.remote is a pass-through decorator; pysam.FastxFile reads FASTA and FASTQ
(name up to the first whitespace, multi-line sequences joined); edlib.align(pattern, query, task="path",
mode="HW", k, additionalEqualities) returns {"editDistance", "locations"} from oracle/extract.hw_locate -- the
restatement of edlib's HW/path semantics, so the search itself stays parity-unpinned against edlib (it checks
that the equalities passed are the ones the restatement uses).  Only data is written to the fixtures.

Usage: python tests/golden/make_golden_extract.py  (requires /root/reference)
"""
from __future__ import annotations

import json
import os
import random
import shutil
import sys
import tempfile
import types

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import extract as ox  # noqa: E402  (the edlib HW/path restatement)
import make_golden  # noqa: E402  (the module loader)

FWD = "TTTVVVVTTVVVVTTVVVVTTVVVVTTT"
REV = "AAABBBBAABBBBAABBBBAABBBBAAA"


def _stubs():
    ray = types.ModuleType("ray")
    ray.remote = lambda *a, **k: (a[0] if a and callable(a[0]) else (lambda f: f))
    sys.modules["ray"] = ray

    pysam = types.ModuleType("pysam")

    class _Rec:
        def __init__(self, name, seq):
            self.name = name
            self.sequence = seq

    class FastxFile:
        def __init__(self, path):
            self.path = path

        def __enter__(self):
            return self

        def __exit__(self, *a):
            return False

        def __iter__(self):
            lines = [x.rstrip("\n").rstrip("\r") for x in open(self.path)]
            i = 0
            while i < len(lines) and not lines[i]:
                i += 1
            fastq = i < len(lines) and lines[i].startswith("@")
            while i < len(lines):
                if not lines[i]:
                    i += 1
                    continue
                name = lines[i][1:].split()[0] if lines[i][1:].split() else ""
                i += 1
                seq = []
                while i < len(lines) and not lines[i].startswith(">") and not (fastq and lines[i].startswith("+")):
                    seq.append(lines[i].strip())
                    i += 1
                s = "".join(seq)
                if fastq:
                    i += 1  # '+' line
                    q = 0
                    while i < len(lines) and q < len(s):
                        q += len(lines[i])
                        i += 1
                yield _Rec(name, s)

    pysam.FastxFile = FastxFile
    pysam.libcfaidx = types.SimpleNamespace(FastxRecord=_Rec)
    sys.modules["pysam"] = pysam

    edlib = types.ModuleType("edlib")

    def align(pattern, query, task="distance", mode="NW", k=-1, additionalEqualities=()):
        assert task == "path" and mode == "HW"
        assert sorted(additionalEqualities) == sorted(ox.IUPAC_EQ)
        r = ox.hw_locate(pattern, query, k)
        if r is None:
            return {"editDistance": -1, "locations": [], "cigar": None}
        d, s, e = r
        return {"editDistance": d, "locations": [(s, e)], "cigar": None}

    edlib.align = align
    sys.modules["edlib"] = edlib


def _mut(rng, s, n):
    s = list(s)
    for _ in range(n):
        x = rng.randrange(len(s))
        u = rng.random()
        if u < 0.4:
            s[x] = rng.choice("ACGT")
        elif u < 0.7:
            s.insert(x, rng.choice("ACGT"))
        elif len(s) > 1:
            del s[x]
    return "".join(s)


def _inst(rng, pat):
    return "".join(rng.choice("ACG") if c == "V" else rng.choice("CGT") if c == "B" else c for c in pat)


def _reads(rng, n, fwd=FWD, rev=REV, unannotated_at=None, tail_fields=False):
    out = []
    for i in range(n):
        body = "".join(rng.choice("ACGT") for _ in range(rng.randint(60, 300)))
        pre = "".join(rng.choice("ACGT") for _ in range(rng.randint(0, 40)))
        suf = "".join(rng.choice("ACGT") for _ in range(rng.randint(0, 30)))
        u5 = _mut(rng, _inst(rng, fwd), rng.choice([0, 0, 1, 2, 3, 4]))
        u3 = _mut(rng, _inst(rng, rev), rng.choice([0, 0, 1, 2, 3, 5]))
        kind = rng.random()
        if kind < 0.1:
            seq = body
        elif kind < 0.15:
            seq = (pre + u5 + body + u3 + suf).lower()
        elif kind < 0.2:
            seq = pre + u5[:rng.randint(5, 25)]
        else:
            seq = pre + u5 + body + u3 + suf
        if rng.random() < 0.05:
            x = rng.randrange(len(seq))
            seq = seq[:x] + "N" + seq[x + 1:]
        strand = "+" if rng.random() < 0.5 else "-"
        name = f"read{i};strand={strand}" + (";ch=7" if tail_fields and i % 3 == 0 else "")
        if i == unannotated_at:
            name = f"read{i}"
        out.append((name, seq))
    return out


def _fasta(recs, width=0):
    lines = []
    for name, seq in recs:
        lines.append(f">{name}\n")
        if width and seq:
            lines += [seq[j:j + width] + "\n" for j in range(0, len(seq), width)]
        else:
            lines.append(seq + "\n")
    return "".join(lines)


def _fastq(recs, width=0):
    lines = []
    for name, seq in recs:
        q = "".join(chr(33 + (j * 7) % 40) for j in range(len(seq)))
        lines.append(f"@{name} some comment\n")
        if width and seq:
            lines += [seq[j:j + width] + "\n" for j in range(0, len(seq), width)]
            lines.append("+\n")
            lines += [q[j:j + width] + "\n" for j in range(0, len(q), width)]
        else:
            lines += [seq + "\n", "+\n", q + "\n"]
    return "".join(lines)


def run_case(mod, case):
    tmp = tempfile.mkdtemp(prefix="ext_")
    try:
        src = os.path.join(tmp, case["file_name"])
        with open(src, "w") as fh:
            fh.write(case["input"])
        out_dir = os.path.join(tmp, "out")
        os.mkdir(out_dir)
        res = dict(case)
        try:
            ret = mod.extract_umis(src, out_dir, **case["args"])
            res["returned"] = None if ret is None else os.path.relpath(ret, out_dir)
            res["error"] = None
        except Exception as e:  # noqa: BLE001 -- "Read strand not annotated!"
            res["returned"] = None
            res["error"] = str(e)
        res["files"] = {fn: open(os.path.join(out_dir, fn)).read() for fn in sorted(os.listdir(out_dir))}
        return res
    finally:
        shutil.rmtree(tmp)


def main():
    _stubs()
    mod = make_golden._load("extract_umis")
    rng = random.Random(20261017)
    long_fwd, long_rev = "TTTVVTTVVVVTTVVVVTTVVVVTTVVVVTTT", "AAABBBBAABBBBAABBBBAABBBBAABBAAA"
    cases = [
        dict(name="fasta_defaults", file_name="region_cluster7.fasta", input=_fasta(_reads(rng, 300)),
             args=dict(write_region=True)),
        dict(name="fastq_multiline", file_name="region_cluster12.fastq.gz.part",
             input=_fastq(_reads(rng, 150), width=50), args=dict(write_region=True)),
        dict(name="no_region", file_name="reads.fa", input=_fasta(_reads(rng, 80), width=60),
             args=dict(write_region=False)),
        dict(name="window3_zero", file_name="region_cluster1.fasta", input=_fasta(_reads(rng, 60)),
             args=dict(write_region=True, adapter_length_3_end=0)),
        dict(name="window5_zero", file_name="region_cluster2.fasta", input=_fasta(_reads(rng, 40)),
             args=dict(write_region=True, adapter_length_5_end=0)),
        dict(name="k0_run_config_patterns", file_name="region_cluster3.fasta",
             input=_fasta(_reads(rng, 120, long_fwd, long_rev)),
             args=dict(write_region=True, adapter_length_5_end=81, adapter_length_3_end=76, max_pattern_dist=0,
                       umi_fwd=long_fwd, umi_rev=long_rev)),
        dict(name="k3_run_config_patterns", file_name="region_cluster4.fasta",
             input=_fasta(_reads(rng, 120, long_fwd, long_rev, tail_fields=True)),
             args=dict(write_region=True, adapter_length_5_end=81, adapter_length_3_end=76, max_pattern_dist=3,
                       umi_fwd=long_fwd, umi_rev=long_rev)),
        dict(name="none_found", file_name="region_cluster5.fasta",
             input=_fasta([(f"r{i};strand=+", "ACGT" * 30) for i in range(10)]), args=dict(write_region=True)),
        dict(name="unannotated_strand", file_name="region_cluster6.fasta",
             input=_fasta(_reads(rng, 50, unannotated_at=31)), args=dict(write_region=True)),
    ]
    od = os.path.join(HERE, "extract")
    os.makedirs(od, exist_ok=True)
    for c in cases:
        res = run_case(mod, c)
        with open(os.path.join(od, c["name"] + ".json"), "w") as fh:
            json.dump(res, fh, indent=0, sort_keys=True)
        print(c["name"], res["returned"], res["error"], {k: v.count(">") for k, v in res["files"].items()})


if __name__ == "__main__":
    main()
