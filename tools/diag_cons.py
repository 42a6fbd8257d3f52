"""Diagnostic: recompute the consensus of the largest GPU clusters at full scale on the CPU.

Uses the GPU's own membership/strands and the oracle's aligner + the Python MSA restatement, so it
checks K3T (traceback) + K4 (consensus) independently of the greedy.  Test infrastructure only.

    python tools/diag_cons.py [config] [n_clusters] [scale]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ont-tcrconsensus_amd"), os.path.join(ROOT, "oracle")]

import orc  # noqa: E402
import pyref  # noqa: E402
from umiclust import _lib, synth  # noqa: E402


def main():
    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    ncheck = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    scale = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0
    u = synth.config_umis(cfg, scale)
    seqs = u.as_list()
    ident = 0.90
    with _lib.Context(0) as ctx:
        ctx.load(_lib.params(1, ident, 58, 68), buf=u.seq, off=u.off)
        st = ctx.cluster()
        a = ctx.fetch()
    print("stats", {k: st[k] for k in ("n_kept", "n_clusters", "n_alignments")}, flush=True)
    lens = np.array([len(s) for s in seqs])
    bad = [(c, len(s)) for c, s in enumerate(a["consensus"]) if not 56 <= len(s) <= 72]
    print("bad consensus lengths:", len(bad), bad[:20], flush=True)
    keep = [i for i in range(len(seqs)) if 58 <= lens[i] <= 68]
    order = sorted(keep, key=lambda i: -lens[i])
    pos = {i: s for s, i in enumerate(order)}
    cl = a["cluster"]
    members = {}
    for i in order:
        c = int(cl[i])
        members.setdefault(c, []).append(i)
    op = orc.params(1, ident, 58, 68)
    targets = sorted(set(range(min(ncheck, a["n_clusters"]))) | {c for c, _ in bad[:50]})
    nbad = 0
    for c in targets:
        mem = members[c]
        cen = [i for i in mem if a["centroid"][i]]
        assert len(cen) == 1, (c, cen)
        cen = cen[0]
        mem = [cen] + [i for i in mem if i != cen]
        db = {i: orc.dust(seqs[i]) for i in mem}
        strand = {i: int(a["strand"][i]) for i in mem}
        cig = {}
        for i in mem[1:]:
            q = db[i] if not strand[i] else pyref.revcomp(db[i])
            cig[i] = orc.align(op, q, db[cen])["cigar"]
        cons = pyref.msa(db, mem, strand, cig)
        if cons != a["consensus"][c]:
            nbad += 1
            if nbad <= 5:
                print(f"cluster {c} size {len(mem)} cen_len {len(seqs[cen])}:\n gpu {a['consensus'][c]}\n cpu {cons}",
                      flush=True)
                print("  members (pos, strand, len, cigar):",
                      [(pos[i], strand[i], lens[i], cig.get(i)) for i in mem[:12]], flush=True)
    print(f"checked {len(targets)} clusters, {nbad} consensus mismatches", flush=True)


if __name__ == "__main__":
    main()
