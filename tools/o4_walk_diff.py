"""Parity debugging aid: per-query walked-alignment counts of the GPU path (UMICLUST_WALK_DUMP) against the oracle
(ORC_WALK_DUMP) on a BASELINE config sample under O4 (vsearch --threads T).  Prints membership equality and the first
queries whose counts differ.  Usage: python tools/o4_walk_diff.py CONFIG SCALE IDENTITY T [MIXLEN] [BLOCK]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ont-tcrconsensus_amd"), os.path.join(ROOT, "oracle")]
import orc  # noqa: E402
from umiclust import _lib, synth  # noqa: E402


def main():
    cfg, scale, idn, T = int(sys.argv[1]), float(sys.argv[2]), float(sys.argv[3]), int(sys.argv[4])
    mix = sys.argv[5] if len(sys.argv) > 5 else ""
    block = sys.argv[6] if len(sys.argv) > 6 else ""
    lo, hi = synth.CONFIG_LENGTHS[cfg]
    out = os.path.join(ROOT, "gpurun_out", "o4diff")
    os.makedirs(out, exist_ok=True)
    seqs = synth.config_umis(cfg, scale).as_list()
    if mix:
        os.environ["UMICLUST_MIXLEN"] = mix
    if block:
        os.environ["UMICLUST_BLOCK"] = block
    tag = f"c{cfg}_{scale}_{idn}_{T}_{mix or 'd'}_{block or 'd'}"
    gf, of = os.path.join(out, f"gpu_{tag}.bin"), os.path.join(out, f"orc_{tag}.bin")
    os.environ["UMICLUST_WALK_DUMP"] = gf
    p = _lib.params(1, idn, lo, hi, threads=T)
    with _lib.Context(0) as ctx:
        ctx.load(p, seqs)
        st = ctx.cluster()
        g = ctx.fetch()
    os.environ["ORC_WALK_DUMP"] = of
    op = orc.params(1, idn, lo, hi)
    if T > 1:
        op.threads, op.policy_threads = T, 1
    o = orc.cluster(op, seqs)
    gw = np.fromfile(gf, dtype=np.int16).reshape(-1, 4)
    ow = np.fromfile(of, dtype=np.int16).reshape(-1, 2)
    print(f"{tag}: gpu alignments {st['n_alignments']} oracle {o['stats']['alignments']} blocks {st['n_blocks']} "
          f"reruns {st['n_reruns']} membership equal {np.array_equal(g['cluster'], o['cluster'])} "
          f"strand equal {np.array_equal(g['strand'], o['strand'])} n {len(ow)}")
    lens = np.array(sorted((len(s) for s in seqs if lo <= len(s) <= hi), reverse=True))
    bad = np.nonzero((gw[:, :2] != ow).any(axis=1))[0]
    print(f"{len(bad)} queries differ")
    for s in bad[:60]:
        print(f"  seqno {s} len {lens[s]} round {s // T if T > 1 else '-'} (pos {s % T if T > 1 else '-'}) gpu "
              f"{gw[s, :2].tolist()} path {gw[s, 2:].tolist()} oracle {ow[s].tolist()}")


if __name__ == "__main__":
    main()
