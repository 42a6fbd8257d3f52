"""Parity debugging aid: per-query walked-alignment counts of the GPU path (UMICLUST_WALK_DUMP) against the oracle
(ORC_WALK_DUMP) on the deep-cluster O4 input of tests/test_gpu_o4.py::test_batched_rounds_deep_clusters.
Prints the first queries whose counts differ.  Usage: python tools/o4_walk_debug.py [mix] [T] [block]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ont-tcrconsensus_amd"), os.path.join(ROOT, "oracle")]
import orc  # noqa: E402
from umiclust import _lib, synth  # noqa: E402


def params(lib, T, idn=0.75, lens=(80, 110)):
    p = lib.params(1, idn, *lens)
    p.threads, p.policy_threads = T, (1 if T > 1 else 0)
    return p


def main():
    mix = sys.argv[1] if len(sys.argv) > 1 else "1"
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    block = sys.argv[3] if len(sys.argv) > 3 else "256"
    out = os.path.join(ROOT, "gpurun_out", "o4dbg")
    os.makedirs(out, exist_ok=True)
    seqs = synth.make_umis(8, seed=31, max_reads=2500, orient_mix=0.3, mean_reads=1500.0, error_rate=0.15,
                           split=(0.0, 0.5, 0.5), max_edits=4, pattern_fwd=synth.UMI_FWD_LONG,
                           pattern_rev=synth.UMI_REV_LONG).as_list()
    os.environ["UMICLUST_BLOCK"] = block
    os.environ["UMICLUST_MIXLEN"] = mix
    gf, of = os.path.join(out, f"gpu_{mix}_{T}.bin"), os.path.join(out, f"orc_{T}.bin")
    os.environ["UMICLUST_WALK_DUMP"] = gf
    with _lib.Context(0) as ctx:
        ctx.load(params(_lib, T), seqs)
        st = ctx.cluster()
        g = ctx.fetch()
    os.environ["ORC_WALK_DUMP"] = of
    o = orc.cluster(params(orc, T), seqs)
    gw = np.fromfile(gf, dtype=np.int16).reshape(-1, 4)
    ow = np.fromfile(of, dtype=np.int16).reshape(-1, 2)
    print(f"mix {mix} T {T} block {block}: gpu alignments {st['n_alignments']} oracle {o['stats']['alignments']} "
          f"membership equal {np.array_equal(g['cluster'], o['cluster'])} n {len(ow)}")
    lens = np.array(sorted((len(s) for s in seqs if 80 <= len(s) <= 110), reverse=True))
    bad = np.nonzero((gw[:, :2] != ow).any(axis=1))[0]
    print(f"{len(bad)} queries differ")
    for s in bad[:40]:
        print(f"  seqno {s} len {lens[s]} round {s // T if T > 1 else '-'} gpu {gw[s, :2].tolist()} path "
              f"{gw[s, 2:].tolist()} oracle {ow[s].tolist()}")


if __name__ == "__main__":
    main()
