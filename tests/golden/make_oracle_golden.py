"""Generate tests/golden/oracle_config<N>.json: digests of the CPU oracle's clustering of the synthetic
BASELINE config-1 bin (100k reads, the reference's CPU-runnable case), so the GPU parity test can check a
full config-1-sized bin without re-running the ~1 min CPU oracle on the GPU box.

Test infrastructure only.  Run:  python tests/golden/make_oracle_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "ont-tcrconsensus_amd"), os.path.join(ROOT, "oracle")]


def digest(res: dict) -> dict:
    """Size-independent digest of a clustering result (same keys for the GPU and the oracle)."""
    h = lambda b: hashlib.sha256(b).hexdigest()  # noqa: E731
    return dict(n_clusters=int(res["n_clusters"]),
                cluster=h(np.ascontiguousarray(res["cluster"], np.int32).tobytes()),
                strand=h(np.ascontiguousarray(res["strand"], np.uint8).tobytes()),
                centroid=h(np.ascontiguousarray(res["centroid"], np.uint8).tobytes()),
                consensus=h("\n".join(res["consensus"]).encode()))


CASES = {
    # name: (config, scale, preset, identity)
    "config1_round1_id093": (1, 1.0, 1, 0.93),
    "config1_round1_id090": (1, 1.0, 1, 0.90),
    "config1_round2_id097": (1, 1.0, 2, 0.97),
}


def main():
    import orc
    from umiclust import synth
    out = {}
    for name, (cfg, scale, preset, idn) in CASES.items():
        seqs = synth.config_umis(cfg, scale).as_list()
        r = orc.cluster(orc.params(preset, idn, 58, 68), seqs)
        d = digest(r)
        d.update(config=cfg, scale=scale, preset=preset, identity=idn, n_reads=len(seqs),
                 alignments=r["stats"]["alignments"], cells=r["stats"]["cells"])
        out[name] = d
        print(name, d, flush=True)
    with open(os.path.join(HERE, "oracle_config1.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
