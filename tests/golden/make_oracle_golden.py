"""Generate tests/golden/oracle_config<N>.json: digests of the CPU oracle's clustering of the synthetic
BASELINE config-1 bin (100k reads, the reference's CPU-runnable case) and of samples of the config-5
stress bin (~96-nt UMIs, 15 % indels, clusters of >1k members), so the GPU parity test can check them
without re-running the CPU oracle (~1 min per config-1 case) on the GPU box.

Test infrastructure only.  Run:  python tests/golden/make_oracle_golden.py [config ...]
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
    # config 5: at id 0.75 the deep clusters form (2 clusters > 1k members at scale 0.1); at id 0.90
    # almost every read is a centroid (long candidate lists, many new-centroid alignments)
    "config5_round1_id075": (5, 0.1, 1, 0.75),
    "config5_round1_id090": (5, 0.02, 1, 0.90),
    "config5_round2_id075": (5, 0.02, 2, 0.75),
}


def main(configs):
    import orc
    from umiclust import synth
    out = {}
    for name, (cfg, scale, preset, idn) in CASES.items():
        if cfg not in configs:
            continue
        lo, hi = synth.CONFIG_LENGTHS[cfg]
        seqs = synth.config_umis(cfg, scale).as_list()
        r = orc.cluster(orc.params(preset, idn, lo, hi), seqs)
        d = digest(r)
        d.update(config=cfg, scale=scale, preset=preset, identity=idn, minlen=lo, maxlen=hi, n_reads=len(seqs),
                 alignments=r["stats"]["alignments"], cells=r["stats"]["cells"],
                 max_cluster=int(np.bincount(np.asarray(r["cluster"])).max()) if len(seqs) else 0)
        out.setdefault(cfg, {})[name] = d
        print(name, d, flush=True)
    for cfg, cases in out.items():
        with open(os.path.join(HERE, f"oracle_config{cfg}.json"), "w") as f:
            json.dump(cases, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main([int(a) for a in sys.argv[1:]] or sorted({c[0] for c in CASES.values()}))
