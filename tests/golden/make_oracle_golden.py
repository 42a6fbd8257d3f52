"""Generate tests/golden/oracle_config<N>.json: digests of the CPU oracle's clustering of the synthetic
BASELINE config-1 bin (100k reads, the reference's CPU-runnable case) and of samples of the config-5
stress bin (~96-nt UMIs, 15 % indels, clusters of >1k members), so the GPU parity test can check them
without re-running the CPU oracle (~1 min per config-1 case) on the GPU box.

Test infrastructure only.  Run:  python tests/golden/make_oracle_golden.py [config ...] | multibin [name ...] |
segments | o4 [name ...]

o4: the same digests under policy O4 (vsearch --threads T, the mode the reference runs every bin
in: vsearch_umi_cluster.py:33-34,83-84, utils.py:56-63) -> oracle_o4.json.  The oracle's round searches run on
ORC_WORKERS OpenMP threads (default: every host CPU); results do not depend on the worker count.
"""
import hashlib
import json
import os
import platform
import sys
import time

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
    # the headline bin (BASELINE config 2, 2M reads, id 0.90) at full size; its wall time is also the
    # full-bin CPU baseline (1 thread, recorded with the host CPU model)
    "config2_round1_id090": (2, 1.0, 1, 0.90),
    "config1_round1_id090": (1, 1.0, 1, 0.90),
    "config1_round2_id097": (1, 1.0, 2, 0.97),
    # config 5: at id 0.75 the deep clusters form (2 clusters > 1k members at scale 0.1); at id 0.90
    # almost every read is a centroid (long candidate lists, many new-centroid alignments)
    "config5_round1_id075": (5, 0.1, 1, 0.75),
    "config5_round1_id090": (5, 0.02, 1, 0.90),
    "config5_round2_id075": (5, 0.02, 2, 0.75),
}


def _max_cluster(cluster) -> int:
    cl = np.asarray(cluster)
    cl = cl[cl >= 0]  # length-filtered records are -1
    return int(np.bincount(cl).max()) if len(cl) else 0


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


# multi-bin BASELINE configs at reduced scale: every bin clustered by the oracle, a checksum of the per-bin
# digests (membership, strands, centroids, consensus) per round; config 4 chains round 2 on the round-1
# consensus UMIs of every bin (umiclust.binset.round2_binset)
MULTIBIN_CASES = {
    # name: (config, scale)
    "config3_bins_s001": (3, 0.01),
    "config4_rounds_s0002": (4, 0.002),
}


def multibin_golden(cfg: int, scale: float) -> dict:
    import orc
    from umiclust import binset, synth
    lo, hi = synth.CONFIG_LENGTHS[cfg]
    bs = synth.concat_bins(synth.config_bins(cfg, scale, workers=4))
    out = dict(config=cfg, scale=scale, n_bins=len(bs.bins), n_reads=int(bs.n), minlen=lo, maxlen=hi)
    rounds = [("round1", binset.ROUND1)] + ([("round2", binset.ROUND2)] if cfg == 4 else [])
    t0 = time.perf_counter()
    for name, prm in rounds:
        op = orc.params(prm["preset"], prm["identity"], lo, hi)
        res, alignments, cells = [], 0, 0
        for b in bs.bins:
            r = orc.cluster(op, b.umis.as_list())
            res.append(r)
            alignments += r["stats"]["alignments"]
            cells += r["stats"]["cells"]
        dg = [binset.digest(r) for r in res]
        out[name] = dict(preset=prm["preset"], identity=prm["identity"], n_reads=int(bs.n),
                         combined=binset.combine(dg), n_clusters=[d["n_clusters"] for d in dg],
                         alignments=alignments, cells=cells)
        print(name, out[name]["combined"], sum(out[name]["n_clusters"]), flush=True)
        if name == "round1" and len(rounds) > 1:
            bs = binset.round2_binset(bs, res)
    out.update(oracle_seconds=round(time.perf_counter() - t0, 2), oracle_threads=1, host_cpu=_cpu_model())
    return out


def main_multibin(names):
    for name in names:
        cfg, scale = MULTIBIN_CASES[name]
        d = multibin_golden(cfg, scale)
        with open(os.path.join(HERE, f"oracle_{name}.json"), "w") as f:
            json.dump({name: d}, f, indent=1, sort_keys=True)


def main(configs):
    import orc
    from umiclust import synth
    out = {}
    for name, (cfg, scale, preset, idn) in CASES.items():
        if cfg not in configs:
            continue
        lo, hi = synth.CONFIG_LENGTHS[cfg]
        seqs = synth.config_umis(cfg, scale).as_list()
        t0 = time.perf_counter()
        r = orc.cluster(orc.params(preset, idn, lo, hi), seqs)
        dt = time.perf_counter() - t0
        d = digest(r)
        d.update(config=cfg, scale=scale, preset=preset, identity=idn, minlen=lo, maxlen=hi, n_reads=len(seqs),
                 alignments=r["stats"]["alignments"], cells=r["stats"]["cells"],
                 max_cluster=_max_cluster(r["cluster"]),
                 oracle_seconds=round(dt, 2), oracle_threads=1, host_cpu=_cpu_model())
        out.setdefault(cfg, {})[name] = d
        print(name, d, flush=True)
    for cfg, cases in out.items():
        with open(os.path.join(HERE, f"oracle_config{cfg}.json"), "w") as f:
            json.dump(cases, f, indent=1, sort_keys=True)


# O4 cases: name -> (config, scale, preset, identity, T) for single bins, (config, scale, None, None, T) for the
# multi-bin configs (every bin of config 3 / both rounds of config 4 under O4)
O4_CASES = {
    "config1_round1_id093_o4T25": (1, 1.0, 1, 0.93, 25),
    "config1_round2_id097_o4T25": (1, 1.0, 2, 0.97, 25),
    "config5_round1_id075_o4T25": (5, 0.1, 1, 0.75, 25),
    "config5_round1_id090_o4T25": (5, 0.02, 1, 0.90, 25),
    "config3_bins_s001_o4T25": (3, 0.01, None, None, 25),
    "config4_rounds_s0002_o4T25": (4, 0.002, None, None, 25),
    # the headline bin (BASELINE config 2, 2M reads, id 0.90) at full size under --threads 25
    "config2_round1_id090_o4T25": (2, 1.0, 1, 0.90, 25),
    # round 6: the sizes bench.py runs -- config 3 whole (960 bins, ~9.9M reads), config 4 at
    # 2 % scale both rounds, config 5's 300k-read bench bin at --id 0.75
    "config3_bins_s1_o4T25": (3, 1.0, None, None, 25),
    "config4_rounds_s002_o4T25": (4, 0.02, None, None, 25),
    "config5_round1_id075_s1_o4T25": (5, 1.0, 1, 0.75, 25),
}
# single bins of a multi-bin config at full size, both rounds: name -> (config, scale, shard ids, T).  Bin 200
# (barcode 6, region 0: 792k reads, a giant molecule) is config 4's slowest unit, where bench.py partially resolves
# overflowing blocks, re-runs their rest and regrows the block size
O4_BIN_CASES = {
    "config4_bin200_rounds_o4T25": (4, 1.0, [200], 25),
}


def _o4(p, T: int):
    p.threads, p.policy_threads = T, 1
    return p


def main_o4(names):
    import orc
    from umiclust import binset, synth
    os.environ.setdefault("ORC_WORKERS", str(os.cpu_count() or 1))
    path = os.path.join(HERE, "oracle_o4.json")
    out = json.load(open(path)) if os.path.exists(path) else {}
    for name in names:
        sids = None
        if name in O4_BIN_CASES:
            cfg, scale, sids, T = O4_BIN_CASES[name]
            preset = idn = None
        else:
            cfg, scale, preset, idn, T = O4_CASES[name]
        lo, hi = synth.CONFIG_LENGTHS[cfg]
        t0 = time.perf_counter()
        if preset is None:
            bs = synth.concat_bins(synth.config_bins(cfg, scale, workers=4, shard_ids=sids))
            d = dict(config=cfg, scale=scale, n_bins=len(bs.bins), n_reads=int(bs.n), minlen=lo, maxlen=hi, T=T)
            if sids is not None:
                d["shard_ids"] = list(sids)
            rounds = [("round1", binset.ROUND1)] + ([("round2", binset.ROUND2)] if cfg == 4 else [])
            for rname, prm in rounds:
                op = _o4(orc.params(prm["preset"], prm["identity"], lo, hi), T)
                res = [orc.cluster(op, b.umis.as_list()) for b in bs.bins]
                dg = [binset.digest(r) for r in res]
                d[rname] = dict(preset=prm["preset"], identity=prm["identity"], n_reads=int(bs.n),
                                combined=binset.combine(dg), n_clusters=[x["n_clusters"] for x in dg],
                                alignments=sum(r["stats"]["alignments"] for r in res),
                                cells=sum(r["stats"]["cells"] for r in res))
                if rname == "round1" and len(rounds) > 1:
                    bs = binset.round2_binset(bs, res)
        else:
            seqs = synth.config_umis(cfg, scale).as_list()
            r = orc.cluster(_o4(orc.params(preset, idn, lo, hi), T), seqs)
            d = digest(r)
            d.update(config=cfg, scale=scale, preset=preset, identity=idn, minlen=lo, maxlen=hi, n_reads=len(seqs),
                     T=T, alignments=r["stats"]["alignments"], cells=r["stats"]["cells"],
                     max_cluster=_max_cluster(r["cluster"]))
        d.update(oracle_seconds=round(time.perf_counter() - t0, 2), oracle_workers=int(os.environ["ORC_WORKERS"]),
                 host_cpu=_cpu_model())
        out[name] = d
        print(name, {k: v for k, v in d.items() if k not in ("round1", "round2")}, flush=True)
        with open(path, "w") as f:
            json.dump(out, f, indent=1, sort_keys=True)


def main_segments():
    """oracle_segments.json: synth.segment_stress() (a bin past one 7 x 65,536-centroid counter segment)."""
    import orc
    from umiclust import synth
    buf, off = synth.segment_stress()
    raw = buf.tobytes()
    seqs = [raw[off[i]:off[i + 1]].decode() for i in range(len(off) - 1)]
    t0 = time.perf_counter()
    r = orc.cluster(orc.params(1, 0.90, 58, 68), seqs)
    dt = time.perf_counter() - t0
    d = digest(r)
    d.update(preset=1, identity=0.90, minlen=58, maxlen=68, n_reads=len(seqs), alignments=r["stats"]["alignments"],
             cells=r["stats"]["cells"], oracle_seconds=round(dt, 2), oracle_threads=1, host_cpu=_cpu_model())
    with open(os.path.join(HERE, "oracle_segments.json"), "w") as f:
        json.dump({"segments_round1_id090": d}, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    args = sys.argv[1:]
    if args and args[0] == "o4":
        main_o4(args[1:] or list(O4_CASES) + list(O4_BIN_CASES))
    elif args and args[0] == "segments":
        main_segments()
    elif args and args[0] == "multibin":
        main_multibin(args[1:] or sorted(MULTIBIN_CASES))
    else:
        main([int(a) for a in args] or sorted({c[0] for c in CASES.values()}))
