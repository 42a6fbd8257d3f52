"""Record resolve_block calls of real clustering runs on the GPU (UMICLUST_RESOLVE_DUMP, driver.cpp
write_resolve_dump) for the host-only ThreadSanitizer replay (tools/resolve_tsan_main.cpp,
tests/test_sanitizers_cpu.py).  Run on the GPU box; the dumps (gzip) are committed under tests/golden/resolve/.

    python tests/golden/make_resolve_dumps.py <out_dir>

Cases: a config-2-like bin (300k reads, blocks of 4,096, split passes), a bin of few, deep molecules whose new-centroid
rate falls below the lazy-peer threshold (5 per mille: lazy passes, deferred queries and round B), a config-5-like
deep-cluster bin (long UMIs, 15 % indels) and batched rounds (policy O4, T = 25).  The lazy cases assert that the
recorded passes are lazy (the UMICLUST_LAZY switch that forced it before round 5 is gone)."""
import gzip
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "ont-tcrconsensus_amd"))
from umiclust import _lib, synth  # noqa: E402


def run(name, umis, params, env, passes):
    out = sys.argv[1]
    prefix = os.path.join(out, name)
    old = {k: os.environ.get(k) for k in list(env) + ["UMICLUST_RESOLVE_DUMP"]}
    os.environ.update(env)
    os.environ["UMICLUST_RESOLVE_DUMP"] = prefix + ":" + ",".join(str(p) for p in passes)
    try:
        with _lib.Context(0) as ctx:
            ctx.load(params, buf=umis.seq, off=umis.off)
            st = ctx.cluster()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    for p in passes:
        f = f"{prefix}.{p}.bin"
        if os.path.exists(f):
            with open(f, "rb") as fi, gzip.open(f + ".gz", "wb", compresslevel=9) as fo:
                shutil.copyfileobj(fi, fo)
            os.remove(f)
            print(name, p, os.path.getsize(f + ".gz"), "bytes", flush=True)
    print(name, {k: st[k] for k in ("n_kept", "n_clusters", "n_alignments", "n_deferred", "pairs_round_b",
                                    "n_lazy_passes", "n_blocks")}, flush=True)
    return st


def main():
    os.makedirs(sys.argv[1], exist_ok=True)
    u2 = synth.make_umis(15000, seed=2024, max_reads=300_000)
    p2 = _lib.params(_lib.PRESET_ROUND1, 0.90, 58, 68)
    run("c2", u2, p2, {"UMICLUST_BLOCK": "4096"}, [8, 40])
    # ~300 molecules of ~500 reads: after the first blocks almost every query joins a cluster (lazy passes)
    ul = synth.make_umis(300, seed=2025, mean_reads=500.0, max_reads=150_000)
    st = run("c2lazy", ul, p2, {"UMICLUST_BLOCK": "2048"}, [45, 65])
    assert st["n_lazy_passes"] > 30, st  # 44 of 74 passes lazy on the GPU box (round 6): the recorded ones are
    u5 = synth.make_umis(40, seed=1005, mean_reads=1500.0, error_rate=0.15, split=(0.0, 0.5, 0.5), max_edits=4,
                         pattern_fwd=synth.UMI_FWD_LONG, pattern_rev=synth.UMI_REV_LONG, max_reads=30_000)
    run("c5", u5, _lib.params(_lib.PRESET_ROUND1, 0.75, 80, 110), {"UMICLUST_BLOCK": "1024"}, [6, 20])
    p4 = _lib.params(_lib.PRESET_ROUND1, 0.93, 58, 68)
    p4.threads, p4.policy_threads = 25, 1
    u4 = synth.make_umis(3000, seed=77, max_reads=60_000, error_rate=0.03)
    run("o4", u4, p4, {"UMICLUST_BLOCK": "2048"}, [5, 15])


if __name__ == "__main__":
    main()
