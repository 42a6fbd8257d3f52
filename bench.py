"""Benchmark: UMIs clustered/s (+ GCUPS) of the vsearch --cluster_fast drop-in on MI355X.

Workload (BASELINE.json configs[1]): one synthetic region bin of 2M dual-UMI reads per
GPU (seed 1002 for rank 0, 1002*1_000_003 + rank for other ranks: weak scaling, one independent bin
per GPU, no collective on the data path), --id 0.90, round-1 scoring (vsearch_umi_cluster.py:44-50).
A step = one full pass of the hot path over the bin, with the sequences already resident in HBM:
K1 prep/DUST/k-mers, greedy blocks of K2 prefilter + K3 walk alignment + host resolution, K3T
traceback for members, K4 consensus, and the result download.

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ont-tcrconsensus_amd"))

METRIC = "UMIs clustered/sec + banded-NW GCUPS (whole node, 1/2/4/8 MI355X)"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)


def cpu_baseline(umis, n_sample: int, identity: float, lens=(58, 68)) -> dict:
    """The C oracle (oracle/, 1 thread) on the first n_sample reads of the same workload."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import orc
    seqs = umis.as_list()[:n_sample]
    t0 = time.perf_counter()
    r = orc.cluster(orc.params(1, identity, *lens), seqs)
    dt = time.perf_counter() - t0
    return dict(value=r["stats"]["kept"] / dt, unit="UMIs/s", cores=1, kind="port",
                sample=f"first {n_sample} reads of the rank-0 bin ({r['stats']['kept']} kept, "
                       f"{r['n_clusters']} clusters) clustered by the C oracle restatement, 1 thread, "
                       f"{dt:.1f} s; CPU cost grows ~N*C so a full 2M-read bin is slower per UMI",
                seconds=dt, n_kept=r["stats"]["kept"])


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", type=int, default=2, choices=(2, 5),
                    help="2: the headline bin (default); 5: the long-UMI high-error stress bin")
    ap.add_argument("--scale", type=float, default=1.0, help="fraction of the bin (testing only)")
    ap.add_argument("--identity", type=float, default=None, help="default 0.90 (config 2), 0.75 (config 5)")
    ap.add_argument("--cpu-sample", type=int, default=40000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_latest.json"),
                    help="measured HBM bytes per prefilter launch (rocprofv3 PMC pass), if present")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        backend = "nccl" if torch.cuda.is_available() else "gloo"
        dist.init_process_group(backend=backend)
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a HIP device (there is no CPU backend)")
    torch.cuda.set_device(local_rank)

    from umiclust import _lib, synth
    if args.identity is None:
        args.identity = 0.90 if args.config == 2 else 0.75
    lens = synth.CONFIG_LENGTHS[args.config]
    seed = (1000 + args.config) if rank == 0 else (1000 + args.config) * 1_000_003 + rank
    if args.config == 2:
        umis = synth.make_umis(int(100_000 * args.scale), seed=seed, max_reads=int(2_000_000 * args.scale))
        workload = ("BASELINE config 2: synthetic 2M dual-UMI reads per GPU, one region bin, "
                    f"--id {args.identity:.2f}, round-1 scoring (match 10, mismatch -40, gapopen 0E/40I)")
    else:
        umis = synth.make_umis(max(1, int(200 * args.scale)), seed=seed, mean_reads=1500.0, error_rate=0.15,
                               split=(0.0, 0.5, 0.5), max_edits=4, pattern_fwd=synth.UMI_FWD_LONG,
                               pattern_rev=synth.UMI_REV_LONG, max_reads=int(300_000 * args.scale))
        workload = ("BASELINE config 5 stress: synthetic 300k long (~96-nt) UMIs per GPU, 15% indels, deep "
                    f"clusters (NegBin mean 1500 reads/molecule), --id {args.identity:.2f}, "
                    f"--minseqlength {lens[0]} --maxseqlength {lens[1]}, round-1 scoring")
    ctx = _lib.Context(local_rank)
    params = _lib.params(_lib.PRESET_ROUND1, args.identity, *lens)
    ctx.load(params, buf=umis.seq, off=umis.off)

    def barrier():
        if dist is not None:
            dist.barrier()

    for _ in range(args.warmup):
        ctx.cluster()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    stats = []
    for _ in range(args.steps):
        stats.append(ctx.cluster())
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    t_max = elapsed
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        t_max = float(t.item())
    st = stats[-1]
    n_kept = st["n_kept"]
    total_umis = n_kept * world * args.steps
    cells = st["cells"]
    value = total_umis / t_max
    gcups = cells * world * args.steps / t_max / 1e9

    if rank == 0:
        # roofline of the dominant kernel, from HIP-event kernel times accumulated by the driver
        t_pf = sum(s["t_prefilter_s"] for s in stats) / args.steps
        t_al = sum(s["t_align_s"] for s in stats) / args.steps
        n_launch = st["n_blocks"]
        # prefilter algorithmic bytes: u16 postings streamed + 2 CSR offsets per (k-mer, tile)
        pf_bytes = st["kmer_postings"] * 2
        traffic = None
        if os.path.exists(args.traffic_json):
            try:
                tj = json.load(open(args.traffic_json))
                # PMC traffic is per workload: only report it for the config it was counted on
                if tj.get("config", 2) == args.config:
                    traffic = tj.get("prefilter_hbm_bytes_per_launch")
            except Exception:
                traffic = None
        achieved = pf_bytes / n_launch / (t_pf / n_launch) / 1e9 if t_pf > 0 else 0.0
        roof = dict(kernel="k_prefilter", bound="hbm", achieved=achieved, peak=HBM_PEAK_GBS, unit="GB/s",
                    frac=achieved / HBM_PEAK_GBS, traffic=traffic,
                    bytes_per_launch=pf_bytes / max(1, n_launch), launches=n_launch,
                    avg_launch_ms=1e3 * t_pf / max(1, n_launch))
        # the alignment kernel is integer-VALU bound (no MFMA): reported beside the roofline
        align_info = dict(kernel="k_align", seconds_per_step=t_al, gcups_kernel=cells / t_al / 1e9 if t_al else 0,
                          cells_per_step=cells, cells_computed=st["cells_computed"])
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(umis, args.cpu_sample, args.identity, lens)
        out = {
            "metric": METRIC, "value": value, "unit": "UMIs/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": 1e3 * t_max / args.steps, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "int32", "data": "synthetic",
            "config": {"workload": workload,
                       "reads_per_gpu": int(umis.n), "umis_kept_per_gpu": int(n_kept), "clusters": st["n_clusters"],
                       "parallelism": f"{world} independent bins (1 per GPU), no data-path collective"},
            "gcups": gcups,
            "breakdown_s_per_step": {"total": t_max / args.steps, "prefilter_kernels": t_pf, "align_kernels": t_al,
                                     "consensus_kernels": st["t_consensus_s"], "index_kernels": st["t_index_s"],
                                     "host_resolve": st["t_host_s"], "host_pass1": st["t_host_pass1_s"],
                                     "host_wait_d2h": st["t_sync_s"]},
            "merged_walks": st["n_merged_walks"], "t_merged_walks": st["t_merged_s"],
            "deferred_queries": st["n_deferred"], "pairs_round_b": st["pairs_round_b"],
            "pairs_peer": st["pairs_peer"],
            "alignments_per_step": st["n_alignments"],
            "roofline": roof,
            "align": align_info,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
