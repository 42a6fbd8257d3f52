"""Multi-GPU execution of many region bins.

Every (library x region bin) is an independent vsearch invocation in the reference
(/root/reference/ont_tcr_consensus/tcr_consensus.py:231-245 round 1, :411-427 round 2), with its own
input FASTA and output directory, so bins shard across GPUs with no data exchange: one process per
GPU (`torch.distributed.run --nproc-per-node N`), a deterministic LPT assignment that every rank
computes identically, each rank clusters its bins on its own device, and a final gather of per-bin
statistics (host objects only; no RCCL collective on the data path).  Outputs are per-bin files, so
they are byte-identical for any number of GPUs.

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        -m umiclust.shard --round 1 --identity 0.93 in1.fa:out1 in2.fa:out2 ...
"""
from __future__ import annotations

import argparse
import os
from typing import Callable, Sequence


def bin_cost(n_reads: int, reads_per_molecule: float = 20.0) -> float:
    """Cost model of one bin: prefilter ~ N * C (C ~ N / reads_per_molecule centroids) plus
    alignment ~ N * 64^2 cells."""
    n = float(n_reads)
    return n * n / reads_per_molecule + n * 64.0 * 64.0


def lpt_assign(costs: Sequence[float], world: int) -> list[list[int]]:
    """Longest-processing-time-first: bins by cost desc (ties: lower index), each to the least
    loaded rank (ties: lower rank).  Deterministic, so every rank derives the same plan."""
    if world < 1:
        raise ValueError("world must be >= 1")
    order = sorted(range(len(costs)), key=lambda i: (-costs[i], i))
    load = [0.0] * world
    plan: list[list[int]] = [[] for _ in range(world)]
    for i in order:
        r = min(range(world), key=lambda k: (load[k], k))
        plan[r].append(i)
        load[r] += costs[i]
    for p in plan:
        p.sort()
    return plan


def count_fasta_records(path: str) -> int:
    n = 0
    with open(path, "rb") as fh:
        for line in fh:
            n += line.startswith(b">")
    return n


def run_bins(bins: Sequence[tuple[str, str]], worker: Callable[[str, str], dict], rank: int = 0,
             world: int = 1, costs: Sequence[float] | None = None, gather: Callable | None = None) -> list:
    """Run `worker(in_fasta, out_dir) -> stats` on this rank's share of `bins`; if `gather` (e.g.
    torch.distributed.all_gather_object) is given, return every rank's results in bin order."""
    if costs is None:
        costs = [bin_cost(count_fasta_records(b[0])) for b in bins]
    plan = lpt_assign(costs, world)
    mine = [(i, worker(*bins[i])) for i in plan[rank]]
    if gather is None:
        return mine
    allres = [None] * world
    gather(allres, mine)
    out = [None] * len(bins)
    for part in allres:
        for i, st in part:
            out[i] = st
    return out


def hip_worker(round_: int = 1, identity: float | None = None, min_len: int = 58, max_len: int = 68,
               threads: int = 25):
    """The per-bin worker on this process's GPU: the reference's exact vsearch argv for the round
    (vsearch_umi_cluster.py:22-53 / :72-96) through umiclust_run_argv; returns the bin's stats.  threads = the
    argv's --threads (the reference passes max(cpus // bins, 25), utils.py:56-63; > 1 = vsearch's multithreaded
    clustering, policy O4)."""
    from . import vsearch_umi_cluster as v
    ident = identity if identity is not None else (0.93 if round_ == 1 else 0.97)
    fn = v.round1_argv if round_ == 1 else v.round2_argv

    def worker(fa, out):
        os.makedirs(out, exist_ok=True)
        st = v.context().run_argv(fn(fa, out, threads, min_len, max_len, ident))
        return dict(n_kept=int(st["n_kept"]), n_clusters=int(st["n_clusters"]), cells=int(st["cells"]),
                    seconds=float(st["t_run_s"]))
    return worker


def _main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--round", type=int, default=1, choices=(1, 2))
    ap.add_argument("--identity", type=float, default=None)
    ap.add_argument("--min-len", type=int, default=58)
    ap.add_argument("--max-len", type=int, default=68)
    ap.add_argument("bins", nargs="+", help="in_fasta:out_dir")
    a = ap.parse_args()
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group(backend="gloo")  # host objects only: the data path has no collective
    os.environ.setdefault("UMICLUST_DEVICE", os.environ.get("LOCAL_RANK", "0"))
    worker = hip_worker(a.round, a.identity, a.min_len, a.max_len)
    bins = [tuple(b.split(":", 1)) for b in a.bins]
    res = run_bins(bins, worker, rank, world, gather=dist.all_gather_object if world > 1 else None)
    if rank == 0:
        tot = sum(r["n_kept"] for r in res if r)
        print(f"clustered {tot} UMIs in {len(bins)} bins on {world} GPU(s)")
    if world > 1:
        dist.destroy_process_group()
    del torch


if __name__ == "__main__":
    _main()
