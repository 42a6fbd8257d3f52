"""Bin sharding across ranks on CPU: LPT plan properties and a world_size-2 gloo run
whose per-bin outputs must equal the world_size-1 run (the per-bin worker here is the CPU oracle,
standing in for the GPU so the orchestration can be tested without a device)."""
import os
import socket

import orc
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp
from umiclust import synth
from umiclust.shard import bin_cost, lpt_assign, run_bins


def test_lpt_covers_every_bin_once():
    costs = [bin_cost(n) for n in [5, 100_000, 3, 2_000_000, 70, 70, 1_000]]
    for world in (1, 2, 3, 8):
        plan = lpt_assign(costs, world)
        flat = sorted(i for p in plan for i in p)
        assert flat == list(range(len(costs)))
        assert plan == lpt_assign(costs, world)  # deterministic


def test_lpt_balances():
    costs = [10, 9, 8, 7, 6, 5, 4, 3, 2, 1]
    plan = lpt_assign(costs, 2)
    loads = [sum(costs[i] for i in p) for p in plan]
    assert abs(loads[0] - loads[1]) <= 1


def _make_bins(tmp, kind="small"):
    bins = []
    if kind == "config3":
        # BASELINE config 3's bin structure (Zipf(1.1) sizes over 40 region bins) for two barcodes, scaled
        # down so the oracle worker runs in seconds
        for b in synth.config_bins(3, 0.002, barcodes=[0, 5]):
            fa = os.path.join(tmp, f"bc{b.barcode}_region{b.region}.fasta")
            synth.write_umi_fasta(fa, b.umis)
            bins.append(fa)
        return bins
    for b in range(5):
        u = synth.make_umis(20 + 10 * b, seed=500 + b, max_reads=200 + 100 * b)
        fa = os.path.join(tmp, f"bin{b}.fasta")
        synth.write_umi_fasta(fa, u)
        bins.append(fa)
    return bins


def _worker_factory(outroot):
    def worker(fa, tag):
        out = os.path.join(outroot, tag)
        os.makedirs(out, exist_ok=True)
        r = orc.run_fasta(orc.params(1, 0.93, 58, 68), fa, out + "/cluster", out + "/umi_clusters_consensus.fasta")
        return dict(n_kept=r["kept"], n_clusters=r["n_clusters"])
    return worker


def _rank_main(rank, world, port, tmp, bins):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res = run_bins([(fa, f"bin{i}") for i, fa in enumerate(bins)], _worker_factory(os.path.join(tmp, "w2")),
                   rank, world, gather=dist.all_gather_object)
    if rank == 0:
        import json
        with open(os.path.join(tmp, "res2.json"), "w") as fh:
            json.dump(res, fh)
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(300)
@pytest.mark.parametrize("kind", ["small", "config3"])
def test_two_rank_gloo_matches_single_rank(tmp_path, kind):
    import json
    tmp = str(tmp_path)
    bins = _make_bins(tmp, kind)
    res1 = run_bins([(fa, f"bin{i}") for i, fa in enumerate(bins)], _worker_factory(os.path.join(tmp, "w1")))
    mp.spawn(_rank_main, args=(2, _free_port(), tmp, bins), nprocs=2, join=True)
    res2 = json.load(open(os.path.join(tmp, "res2.json")))
    assert [r for _, r in res1] == res2
    for i in range(len(bins)):
        d1, d2 = os.path.join(tmp, "w1", f"bin{i}"), os.path.join(tmp, "w2", f"bin{i}")
        assert sorted(os.listdir(d1)) == sorted(os.listdir(d2))
        for fn in os.listdir(d1):
            assert open(os.path.join(d1, fn), "rb").read() == open(os.path.join(d2, fn), "rb").read()


def test_config3_lpt_plan_is_balanced():
    """The Zipf(1.1) bin mix of config 3 on 2/4/8 ranks: every bin once, and the LPT makespan within the
    classic 4/3 bound of the ideal (sum / world, or the largest bin)."""
    sizes = synth.zipf_bin_sizes(10_000_000).ravel()
    costs = [bin_cost(int(n)) for n in sizes]
    for world in (2, 4, 8):
        plan = lpt_assign(costs, world)
        assert sorted(i for p in plan for i in p) == list(range(len(costs)))
        span = max(sum(costs[i] for i in p) for p in plan)
        ideal = max(sum(costs) / world, max(costs))
        assert span <= 4 / 3 * ideal
