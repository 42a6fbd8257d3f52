"""shard.py on the device: BASELINE config 3's bin structure (Zipf(1.1) region bins,
two barcodes, reduced scale) through shard.run_bins with the real HIP worker (the reference's vsearch argv
through umiclust_run_argv).  Every bin's files are byte-identical to the CPU oracle's, and a two-rank
run (two processes on the one GPU, gloo for the final gather only) writes byte-identical files."""
import json
import os
import socket

import orc
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp
from umiclust import synth
from umiclust.shard import hip_worker, run_bins

pytestmark = pytest.mark.gpu


def _bins(tmp):
    out = []
    for b in synth.config_bins(3, 0.004, barcodes=[2, 17]):
        fa = os.path.join(tmp, f"bc{b.barcode}_region{b.region}.fasta")
        synth.write_umi_fasta(fa, b.umis)
        out.append((fa, f"bc{b.barcode}/region_cluster{b.region}"))
    return out


def _read_dir(d):
    return {fn: open(os.path.join(d, fn), "rb").read() for fn in sorted(os.listdir(d)) if not fn.endswith(".log")}


def _rank_main(rank, world, port, tmp, bins):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), UMICLUST_DEVICE="0")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    w = hip_worker(1)
    res = run_bins([(fa, os.path.join(tmp, "w2", tag)) for fa, tag in bins], w, rank, world,
                   gather=dist.all_gather_object)
    if rank == 0:
        with open(os.path.join(tmp, "res2.json"), "w") as fh:
            json.dump([(r["n_kept"], r["n_clusters"], r["cells"]) for r in res], fh)
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(600)
def test_config3_bins_through_shard_on_gpu(tmp_path):
    tmp = str(tmp_path)
    bins = _bins(tmp)
    w = hip_worker(1)
    res1 = run_bins([(fa, os.path.join(tmp, "w1", tag)) for fa, tag in bins], w)
    assert len(res1) == len(bins)
    op = orc.params(1, 0.93, 58, 68)
    op.threads, op.policy_threads = 25, 1  # the worker's argv carries --threads 25 (vsearch's multithreaded mode)
    for fa, tag in bins:
        ref = os.path.join(tmp, "oracle", tag)
        os.makedirs(ref)
        orc.run_fasta(op, fa, ref + "/cluster", os.path.join(ref, "umi_clusters_consensus.fasta"))
        assert _read_dir(os.path.join(tmp, "w1", tag)) == _read_dir(ref), tag
    mp.spawn(_rank_main, args=(2, _free_port(), tmp, bins), nprocs=2, join=True)
    res2 = json.load(open(os.path.join(tmp, "res2.json")))
    assert [[r["n_kept"], r["n_clusters"], r["cells"]] for _, r in sorted(res1, key=lambda x: x[0])] == res2
    for _, tag in bins:
        assert _read_dir(os.path.join(tmp, "w1", tag)) == _read_dir(os.path.join(tmp, "w2", tag)), tag


@pytest.mark.timeout(600)
def test_bench_two_ranks_partition_and_digests(tmp_path):
    """bench.py's own N-rank path: `--gpus 2` relaunches itself through torch.distributed.run,
    the ranks rendezvous over gloo (no RCCL communicator: the only cross-rank operations are a barrier and two
    host-scalar reductions), each rank clusters its LPT share of config 3's 960 bins (both ranks on device 0 here).
    The ranks' shares partition the bins, the JSON line reports n_gpus 2, and the per-bin digests, put back in bin
    order, equal the O4 oracle golden of the whole set (tests/golden/oracle_o4.json config3_bins_s001_o4T25)."""
    import subprocess
    import sys
    from umiclust import binset
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    gold = json.load(open(os.path.join(root, "tests", "golden", "oracle_o4.json")))["config3_bins_s001_o4T25"]
    dg = str(tmp_path / "dg")
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--config", "3", "--scale",
                        str(gold["scale"]), "--steps", "1", "--warmup", "0", "--ranks-share-device", "--digest-out", dg,
                        "--no-cpu-baseline"], capture_output=True, text=True, timeout=540, env=env, cwd=root)
    assert p.returncode == 0, p.stderr[-4000:]
    line = json.loads([x for x in p.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["value"] > 0 and line["scaling"] == "strong"
    ranks = [json.load(open(f"{dg}.rank{r}.json")) for r in range(2)]
    b0, b1 = set(ranks[0]["bins"]), set(ranks[1]["bins"])
    assert not (b0 & b1) and b0 | b1 == set(range(gold["n_bins"])) and b0 and b1
    per_bin = {**ranks[0]["rounds"][0], **ranks[1]["rounds"][0]}
    dgs = [per_bin[str(b)] for b in range(gold["n_bins"])]
    assert [d["n_clusters"] for d in dgs] == gold["round1"]["n_clusters"]
    assert binset.combine(dgs) == gold["round1"]["combined"]
