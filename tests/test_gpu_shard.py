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
