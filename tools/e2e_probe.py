"""Where the drop-in's file-boundary time goes on the GPU box (measurement only): writes the config-2 bin as a FASTA
with 1,500-nt seq= reads to /dev/shm, then runs umiclust_run_fasta (cluster<N> files + consout) and
umiclust_run_fasta_parse (the fused drop-in) twice each with UMICLUST_DEBUG=1 (phase times on stderr), and
tools/read_probe on the same file.  Usage: python tools/e2e_probe.py <out.json>"""
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ont-tcrconsensus_amd"))
os.environ["UMICLUST_DEBUG"] = "1"
from umiclust import _lib, synth  # noqa: E402

d = tempfile.mkdtemp(prefix="e2e_probe_", dir="/dev/shm")
out = {}
try:
    fa = os.path.join(d, "in.fasta")
    u = synth.config_umis(2, 1.0)
    synth.write_umi_fasta_fast(fa, u, read_len=1500)
    out["fasta_bytes"] = os.path.getsize(fa)
    rp = subprocess.run([os.path.join(ROOT, "tools", "read_probe"), fa, "16"], capture_output=True, text=True)
    out["read_probe"] = [json.loads(x) for x in rp.stdout.splitlines() if x.startswith("{")]
    p = _lib.params(_lib.PRESET_ROUND1, 0.90, 58, 68, threads=25)
    runs = []
    with _lib.Context(0) as ctx:
        for rep in range(2):
            o = os.path.join(d, f"out{rep}")
            os.mkdir(o)
            os.sync()
            t0 = time.perf_counter()
            st = ctx.run_fasta(p, fa, os.path.join(o, "cluster"), os.path.join(o, "umi_clusters_consensus.fasta"),
                               os.path.join(o, "vsearch_cluster.log"))
            runs.append(dict(kind="run_fasta", seconds=time.perf_counter() - t0, t_read_s=st["t_read_s"],
                             t_cluster_s=st["t_total_s"], t_write_s=st["t_write_s"]))
            shutil.rmtree(o)
            w = os.path.join(d, f"work{rep}")
            os.mkdir(w)
            os.sync()
            pp = _lib.ParseParams(min_reads_per_cluster=4, max_reads_per_cluster=60, balance_strands=0, max_clusters=0)
            t0 = time.perf_counter()
            st, pr = ctx.run_fasta_parse(p, fa, None, os.path.join(w, "umi_clusters_consensus.fasta"),
                                         os.path.join(w, "vsearch_cluster.log"), pp, w)
            runs.append(dict(kind="fused", seconds=time.perf_counter() - t0, t_read_s=st["t_read_s"],
                             t_cluster_s=st["t_total_s"], t_write_s=st["t_write_s"]))
            shutil.rmtree(w)
            print(runs[-2:], flush=True)
    out["runs"] = runs
finally:
    shutil.rmtree(d, ignore_errors=True)
json.dump(out, open(sys.argv[1], "w"), indent=1)
