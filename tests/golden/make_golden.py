"""Generate the committed golden fixtures from the REFERENCE itself (run here, not on the GPU box).

  * tests/golden/parse/*.json: inputs (consout + cluster<N> files + arguments) and the exact files
    /root/reference/ont_tcr_consensus/parse_umi_clusters.py writes for them.
  * tests/golden/argv.json: the exact vsearch argv vsearch_umi_cluster.py builds for both rounds
    (captured by stubbing subprocess.run).

`ray` and `pysam` are not installed (ordinary ModuleNotFoundError); they are
replaced by minimal stand-ins that execute nothing from the reference's data: ray.remote is a
pass-through decorator, pysam.FastxFile a FASTA iterator yielding .name (header up to the first
whitespace) and .sequence.  Only data (inputs and outputs) is written to the fixtures.

Usage: python tests/golden/make_golden.py  (requires /root/reference)
"""
from __future__ import annotations

import importlib.util
import json
import os
import random
import shutil
import subprocess
import sys
import tempfile
import types

REF = "/root/reference/ont_tcr_consensus"
HERE = os.path.dirname(os.path.abspath(__file__))


def _stub_modules():
    ray = types.ModuleType("ray")
    ray.remote = lambda *a, **k: (a[0] if a and callable(a[0]) else (lambda f: f))
    sys.modules["ray"] = ray

    pysam = types.ModuleType("pysam")

    class _Rec:
        def __init__(self, name, seq):
            self.name = name
            self.sequence = seq

    class FastxFile:
        def __init__(self, path):
            self.path = path

        def __enter__(self):
            return self

        def __exit__(self, *a):
            return False

        def __iter__(self):
            name, parts = None, []
            with open(self.path) as fh:
                for line in fh:
                    line = line.rstrip("\n")
                    if line.startswith(">"):
                        if name is not None:
                            yield _Rec(name, "".join(parts))
                        name, parts = line[1:].split()[0] if line[1:].split() else "", []
                    elif name is not None:
                        parts.append(line.strip())
            if name is not None:
                yield _Rec(name, "".join(parts))

    pysam.FastxFile = FastxFile
    pysam.libcfaidx = types.SimpleNamespace(FastxRecord=_Rec)
    sys.modules["pysam"] = pysam


def _load(name):
    spec = importlib.util.spec_from_file_location(f"ref_{name}", os.path.join(REF, name + ".py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _header(rid, strand, rng):
    u = "".join(rng.choice("ACGT") for _ in range(64))
    read = "".join(rng.choice("ACGT") for _ in range(rng.randint(20, 40)))
    return (f"{rid};strand={strand};umi_fwd_dist={rng.randint(0, 3)};umi_rev_dist={rng.randint(0, 3)};"
            f"umi_fwd_seq={u[:32]};umi_rev_seq={u[32:]};seq={read}"), u


def make_case(rng, n_clusters, strands_per_cluster, dup_ids=False):
    clusters, cons = {}, []
    order = list(range(n_clusters))
    rng.shuffle(order)  # consout order need not be id order
    for cid in range(n_clusters):
        lines = []
        for k, st in enumerate(strands_per_cluster[cid]):
            rid = f"r{cid}_{k if not dup_ids else k // 2}"
            h, u = _header(rid, st, rng)
            lines.append(f">{h}\n{u}\n")
        clusters[f"cluster{cid}"] = "".join(lines)
    for cid in order:
        cons.append(f">centroid=x{cid};seqs={len(strands_per_cluster[cid])};clusterid={cid}\n"
                    + "".join(rng.choice("ACGT") for _ in range(64)) + "\n")
    return clusters, "".join(cons)


def run_parse(parse_mod, clusters, consout, args, region="region_cluster3", region_json=None):
    tmp = tempfile.mkdtemp(prefix="golden_")
    try:
        d = os.path.join(tmp, region)
        os.mkdir(d)
        for fn, text in clusters.items():
            with open(os.path.join(d, fn), "w") as fh:
                fh.write(text)
        cpath = os.path.join(d, "umi_clusters_consensus.fasta")
        with open(cpath, "w") as fh:
            fh.write(consout)
        wo = os.path.join(tmp, "regions_wo_clusters.txt")
        kw = dict(args)
        if region_json is not None:
            jp = os.path.join(tmp, "region_split_dict.json")
            with open(jp, "w") as fh:
                json.dump(region_json, fh)
            kw["region_cluster_dict_json"] = jp
        ret = parse_mod.parse_umi_clusters(cpath, wo, **kw)
        files = {}
        for root, _dirs, fns in os.walk(d):
            for fn in fns:
                p = os.path.join(root, fn)
                rel = os.path.relpath(p, d)
                if rel in clusters or rel == "umi_clusters_consensus.fasta":
                    continue
                with open(p) as fh:
                    files[rel] = fh.read().replace(d, "{DIR}")
        wo_text = open(wo).read() if os.path.exists(wo) else None
        return dict(returned=None if ret is None else os.path.relpath(ret, d), files=files, regions_wo=wo_text)
    finally:
        shutil.rmtree(tmp)


def main():
    _stub_modules()
    parse_mod = _load("parse_umi_clusters")
    rng = random.Random(20251015)
    cases = []
    # 1. SURVEY §8c example: cluster0 strands ++-+-, cluster1 one read, min 1 max 4
    cl, co = make_case(rng, 2, [list("++-+-"), list("+")])
    cases.append(("survey_example", cl, co, dict(min_reads_per_cluster=1, max_reads_per_cluster=4), None))
    # 2. reference round-1 settings (config: 4 / 60 / balance false) with caps hit
    strands = [["+"] * 70 + ["-"] * 3, ["-"] * 40 + ["+"] * 45, ["+", "-", "+"], ["-"] * 5, ["+"] * 2]
    cl, co = make_case(rng, 5, strands)
    cases.append(("round1_caps", cl, co, dict(min_reads_per_cluster=4, max_reads_per_cluster=60), None))
    # 3. balance_strands true
    cl, co = make_case(rng, 5, strands)
    cases.append(("balance", cl, co, dict(min_reads_per_cluster=4, max_reads_per_cluster=60,
                                          balance_strands=True), None))
    # 4. round-2 settings (min 1, balance false)
    cl, co = make_case(rng, 4, [list("+-"), list("-"), list("++++"), list("-+-+-+")])
    cases.append(("round2", cl, co, dict(min_reads_per_cluster=1, max_reads_per_cluster=60), None))
    # 5. nothing written -> regions_wo_clusters
    cl, co = make_case(rng, 3, [list("+"), list("-"), list("+-")])
    cases.append(("none_written", cl, co, dict(min_reads_per_cluster=20, max_reads_per_cluster=60), None))
    # 6. nothing written + region json
    cl, co = make_case(rng, 2, [list("+"), list("-")])
    cases.append(("none_written_json", cl, co, dict(min_reads_per_cluster=20, max_reads_per_cluster=60),
                  {"TRBV1": 3, "TRBV2": 3, "TRBV9": 1}))
    # 7. max_clusters break
    cl, co = make_case(rng, 6, [list("++--")] * 6)
    cases.append(("max_clusters", cl, co, dict(min_reads_per_cluster=1, max_reads_per_cluster=60,
                                               max_clusters=2), None))
    # 8. duplicate read ids within a cluster
    cl, co = make_case(rng, 2, [list("++++--"), list("+-+-")], dup_ids=True)
    cases.append(("dup_ids", cl, co, dict(min_reads_per_cluster=1, max_reads_per_cluster=3), None))
    # 9-12. random
    for r in range(4):
        n = rng.randint(3, 12)
        strands = [[rng.choice("+-") for _ in range(rng.randint(1, 90))] for _ in range(n)]
        args = dict(min_reads_per_cluster=rng.choice([1, 4, 20]), max_reads_per_cluster=rng.choice([4, 60]),
                    balance_strands=rng.random() < 0.5)
        cl, co = make_case(rng, n, strands)
        cases.append((f"random{r}", cl, co, args, None))
    os.makedirs(os.path.join(HERE, "parse"), exist_ok=True)
    for name, cl, co, args, rj in cases:
        out = run_parse(parse_mod, cl, co, args, region_json=rj)
        with open(os.path.join(HERE, "parse", f"{name}.json"), "w") as fh:
            json.dump(dict(name=name, inputs=dict(clusters=cl, consout=co, args=args, region="region_cluster3",
                                                  region_json=rj), outputs=out), fh, indent=1, sort_keys=True)

    # vsearch argv of both rounds, captured from the reference module
    captured = []
    real_run = subprocess.run
    subprocess.run = lambda argv, *a, **k: captured.append(list(argv))
    try:
        vmod = _load("vsearch_umi_cluster")
        r1 = vmod.vsearch_cluster("in.fa", "/tmp/out", 25, 58, 68, 0.93)
        r2 = vmod.vsearch_cluster_consensus("in2.fa", "/tmp/out2", 25, 58, 68, 0.97)
        r3 = vmod.vsearch_cluster("x.fa", "/tmp/o3", 8)  # defaults 50/60/0.94
        r4 = vmod.vsearch_cluster_consensus("y.fa", "/tmp/o4", 8)  # defaults 50/60/0.97
    finally:
        subprocess.run = real_run
    with open(os.path.join(HERE, "argv.json"), "w") as fh:
        json.dump(dict(calls=[
            dict(fn="vsearch_cluster", args=["in.fa", "/tmp/out", 25, 58, 68, 0.93], argv=captured[0], ret=r1),
            dict(fn="vsearch_cluster_consensus", args=["in2.fa", "/tmp/out2", 25, 58, 68, 0.97], argv=captured[1],
                 ret=r2),
            dict(fn="vsearch_cluster", args=["x.fa", "/tmp/o3", 8], argv=captured[2], ret=r3),
            dict(fn="vsearch_cluster_consensus", args=["y.fa", "/tmp/o4", 8], argv=captured[3], ret=r4),
        ]), fh, indent=1)
    print(f"wrote {len(cases)} parse fixtures and argv.json")


if __name__ == "__main__":
    main()
