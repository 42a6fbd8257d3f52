"""Generate tests/golden/region_split/*.json from the REFERENCE itself (run here, not on the GPU box): inputs
and outputs of filter_and_split_reads_by_region_cluster (/root/reference/ont_tcr_consensus/region_split.py:
219-333).

pysam is not installed (ordinary ModuleNotFoundError): pysam.AlignmentFile is replaced by the
BAM reader of oracle/bam.py (SAM/BAM specification restated) and pysam.FastxFile by make_golden.py's FASTA
iterator.  The BAM inputs are written by oracle/bam.py from the records stored in the fixture, so the fixture
holds data only (records, reference regions, parameters, output files).

Usage: python tests/golden/make_golden_region_split.py  (requires /root/reference)
"""
from __future__ import annotations

import json
import os
import random
import shutil
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [HERE, os.path.join(ROOT, "oracle")]
import bam  # noqa: E402
import make_golden  # noqa: E402


def make_case(rng, name, n_regions, n_reads, minimal_region_overlap=0.95, s5=73, s3=68, pre_existing=False,
              unknown_ref=False, no_cigar_at=None):
    regions = []
    for r in range(n_regions):
        suffix = rng.choice(["", "", "", "_v_n", "cdr3j_n", "full_n"]) if r > 1 else ""
        regions.append((f"TRBV{r}_{rng.randint(1, 99)}{suffix}", rng.randint(300, 700)))
    clusters = {}
    k = 0
    for nm, _ in regions:  # some regions share a cluster (the homology clustering's output)
        if clusters and rng.random() < 0.3:
            clusters[nm] = rng.choice(list(clusters.values()))
        else:
            clusters[nm] = k
            k += 1
    refs = list(regions)
    if unknown_ref:
        refs.append(("not_in_reference", 500))
    records = []
    for i in range(n_reads):
        ref = rng.randrange(len(refs))
        rlen = refs[ref][1]
        kind = rng.random()
        flag = 0
        if kind < 0.05:
            flag = 4
        elif kind < 0.1:
            flag = 256
        elif kind < 0.13:
            flag = 2048
        if rng.random() < 0.5:
            flag |= 16
        aln = int(rlen * rng.choice([1.0, 0.99, 0.97, 0.96, 0.9, 0.6])) if flag & 4 == 0 else 0
        clip5, clip3 = rng.randint(0, 90), rng.randint(0, 80)
        extra = rng.choice([0, 0, 0, 5, rlen])  # an occasional far-too-long read
        cigar = ([("S", clip5)] if clip5 else []) + [("M", aln + extra)] + ([("S", clip3)] if clip3 else []) \
            if aln else []
        if aln and rng.random() < 0.3:
            cigar = cigar[:-1] + [("D", 3), ("I", 2)] + cigar[-1:]
        qlen = sum(ln for op, ln in cigar if op in "MIS=X") if cigar else rng.randint(50, 300)
        alpha = "ACGTN" if rng.random() < 0.1 else "ACGT"
        seq = "".join(rng.choice(alpha) for _ in range(qlen))
        if flag & 256 and rng.random() < 0.5:
            seq = ""  # secondary without a stored sequence
        records.append(dict(name=f"read{i:05d}", flag=flag, ref=ref if not flag & 4 or rng.random() < 0.5 else -1,
                            pos=rng.randint(0, 20), cigar=cigar, seq=seq))
        if i == no_cigar_at:  # a mapped primary record without a CIGAR: reference_length 1 (htslib bam_endpos)
            records[-1].update(flag=16, ref=0, cigar=[])
    pre = {}
    if pre_existing:  # the reference appends to region_cluster<k>.fasta
        pre = {f"region_cluster{clusters[regions[0][0]]}.fasta": ">old;strand=+\nACGT\n"}
    return dict(name=name, regions=regions, refs=refs, clusters=clusters, records=records, pre_existing=pre,
                minimal_region_overlap=minimal_region_overlap, max_softclip_5_end=s5, max_softclip_3_end=s3)


def write_inputs(case, d):
    """BAM, reference FASTA, cluster JSON, output dir (with any pre-existing files), logs dir."""
    os.makedirs(d, exist_ok=True)
    bam_path = os.path.join(d, "barcode07.sorted.bam")
    bam.write_bam(bam_path, [tuple(r) for r in case["refs"]], case["records"])
    ref_fa = os.path.join(d, "reference.fa")
    rng = random.Random(len(case["regions"]))
    with open(ref_fa, "w") as fh:
        for nm, ln in case["regions"]:
            s = "".join(rng.choice("ACGT") for _ in range(ln))
            fh.write(f">{nm}\n" + "\n".join(s[i:i + 60] for i in range(0, ln, 60)) + "\n")
    js = os.path.join(d, "region_cluster_dict.json")
    with open(js, "w") as fh:
        json.dump(case["clusters"], fh)
    out = os.path.join(d, "out")
    logs = os.path.join(d, "logs")
    os.makedirs(out)
    os.makedirs(logs)
    for fn, txt in case["pre_existing"].items():
        with open(os.path.join(out, fn), "w") as fh:
            fh.write(txt)
    return bam_path, ref_fa, js, out, logs


def run_reference(mod, case):
    tmp = tempfile.mkdtemp(prefix="rs_")
    try:
        bam_path, ref_fa, js, out, logs = write_inputs(case, tmp)
        res = dict(case)
        try:
            ret = mod.filter_and_split_reads_by_region_cluster(
                bam_file=bam_path, region_cluster_dict_json=js, reference=ref_fa, logs_dir=logs,
                region_fasta_out_dir=out, minimal_region_overlap=case["minimal_region_overlap"],
                max_softclip_5_end=case["max_softclip_5_end"], max_softclip_3_end=case["max_softclip_3_end"])
            res["result"] = sorted(os.path.relpath(p, tmp) for p in ret)
            res["error"] = None
        except KeyError as e:
            res["result"] = None
            res["error"] = f"KeyError: {e}"
        except TypeError as e:  # None < float: a mapped primary record without a CIGAR
            res["result"] = None
            res["error"] = f"TypeError: {e}"
        res["out_files"] = {fn: open(os.path.join(out, fn)).read() for fn in sorted(os.listdir(out))}
        res["log_files"] = {fn: open(os.path.join(logs, fn)).read() for fn in sorted(os.listdir(logs))}
        return res
    finally:
        shutil.rmtree(tmp)


def main():
    make_golden._stub_modules()
    sys.modules["pysam"].AlignmentFile = bam.AlignmentFile
    mod = make_golden._load("region_split")
    rng = random.Random(20261016)
    cases = [make_case(rng, "small", 6, 150), make_case(rng, "many_regions", 30, 500),
             make_case(rng, "loose_overlap", 8, 250, minimal_region_overlap=0.5, s5=10, s3=10),
             make_case(rng, "append_existing", 5, 150, pre_existing=True),
             make_case(rng, "unknown_reference", 5, 150, unknown_ref=True),
             make_case(rng, "no_cigar", 5, 150, no_cigar_at=97)]
    od = os.path.join(HERE, "region_split")
    os.makedirs(od, exist_ok=True)
    for c in cases:
        r = run_reference(mod, c)
        with open(os.path.join(od, c["name"] + ".json"), "w") as fh:
            json.dump(r, fh, indent=0, sort_keys=True)
        print(c["name"], r["result"], r["error"], list(r["log_files"]))


if __name__ == "__main__":
    main()
