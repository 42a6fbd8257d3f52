"""Consumer of the hot path's files: behaviour-for-behaviour counterpart of
/root/reference/ont_tcr_consensus/parse_umi_clusters.py.

It reads `umi_clusters_consensus.fasta` in file order, takes each record's cluster id from the
last `;` field (`clusterid=<N>`, :197-200), opens `<dir>/cluster<N>` and writes
`clusters_fa/cluster<N>.fasta`, `smolecule_clusters.fa`, `vsearch_cluster_stats.tsv` and
`parse_cluster.log` byte-for-byte like the reference, including its quirks:
the per-cluster return value overwrites the running read totals (:206, :220-221), so the log's
"Reads: X found" reports the last cluster's count and the empty-region test uses it.

pysam is not required: records are read with a minimal FASTA reader whose `name` is the header up
to the first whitespace and `sequence` the concatenated sequence lines (pysam.FastxFile's view).
"""
from __future__ import annotations

import collections
import json
import os
from typing import Iterator, NamedTuple, TextIO, Union


class FastaRecord(NamedTuple):
    name: str
    sequence: str


def read_fasta(path: Union[str, os.PathLike[str]]) -> Iterator[FastaRecord]:
    name = None
    parts: list[str] = []
    with open(path) as fh:
        for line in fh:
            line = line.rstrip("\r\n")
            if line.startswith(">"):
                if name is not None:
                    yield FastaRecord(name, "".join(parts))
                hdr = line[1:]
                name = hdr.split(None, 1)[0] if hdr.split() else ""
                parts = []
            elif name is not None:
                parts.append(line.strip())
    if name is not None:
        yield FastaRecord(name, "".join(parts))


def _strand_caps(n_fwd: int, n_rev: int, min_reads: int, max_reads: int, balance: bool):
    """Per-strand minimum and maximum read counts (parse_umi_clusters.py:66-87)."""
    if balance:
        half_min = int(min_reads / 2)
        capped = min(n_fwd * 2, n_rev * 2, max_reads)
        return half_min, half_min, int(capped / 2), int(capped / 2)
    if n_fwd > n_rev:
        max_rev = min(n_rev, int(max_reads / 2))
        return 0, 0, min(max_reads - max_rev, n_fwd), max_rev
    max_fwd = min(n_fwd, int(max_reads / 2))
    return 0, 0, max_fwd, min(max_reads - max_fwd, n_rev)


def polish_cluster(
    id_cluster: int,
    clustering_out_dir: Union[str, os.PathLike[str]],
    polish_cluster_out_dir: Union[str, os.PathLike[str]],
    stat_out: TextIO,
    smolecule_out: TextIO,
    logging_str: str,
    min_reads_per_cluster: int = 20,
    max_reads_per_cluster: int = 60,
    balance_strands: bool = False,
    cons_umi: str = None,
):
    """One cluster file -> capped per-strand read sets (parse_umi_clusters.py:10-140)."""
    out_fasta = os.path.join(polish_cluster_out_dir, f"cluster{id_cluster}.fasta")
    kept = {"+": {}, "-": {}}
    seen = {"+": 0, "-": 0}
    found = 0
    for rec in read_fasta(os.path.join(clustering_out_dir, f"cluster{id_cluster}")):
        fields = rec.name.split(";")
        if len(fields) != 7:
            raise Exception(id_cluster, "cluster fasta entry header has", len(fields),
                            "cols while it should contain 7!", rec.name, fields)
        strand = fields[1].split("strand=")[1]
        found += 1
        if strand not in kept:
            raise Exception("Strand annotation is", strand, "but only - or + are allowed!")
        # the first max_reads_per_cluster reads of each strand, keyed (and de-duplicated) by read id
        if seen[strand] < max_reads_per_cluster:
            kept[strand][fields[0]] = rec
        seen[strand] += 1
    n_fwd, n_rev = seen["+"], seen["-"]
    min_fwd, min_rev, max_fwd, max_rev = _strand_caps(n_fwd, n_rev, min_reads_per_cluster,
                                                      max_reads_per_cluster, balance_strands)
    n_reads = max_fwd + max_rev
    if n_reads > max_reads_per_cluster:
        raise Exception("n_reads is higher than max_reads_per_cluster! max_fwd and max_rev calculation is incorrect!")
    logging_str += f"Cluster: {out_fasta} has {n_fwd}/{max_fwd} fwd and {n_rev}/{max_rev} rev reads\n"
    if n_fwd >= min_fwd and n_rev >= min_rev and n_reads >= min_reads_per_cluster:
        fwd = list(kept["+"].values())[:max_fwd]
        rev = list(kept["-"].values())[:max_rev]
        chosen = (fwd + rev)[:max_reads_per_cluster]
        w_fwd, w_rev, w_all, written = len(fwd), len(rev), len(chosen), 1
        lines = []
        for rec in chosen:
            fields = rec.name.split(";")
            read = fields[6].split("seq=")[1]
            lines.append(f">{fields[0]}\n{read}\n")
            if smolecule_out:
                smolecule_out.write(f">{id_cluster}\n{read}\n")
        with open(out_fasta, "w") as fh:
            fh.write("".join(lines))
    else:
        w_fwd = w_rev = w_all = written = 0
        logging_str += f"Cluster {id_cluster} skipped\n"
    logging_str += f"Cluster: {out_fasta} has {w_all} reads written: {w_fwd} fwd - {w_rev} rev\n"
    stat_out.write("\t".join(str(x) for x in (f"cluster{id_cluster}", n_fwd, n_rev, w_fwd, w_rev, found,
                                              w_all, written)) + "\n")
    return written, found, w_all, logging_str


def _parse_umi_clusters(
    consensus_umi_fasta: Union[str, os.PathLike[str]],
    regions_wo_clusters_txt: Union[str, os.PathLike[str]],
    min_reads_per_cluster: int = 20,
    max_reads_per_cluster: int = 60,
    region_cluster_dict_json: Union[str, os.PathLike[str]] = None,
    balance_strands: bool = False,
    max_clusters: int = None,
):
    """consout -> smolecule FASTA + stats + log (parse_umi_clusters.py:143-242)."""
    by_cluster = None
    if region_cluster_dict_json:
        with open(region_cluster_dict_json) as fh:
            mapping = json.load(fh)
        by_cluster = collections.defaultdict(list)
        for region, rc in mapping.items():
            by_cluster[rc].append(region)
    work_dir = os.path.dirname(consensus_umi_fasta)
    region = os.path.basename(work_dir)
    fa_dir = os.path.join(work_dir, "clusters_fa")
    smolecule_fa = os.path.join(work_dir, "smolecule_clusters.fa")
    if os.path.exists(fa_dir):
        raise Exception(fa_dir, "should not exist yet but does exist!")
    os.mkdir(fa_dir)
    n_clusters = sum(1 for _ in read_fasta(consensus_umi_fasta))
    n_written = reads_found = reads_written = 0
    log = ""
    with open(os.path.join(work_dir, "vsearch_cluster_stats.tsv"), "w") as stats, \
            open(smolecule_fa, "w") as smol:
        stats.write("id_cluster\tn_fwd\tn_rev\twritten_fwd\twritten_rev\tn\twritten\tcluster_written\n")
        for rec in read_fasta(consensus_umi_fasta):
            cid = int(rec.name.split(";")[-1].split("=")[1])
            written, reads_found, reads_written, log = polish_cluster(
                id_cluster=cid, clustering_out_dir=work_dir, polish_cluster_out_dir=fa_dir, logging_str=log,
                min_reads_per_cluster=min_reads_per_cluster, max_reads_per_cluster=max_reads_per_cluster,
                stat_out=stats, smolecule_out=smol, balance_strands=balance_strands, cons_umi=None)
            n_written += written
            # reference quirk (:219-221): the running totals are overwritten, then doubled
            reads_found += reads_found
            reads_written += reads_written
            if max_clusters and n_written > max_clusters:
                break
    if n_written == 0 or reads_found == 0:
        with open(regions_wo_clusters_txt, "a") as fh:
            if region_cluster_dict_json:
                fh.write(f"{region} {by_cluster[int(region.split('region_cluster')[1])]}\n")
            else:
                fh.write(f"{region}\n")
        return None
    log += f"Clusters: {int(n_written * 100.0 / n_clusters)}% written ({n_written})\n"
    log += f"Reads: {reads_found} found\n"
    log += f"Reads: {int(reads_written * 100.0 / reads_found)}% in written clusters\n"
    if log:
        with open(os.path.join(work_dir, "parse_cluster.log"), "w") as fh:
            fh.write(log)
    return smolecule_fa


def _append_empty_region(regions_wo_clusters_txt, work_dir, region_cluster_dict_json) -> None:
    """parse_umi_clusters.py:224-231: record a region that produced no written cluster."""
    region = os.path.basename(work_dir)
    with open(regions_wo_clusters_txt, "a") as fh:
        if region_cluster_dict_json:
            with open(region_cluster_dict_json) as jf:
                mapping = json.load(jf)
            by_cluster = collections.defaultdict(list)
            for reg, rc in mapping.items():
                by_cluster[rc].append(reg)
            fh.write(f"{region} {by_cluster[int(region.split('region_cluster')[1])]}\n")
        else:
            fh.write(f"{region}\n")


def _vsearch_cluster_and_parse(
    umi_fasta: Union[str, os.PathLike[str]],
    clustering_out_dir: Union[str, os.PathLike[str]],
    threads: int,
    regions_wo_clusters_txt: Union[str, os.PathLike[str]],
    min_umi_length: int = 50,
    max_umi_length: int = 60,
    identity: float = 0.94,
    min_reads_per_cluster: int = 20,
    max_reads_per_cluster: int = 60,
    region_cluster_dict_json: Union[str, os.PathLike[str]] = None,
    balance_strands: bool = False,
    max_clusters: int = None,
    round_: int = 1,
    write_cluster_files: bool = True,
):
    """`vsearch_cluster` (round_=1) or `vsearch_cluster_consensus` (round_=2) followed by
    `parse_umi_clusters` on its consout (tcr_consensus.py:237-265 round 1, :419-444 round 2), fused:
    the consumer's outputs (clusters_fa/, smolecule_clusters.fa, vsearch_cluster_stats.tsv,
    parse_cluster.log) are written by the native library straight from the in-memory clusters, byte-
    identical to the two-step path.  With write_cluster_files=False the per-cluster `cluster<N>` files,
    which the consumer only re-reads, are skipped.  Returns the
    smolecule_clusters.fa path, or None for a region without written clusters, like parse_umi_clusters."""
    from . import _lib
    from .vsearch_umi_cluster import context, round1_argv, round2_argv
    build = round1_argv if round_ == 1 else round2_argv
    argv = build(os.fspath(umi_fasta), os.fspath(clustering_out_dir), threads, min_umi_length, max_umi_length,
                 identity)
    p, paths = _lib.params_from_argv(argv)
    pp = _lib.ParseParams(min_reads_per_cluster, max_reads_per_cluster, int(bool(balance_strands)),
                          int(max_clusters) if max_clusters else 0)
    work_dir = os.path.dirname(paths["consout"])
    _, res = context().run_fasta_parse(p, paths["in_fasta"], paths["clusters_prefix"] if write_cluster_files else None,
                                       paths["consout"], paths["log"], pp, work_dir)
    if res["empty_region"]:
        _append_empty_region(regions_wo_clusters_txt, work_dir, region_cluster_dict_json)
        return None
    return os.path.join(work_dir, "smolecule_clusters.fa")


try:  # pragma: no cover - ray is not installed in this image
    import ray as _ray

    parse_umi_clusters = _ray.remote(_parse_umi_clusters)
    vsearch_cluster_and_parse = _ray.remote(_vsearch_cluster_and_parse)
except ImportError:
    from .vsearch_umi_cluster import _LocalRemote

    parse_umi_clusters = _LocalRemote(_parse_umi_clusters)
    vsearch_cluster_and_parse = _LocalRemote(_vsearch_cluster_and_parse)
