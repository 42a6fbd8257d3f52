"""Drop-in for filter_and_split_reads_by_region_cluster of /root/reference/ont_tcr_consensus/region_split.py
(:219-333): the region binning that produces the hot path's shards.

Same signature, defaults, files (append-mode region_cluster<k>.fasta, the
<bam>_filter_and_split_reads_by_region_cluster.err log) and return value (the list of cluster FASTA paths, a
set's order).  The BAM record loop runs in the library (umiclust_region_split: BGZF inflated on the host
threads, records classified and FASTA records built on the GPU); the log is formatted here with the same
Python expressions as the reference.  No CPU fallback.
"""
from __future__ import annotations

import collections
import json
import os
from typing import Union

import numpy as np

from . import vsearch_umi_cluster as _v

NEGATIVE_CONTROL_SUFFIXES = ("_v_n", "cdr3j_n", "full_n")  # region_split.py:305


def _fasta_entries(path):
    """(name, sequence) of a FASTA file as pysam.FastxFile yields them (name = header up to whitespace)."""
    name, parts = None, []
    with open(path) as fh:
        for line in fh:
            line = line.rstrip("\n")
            if line.startswith(">"):
                if name is not None:
                    yield name, "".join(parts)
                toks = line[1:].split()
                name, parts = (toks[0] if toks else ""), []
            elif name is not None:
                parts.append(line.strip())
    if name is not None:
        yield name, "".join(parts)


def generate_regions_set_from_ref_fa(reference, remove_negative_control_regions=False,
                                     negative_control_regions_suffix_str_tuple=None):
    """region_split.py:29-49."""
    if remove_negative_control_regions:
        return {n for n, _ in _fasta_entries(reference) if not n.endswith(negative_control_regions_suffix_str_tuple)}
    return {n for n, _ in _fasta_entries(reference)}


def generate_region_length_dict_from_ref_fa(reference):
    """region_split.py:52-58."""
    return {n: len(s) for n, s in _fasta_entries(reference)}


def filter_and_split_reads_by_region_cluster(bam_file: Union[str, os.PathLike[str]],
                                             region_cluster_dict_json: Union[str, os.PathLike[str]],
                                             reference: Union[str, os.PathLike[str]],
                                             logs_dir: Union[str, os.PathLike[str]],
                                             region_fasta_out_dir: Union[str, os.PathLike[str]],
                                             minimal_region_overlap: float = 0.95, max_softclip_5_end: int = 73,
                                             max_softclip_3_end: int = 68):
    log_file = os.path.join(logs_dir,
                            os.path.basename(bam_file).split(".")[0] + "_filter_and_split_reads_by_region_cluster.err")
    with open(region_cluster_dict_json, "r") as json_in:
        region_cluster_dict = json.load(json_in)
    region_length_dict = generate_region_length_dict_from_ref_fa(reference=reference)
    names = list(region_length_dict)
    counts, per_cluster, detected = _v.context().region_split(
        os.fspath(bam_file), names, [region_length_dict[n] for n in names],
        [int(region_cluster_dict[n]) if n in region_cluster_dict else -1 for n in names], minimal_region_overlap,
        max_softclip_5_end, max_softclip_3_end, os.fspath(region_fasta_out_dir))
    n_unmapped, n_primary_mapped, n_short, n_long = (int(x) for x in counts)
    n_reads_region_cluster_counter = collections.defaultdict(int)
    for k, v in enumerate(per_cluster):
        if v:
            n_reads_region_cluster_counter[k] = int(v)
    region_cluster_fasta_set = {os.path.join(region_fasta_out_dir, "region_cluster{}.fasta".format(k))
                                for k in n_reads_region_cluster_counter}
    detected_regions_set = {names[r] for r, d in enumerate(detected) if d}

    # the log, as region_split.py:285-331 builds it
    logging_str = "Total # primary alignments in bam file: " + str(n_primary_mapped) + "\n"
    logging_str += (
        "median # of primary alignments in region clusters that have minimal region overlap and are not too long: "
        + str(round(np.median(list(n_reads_region_cluster_counter.values())), 3)) + "\n")
    logging_str += ("% of primary alignments that have shorter overlap than minimal region overlap: "
                    + str(round(100 * n_short / n_primary_mapped, 2)) + "\n")
    logging_str += "% of primary alignments that have too long reads: " + str(round(100 * n_long / n_primary_mapped, 2)) + "\n"
    regions_set = generate_regions_set_from_ref_fa(reference=reference, remove_negative_control_regions=True,
                                                   negative_control_regions_suffix_str_tuple=NEGATIVE_CONTROL_SUFFIXES)
    detected_regions_set = set([r for r in detected_regions_set if not r.endswith(NEGATIVE_CONTROL_SUFFIXES)])
    fraction_regions_detected = len(regions_set.intersection(detected_regions_set)) / len(regions_set)
    number_missing_regions = len(regions_set.difference(detected_regions_set))
    missing_regions = regions_set.difference(detected_regions_set)
    logging_str += ("fraction detected regions of total regions in reference in initial non-polished read alignments: "
                    + str(round(fraction_regions_detected, 4)) + "\n")
    logging_str += ("# of missing regions from reference in initial non-polished read alignments: "
                    + str(number_missing_regions) + "\n")
    logging_str += ("missing/non-detected regions from reference in initial non-polished read alignments: "
                    + str(missing_regions) + "\n")
    with open(log_file, "w") as ferr:
        ferr.write(logging_str)
    del n_unmapped
    return list(region_cluster_fasta_set)
