"""Drop-in for the region-vs-region UMI overlap count of /root/reference/ont_tcr_consensus/extract_umis.py
(SURVEY.md §8f row f3), on the GPU.

Same names, arguments, files and return values as the reference:
  * count_single_umi_overlaps(umi_1_seq, umi_fasta_region_2_seqs, overlapping_umi_edit_threshold) (:270-290):
    the number of region-2 sequences string-equal to umi_1_seq (the edlib comparison is commented out
    upstream, so the edit threshold is accepted and unused, as there);
  * count_overlapping_umis_between_2_regions(region_1_dir, region_2_dir, regions_w_overlapping_umis_tsv,
    overlapping_umi_edit_threshold) (:293-342): reads both regions' umi_clusters_consensus.fasta, appends the
    warning line to <logs>/region_region_umi_comparison.stderr when a region-1 UMI matches more than one
    region-2 UMI, appends `region_1 region_2 count` to the TSV when the count is non-zero, returns bool;
    an empty region 1 raises ValueError (upstream's max() of an empty list);
  * count_overlapping_umis_between_all_regions(smolecule_filtered_fa_list, overlapping_umi_edit_threshold,
    logs_dir) (:345-369): the TSV header, then every itertools.combinations pair -- all pairs in ONE GPU hash
    join (umiclust_overlap_regions) instead of one Ray task per pair and one per UMI; past
    UMICLUST_OVERLAP_MAX_REGIONS regions, row blocks of regions joined with every later block.  A pair with an
    empty region 1 raises ValueError, as upstream's task does, after every other pair has been reported (the
    other Ray tasks still run and append their rows before ray.get raises).
Rows are written in combinations order (upstream: Ray completion order).  No CPU fallback: without the
library or a device every call raises.
"""
from __future__ import annotations

import os
from typing import Union

import numpy as np

from . import _lib
from . import vsearch_umi_cluster as _v

CONSOUT = "umi_clusters_consensus.fasta"


def read_fasta_seqs(path) -> list:
    """Sequences of a FASTA file in order, multi-line records joined (pysam.FastxFile `.sequence`)."""
    seqs, cur = [], None
    with open(path) as fh:
        for line in fh:
            line = line.rstrip("\r\n")
            if line.startswith(">"):
                if cur is not None:
                    seqs.append("".join(cur))
                cur = []
            elif cur is not None:
                cur.append(line.strip())
    if cur is not None:
        seqs.append("".join(cur))
    return seqs


def count_single_umi_overlaps(umi_1_seq: str, umi_fasta_region_2_seqs: list, overlapping_umi_edit_threshold: int):
    return int(_v.context().overlap_counts([umi_1_seq], umi_fasta_region_2_seqs)[0])


def _report(region_1, region_2, total, maxcount, logs_dir, tsv):
    if maxcount > 1:
        with open(os.path.join(logs_dir, "region_region_umi_comparison.stderr"), "a") as ferr:
            print("WARNING: there are UMIs from", region_1, "that match more than 1 UMI within", region_2, file=ferr)
    if total:
        with open(tsv, "a") as tsv_out:
            print(region_1, region_2, str(total), sep="\t", file=tsv_out)
    return bool(total)


def count_overlapping_umis_between_2_regions(region_1_dir: Union[str, os.PathLike], region_2_dir: Union[str, os.PathLike],
                                             regions_w_overlapping_umis_tsv: Union[str, os.PathLike],
                                             overlapping_umi_edit_threshold: int):
    region_1, region_2 = os.path.basename(region_1_dir), os.path.basename(region_2_dir)
    logs_dir = os.path.dirname(regions_w_overlapping_umis_tsv)
    s2 = read_fasta_seqs(os.path.join(region_2_dir, CONSOUT))
    s1 = read_fasta_seqs(os.path.join(region_1_dir, CONSOUT))
    counts = _v.context().overlap_counts(s1, s2)
    mx = max(counts.tolist())  # ValueError on an empty region 1, as upstream
    return _report(region_1, region_2, int(counts.sum()), mx, logs_dir, regions_w_overlapping_umis_tsv)


def count_overlapping_umis_between_all_regions(smolecule_filtered_fa_list: list, overlapping_umi_edit_threshold: int,
                                               logs_dir: Union[str, os.PathLike]):
    region_dirs = [os.path.dirname(fa) for fa in smolecule_filtered_fa_list]
    tsv = os.path.join(logs_dir, "regions_w_overlapping_umis.tsv")
    with open(tsv, "a") as tsv_out:
        print("region_1", "region_2", "umi_overlap_count", sep="\t", file=tsv_out)
    seqs = [read_fasta_seqs(os.path.join(d, CONSOUT)) for d in region_dirs]
    R = len(region_dirs)
    out = []
    if R < 2:
        return out
    names = [os.path.basename(d) for d in region_dirs]
    empty_region_1 = False
    # one GPU join over every region when they fit one call; beyond that, row blocks of regions joined with each
    # later block (every pair of the union is counted; the pairs of the row block are kept)
    B = _lib.OVERLAP_MAX_REGIONS // 2 if R > _lib.OVERLAP_MAX_REGIONS else R
    for i0 in range(0, R, B):
        rows = range(i0, min(R, i0 + B))
        tot = np.zeros((len(rows), R), np.int64)
        mxc = np.zeros((len(rows), R), np.int32)
        for j0 in range(i0, R, B):
            cols = list(rows) if j0 == i0 else list(rows) + list(range(j0, min(R, j0 + B)))
            t, m = _v.context().overlap_regions([seqs[x] for x in cols])
            tot[:, cols] = np.maximum(tot[:, cols], t[:len(rows)])
            mxc[:, cols] = np.maximum(mxc[:, cols], m[:len(rows)])
        for r, a in enumerate(rows):
            for b in range(a + 1, R):
                if not seqs[a]:
                    # upstream: max() of an empty region 1 raises inside that pair's task; the other tasks still run
                    # and append their rows, and ray.get raises afterwards
                    empty_region_1 = True
                    continue
                out.append(_report(names[a], names[b], int(tot[r, b]), int(mxc[r, b]), logs_dir, tsv))
    if empty_region_1:
        raise ValueError("max() arg is an empty sequence")
    return out


# ray-style call syntax (the reference's functions are ray.remote tasks)
class _LocalRemote:
    def __init__(self, fn):
        self._fn = fn
        self.__doc__ = fn.__doc__

    def options(self, **_kw):
        return self

    def remote(self, *a, **kw):
        return self._fn(*a, **kw)

    def __call__(self, *a, **kw):
        return self._fn(*a, **kw)


count_single_umi_overlaps_task = _LocalRemote(count_single_umi_overlaps)
count_overlapping_umis_between_2_regions_task = _LocalRemote(count_overlapping_umis_between_2_regions)
