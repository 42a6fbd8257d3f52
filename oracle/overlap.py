"""CPU restatement of the region-vs-region UMI overlap count.

TEST INFRASTRUCTURE ONLY: the checker for the future GPU hash join, never the product path.
Follows ont_tcr_consensus/extract_umis.py:
  - count_single_umi_overlaps               extract_umis.py:270-290 (exact string equality; the edlib
                                            HW alignment with IUPAC equalities is commented out
                                            upstream, so `overlapping_umi_edit_threshold` is unused)
  - count_overlapping_umis_between_2_regions extract_umis.py:296-342
  - count_overlapping_umis_between_all_regions extract_umis.py:345-369
The O(n*m) per-UMI scan becomes a multiset join (count of region-2 sequences equal to each region-1
sequence), which gives the same per-UMI counts.  Upstream appends TSV rows in Ray completion order;
here rows follow itertools.combinations order (the only deterministic choice).
Parity pinned: tests/golden/overlap/*.json are the outputs of the reference's own extract_umis.py, run here
with pass-through stand-ins for the uninstalled ray/pysam/edlib (tests/golden/make_golden_overlap.py);
tests/test_overlap_cpu.py checks this restatement against them (return list, TSV, warning file, the
empty-region-1 ValueError) and against a literal pairwise restatement of extract_umis.py:280-288.
"""
from __future__ import annotations

import itertools
import os
from collections import Counter


def read_fasta_seqs(path):
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
                cur.append(line)
    if cur is not None:
        seqs.append("".join(cur))
    return seqs


def count_single_umi_overlaps(umi_1_seq, umi_fasta_region_2_seqs, overlapping_umi_edit_threshold=0):
    """extract_umis.py:270-290: number of region-2 sequences string-equal to umi_1_seq."""
    return sum(1 for s in umi_fasta_region_2_seqs if s == umi_1_seq)


def overlap_counts(region_1_seqs, region_2_seqs):
    """Per-region-1-UMI overlap counts via a multiset join (same values as the pairwise scan)."""
    c2 = Counter(region_2_seqs)
    return [c2.get(s, 0) for s in region_1_seqs]


def count_overlapping_umis_between_2_regions(region_1_dir, region_2_dir, regions_w_overlapping_umis_tsv,
                                             overlapping_umi_edit_threshold=0):
    """extract_umis.py:296-342.  An empty region 1 raises ValueError, as upstream's max([]) does."""
    region_1 = os.path.basename(region_1_dir)
    region_2 = os.path.basename(region_2_dir)
    logs_dir = os.path.dirname(regions_w_overlapping_umis_tsv)
    s2 = read_fasta_seqs(os.path.join(region_2_dir, "umi_clusters_consensus.fasta"))
    s1 = read_fasta_seqs(os.path.join(region_1_dir, "umi_clusters_consensus.fasta"))
    counts = overlap_counts(s1, s2)
    if max(counts) > 1:
        with open(os.path.join(logs_dir, "region_region_umi_comparison.stderr"), "a") as ferr:
            print("WARNING: there are UMIs from", region_1, "that match more than 1 UMI within", region_2,
                  file=ferr)
    total = sum(counts)
    if total:
        with open(regions_w_overlapping_umis_tsv, "a") as tsv_out:
            print(region_1, region_2, str(total), sep="\t", file=tsv_out)
    return bool(total)


def count_overlapping_umis_between_all_regions(smolecule_filtered_fa_list, overlapping_umi_edit_threshold,
                                               logs_dir):
    """extract_umis.py:345-369: header row, then one task per unordered region pair; ray.get raises the first
    task's exception (an empty region 1's ValueError) after every task has run and appended its rows."""
    region_dirs = [os.path.dirname(fa) for fa in smolecule_filtered_fa_list]
    tsv = os.path.join(logs_dir, "regions_w_overlapping_umis.tsv")
    with open(tsv, "a") as tsv_out:
        print("region_1", "region_2", "umi_overlap_count", sep="\t", file=tsv_out)
    out, first_exc = [], None
    for r1, r2 in itertools.combinations(region_dirs, 2):
        try:
            out.append(count_overlapping_umis_between_2_regions(r1, r2, tsv, overlapping_umi_edit_threshold))
        except ValueError as e:
            first_exc = first_exc or e
    if first_exc is not None:
        raise first_exc
    return out
