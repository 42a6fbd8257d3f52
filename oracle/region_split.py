"""CPU restatement of the region-binning record loop -- TEST INFRASTRUCTURE ONLY.

The checker and CPU baseline for the GPU path (umiclust_region_split), never the product.  Follows
/root/reference/ont_tcr_consensus/region_split.py:219-333 (filter_and_split_reads_by_region_cluster), over
records read by oracle/bam.py (pysam is not installed):
  - unmapped records are counted and skipped (:254-256), secondary / supplementary skipped (:257-258);
  - a primary record counts as mapped (:259), then `short` if its reference_length is below
    region_length * minimal_region_overlap (:261-263), `long` if its query_length exceeds
    region_length * (2 - minimal_region_overlap) + max_softclip_5_end + max_softclip_3_end (:264-269);
  - a kept record goes to region_cluster<k>.fasta as `>{query_name};strand={+|-}` and its forward sequence
    (`None` when the record stores none, as print() writes it) (:271-283);
  - the region-length and cluster lookups raise KeyError for a reference missing from them (:261, :271);
  - a mapped primary record without a CIGAR has reference_length 1 (pysam's bam_endpos - pos; htslib's
    bam_endpos counts a zero reference span as 1), so it drops as short.
Pinned by tests/golden/region_split/*.json, the reference's own outputs (tests/test_region_split_cpu.py).
With `out_dir` the records are appended one open() per record, as the reference does (:273-280): the
CPU baseline of bench_rows.py times exactly that loop.
"""
from __future__ import annotations

import collections
import os


def split_records(records, region_length: dict, region_cluster: dict, minimal_region_overlap: float = 0.95,
                  max_softclip_5_end: int = 73, max_softclip_3_end: int = 68, out_dir: str | None = None):
    """Returns (counts {unmapped, primary, short, long}, reads per cluster, FASTA text per cluster (empty when
    written to out_dir), detected region names).  A KeyError propagates after the earlier records."""
    counts = dict(unmapped=0, primary=0, short=0, long=0)
    per_cluster = collections.defaultdict(int)
    texts = collections.defaultdict(list)
    detected = set()
    slack = max_softclip_5_end + max_softclip_3_end
    for e in records:
        if e.is_unmapped:
            counts["unmapped"] += 1
            continue
        if e.is_secondary or e.is_supplementary:
            continue
        counts["primary"] += 1
        length = region_length[e.reference_name]
        if e.reference_length < length * minimal_region_overlap:
            counts["short"] += 1
            continue
        if e.query_length > length * (2 - minimal_region_overlap) + slack:
            counts["long"] += 1
            continue
        k = region_cluster[e.reference_name]
        per_cluster[k] += 1
        seq = e.get_forward_sequence() if e.is_reverse else e.query_sequence
        rec = f">{e.query_name};strand={'-' if e.is_reverse else '+'}\n{seq}\n"
        if out_dir is not None:
            with open(os.path.join(out_dir, f"region_cluster{k}.fasta"), "a") as fh:
                fh.write(rec)
        else:
            texts[k].append(rec)
        detected.add(e.reference_name)
    return counts, dict(per_cluster), {k: "".join(v) for k, v in texts.items()}, detected
