"""Drop-in for the UMI extraction of /root/reference/ont_tcr_consensus/extract_umis.py,
on the GPU: the producer of the clustering hot path's input (`<region>_detected_umis.fasta`).

`extract_umis(fastx_file, umi_fasta_out_dir, write_region, adapter_length_5_end=73, adapter_length_3_end=68,
max_pattern_dist=3, umi_fwd=..., umi_rev=...)` keeps the reference's signature, defaults, output path rule and
return value (:189-267): the output FASTA path if at least one read has both UMIs, else None.  The per-read
edlib search (:19-107) runs as a Myers bit-vector kernel (csrc/extract.hip) over every read's two adapter
windows at once, and the records of write_fasta (:154-186) are written by the library
(umiclust_extract_umis_file).  `extract_umi(query_seq, pattern, max_edit_dist)` is the single-window form.
No CPU fallback: without the library or a device every call raises.
"""
from __future__ import annotations

import os
from typing import Union

from . import vsearch_umi_cluster as _v

UMI_FWD_DEFAULT = "TTTVVVVTTVVVVTTVVVVTTVVVVTTT"
UMI_REV_DEFAULT = "AAABBBBAABBBBAABBBBAABBBBAAA"


def extract_umi(query_seq: str, pattern: str, max_edit_dist: int):
    """(edit distance, UMI) of edlib.align(pattern, query_seq, mode="HW", task="path", k=max_edit_dist, IUPAC
    equalities) -- (None, None) when no location is within max_edit_dist (extract_umis.py:19-107)."""
    r = _v.context().extract_umis([query_seq], len(query_seq), 0, max_edit_dist, pattern, pattern)[0]
    if r[0] < 0:
        return None, None
    return int(r[0]), query_seq[r[1]:r[2] + 1]


def _extract_umis(fastx_file: Union[str, os.PathLike[str]], umi_fasta_out_dir: Union[str, os.PathLike[str]],
                  write_region: bool, adapter_length_5_end: int = 73, adapter_length_3_end: int = 68,
                  max_pattern_dist: int = 3, umi_fwd: str = UMI_FWD_DEFAULT, umi_rev: str = UMI_REV_DEFAULT):
    if write_region:
        region = os.path.basename(fastx_file).split(".")[0]
        out = os.path.join(umi_fasta_out_dir, region + "_detected_umis.fasta")
    else:
        out = os.path.join(umi_fasta_out_dir, "_detected_umis.fasta")
    n_both_umi = _v.context().extract_umis_file(os.fspath(fastx_file), out, adapter_length_5_end, adapter_length_3_end,
                                               max_pattern_dist, umi_fwd, umi_rev)
    return out if n_both_umi else None


extract_umis = _v._LocalRemote(_extract_umis)
