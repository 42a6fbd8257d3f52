"""CPU restatement of UMI extraction: /root/reference/ont_tcr_consensus/extract_umis.py.

TEST INFRASTRUCTURE ONLY: the checker for the GPU Myers kernel (umiclust_extract_umis*), never the product.
Follows:
  - extract_umi (extract_umis.py:19-107): edlib.align(pattern, window, task="path", mode="HW",
    k=max_edit_dist, additionalEqualities=IUPAC pairs) -> (editDistance, window[start:end+1]) or (None, None)
  - extract_adapters (:110-126): the first adapter_length_5_end and the last adapter_length_3_end bases
  - get_read_name / get_read_strand (:129-137), combine_umis_fasta (:140-151), write_fasta (:154-186)
  - extract_umis (:189-267)
The alignment arithmetic lives in the third-party edlib (python-edlib >= 1.3.9, pyproject.toml:34), which is
not installed here and not vendored in the reference.  Its published semantics are restated as a plain
O(m n) dynamic program:
  * HW ("infix"): D[0][j] = 0 (free target prefix), D[i][0] = i, unit costs; the edit distance is
    min_j D[m][j] over target end positions, reported only if <= k; the end locations are every target
    position with that distance, ascending; locations[0] is the first.
  * the start of an end location e (edlib.cpp obtainLocations, mode HW): SHW on the reversed pattern and the
    reversed target prefix [0, e]: among the reversed positions p with distance = the edit distance, the
    LAST (largest) one, start = e - p ("ensures that alignment will not start with insertion").
  * equality: identical bytes, or a pair of additionalEqualities, in either order.
PARITY UNPINNED against edlib itself (no binary, no fixture); the tests pin it on hand-derived cases.
"""
from __future__ import annotations

IUPAC_EQ = [("M", "A"), ("M", "C"), ("R", "A"), ("R", "G"), ("W", "A"), ("W", "T"), ("S", "C"), ("S", "G"),
            ("Y", "C"), ("Y", "T"), ("K", "G"), ("K", "T"), ("V", "A"), ("V", "C"), ("V", "G"), ("H", "A"),
            ("H", "C"), ("H", "T"), ("D", "A"), ("D", "G"), ("D", "T"), ("B", "C"), ("B", "G"), ("B", "T"),
            ("N", "A"), ("N", "C"), ("N", "G"), ("N", "T"), ("m", "a"), ("m", "c"), ("r", "a"), ("r", "g"),
            ("w", "a"), ("w", "t"), ("s", "c"), ("s", "g"), ("y", "c"), ("y", "t"), ("k", "g"), ("k", "t"),
            ("v", "a"), ("v", "c"), ("v", "g"), ("h", "a"), ("h", "c"), ("h", "t"), ("d", "a"), ("d", "g"),
            ("d", "t"), ("b", "c"), ("b", "g"), ("b", "t"), ("n", "a"), ("n", "c"), ("n", "g"), ("n", "t"),
            ("a", "A"), ("c", "C"), ("t", "T"), ("g", "G")]
_EQ = set(IUPAC_EQ) | {(b, a) for a, b in IUPAC_EQ}


def eq(a: str, b: str) -> bool:
    return a == b or (a, b) in _EQ


def _last_row(pattern: str, target: str, free_start: bool) -> list:
    """D[m][j] for j = 0..len(target) (HW: free_start, SHW: D[0][j] = j)."""
    m = len(pattern)
    prev = [0 if free_start else j for j in range(len(target) + 1)]
    for i in range(1, m + 1):
        cur = [i] + [0] * len(target)
        pc = pattern[i - 1]
        for j in range(1, len(target) + 1):
            cur[j] = min(prev[j - 1] + (0 if eq(pc, target[j - 1]) else 1), prev[j] + 1, cur[j - 1] + 1)
        prev = cur
    return prev


def hw_locate(pattern: str, target: str, k: int):
    """edlib HW with task path: (edit distance, start, end) of locations[0], or None."""
    row = _last_row(pattern, target, True)
    best = min(row[1:]) if len(target) else len(pattern)
    if best > k or not len(target):
        return None
    end = next(j - 1 for j in range(1, len(target) + 1) if row[j] == best)
    rrow = _last_row(pattern[::-1], target[:end + 1][::-1], False)
    p = max(j - 1 for j in range(1, end + 2) if rrow[j] == best)
    return best, end - p, end


def extract_umi(query_seq: str, pattern: str, max_edit_dist: int):
    r = hw_locate(pattern, query_seq, max_edit_dist)
    if r is None:
        return None, None
    d, s, e = r
    return d, query_seq[s:e + 1]


def reverse_complement(seq: str) -> str:
    return seq.translate(str.maketrans("ACTG", "TGAC"))[::-1]


def combine(seq_5p: str, seq_3p: str, strand: str) -> str:
    return seq_5p + seq_3p if strand == "+" else reverse_complement(seq_3p) + reverse_complement(seq_5p)


def extract_records(records, adapter_length_5_end=73, adapter_length_3_end=68, max_pattern_dist=3,
                    umi_fwd="TTTVVVVTTVVVVTTVVVVTTVVVVTTT", umi_rev="AAABBBBAABBBBAABBBBAABBBBAAA"):
    """records: (name, sequence) pairs as pysam yields them.  Returns the output FASTA text and the count."""
    out, n = [], 0
    for name, seq in records:
        parts = name.split("strand=")
        if not len(parts) > 1:
            raise Exception("Read strand not annotated!")
        strand = parts[1]
        rid = name.split(";")[0]
        w5, w3 = seq[:adapter_length_5_end], seq[-adapter_length_3_end:]
        d5, u5 = extract_umi(w5, umi_fwd, max_pattern_dist)
        d3, u3 = extract_umi(w3, umi_rev, max_pattern_dist)
        if not u5 or not u3:
            continue
        n += 1
        out.append(f">{rid};strand={strand};umi_fwd_dist={d5};umi_rev_dist={d3};umi_fwd_seq={u5};"
                   f"umi_rev_seq={u3};seq={seq}\n{combine(u5, u3, strand)}\n")
    return "".join(out), n
