"""Oracle for SURVEY.md §8f row f1 (extract_umis, /root/reference/ont_tcr_consensus/extract_umis.py:19-267).

The edlib HW/path semantics restated in oracle/extract.py are checked on hand-derived cases.  Parity against
edlib itself is unpinned: python-edlib (pyproject.toml:34) is not installed and the reference has no fixture.
"""
import extract as ox
import pytest

FWD = "TTTVVTTVVVVTTVVVVTTVVVVTTVVVVTTT"  # run_config.json:11


def test_exact_match_span():
    u = "TTTACTTGACGTTCAGCTTGGAATTACGCTTT"  # FWD instantiated
    w = "GGCCGGCC" + u + "GGCCGG"
    assert ox.extract_umi(w, FWD, 3) == (0, u)


def test_iupac_equalities():
    assert ox.eq("V", "A") and ox.eq("A", "V") and ox.eq("v", "a") and ox.eq("a", "A")
    assert not ox.eq("V", "T") and not ox.eq("V", "a") and not ox.eq("N", "n")
    # a T where the pattern has V is a substitution
    u = "TTTATTTGACGTTCAGCTTGGAATTACGCTTT"
    assert ox.extract_umi("GGGGCCCC" + u + "CCCC", FWD, 3)[0] == 1


def test_insertion_and_deletion():
    u = "TTTACTTGACGTTCAGCTTGGAATTACGCTTT"
    ins = u[:10] + "A" + u[10:]
    d, got = ox.extract_umi("GGCCGGCC" + ins + "GGCC", FWD, 3)
    assert d == 1 and got == ins
    dele = u[:12] + u[13:]
    d, got = ox.extract_umi("GGCCGGCC" + dele + "GGCC", FWD, 3)
    assert d == 1 and got == dele


def test_beyond_k_is_none():
    assert ox.extract_umi("ACGT" * 20, FWD, 3) == (None, None)


def test_first_end_and_leftmost_start():
    # pattern "AAC", target "AACAAC": two exact ends (2 and 5); locations[0] is the first
    assert ox.hw_locate("AAC", "AACAAC", 0) == (0, 0, 2)
    # pattern "TA", target "TTA": end 2 (0 edits); the start of the optimal alignment is 1
    assert ox.hw_locate("TA", "TTA", 1) == (0, 1, 2)
    # one edit: pattern "ACG" vs "AG": end 1, SHW picks the last reversed column -> the leftmost start 0
    assert ox.hw_locate("ACG", "AG", 1) == (1, 0, 1)


def test_records_and_strand():
    u5 = "TTTACTTGACGTTCAGCTTGGAATTACGCTTT"
    u3 = "AAACGTCAACTGCAATGTCAAGGCTAACTAAA"
    rev = "AAABBBBAABBBBAABBBBAABBBBAABBAAA"
    seq = "GG" + u5 + "C" * 60 + u3 + "G"
    txt, n = ox.extract_records([("r1;strand=-", seq)], 73, 68, 3, FWD, rev)
    assert n == 1
    assert txt.startswith(f">r1;strand=-;umi_fwd_dist=0;umi_rev_dist=0;umi_fwd_seq={u5};umi_rev_seq={u3};seq={seq}\n")
    assert txt.endswith(ox.reverse_complement(u3) + ox.reverse_complement(u5) + "\n")
    with pytest.raises(Exception):
        ox.extract_records([("r1", seq)], 73, 68, 3, FWD, rev)


# ---- pinned by the reference itself: tests/golden/extract (make_golden_extract.py ran extract_umis.py here) ----
import glob as _glob
import json as _json
import os as _os

EXTRACT_FIX = sorted(_glob.glob(_os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "golden", "extract",
                                              "*.json")))


def _records(text):
    """pysam.FastxFile's view of a FASTA/FASTQ text: (name up to whitespace, joined sequence)."""
    lines = [x.rstrip("\r") for x in text.split("\n")]
    fastq = any(x for x in lines) and next(x for x in lines if x).startswith("@")
    recs, i = [], 0
    while i < len(lines):
        if not lines[i]:
            i += 1
            continue
        name = lines[i][1:].split()[0]
        i += 1
        seq = []
        while i < len(lines) and not lines[i].startswith(">") and not (fastq and lines[i].startswith("+")):
            seq.append(lines[i].strip())
            i += 1
        s = "".join(seq)
        if fastq:
            i += 1
            q = 0
            while i < len(lines) and q < len(s):
                q += len(lines[i])
                i += 1
        recs.append((name, s))
    return recs


@pytest.mark.parametrize("path", EXTRACT_FIX, ids=[_os.path.basename(p)[:-5] for p in EXTRACT_FIX])
def test_oracle_glue_matches_reference_fixtures(path):
    """The oracle's restated glue (oracle/extract.extract_records: strand split, read name, windows, skips,
    header and combined-UMI format) reproduces the reference's output records."""
    case = _json.load(open(path))
    a = dict(case["args"])
    a.pop("write_region")
    recs = _records(case["input"])
    want = list(case["files"].values())[0]
    if case["error"]:
        bad = next(i for i, (n, _s) in enumerate(recs) if "strand=" not in n)
        got, _n = ox.extract_records(recs[:bad], **a)
        with pytest.raises(Exception, match="Read strand not annotated!"):
            ox.extract_records(recs, **a)
    else:
        got, _n = ox.extract_records(recs, **a)
    assert got == want
