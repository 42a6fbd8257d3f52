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
