"""SURVEY.md §8f row f4 test infrastructure on CPU: the BAM writer/reader of oracle/bam.py round-trips the
fixture records (tests/golden/region_split/*.json hold the reference's own outputs for them,
tests/golden/make_golden_region_split.py)."""
import glob
import json
import os

import bam
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "region_split")


def cases():
    return [json.load(open(p)) for p in sorted(glob.glob(os.path.join(GOLD, "*.json")))]


@pytest.mark.parametrize("case", cases(), ids=[c["name"] for c in cases()])
def test_bam_round_trip(tmp_path, case):
    p = str(tmp_path / "x.bam")
    bam.write_bam(p, [tuple(r) for r in case["refs"]], case["records"])
    refs, recs = bam.read_bam(p)
    assert [list(r) for r in refs] == [list(r) for r in case["refs"]]
    assert len(recs) == len(case["records"])
    for a, r in zip(recs, case["records"]):
        assert a.query_name == r["name"] and a.flag == r["flag"] and a.reference_id == r["ref"]
        assert (a.query_sequence or "") == r["seq"]
        assert [("MIDNSHP=X"[op], ln) for op, ln in a.cigartuples] == [tuple(x) for x in r["cigar"]]


def test_fixtures_cover_the_branches():
    cs = {c["name"]: c for c in cases()}
    assert cs["unknown_reference"]["error"].startswith("KeyError")
    nc = cs["no_cigar"]
    assert nc["error"] is None and any(r["flag"] == 16 and not r["cigar"] for r in nc["records"])
    assert cs["append_existing"]["out_files"][next(iter(cs["append_existing"]["pre_existing"]))].startswith(">old")
    flags = {r["flag"] & 0x914 for c in cs.values() for r in c["records"]}
    assert {0, 4, 16, 256, 2048} <= flags | {x & ~16 for x in flags}


@pytest.mark.parametrize("case", cases(), ids=[c["name"] for c in cases()])
def test_oracle_restatement_vs_reference_fixtures(case):
    """oracle/region_split.py (the f4 checker and CPU baseline) reproduces the reference's files and counts."""
    import region_split as ors
    recs = [bam.AlignedSegment([tuple(r) for r in case["refs"]], r["ref"], r["pos"], r["flag"], r["name"],
                               [("MIDNSHP=X".index(op), ln) for op, ln in r["cigar"]], r["seq"] or None)
            for r in case["records"]]
    lengths = {nm: ln for nm, ln in case["regions"]}
    kw = dict(minimal_region_overlap=case["minimal_region_overlap"], max_softclip_5_end=case["max_softclip_5_end"],
              max_softclip_3_end=case["max_softclip_3_end"])
    if case["error"]:
        exc = KeyError
        with pytest.raises(exc) as e:
            ors.split_records(recs, lengths, case["clusters"], **kw)
        assert f"{exc.__name__}: {e.value}" == case["error"]
        return
    counts, per_cluster, texts, _ = ors.split_records(recs, lengths, case["clusters"], **kw)
    want = {fn: t[len(case["pre_existing"].get(fn, "")):] for fn, t in case["out_files"].items()}
    assert {f"region_cluster{k}.fasta": t for k, t in texts.items()} == want
    log = next(iter(case["log_files"].values()))
    assert f"Total # primary alignments in bam file: {counts['primary']}\n" in log
