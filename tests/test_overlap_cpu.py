"""Oracle for SURVEY.md §8f row f3 (count_overlapping_umis_between_2_regions, extract_umis.py:270-369).

The multiset join in oracle/overlap.py is checked against a literal restatement of the reference's
pairwise equality scan (extract_umis.py:280-288), and the file-level behaviour (TSV rows, warning
file, bool list, empty-region error) against hand-computed expectations.  Parity unpinned against
the reference itself: it ships no fixture for this function.
"""
import os
import random

import overlap
import pytest


def _rand_umis(rng, n, pool):
    return [rng.choice(pool) for _ in range(n)]


def _write_consout(d, seqs, width=0):
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "umi_clusters_consensus.fasta"), "w") as fh:
        for i, s in enumerate(seqs):
            fh.write(f">centroid=u{i};seqs=1;clusterid={i}\n")
            if width:
                for j in range(0, len(s), width):
                    fh.write(s[j:j + width] + "\n")
            else:
                fh.write(s + "\n")


@pytest.mark.parametrize("seed", range(5))
def test_join_matches_pairwise_scan(seed):
    rng = random.Random(seed)
    pool = ["".join(rng.choice("ACGT") for _ in range(rng.randint(55, 70))) for _ in range(40)]
    r1, r2 = _rand_umis(rng, 120, pool), _rand_umis(rng, 90, pool)
    want = [overlap.count_single_umi_overlaps(s, r2, 1) for s in r1]
    assert overlap.overlap_counts(r1, r2) == want


def test_all_regions_files(tmp_path):
    a, b, c = (str(tmp_path / r) for r in ("regA", "regB", "regC"))
    _write_consout(a, ["ACGTACGT", "TTTTGGGG", "CCCCAAAA"])
    _write_consout(b, ["ACGTACGT", "ACGTACGT", "GGGGCCCC"], width=3)  # multi-line records join
    _write_consout(c, ["AAAACCCC"])
    logs = tmp_path / "logs"
    logs.mkdir()
    fas = [os.path.join(d, "smolecule_filtered.fa") for d in (a, b, c)]
    got = overlap.count_overlapping_umis_between_all_regions(fas, 0, str(logs))
    assert got == [True, False, False]
    rows = (logs / "regions_w_overlapping_umis.tsv").read_text().splitlines()
    assert rows == ["region_1\tregion_2\tumi_overlap_count", "regA\tregB\t2"]
    warn = (logs / "region_region_umi_comparison.stderr").read_text()
    assert warn.strip() == "WARNING: there are UMIs from regA that match more than 1 UMI within regB"


def test_empty_region_1_raises(tmp_path):
    a, b = str(tmp_path / "a"), str(tmp_path / "b")
    _write_consout(a, [])
    _write_consout(b, ["ACGT"])
    with pytest.raises(ValueError):
        overlap.count_overlapping_umis_between_2_regions(a, b, str(tmp_path / "t.tsv"), 0)


def _golden():
    import glob
    import json
    d = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "overlap")
    return [json.load(open(p)) for p in sorted(glob.glob(os.path.join(d, "*.json")))]


def materialize(tmp_path, case):
    """Write a fixture's regions as <region>/umi_clusters_consensus.fasta (its own wrap width)."""
    dirs = []
    for reg in case["regions"]:
        d = tmp_path / reg["name"]
        d.mkdir()
        with open(d / "umi_clusters_consensus.fasta", "w") as fh:
            for i, s in enumerate(reg["seqs"]):
                fh.write(f">centroid=r{i};strand=+;seqs={1 + i % 5};clusterid={i}\n")
                for j in range(0, max(1, len(s)), case["width"]):
                    fh.write(s[j:j + case["width"]] + "\n")
        dirs.append(str(d))
    logs = tmp_path / "logs"
    logs.mkdir()
    return [os.path.join(d, "smolecule_filtered.fa") for d in dirs], str(logs)


def run_and_compare(fn, tmp_path, case):
    fas, logs = materialize(tmp_path, case)
    if case["error"]:
        with pytest.raises(ValueError):
            fn(fas, 2, logs)
    else:
        assert fn(fas, 2, logs) == case["result"]
    got = {f: open(os.path.join(logs, f)).read() for f in sorted(os.listdir(logs))}
    assert got == case["files"]


@pytest.mark.parametrize("case", _golden(), ids=[c["name"] for c in _golden()])
def test_oracle_matches_reference_fixtures(tmp_path, case):
    """Pinned: tests/golden/overlap/*.json are the reference's own outputs (make_golden_overlap.py)."""
    run_and_compare(overlap.count_overlapping_umis_between_all_regions, tmp_path, case)
