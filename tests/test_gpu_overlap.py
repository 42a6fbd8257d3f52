"""§8f row f3 on the GPU: the hash join (umiclust_overlap_counts / umiclust_overlap_regions through
umiclust.overlap) against the reference's own outputs (tests/golden/overlap, made by running
extract_umis.py here) and against the CPU oracle on larger seeded inputs."""
import os
import random

import numpy as np
import overlap as oracle
import pytest
from test_overlap_cpu import _golden, run_and_compare
from umiclust import overlap

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", _golden(), ids=[c["name"] for c in _golden()])
def test_all_regions_vs_reference_fixtures(tmp_path, case):
    run_and_compare(overlap.count_overlapping_umis_between_all_regions, tmp_path, case)


def _sets(seed, n1, n2, pool_n):
    rng = random.Random(seed)
    pool = ["".join(rng.choice("ACGTN") for _ in range(rng.randint(1, 120))) for _ in range(pool_n)]
    pick = lambda n: [rng.choice(pool) if rng.random() < 0.7 else  # noqa: E731
                      "".join(rng.choice("ACGT") for _ in range(rng.randint(50, 70))) for _ in range(n)]
    return pick(n1), pick(n2)


@pytest.mark.parametrize("seed,n1,n2,pool", [(1, 0, 10, 5), (2, 10, 0, 5), (3, 500, 700, 50), (4, 20000, 30000, 3000)])
def test_counts_vs_oracle(gpu_ctx, seed, n1, n2, pool):
    s1, s2 = _sets(seed, n1, n2, pool)
    got = gpu_ctx.overlap_counts(s1, s2)
    assert got.tolist() == oracle.overlap_counts(s1, s2)


def test_single_umi_matches_pairwise_scan(gpu_ctx):
    s1, s2 = _sets(7, 30, 200, 10)
    for u in s1:
        assert overlap.count_single_umi_overlaps(u, s2, 2) == oracle.count_single_umi_overlaps(u, s2, 2)


def test_regions_vs_oracle_large(gpu_ctx):
    rng = random.Random(11)
    pool = ["".join(rng.choice("ACG") for _ in range(64)) for _ in range(20000)]
    regions = [[rng.choice(pool) for _ in range(rng.randint(0, 4000))] for _ in range(60)]
    total, maxc = gpu_ctx.overlap_regions(regions)
    for a in range(len(regions)):
        for b in range(a + 1, len(regions)):
            c = oracle.overlap_counts(regions[a], regions[b])
            assert total[a, b] == sum(c) and maxc[a, b] == (max(c) if c else 0), (a, b)
    assert not np.any(np.tril(total)) and not np.any(np.tril(maxc))


def test_hash_collision_reseeds_exactly(monkeypatch):
    """The first table pass with 8-bit hashes collides on purpose; the re-seeded pass must be exact."""
    from umiclust import _lib
    monkeypatch.setenv("UMICLUST_OVERLAP_TEST_COLLIDE", "1")
    s1, s2 = _sets(5, 3000, 4000, 400)
    with _lib.Context(0) as ctx:
        got = ctx.overlap_counts(s1, s2)
    assert got.tolist() == oracle.overlap_counts(s1, s2)


def test_regions_shared_artifact_umi(gpu_ctx):
    """one consensus UMI present in hundreds of regions (an adapter artifact) -- its bucket goes to the
    workgroup-per-bucket path (k_ov_pairs_big) instead of one thread's quadratic loops; exact against the oracle."""
    rng = random.Random(13)
    art = "ACGT" * 16
    pool = ["".join(rng.choice("ACG") for _ in range(60)) for _ in range(300)]
    regions = []
    for r in range(400):
        seqs = [rng.choice(pool) for _ in range(rng.randint(0, 6))] + [art] * rng.randint(0, 3)
        rng.shuffle(seqs)
        regions.append(seqs)
    total, maxc = gpu_ctx.overlap_regions(regions)
    for a in range(len(regions)):
        for b in range(a + 1, len(regions)):
            c = oracle.overlap_counts(regions[a], regions[b])
            assert total[a, b] == sum(c) and maxc[a, b] == (max(c) if c else 0), (a, b)


def test_all_regions_in_blocks_past_the_region_cap(tmp_path, monkeypatch):
    """More regions than one join holds (UMICLUST_OVERLAP_MAX_REGIONS; lowered here to 8): row blocks joined with
    every later block give the same files and results as the oracle, and an empty region 1 in the middle still
    lets every other pair report before the ValueError."""
    from test_overlap_cpu import materialize
    from umiclust import _lib
    monkeypatch.setattr(_lib, "OVERLAP_MAX_REGIONS", 8)
    rng = random.Random(17)
    pool = ["".join(rng.choice("ACGT") for _ in range(rng.randint(56, 70))) for _ in range(40)]
    for empty in (None, 7):
        regions = [dict(name=f"region_cluster{r}", seqs=[] if r == empty else
                        [rng.choice(pool) for _ in range(rng.randint(1, 12))]) for r in range(21)]
        case = dict(width=80, regions=regions)
        d_gpu, d_orc = tmp_path / f"g{empty}", tmp_path / f"o{empty}"
        d_gpu.mkdir()
        d_orc.mkdir()
        res = {}
        for d, fn in ((d_gpu, overlap.count_overlapping_umis_between_all_regions),
                      (d_orc, oracle.count_overlapping_umis_between_all_regions)):
            fas, logs = materialize(d, case)
            try:
                res[str(d)] = ("ok", fn(fas, 2, logs))
            except ValueError:
                res[str(d)] = ("ValueError", None)
            res[str(d)] += (tuple(open(os.path.join(logs, f)).read() for f in sorted(os.listdir(logs))),)
        assert res[str(d_gpu)] == res[str(d_orc)]
        assert res[str(d_gpu)][0] == ("ok" if empty is None else "ValueError")
