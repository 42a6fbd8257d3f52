"""BinRunner's grouping of a lane's bins into packs (umiclust_cluster_pack), on CPU: every bin in exactly one pack, in
lane order, consecutive bins up to pack_reads reads (a bin larger than that alone), one bin per call when off."""
from types import SimpleNamespace

import pytest
from umiclust.binset import BinRunner


def _stub(sizes, plan, pack_reads):
    bins = [SimpleNamespace(umis=SimpleNamespace(n=n)) for n in sizes]
    return SimpleNamespace(plan=plan, pack_reads=pack_reads, binset=SimpleNamespace(bins=bins))


@pytest.mark.parametrize("pack_reads", [0, 1, 100, 250, 10**9])
def test_packs_cover_lane_in_order(pack_reads):
    sizes = [300, 5, 120, 120, 0, 40, 60, 900, 1, 1]
    plan = [[7, 0, 2, 3, 6, 5, 1, 8, 9, 4]]  # a lane's bins, largest first (LPT order), as loaded
    st = _stub(sizes, plan, pack_reads)
    packs = BinRunner.packs(st, 0)
    flat = [j for first, m in packs for j in range(first, first + m)]
    assert flat == list(range(len(plan[0])))  # load positions, each once, in order
    for first, m in packs:
        reads = sum(sizes[plan[0][j]] for j in range(first, first + m))
        if pack_reads <= 0:
            assert m == 1
        elif m > 1:
            assert reads <= pack_reads
    if pack_reads >= sum(sizes):
        assert packs == [(0, len(sizes))]


def test_pack_boundaries():
    st = _stub([60, 50, 40, 30, 20], [[0, 1, 2, 3, 4]], 100)
    assert BinRunner.packs(st, 0) == [(0, 1), (1, 2), (3, 2)]
