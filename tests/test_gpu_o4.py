"""SURVEY Appendix C O4 on the GPU: the batched restatement of vsearch's multithreaded cluster_fast
(umiclust_params.policy_threads = 1, rounds of `threads` queries; oracle/umiclust_oracle.c cluster_core_parallel
branch) against the oracle, bit-exact: membership, strands, centroids, consensus, alignment count and cells.
Rounds are cut from the bin's first sorted query regardless of the greedy blocks, so small blocks and rounds
spanning several lengths and blocks exercise the round windows (driver.cpp round_window) and the held-back
index appends."""
import numpy as np
import orc
import pytest
from umiclust import _lib, synth

pytestmark = pytest.mark.gpu


def _cmp(g, o):
    assert g["n_clusters"] == o["n_clusters"]
    assert np.array_equal(g["cluster"], o["cluster"])
    assert np.array_equal(g["strand"], o["strand"])
    assert np.array_equal(g["centroid"], o["centroid"])
    assert g["consensus"] == o["consensus"]


def _params(lib, preset, idn, T, lens=(58, 68)):
    p = lib.params(preset, idn, *lens)
    p.threads, p.policy_threads = T, 1
    return p


@pytest.mark.parametrize("T", [2, 25, 100])
@pytest.mark.parametrize("block", ["default", "7", "64"])
def test_batched_rounds_vs_oracle(T, block, monkeypatch):
    seqs = synth.make_umis(400, seed=7, max_reads=8000, error_rate=0.04, orient_mix=0.2).as_list()
    if block != "default":
        monkeypatch.setenv("UMICLUST_BLOCK", block)
    with _lib.Context(0) as ctx:
        ctx.load(_params(_lib, 1, 0.93, T), seqs)
        st = ctx.cluster()
        g = ctx.fetch()
    o = orc.cluster(_params(orc, 1, 0.93, T), seqs)
    _cmp(g, o)
    assert st["n_alignments"] == o["stats"]["alignments"] and st["cells"] == o["stats"]["cells"]


def test_batched_rounds_differ_from_sequential(gpu_ctx):
    """The policy switch changes results on this input (the oracle says so; the GPU follows both ways)."""
    seqs = synth.make_umis(1000, seed=7, max_reads=20000, error_rate=0.04).as_list()
    gpu_ctx.load(_params(_lib, 1, 0.93, 25), seqs)
    gpu_ctx.cluster()
    gb = gpu_ctx.fetch()
    gpu_ctx.load(_lib.params(1, 0.93, 58, 68), seqs)
    gpu_ctx.cluster()
    gs = gpu_ctx.fetch()
    _cmp(gb, orc.cluster(_params(orc, 1, 0.93, 25), seqs))
    _cmp(gs, orc.cluster(orc.params(1, 0.93, 58, 68), seqs))
    assert not np.array_equal(gb["cluster"], gs["cluster"])


def test_batched_rounds_ragged_small_bins():
    """Many tiny bins with ragged lengths: rounds span several one-length blocks (round tiles over several
    lengths), through the multi-bin load."""
    rng = np.random.default_rng(5)
    bins, seqs = [0], []
    for b in range(12):
        u = synth.make_umis(int(rng.integers(2, 12)), seed=500 + b, max_reads=int(rng.integers(20, 300)),
                            error_rate=0.05, orient_mix=0.3)
        seqs += u.as_list()
        bins.append(len(seqs))
    buf, off = _lib._pack(seqs)
    with _lib.Context(0) as ctx:
        ctx.load_bins(_params(_lib, 1, 0.93, 25), buf, off, bins)
        for b in range(len(bins) - 1):
            st = ctx.cluster_bin(b)
            g = ctx.fetch_bin(b)
            o = orc.cluster(_params(orc, 1, 0.93, 25), seqs[bins[b]:bins[b + 1]])
            _cmp(g, o)
            assert st["n_alignments"] == o["stats"]["alignments"]


def _deep(seed=31, n=2500):
    return synth.make_umis(8, seed=seed, max_reads=n, orient_mix=0.3, mean_reads=1500.0, error_rate=0.15,
                           split=(0.0, 0.5, 0.5), max_edits=4, pattern_fwd=synth.UMI_FWD_LONG,
                           pattern_rev=synth.UMI_REV_LONG).as_list()


@pytest.mark.parametrize("mix", ["0", "1"])
@pytest.mark.parametrize("T", [1, 25])
def test_batched_rounds_deep_clusters(mix, T, monkeypatch):
    """Config-5 style deep clusters: peer lists overflow and blocks re-run alone, in batched mode and (T = 1) in the
    sequential one, with blocks of one length or across length changes (UMICLUST_MIXLEN=1: the per-length pair
    segments); alignment count and cells equal the oracle's.  (Round 3 excluded mixed blocks under O4 after one run
    of this case gave 7,595 vs 7,574 alignments; per-query walk dumps, tools/o4_walk_debug.py, show every query's
    count equal with mixed blocks forced on the round-4 code.)"""
    seqs = _deep()
    monkeypatch.setenv("UMICLUST_BLOCK", "256")
    monkeypatch.setenv("UMICLUST_MIXLEN", mix)
    with _lib.Context(0) as ctx:
        ctx.load(_params(_lib, 1, 0.75, T, (80, 110)), seqs)
        st = ctx.cluster()
        g = ctx.fetch()
    o = orc.cluster(_params(orc, 1, 0.75, T, (80, 110)), seqs)
    _cmp(g, o)
    assert st["n_alignments"] == o["stats"]["alignments"] and st["cells"] == o["stats"]["cells"]


@pytest.mark.parametrize("T", [2, 25, 100])
@pytest.mark.parametrize("block", ["default", "64"])
def test_batched_rounds_mixed_blocks(T, block, monkeypatch):
    """Blocks across query-length changes forced on (ragged lengths 58-68, rounds spanning several lengths and
    blocks): batched rounds equal the oracle, alignment count and cells included."""
    seqs = synth.make_umis(400, seed=9, max_reads=8000, error_rate=0.06, orient_mix=0.2).as_list()
    monkeypatch.setenv("UMICLUST_MIXLEN", "1")
    if block != "default":
        monkeypatch.setenv("UMICLUST_BLOCK", block)
    with _lib.Context(0) as ctx:
        ctx.load(_params(_lib, 1, 0.93, T), seqs)
        st = ctx.cluster()
        g = ctx.fetch()
    o = orc.cluster(_params(orc, 1, 0.93, T), seqs)
    _cmp(g, o)
    assert st["n_alignments"] == o["stats"]["alignments"] and st["cells"] == o["stats"]["cells"]


@pytest.mark.parametrize("packs", [[(0, 12)], [(0, 5), (5, 7)], [(3, 4), (0, 3), (7, 5)]])
@pytest.mark.parametrize("T", [2, 25])
def test_batched_rounds_packs(packs, T):
    """Packs of bins (umiclust_cluster_pack: one greedy order over several bins, blocks across bin boundaries) under
    batched rounds: every bin's rounds are counted from its own first sorted query, so every bin equals the oracle
    run on that bin alone, alignment count included (summed over the pack)."""
    rng = np.random.default_rng(15)
    bins, seqs = [0], []
    for b in range(12):
        u = synth.make_umis(int(rng.integers(2, 30)), seed=700 + b, max_reads=int(rng.integers(20, 700)),
                            error_rate=0.05, orient_mix=0.3)
        seqs += u.as_list()
        bins.append(len(seqs))
    buf, off = _lib._pack(seqs)
    with _lib.Context(0) as ctx:
        ctx.load_bins(_params(_lib, 1, 0.93, T), buf, off, bins)
        for first, m in packs:
            st = ctx.cluster_pack(first, m)
            want = 0
            for b in range(first, first + m):
                o = orc.cluster(_params(orc, 1, 0.93, T), seqs[bins[b]:bins[b + 1]])
                _cmp(ctx.fetch_bin(b), o)
                want += o["stats"]["alignments"]
            assert st["n_alignments"] == want
