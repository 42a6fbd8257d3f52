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


def _o4_golden():
    import json
    import os
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "oracle_o4.json")
    return sorted(json.load(open(path)).items()) if os.path.exists(path) else []


_O4_SINGLE = [(k, v) for k, v in _o4_golden() if "n_bins" not in v]
_O4_MULTI = [(k, v) for k, v in _o4_golden() if "n_bins" in v]


@pytest.mark.parametrize("name,gold", _O4_SINGLE, ids=[k for k, _ in _O4_SINGLE])
def test_o4_config_vs_oracle_golden(gpu_ctx, name, gold):
    """The reference's operating mode at BASELINE sizes: vsearch --threads 25 (vsearch_umi_cluster.py:33-34,
    utils.py:56-63; policy O4) on config 1 both rounds (100k reads), config 2 (the headline bin: 2M reads, --id 0.90;
    the oracle's OpenMP workers took ~21 min on 7 cores) and config-5 stress samples, default blocks: alignment
    count, cells and the digests of membership, strands, centroids and consensus equal the oracle's
    (tests/golden/make_oracle_golden.py o4)."""
    from make_oracle_golden import digest
    u = synth.config_umis(gold["config"], gold["scale"])
    gpu_ctx.load(_lib.params(gold["preset"], gold["identity"], gold["minlen"], gold["maxlen"], threads=gold["T"]),
                 buf=u.seq, off=u.off)
    st = gpu_ctx.cluster()
    d = digest(gpu_ctx.fetch())
    assert st["n_alignments"] == gold["alignments"] and st["cells"] == gold["cells"]
    for k in ("n_clusters", "cluster", "strand", "centroid", "consensus"):
        assert d[k] == gold[k], k


def _structure_ok(res, lens):
    """--clusterout_sort order, one centroid per cluster, every member no longer than its centroid."""
    cl = np.asarray(res["cluster"])
    k = int(res["n_clusters"])
    kept = cl >= 0
    sizes = np.bincount(cl[kept], minlength=k)
    cen = np.asarray(res["centroid"]) == 1
    cen_len = np.zeros(k, np.int64)
    cen_len[cl[cen]] = lens[cen]
    return (bool(np.all(np.diff(sizes) <= 0)) and int(cen.sum()) == k and len(res["consensus"]) == k
            and bool(np.all(lens[kept] <= cen_len[cl[kept]])))


def _multi_cases():
    """(name, gold, lanes, pack): reduced-scale goldens bin by bin on one lane, as bench.py runs them (8 lanes, packs of
    200k reads) and in small packs on 4 lanes; the bench-size goldens (round 6: config 3 whole, config 4 at 2 % and
    its giant-molecule bin 200 at full size) as bench.py runs them, and config 3 also bin by bin."""
    out = []
    for name, gold in _O4_MULTI:
        if gold["scale"] < 0.02:
            combos = [(1, 0), (8, 200000), (4, 3000)]
        elif gold["config"] == 3:
            combos = [(8, 200000), (1, 0)]
        else:
            combos = [(8, 200000)]
        out += [(name, gold, lanes, pack) for lanes, pack in combos]
    return out


_MULTI_CASES = _multi_cases()


@pytest.mark.parametrize("name,gold,lanes,pack", _MULTI_CASES,
                         ids=[f"{n}-l{la}-p{pk}" for n, _, la, pk in _MULTI_CASES])
def test_o4_multibin_vs_oracle_golden(name, gold, lanes, pack, config_binset):
    """Configs 3 (960 Zipf bins) and 4 (both rounds) under --threads 25, as bench.py runs them (8 lanes, packs of
    200k reads, the largest bin's lane prioritised: bench.py's BinRunner call), bin by bin on one lane, and in small
    packs on 4 lanes: every bin's digest and cluster count, the alignment count and cells equal the oracle's
    (tests/golden/make_oracle_golden.py o4).  At bench size: config 3 whole (~9.9M reads), config 4 at 2 % scale and
    config 4's bin 200 alone at full size (792k reads with a giant molecule), whose round 1 overflows peer lists,
    resolves the overflowing blocks up to the overflow, re-runs the rest and regrows the halved block size."""
    from umiclust import binset
    bs = config_binset(gold["config"], gold["scale"], gold.get("shard_ids"))
    assert len(bs.bins) == gold["n_bins"] and bs.n == gold["n_reads"]
    rounds = [("round1", binset.ROUND1)] + ([("round2", binset.ROUND2)] if "round2" in gold else [])
    for rname, prm in rounds:
        g = gold[rname]
        with _lib.Context(0) as ctx:
            run = binset.BinRunner(ctx, bs, prm["preset"], prm["identity"], gold["minlen"], gold["maxlen"],
                                   lanes=lanes, pack_reads=pack, threads=gold["T"])
            st = run.cluster_all()
            res = run.results()
            run.close()
        dg = [binset.digest(r) for r in res]
        assert [x["n_clusters"] for x in dg] == g["n_clusters"], rname
        assert sum(x["n_alignments"] for x in st) == g["alignments"] and sum(x["cells"] for x in st) == g["cells"]
        assert binset.combine(dg) == g["combined"], rname
        for b, r in enumerate(res):  # (the full-size config-3 run of round 5 checked only this, sequential policy)
            assert _structure_ok(r, np.diff(bs.bins[b].umis.off)), (rname, b)
        if gold.get("shard_ids") == [200] and rname == "round1":
            # the production-depth mechanisms are exercised: overflow re-runs after partial resolution, regrowth
            assert sum(x["n_reruns"] for x in st) > 0 and sum(x["n_regrows"] for x in st) > 0, st
        if rname == "round1":
            bs = binset.round2_binset(bs, res)


@pytest.mark.parametrize("mix", ["0", "1"])
@pytest.mark.parametrize("T", [7, 25])
def test_o4_rerun_after_queued_pass(mix, T, monkeypatch):
    """Regression (round 5): a block that overflows a peer list is re-run alone after the next block's pass was
    queued; the re-run must search an index holding no centroid of its own first round.  Round 4 synced the index for
    the queued pass up to the overflowing block's start, so its re-run met centroids of the round straddling that
    start (config 5 at --id 0.90: 15-50 extra alignments, reads moved between clusters).  The bin re-runs 18-24
    blocks here, with blocks of one length and across length changes; every query's walk equals the oracle's."""
    monkeypatch.setenv("UMICLUST_MIXLEN", mix)
    monkeypatch.setenv("ORC_WORKERS", "8")
    lo, hi = synth.CONFIG_LENGTHS[5]
    seqs = synth.config_umis(5, 0.02).as_list()
    with _lib.Context(0) as ctx:
        ctx.load(_lib.params(1, 0.90, lo, hi, threads=T), seqs)
        st = ctx.cluster()
        g = ctx.fetch()
    assert st["n_reruns"] > 0  # the mechanism is exercised
    o = orc.cluster(_params(orc, 1, 0.90, T, (lo, hi)), seqs)
    _cmp(g, o)
    assert st["n_alignments"] == o["stats"]["alignments"] and st["cells"] == o["stats"]["cells"]


def test_o4_partial_resolution_and_regrowth(monkeypatch):
    """Round 5: a block whose peer list overflows is resolved up to its first overflowing query and only the rest is
    re-run; blocks halved by overflows grow again after `UMICLUST_REGROW` clean, shallow blocks.  A deep molecule's
    long reads sort first (overflowing windows), then shallow short reads (regrowth: fewer blocks than without it);
    with regrowth off, after 1 and after 8 clean blocks, every query's walk, the clusters and the alignment totals
    equal the O4 oracle's."""
    monkeypatch.setenv("UMICLUST_BLOCK", "2048")
    monkeypatch.setenv("ORC_WORKERS", "8")
    deep = synth.make_umis(4, seed=61, max_reads=2500, mean_reads=1500.0, error_rate=0.08, split=(0.4, 0.3, 0.3),
                           pattern_fwd=synth.UMI_FWD_LONG, pattern_rev=synth.UMI_REV_LONG, orient_mix=0.2)
    plain = synth.make_umis(900, seed=62, max_reads=12000, orient_mix=0.2)
    seqs = deep.as_list() + plain.as_list()
    lens = (58, 110)
    o = orc.cluster(_params(orc, 1, 0.90, 25, lens), seqs)
    blocks = {}
    for regrow in ("0", "1", "8"):
        monkeypatch.setenv("UMICLUST_REGROW", regrow)
        with _lib.Context(0) as ctx:
            ctx.load(_lib.params(1, 0.90, *lens, threads=25), seqs)
            st = ctx.cluster()
            g = ctx.fetch()
        assert st["n_reruns"] > 0  # overflows happened
        _cmp(g, o)
        assert st["n_alignments"] == o["stats"]["alignments"] and st["cells"] == o["stats"]["cells"]
        blocks[regrow] = st["n_blocks"]
    assert blocks["1"] < blocks["0"], blocks  # the halved blocks grew again


def test_deep_blocks_never_regrow(monkeypatch):
    """Regrowth gate (advisor round 5): a block whose deepest peer list reaches kPeerCap / 4 is not clean, so even with
    UMICLUST_REGROW=1 a bin whose every window is deep (four molecules of ~600 reads) re-runs overflowing blocks but
    never doubles its block size again (umiclust_stats.n_regrows, ABI 9); the clusters equal the O4 oracle's."""
    monkeypatch.setenv("UMICLUST_BLOCK", "2048")
    monkeypatch.setenv("UMICLUST_REGROW", "1")
    monkeypatch.setenv("ORC_WORKERS", "8")
    seqs = synth.make_umis(4, seed=63, max_reads=2400, mean_reads=1500.0, error_rate=0.02, orient_mix=0.2).as_list()
    with _lib.Context(0) as ctx:
        ctx.load(_lib.params(1, 0.90, 58, 68, threads=25), seqs)
        st = ctx.cluster()
        g = ctx.fetch()
    assert st["n_reruns"] > 0 and st["n_regrows"] == 0, st
    o = orc.cluster(_params(orc, 1, 0.90, 25), seqs)
    _cmp(g, o)
    assert st["n_alignments"] == o["stats"]["alignments"] and st["cells"] == o["stats"]["cells"]
