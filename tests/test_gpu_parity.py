"""GPU parity tests: the HIP path (through the C ABI) against the CPU oracle on the same seeded inputs.
Bit-exact for every integer/byte result: alignment score/matches/internal length/ops, DUST masks,
k-mer sets, cluster membership, strands, centroids, consensus bytes and the written files."""
import os
import random

import numpy as np
import orc
import pytest
from umiclust import _lib, synth

pytestmark = pytest.mark.gpu


def _mutate(rng, a, nedits, alphabet="ACGT"):
    b = list(a)
    for _ in range(nedits):
        x = rng.randrange(len(b))
        u = rng.random()
        if u < 0.4:
            b[x] = rng.choice(alphabet)
        elif u < 0.7:
            b.insert(x, rng.choice(alphabet))
        elif len(b) > 1:
            del b[x]
    return "".join(b)


def _expand(cigar):
    import re
    return "".join(o * (int(n) if n else 1) for n, o in re.findall(r"(\d*)([MDI])", cigar))


def _pairs(seed, n, qlens, tl_lo=16, tl_hi=72, ambig=False):
    rng = random.Random(seed)
    qs, ts = [], []
    alpha = "ACGTN" if ambig else "ACGT"
    for _ in range(n):
        ql = rng.choice(qlens)
        q = "".join(rng.choice("ACGT") for _ in range(ql))
        kind = rng.random()
        if kind < 0.6:
            t = _mutate(rng, q, rng.randint(0, 10), alpha)
        elif kind < 0.8:
            t = "".join(rng.choice(alpha) for _ in range(rng.randint(tl_lo, tl_hi)))
        else:
            t = q[rng.randint(0, 6):] + "".join(rng.choice("ACGT") for _ in range(rng.randint(0, 6)))
        t = t[:tl_hi] if len(t) >= 1 else "A"
        if ambig and rng.random() < 0.3:
            x = rng.randrange(len(q))
            q = q[:x] + rng.choice("NRYKM") + q[x + 1:]
        qs.append(q)
        ts.append(t)
    return qs, ts


@pytest.mark.parametrize("preset,ambig,hi", [(1, False, 72), (2, False, 72), (1, True, 72), (2, True, 72),
                                             (1, False, _lib.MAX_LEN), (2, False, _lib.MAX_LEN),
                                             (1, True, _lib.MAX_LEN), (2, True, _lib.MAX_LEN)])
def test_align_pairs_vs_oracle(gpu_ctx, preset, ambig, hi):
    """Every query length 32..hi (one kernel instantiation each), targets 16..hi."""
    p = _lib.params(preset, 0.93, 32, hi)
    op = orc.params(preset, 0.93, 32, hi)
    qs, ts = _pairs(100 + preset + 10 * ambig + hi, 3000, list(range(32, hi + 1)), tl_hi=hi, ambig=ambig)
    r = gpu_ctx.align_pairs(p, qs, ts)
    tb = gpu_ctx.align_pairs(p, qs, ts, with_ops=True)
    for k, (q, t) in enumerate(zip(qs, ts)):
        o = orc.align(op, q, t)
        got = (int(r["score"][k]), int(r["matches"][k]), int(r["internal_len"][k]))
        assert got == (o["score"], o["matches"], o["internal_len"]), (k, q, t, got, o)
        # explicit traceback kernel agrees with both
        assert tb["ops"][k] == _expand(o["cigar"]), (k, q, t)
        assert (int(tb["score"][k]), int(tb["matches"][k]), int(tb["internal_len"][k])) == got


@pytest.mark.parametrize("preset,hi", [(1, 72), (2, _lib.MAX_LEN), (1, _lib.MAX_LEN)])
def test_align_pairs_banded_vs_oracle(preset, hi, monkeypatch):
    """The banded packed kernel (one pair over a group of 4 or 8 lanes, virtual rows on top of lane 0,
    DPP carries between lanes), forced for every launch: every query length 32..hi, targets 1..hi."""
    monkeypatch.setenv("UMICLUST_BAND", str(1 << 30))
    p = _lib.params(preset, 0.93, 32, hi)
    op = orc.params(preset, 0.93, 32, hi)
    qs, ts = _pairs(700 + preset + hi, 4000, list(range(32, hi + 1)), tl_lo=1, tl_hi=hi)
    with _lib.Context(0) as ctx:
        r = ctx.align_pairs(p, qs, ts)
    for k, (q, t) in enumerate(zip(qs, ts)):
        o = orc.align(op, q, t)
        got = (int(r["score"][k]), int(r["matches"][k]), int(r["internal_len"][k]))
        assert got == (o["score"], o["matches"], o["internal_len"]), (k, q, t, got, o)


@pytest.mark.parametrize("deep", [False, True])
def test_cluster_banded_vs_oracle(deep, monkeypatch):
    """Every walk launch on the banded kernel: short UMIs (config-2 style) and config-5 deep clusters."""
    monkeypatch.setenv("UMICLUST_BAND", str(1 << 30))
    if deep:
        u = synth.make_umis(8, seed=37, max_reads=2500, orient_mix=0.3, mean_reads=1500.0, error_rate=0.15,
                            split=(0.0, 0.5, 0.5), max_edits=4, pattern_fwd=synth.UMI_FWD_LONG,
                            pattern_rev=synth.UMI_REV_LONG)
        args = (1, 0.75, 80, 110)
    else:
        u = synth.make_umis(200, seed=29, max_reads=2500, orient_mix=0.2)
        args = (1, 0.93, 58, 68)
    seqs = u.as_list()
    monkeypatch.setenv("UMICLUST_BLOCK", "256")
    with _lib.Context(0) as ctx:
        ctx.load(_lib.params(*args), seqs)
        st = ctx.cluster()
        g = ctx.fetch()
    o = orc.cluster(orc.params(*args), seqs)
    _cmp_cluster(g, o)
    assert st["n_alignments"] == o["stats"]["alignments"] and st["cells"] == o["stats"]["cells"]


def test_align_known_answers(gpu_ctx):
    p = _lib.params(1, 0.93, 32, 72)
    base = "TTTCGTTCCGCTTGGCATTCCAGTTAGCGTTTAAACGGGAATGCTAACGGCAAGCGTAATGAAA"
    qs = [base, base, "TT" + base[:62], base[:40] + base[41:], base, "G" + "A" * 33 + "C"]
    ts = [base, base[:20] + "A" + base[21:], base[:62], base, base + "TT", "G" + "A" * 32 + "C"]
    r = gpu_ctx.align_pairs(p, qs, ts, with_ops=True)
    assert int(r["score"][0]) == 640 and int(r["internal_len"][0]) == 64
    assert int(r["matches"][1]) == 63
    assert r["ops"][2] == "DD" + "M" * 62  # leading overhang: terminal gap, trimmed
    assert int(r["internal_len"][2]) == 62
    assert r["ops"][4] == "M" * 64 + "II"
    assert r["ops"][5] == "M" + "D" + "M" * 33  # tie: gap placed leftmost (backtrack16 order)


def test_prep_vs_oracle(gpu_ctx):
    rng = random.Random(5)
    seqs = ["ACACACACACACACACACACACACACACACGTAGCTAGCTAGCATCGATCGATCGTAGCTAGCA",
            "TTTAAATTTAAATTTAAATTTAAATTTAAATTTAAATTTGGCCGGCCGGCCGGCCGGCAAAAAAAAAAA"[:72]]
    seqs += synth.make_umis(50, seed=9, max_reads=400).as_list()
    seqs += ["".join(rng.choice("AC") for _ in range(rng.randint(16, 72))) for _ in range(100)]
    seqs += ["".join(rng.choice("ACGTN") for _ in range(rng.randint(16, 72))) for _ in range(100)]
    # long UMIs (config 5): DUST over three 64-nt windows, up to 105 k-mers per strand
    seqs += synth.config_umis(5, 0.002).as_list()[:300]
    seqs += ["".join(rng.choice("AC") for _ in range(rng.randint(73, _lib.MAX_LEN))) for _ in range(50)]
    seqs += ["ACG" * 20 + "".join(rng.choice("ACGT") for _ in range(rng.randint(13, _lib.MAX_LEN - 60)))
             for _ in range(50)]
    p = _lib.params(1, 0.93, 1, _lib.MAX_LEN)
    out = gpu_ctx.prep(p, seqs)
    from pyref import revcomp
    for s, m, km in zip(seqs, out["masked"], out["kmers"]):
        om = orc.dust(s)
        assert m == om
        assert sorted(km[0]) == sorted(set(orc.unique_kmers(om, 8, True)))
        assert sorted(km[1]) == sorted(set(orc.unique_kmers(revcomp(om), 8, True)))


def _cmp_cluster(gpu, ora):
    assert gpu["n_clusters"] == ora["n_clusters"]
    assert np.array_equal(gpu["cluster"], ora["cluster"])
    assert np.array_equal(gpu["strand"], ora["strand"])
    assert np.array_equal(gpu["centroid"], ora["centroid"])
    assert gpu["consensus"] == ora["consensus"]


CASES = [
    # (n_molecules, seed, max_reads, preset, identity, orient_mix, error_rate)
    (60, 1, 800, 1, 0.93, 0.0, 0.015),
    (60, 2, 800, 1, 0.93, 0.4, 0.015),
    (300, 3, 4000, 1, 0.90, 0.1, 0.015),
    (300, 4, 4000, 2, 0.97, 0.1, 0.003),
    (100, 5, 3000, 1, 0.93, 0.2, 0.06),
    (1500, 6, 30000, 1, 0.93, 0.0, 0.015),
]
# config-5 style: long UMIs (~96 nt), 15 % indels, (min, max) length 80..110
LONG_CASES = [
    # (n_molecules, seed, max_reads, preset, identity, orient_mix)
    (8, 11, 2000, 1, 0.75, 0.3),
    (30, 12, 1500, 1, 0.90, 0.0),
    (8, 13, 2000, 2, 0.80, 0.2),
]


@pytest.mark.parametrize("case", LONG_CASES, ids=[f"long_m{c[0]}_s{c[1]}_p{c[3]}_id{c[4]}" for c in LONG_CASES])
def test_cluster_long_vs_oracle(gpu_ctx, case):
    nm, seed, mr, preset, idn, mix = case
    u = synth.make_umis(nm, seed=seed, max_reads=mr, orient_mix=mix, mean_reads=1500.0, error_rate=0.15,
                        split=(0.0, 0.5, 0.5), max_edits=4, pattern_fwd=synth.UMI_FWD_LONG,
                        pattern_rev=synth.UMI_REV_LONG)
    seqs = u.as_list()
    gpu_ctx.load(_lib.params(preset, idn, 80, 110), seqs)
    st = gpu_ctx.cluster()
    g = gpu_ctx.fetch()
    o = orc.cluster(orc.params(preset, idn, 80, 110), seqs)
    _cmp_cluster(g, o)
    assert st["n_alignments"] == o["stats"]["alignments"]
    assert st["cells"] == o["stats"]["cells"]


@pytest.mark.parametrize("case", CASES, ids=[f"m{c[0]}_s{c[1]}_p{c[3]}_id{c[4]}" for c in CASES])
def test_cluster_vs_oracle(gpu_ctx, case):
    nm, seed, mr, preset, idn, mix, err = case
    u = synth.make_umis(nm, seed=seed, max_reads=mr, orient_mix=mix, error_rate=err)
    seqs = u.as_list()
    gpu_ctx.load(_lib.params(preset, idn, 58, 68), seqs)
    st = gpu_ctx.cluster()
    g = gpu_ctx.fetch()
    o = orc.cluster(orc.params(preset, idn, 58, 68), seqs)
    _cmp_cluster(g, o)
    assert st["n_alignments"] == o["stats"]["alignments"]
    assert st["cells"] == o["stats"]["cells"]


@pytest.mark.parametrize("block", [1, 7, 64, 1000])
def test_block_size_invariance(block, monkeypatch):
    """Small greedy blocks stress the in-block dependency resolution (deferred queries, peers)."""
    u = synth.make_umis(200, seed=21, max_reads=2500, orient_mix=0.2)
    seqs = u.as_list()
    monkeypatch.setenv("UMICLUST_BLOCK", str(block))
    with _lib.Context(0) as ctx:
        ctx.load(_lib.params(1, 0.93, 58, 68), seqs)
        ctx.cluster()
        g = ctx.fetch()
    _cmp_cluster(g, orc.cluster(orc.params(1, 0.93, 58, 68), seqs))


@pytest.mark.parametrize("split", ["0", "1", "2"])
@pytest.mark.parametrize("block", [7, 64, 1000])
def test_pipeline_modes(split, block, monkeypatch):
    """Whole passes (UMICLUST_SPLIT=0) and split passes -- the counting half against the index before the
    block two ahead is resolved, that block's hits flagged and kept by the merge only if they turn out
    centroids -- on the main stream (1) or on their own stream (2): membership, strands, centroids,
    consensus, alignment count and cells equal the oracle's for any block size."""
    u = synth.make_umis(200, seed=23, max_reads=2500, orient_mix=0.2)
    seqs = u.as_list()
    monkeypatch.setenv("UMICLUST_BLOCK", str(block))
    monkeypatch.setenv("UMICLUST_SPLIT", split)
    with _lib.Context(0) as ctx:
        ctx.load(_lib.params(1, 0.93, 58, 68), seqs)
        st = ctx.cluster()
        g = ctx.fetch()
    o = orc.cluster(orc.params(1, 0.93, 58, 68), seqs)
    _cmp_cluster(g, o)
    assert st["n_alignments"] == o["stats"]["alignments"] and st["cells"] == o["stats"]["cells"]


def _ragged_lengths(seed, n_mol=40, max_reads=3000):
    """Long high-error UMIs cut to random lengths 40..112: bins whose blocks span many query lengths."""
    u = synth.make_umis(n_mol, seed=seed, max_reads=max_reads, orient_mix=0.2, mean_reads=80.0, error_rate=0.05,
                        split=(0.0, 0.5, 0.5), max_edits=3, pattern_fwd=synth.UMI_FWD_LONG, pattern_rev=synth.UMI_REV_LONG)
    rng = np.random.default_rng(seed)
    return [x[:int(rng.integers(40, min(len(x), 112) + 1))] if len(x) > 40 else x for x in u.as_list()]


@pytest.mark.parametrize("mix", ["0", "1"])
@pytest.mark.parametrize("block,split", [("default", "default"), ("300", "0"), ("300", "1"), ("97", "1")])
def test_mixed_length_blocks(mix, block, split, monkeypatch):
    """Greedy blocks across query-length changes (UMICLUST_MIXLEN, default on): the walk and the peer pairs append to
    per-length pair segments, one alignment launch per length and round, round B per run of one length, blocks of
    at most kSegLens (32) lengths -- here 40..112 nt in one bin; equal to the oracle with and without mixing."""
    seqs = _ragged_lengths(41)
    monkeypatch.setenv("UMICLUST_MIXLEN", mix)
    if block != "default":
        monkeypatch.setenv("UMICLUST_BLOCK", block)
    if split != "default":
        monkeypatch.setenv("UMICLUST_SPLIT", split)
    p = (1, 0.85, 32, _lib.MAX_LEN)
    with _lib.Context(0) as ctx:
        ctx.load(_lib.params(*p), seqs)
        st = ctx.cluster()
        g = ctx.fetch()
    o = orc.cluster(orc.params(*p), seqs)
    _cmp_cluster(g, o)
    assert st["n_alignments"] == o["stats"]["alignments"] and st["cells"] == o["stats"]["cells"]


@pytest.mark.parametrize("split", ["0", "1", "2"])
def test_pipeline_modes_deep_clusters(split, monkeypatch):
    """Config-5 style deep clusters (long UMIs, 15 % indels) with small blocks: peer lists overflow, blocks
    re-run alone and the pipeline restarts mid-bin, in every pipeline mode."""
    u = synth.make_umis(8, seed=31, max_reads=2500, orient_mix=0.3, mean_reads=1500.0, error_rate=0.15,
                        split=(0.0, 0.5, 0.5), max_edits=4, pattern_fwd=synth.UMI_FWD_LONG,
                        pattern_rev=synth.UMI_REV_LONG)
    seqs = u.as_list()
    # blocks of 1024: a two-block window holds ~250 reads of each molecule, past the 128-peer cap (kPeerCap)
    monkeypatch.setenv("UMICLUST_BLOCK", "1024")
    monkeypatch.setenv("UMICLUST_SPLIT", split)
    with _lib.Context(0) as ctx:
        ctx.load(_lib.params(1, 0.75, 80, 110), seqs)
        st = ctx.cluster()
        g = ctx.fetch()
    o = orc.cluster(orc.params(1, 0.75, 80, 110), seqs)
    _cmp_cluster(g, o)
    assert st["n_alignments"] == o["stats"]["alignments"] and st["cells"] == o["stats"]["cells"]
    assert st["n_reruns"] > 0  # the overflow re-run and the pipeline restart were exercised


@pytest.mark.parametrize("lanes", [3])
def test_lanes_with_overflowing_bin(lanes, monkeypatch):
    """Several lanes, two of whose bins overflow their peer lists (deep clusters: synchronous re-runs while the other
    lanes keep clustering), and every bin's membership, strands, centroids and consensus equal the oracle's."""
    from umiclust import binset
    deep = lambda seed: synth.make_umis(6, seed=seed, max_reads=1800, orient_mix=0.3, mean_reads=1500.0,  # noqa: E731
                                        error_rate=0.15, split=(0.0, 0.5, 0.5), max_edits=4,
                                        pattern_fwd=synth.UMI_FWD_LONG, pattern_rev=synth.UMI_REV_LONG)
    plain = lambda seed: synth.make_umis(150, seed=seed, max_reads=2500, orient_mix=0.2,  # noqa: E731
                                         pattern_fwd=synth.UMI_FWD_LONG, pattern_rev=synth.UMI_REV_LONG)
    sets = [deep(51), plain(52), deep(53), plain(54), plain(55)]
    bs = synth.concat_bins([synth.Bin(0, i, i, 0, u) for i, u in enumerate(sets)])
    monkeypatch.setenv("UMICLUST_BLOCK", "1024")
    with _lib.Context(0) as ctx:
        run = binset.BinRunner(ctx, bs, 1, 0.75, 80, 110, lanes=lanes)
        st = run.cluster_all()
        res = run.results()
        run.close()
    assert sum(x["n_reruns"] for x in st) > 0
    for u, r in zip(sets, res):
        o = orc.cluster(orc.params(1, 0.75, 80, 110), u.as_list())
        assert binset.digest(r) == binset.digest(o)


@pytest.mark.parametrize("split", ["0", "1"])
def test_two_counter_segments(split, monkeypatch):
    """A bin past one counter segment (> 7 x 65,536 centroids: synth.segment_stress, 470k random 64-mers and
    1-substitution copies of sequences from both segments): the full kernel counts both segments and keeps a
    running top-41 across them (the split pipeline falls back to whole passes once the index spans two
    segments).  Alignment count, cells and the membership / strand / centroid / consensus digests equal the
    oracle's (tests/golden/oracle_segments.json, make_oracle_golden.py segments)."""
    import json
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    from make_oracle_golden import digest
    gold = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                                       "oracle_segments.json")))["segments_round1_id090"]
    buf, off = synth.segment_stress()
    monkeypatch.setenv("UMICLUST_SPLIT", split)
    with _lib.Context(0) as ctx:
        ctx.load(_lib.params(1, 0.90, 58, 68), buf=buf, off=off)
        st = ctx.cluster()
        g = ctx.fetch()
    assert st["n_clusters"] > 7 * 65536  # two counter segments
    d = digest(g)
    assert st["n_alignments"] == gold["alignments"] and st["cells"] == gold["cells"]
    for k in ("n_clusters", "cluster", "strand", "centroid", "consensus"):
        assert d[k] == gold[k], k


def test_edge_inputs(gpu_ctx):
    p = _lib.params(1, 0.93, 58, 68)
    op = orc.params(1, 0.93, 58, 68)
    base = "TTTCGTTCCGCTTGGCATTCCAGTTAGCGTTTAAACGGGAATGCTAACGGCAAGCGTAATGAAA"
    for seqs in ([], ["ACGT"], [base], [base] * 5, [base, base[:57], base + "ACGTA", base[:58], base + "A" * 4],
                 [base.replace("G", "N", 3)] * 3 + [base]):
        gpu_ctx.load(p, seqs)
        gpu_ctx.cluster()
        g = gpu_ctx.fetch()
        o = orc.cluster(op, seqs) if seqs else dict(n_clusters=0, cluster=np.zeros(0, np.int32),
                                                     strand=np.zeros(0, np.uint8),
                                                     centroid=np.zeros(0, np.uint8), consensus=[])
        _cmp_cluster(g, o)


def _read_dir(d):
    return {fn: open(os.path.join(d, fn), "rb").read() for fn in sorted(os.listdir(d)) if not fn.endswith(".log")}


@pytest.mark.parametrize("policy", ["o4", "sequential"])
@pytest.mark.parametrize("round_", [1, 2])
def test_dropin_files_vs_oracle(tmp_path, round_, policy, monkeypatch):
    """The drop-in with the reference's arguments (threads=25): byte-identical files to the oracle in vsearch's
    --threads 25 mode (the default, policy O4) and, with UMICLUST_O4=sequential, in the sequential definition."""
    from umiclust.vsearch_umi_cluster import vsearch_cluster, vsearch_cluster_consensus
    if policy == "sequential":
        monkeypatch.setenv("UMICLUST_O4", "sequential")
    else:
        monkeypatch.delenv("UMICLUST_O4", raising=False)
    u = synth.make_umis(150, seed=31 + round_, max_reads=2500, orient_mix=0.1,
                       error_rate=0.015 if round_ == 1 else 0.002)
    fa = tmp_path / "region_cluster7_detected_umis.fasta"
    synth.write_umi_fasta(str(fa), u)
    out = tmp_path / "gpu"
    out.mkdir()
    if round_ == 1:
        ret = vsearch_cluster.options(num_cpus=25).remote(umi_fasta=str(fa), clustering_out_dir=str(out),
                                                          threads=25, min_umi_length=58, max_umi_length=68,
                                                          identity=0.93)
        log = "vsearch_cluster.log"
    else:
        ret = vsearch_cluster_consensus.options(num_cpus=25).remote(
            umi_fasta=str(fa), clustering_consensus_out_dir=str(out), threads=25, min_umi_length=58,
            max_umi_length=68, identity=0.97)
        log = "vsearch_cluster_consensus.log"
    assert ret == os.path.join(str(out), "umi_clusters_consensus.fasta")
    assert (out / log).exists()
    ref = tmp_path / "oracle"
    ref.mkdir()
    op = orc.params(1 if round_ == 1 else 2, 0.93 if round_ == 1 else 0.97, 58, 68)
    if policy == "o4":
        op.threads, op.policy_threads = 25, 1
    orc.run_fasta(op, str(fa), str(ref) + "/cluster", str(ref / "umi_clusters_consensus.fasta"))
    assert _read_dir(out) == _read_dir(ref)
    # the consumer runs unchanged on the GPU outputs
    from umiclust.parse_umi_clusters import parse_umi_clusters
    sm = parse_umi_clusters.remote(ret, str(tmp_path / "wo.txt"), min_reads_per_cluster=4, max_reads_per_cluster=60)
    assert sm and os.path.exists(sm)


def _tree(d):
    out = {}
    for root, _, files in os.walk(d):
        for fn in files:
            if not fn.endswith(".log") or fn == "parse_cluster.log":
                p = os.path.join(root, fn)
                out[os.path.relpath(p, d)] = open(p, "rb").read()
    return out


PARSE_CASES = [
    # (round, min_reads, max_reads, balance, max_clusters, dup_ids, molecules)
    (1, 4, 60, False, None, False, 120),
    (1, 2, 5, True, None, True, 120),
    (1, 3, 8, False, 5, True, 120),
    (2, 1, 4, False, None, False, 120),
    (1, 100000, 60, False, None, False, 120),  # nothing written: the empty-region branch
    # >= 256 clusters: the parse runs on io_threads() threads (early exit inside a later thread's range)
    (1, 4, 60, False, None, True, 900),
    (1, 2, 8, True, 400, False, 900),
]


@pytest.mark.parametrize("case", PARSE_CASES, ids=[f"r{c[0]}_min{c[1]}_max{c[2]}_b{int(c[3])}_mc{c[4]}_d{int(c[5])}_m{c[6]}"
                                                  for c in PARSE_CASES])
def test_fused_parse_matches_two_step(tmp_path, case):
    """§8f f2: vsearch_cluster_and_parse writes the same bytes as vsearch_cluster followed by the
    (reference-pinned, tests/test_parse_golden.py) parse_umi_clusters restatement, with and without the
    intermediate cluster<N> files."""
    from umiclust.parse_umi_clusters import parse_umi_clusters, vsearch_cluster_and_parse
    from umiclust.vsearch_umi_cluster import vsearch_cluster, vsearch_cluster_consensus
    round_, mn, mx, bal, mc, dup, nmol = case
    u = synth.make_umis(nmol, seed=41 + mn, max_reads=2000 * nmol // 120, orient_mix=0.1,
                        error_rate=0.015 if round_ == 1 else 0.002)
    fa = tmp_path / "in.fasta"
    synth.write_umi_fasta(str(fa), u)
    if dup:  # repeated read ids (kept once per strand, at the first position, with the last record)
        lines = fa.read_text().splitlines(True)
        hdrs = [i for i, ln in enumerate(lines) if ln.startswith(">")]
        rng = random.Random(5)
        for i in rng.sample(hdrs, len(hdrs) // 4):
            j = rng.choice(hdrs)
            lines[i] = lines[j].split(";", 1)[0] + ";" + lines[i].split(";", 1)[1]
        fa.write_text("".join(lines))
    idn = 0.93 if round_ == 1 else 0.97
    kw = dict(min_reads_per_cluster=mn, max_reads_per_cluster=mx, balance_strands=bal, max_clusters=mc)
    a = tmp_path / "region_cluster3"
    a.mkdir()
    if round_ == 1:
        cons = vsearch_cluster.remote(str(fa), str(a), 25, 58, 68, idn)
    else:
        cons = vsearch_cluster_consensus.remote(str(fa), str(a), 25, 58, 68, idn)
    ra = parse_umi_clusters.remote(cons, str(tmp_path / "wo_a.txt"), **kw)
    for write in (True, False):
        b = tmp_path / f"fused{int(write)}" / "region_cluster3"
        b.mkdir(parents=True)
        rb = vsearch_cluster_and_parse.remote(str(fa), str(b), 25, str(tmp_path / f"wo_b{int(write)}.txt"), 58, 68, idn,
                                              round_=round_, write_cluster_files=write, **kw)
        assert (ra is None) == (rb is None)
        ta, tb = _tree(a), _tree(b)
        if not write:
            ta = {k: v for k, v in ta.items() if not (k.startswith("cluster") and "/" not in k)}
        assert sorted(ta) == sorted(tb)
        for k in ta:
            # paths inside the log name the work dir
            assert ta[k].replace(str(a).encode(), b"@") == tb[k].replace(str(b).encode(), b"@"), k
        if ra is None:
            assert open(tmp_path / "wo_a.txt").read() == open(tmp_path / f"wo_b{int(write)}.txt").read()


def test_run_argv_matches_reference_argv(tmp_path):
    """umiclust_run_argv consumes the exact argv the reference passes to vsearch."""
    from umiclust.vsearch_umi_cluster import context, round1_argv
    u = synth.make_umis(40, seed=77, max_reads=600)
    fa = tmp_path / "in.fasta"
    synth.write_umi_fasta(str(fa), u)
    (tmp_path / "o").mkdir()
    st = context().run_argv(round1_argv(str(fa), str(tmp_path / "o"), 25, 58, 68, 0.93))
    op = orc.params(1, 0.93, 58, 68)
    op.threads, op.policy_threads = 25, 1  # --threads 25: vsearch's multithreaded clustering
    o = orc.run_fasta(op, str(fa), None, None)
    assert (st["n_clusters"], st["n_alignments"]) == (o["n_clusters"], o["alignments"])


def test_full_scale_properties():
    """BASELINE config 2 size (2M reads): deterministic across runs and structurally valid."""
    u = synth.config_umis(2)
    with _lib.Context(0) as ctx:
        ctx.load(_lib.params(1, 0.90, 58, 68), buf=u.seq, off=u.off)
        s1 = ctx.cluster()
        a = ctx.fetch()
        s2 = ctx.cluster()
        b = ctx.fetch()
    _cmp_cluster(a, b)
    assert s1["n_alignments"] == s2["n_alignments"] and s1["cells"] == s2["cells"]
    cl = a["cluster"]
    k = a["n_clusters"]
    sizes = np.bincount(cl[cl >= 0], minlength=k)
    assert np.all(np.diff(sizes) <= 0)  # --clusterout_sort
    assert int(a["centroid"].sum()) == k
    lens = np.diff(u.off)
    cen_len = np.zeros(k, np.int64)
    cen_len[cl[a["centroid"] == 1]] = lens[a["centroid"] == 1]
    kept = cl >= 0
    assert np.all(lens[kept] <= cen_len[cl[kept]])  # centroids are the longest of their cluster
    # K3T traceback + K4 consensus of the largest clusters (and of every unusually short consensus,
    # which round-1's free terminal gaps legitimately produce for shifted members), recomputed on the
    # CPU from the GPU's own membership with the oracle aligner and the Python MSA restatement
    seqs = u.as_list()
    short = [c for c, s in enumerate(a["consensus"]) if len(s) < 56][:40]
    _check_consensus_cpu(seqs, a, sorted(set(range(150)) | set(short)), orc.params(1, 0.90, 58, 68))


def _check_consensus_cpu(seqs, a, targets, op):
    import pyref
    lens = np.array([len(s) for s in seqs])
    members = {}
    for i in sorted(range(len(seqs)), key=lambda i: -lens[i]):  # stable: sorted-db order
        if a["cluster"][i] >= 0:
            members.setdefault(int(a["cluster"][i]), []).append(i)
    for c in targets:
        mem = members[c]
        cen = [i for i in mem if a["centroid"][i]]
        assert len(cen) == 1
        mem = cen + [i for i in mem if i != cen[0]]
        db = {i: orc.dust(seqs[i]) for i in mem}
        strand = {i: int(a["strand"][i]) for i in mem}
        cig = {i: orc.align(op, pyref.revcomp(db[i]) if strand[i] else db[i], db[cen[0]])["cigar"] for i in mem[1:]}
        assert pyref.msa(db, mem, strand, cig) == a["consensus"][c], c


def _golden_cases():
    import glob
    import json
    out = {}
    for path in sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                                              "oracle_config*.json"))):
        out.update(json.load(open(path)))
    return sorted((k, v) for k, v in out.items() if "n_bins" not in v)


def _multibin_cases():
    import glob
    import json
    out = {}
    for path in sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                                              "oracle_config*.json"))):
        out.update(json.load(open(path)))
    return sorted((k, v) for k, v in out.items() if "n_bins" in v)


@pytest.mark.parametrize("name,gold", _multibin_cases(), ids=[n for n, _ in _multibin_cases()])
@pytest.mark.parametrize("split,pack", [("default", 0), ("1", 0), ("default", 3000), ("1", 20000), ("0", 1 << 30),
                                        ("lanes4prio", 3000)])
def test_multibin_vs_oracle_golden(name, gold, split, pack, monkeypatch):
    """BASELINE configs 3 (24 barcodes x 40 Zipf bins) and 4 (both rounds, round 2 on the round-1 consensus
    UMIs) at reduced scale: every bin resident in one load, clustered bin by bin or in packs of consecutive bins
    (umiclust_cluster_pack: one greedy order over the pack, blocks across bin boundaries, the prefilter keeping a
    query's own bin; up to 3k / 20k reads per pack, or the whole set as one pack); the checksum of the per-bin
    digests (membership, strands, centroids, consensus) and every bin's cluster count equal the oracle's."""
    from umiclust import binset, synth
    lanes, prio = (4, True) if split == "lanes4prio" else (1, False)  # 4 lanes, the largest bin's on the priority stream
    if split not in ("default", "lanes4prio"):  # multi-bin sets run whole passes unless UMICLUST_SPLIT says otherwise
        monkeypatch.setenv("UMICLUST_SPLIT", split)
    bs = synth.concat_bins(synth.config_bins(gold["config"], gold["scale"], workers=4))
    assert len(bs.bins) == gold["n_bins"] and bs.n == gold["n_reads"]
    rounds = [("round1", binset.ROUND1)] + ([("round2", binset.ROUND2)] if "round2" in gold else [])
    for rname, prm in rounds:
        g = gold[rname]
        with _lib.Context(0) as ctx:
            run = binset.BinRunner(ctx, bs, prm["preset"], prm["identity"], gold["minlen"], gold["maxlen"],
                                   pack_reads=pack, lanes=lanes, critical_priority=prio)
            assert (run.critical_lane is not None) == prio
            st = run.cluster_all()
            res = run.results()
            run.close()
        assert bs.n == g["n_reads"]
        dg = [binset.digest(r) for r in res]
        assert [d["n_clusters"] for d in dg] == g["n_clusters"], rname
        assert sum(x["n_alignments"] for x in st) == g["alignments"] and sum(x["cells"] for x in st) == g["cells"]
        assert binset.combine(dg) == g["combined"], rname
        if rname == "round1":
            bs = binset.round2_binset(bs, res)


@pytest.mark.parametrize("name,gold", _golden_cases(), ids=[n for n, _ in _golden_cases()])
def test_config_vs_oracle_golden(gpu_ctx, name, gold):
    """BASELINE config 1 (100k reads) and config 2 (the headline: 2M reads, one bin, --id 0.90; the oracle took
    7,201 s on one core) at full size, and config-5 stress samples (long UMIs, 15 % indels, clusters of >1k
    members): the alignment count and cells of vsearch's procedure, and the digests of membership, strands,
    centroids and consensus, equal the CPU oracle's (committed by tests/golden/make_oracle_golden.py)."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    from make_oracle_golden import digest
    u = synth.config_umis(gold["config"], gold["scale"])
    gpu_ctx.load(_lib.params(gold["preset"], gold["identity"], gold.get("minlen", 58), gold.get("maxlen", 68)),
                 buf=u.seq, off=u.off)
    st = gpu_ctx.cluster()
    d = digest(gpu_ctx.fetch())
    assert st["n_alignments"] == gold["alignments"] and st["cells"] == gold["cells"]
    for k in ("n_clusters", "cluster", "strand", "centroid", "consensus"):
        assert d[k] == gold[k], k


@pytest.mark.parametrize("packs", [[(0, 7)], [(0, 3), (3, 4)], [(2, 3), (0, 2), (5, 2)]])
def test_pack_edge_cases(gpu_ctx, packs):
    """umiclust_cluster_pack over the same edge-case bins (empty, fully length-filtered, one-record and ordinary bins)
    as the whole load, two packs, or packs clustered out of order: every bin equals the oracle run on it alone."""
    base = "TTTCGTTCCGCTTGGCATTCCAGTTAGCGTTTAAACGGGAATGCTAACGGCAAGCGTAATGAAA"
    groups = [[], ["ACGT", "ACGTACGT"], [base], synth.make_umis(40, seed=61, max_reads=500, orient_mix=0.2).as_list(),
              [], synth.make_umis(25, seed=62, max_reads=300).as_list(), [base[:57], base + "A" * 5]]
    buf, off = _lib._pack([s for g in groups for s in g])
    starts = np.cumsum([0] + [len(g) for g in groups])
    op = orc.params(1, 0.93, 58, 68)
    gpu_ctx.load_bins(_lib.params(1, 0.93, 58, 68), buf, off, starts)
    for first, m in packs:
        gpu_ctx.cluster_pack(first, m)
    for b, g in enumerate(groups):
        got = gpu_ctx.fetch_bin(b)
        want = orc.cluster(op, g) if g else dict(n_clusters=0, cluster=np.zeros(0, np.int32), strand=np.zeros(0, np.uint8),
                                                centroid=np.zeros(0, np.uint8), consensus=[])
        _cmp_cluster(got, want)


def test_pack_errors(gpu_ctx):
    """A pack past the load's bins and an empty pack fail with EINVAL (packs under the batched O4 policy are
    tests/test_gpu_o4.py's)."""
    seqs = synth.make_umis(20, seed=63, max_reads=200).as_list()
    buf, off = _lib._pack(seqs + seqs)
    gpu_ctx.load_bins(_lib.params(1, 0.93, 58, 68), buf, off, [0, len(seqs), 2 * len(seqs)])
    for first, m in [(1, 2), (0, 0), (-1, 2)]:
        with pytest.raises(_lib.UmiclustError):
            gpu_ctx.cluster_pack(first, m)


def test_load_bins_edge_cases(gpu_ctx):
    """umiclust_load_bins: empty bins, bins whose every record is length-filtered, one-record bins and
    ordinary bins in one load; each bin equals the oracle run on that bin alone, in any clustering order."""
    base = "TTTCGTTCCGCTTGGCATTCCAGTTAGCGTTTAAACGGGAATGCTAACGGCAAGCGTAATGAAA"
    groups = [[], ["ACGT", "ACGTACGT"], [base], synth.make_umis(40, seed=61, max_reads=500, orient_mix=0.2).as_list(),
              [], synth.make_umis(25, seed=62, max_reads=300).as_list(), [base[:57], base + "A" * 5]]
    buf, off = _lib._pack([s for g in groups for s in g])
    starts = np.cumsum([0] + [len(g) for g in groups])
    op = orc.params(1, 0.93, 58, 68)
    gpu_ctx.load_bins(_lib.params(1, 0.93, 58, 68), buf, off, starts)
    for b in [5, 0, 3, 1, 6, 2, 4]:  # out of order: bins are independent
        gpu_ctx.cluster_bin(b)
    for b, g in enumerate(groups):
        got = gpu_ctx.fetch_bin(b)
        want = orc.cluster(op, g) if g else dict(n_clusters=0, cluster=np.zeros(0, np.int32), strand=np.zeros(0, np.uint8),
                                                centroid=np.zeros(0, np.uint8), consensus=[])
        _cmp_cluster(got, want)


def test_stage_prepare_equals_load():
    """umiclust_stage + umiclust_prepare (ABI 6; bench.py times prepare + cluster per step) equal umiclust_load:
    preparing the same staged records again, or with other parameters, gives the oracle's result each time; a
    multi-bin staging prepares every bin."""
    seqs = synth.make_umis(300, seed=77, max_reads=6000, error_rate=0.03, orient_mix=0.2).as_list()
    seqs += ["ACGT" * 5, "T" * 80]  # length-filtered at either end
    buf, off = _lib._pack(seqs)
    with _lib.Context(0) as ctx:
        ctx.stage(buf, off)
        for idn, lens in [(0.93, (58, 68)), (0.93, (58, 68)), (0.97, (60, 68))]:
            p = _lib.params(1, idn, *lens)
            ctx.prepare(p)
            st = ctx.cluster()
            o = orc.cluster(orc.params(1, idn, *lens), seqs)
            _cmp_cluster(ctx.fetch(), o)
            assert st["n_alignments"] == o["stats"]["alignments"] and st["n_kept"] == o["stats"]["kept"]
        starts = [0, 2000, 2000, len(seqs)]
        ctx.stage(buf, off, starts)
        ctx.prepare(_lib.params(1, 0.93, 58, 68))
        for b in range(3):
            ctx.cluster_bin(b)
            g = seqs[starts[b]:starts[b + 1]]
            if g:
                _cmp_cluster(ctx.fetch_bin(b), orc.cluster(orc.params(1, 0.93, 58, 68), g))
    with _lib.Context(0) as ctx, pytest.raises(_lib.UmiclustError):
        ctx.prepare(_lib.params(1, 0.93, 58, 68))  # nothing staged


@pytest.mark.parametrize("name", ["config1_round1_id093", "config1_round2_id097"])
def test_parallel_inorder_phase_every_block(name, monkeypatch):
    """The dependency-ordered in-order resolve phase on the pool (resolve.cpp, on by default from 4096 open queries)
    forced onto every block (UMICLUST_PAR_MIN=1) of the full config-1 bin: alignment count, cells and digests equal
    the oracle's (the default-setting case on 8192-query blocks is the config-2 golden above)."""
    from make_oracle_golden import digest
    gold = dict(_golden_cases())[name]
    monkeypatch.setenv("UMICLUST_PAR_MIN", "1")
    u = synth.config_umis(gold["config"], gold["scale"])
    with _lib.Context(0) as ctx:
        ctx.load(_lib.params(gold["preset"], gold["identity"], gold.get("minlen", 58), gold.get("maxlen", 68)),
                 buf=u.seq, off=u.off)
        st = ctx.cluster()
        d = digest(ctx.fetch())
    assert st["n_alignments"] == gold["alignments"] and st["cells"] == gold["cells"]
    for k in ("n_clusters", "cluster", "strand", "centroid", "consensus"):
        assert d[k] == gold[k], k


def test_timeline_union_and_counter_cells():
    """umiclust_timeline: one context's counting launches are serial on its stream, so the union of their HIP-event
    brackets equals their sum (umiclust_stats.t_count_s) and the bracket count equals n_count_launches;
    counter_cells (ABI 8) = sum over the counting launches of query-strands x centroids indexed."""
    u = synth.config_umis(1, 0.1)
    with _lib.Context(0) as ctx:
        ctx.load(_lib.params(_lib.PRESET_ROUND1, 0.93, 58, 68, threads=25), buf=u.seq, off=u.off)
        _lib.timeline(0, reset=True)
        st = ctx.cluster()
        busy, n = _lib.timeline(0)
        abusy, an = _lib.timeline(1)
    assert n == st["n_count_launches"] > 0
    assert abs(busy - st["t_count_s"]) <= 0.02 * st["t_count_s"] + 1e-4
    assert an > 0 and 0 < abusy <= st["t_align_s"] * 1.02 + 1e-4
    assert 0 < st["counter_cells"] <= st["n_count_launches"] * 2 * 8192 * st["n_kept"]


@pytest.mark.parametrize("pf1", ["0", str(1 << 30)])
def test_counting_wave_layouts(pf1, monkeypatch):
    """k_pf_count's two workgroup layouts (4 waves with block-wide scans, or one-wave units, UMICLUST_PF1 = the LDS
    bound below which units run as one wave) forced over the whole config-1 bin: alignment count, cells and digests
    equal the oracle's golden either way."""
    from make_oracle_golden import digest
    gold = dict(_golden_cases())["config1_round1_id093"]
    monkeypatch.setenv("UMICLUST_PF1", pf1)
    u = synth.config_umis(gold["config"], gold["scale"])
    with _lib.Context(0) as ctx:
        ctx.load(_lib.params(gold["preset"], gold["identity"], gold.get("minlen", 58), gold.get("maxlen", 68)),
                 buf=u.seq, off=u.off)
        st = ctx.cluster()
        d = digest(ctx.fetch())
    assert st["n_alignments"] == gold["alignments"] and st["cells"] == gold["cells"]
    for k in ("n_clusters", "cluster", "strand", "centroid", "consensus"):
        assert d[k] == gold[k], k


def test_file_path_releases_input_after_return(tmp_path):
    """The file-path calls release their input on a thread of the context after writing every output
    (umiclust_wait_host): back-to-back calls on one context (the second joins the first's release) write the oracle's
    files, and the input can be replaced between them."""
    u = synth.make_umis(120, seed=77, max_reads=2000, orient_mix=0.1, error_rate=0.01)
    fa = tmp_path / "in.fasta"
    synth.write_umi_fasta(str(fa), u)
    ref = tmp_path / "oracle"
    ref.mkdir()
    op = orc.params(1, 0.93, 58, 68)
    op.threads, op.policy_threads = 25, 1
    orc.run_fasta(op, str(fa), str(ref) + "/cluster", str(ref / "umi_clusters_consensus.fasta"))
    p = _lib.params(_lib.PRESET_ROUND1, 0.93, 58, 68, threads=25)
    with _lib.Context(0) as ctx:
        for rep in range(3):
            out = tmp_path / f"gpu{rep}"
            out.mkdir()
            ctx.run_fasta(p, str(fa), str(out) + "/cluster", str(out / "umi_clusters_consensus.fasta"), None)
            if rep == 1:
                ctx.wait_host()
                tmp = tmp_path / "in.tmp"
                synth.write_umi_fasta(str(tmp), u)
                os.replace(tmp, fa)  # the old file's mapping is gone; the next call maps the new one
            assert _read_dir(out) == _read_dir(ref)
        ctx.wait_host()
        ctx.wait_host()  # idempotent
