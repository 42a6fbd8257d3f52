"""Seeded synthetic UMI workloads.

A molecule's UMI instantiates the reference's default patterns
(`umi_fwd` / `umi_rev`, /root/reference/configs/run_config.json:11-12: V in {A,C,G},
B in {C,G,T}) into a 64-nt combined UMI, written molecule-oriented for both read strands
exactly as `combine_umis_fasta` does (/root/reference/ont_tcr_consensus/extract_umis.py:140-151).
Reads per molecule ~ NegBin(mean, dispersion), >=1; strand ~ Bernoulli(0.5); per-base errors
(substitution : insertion : deletion = 0.4 : 0.3 : 0.3) capped at `max_edits` per 32-nt half
(mirrors `max_pattern_dist`, run_config.json:13).  Everything is vectorised numpy so that the
2M-read configuration generates in seconds.
"""
from __future__ import annotations

import dataclasses
import uuid

import numpy as np

UMI_FWD = "TTTVVTTVVVVTTVVVVTTVVVVTTVVVVTTT"
UMI_REV = "AAABBBBAABBBBAABBBBAABBBBAABBAAA"
ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)
_COMP = np.zeros(256, np.uint8)
for _a, _b in zip(b"ACGTNacgtn", b"TGCANtgcan"):
    _COMP[_a] = _b


@dataclasses.dataclass
class UmiSet:
    """Concatenated UMI bytes + per-record metadata (input order)."""
    seq: np.ndarray          # uint8, concatenated ASCII
    off: np.ndarray          # int64 [n+1]
    molecule: np.ndarray     # int64 [n] true molecule id
    strand: np.ndarray       # uint8 [n] 0 '+', 1 '-'
    fwd_dist: np.ndarray     # int8 [n] edits in 5' half
    rev_dist: np.ndarray     # int8 [n] edits in 3' half

    @property
    def n(self) -> int:
        return len(self.off) - 1

    @property
    def lens(self) -> np.ndarray:
        return np.diff(self.off).astype(np.int32)

    def get(self, i: int) -> str:
        return self.seq[self.off[i]:self.off[i + 1]].tobytes().decode()

    def as_list(self) -> list[str]:
        raw = self.seq.tobytes()
        return [raw[self.off[i]:self.off[i + 1]].decode() for i in range(self.n)]


def _instantiate(pattern: str, n: int, rng: np.random.Generator) -> np.ndarray:
    pat = np.frombuffer(pattern.encode(), np.uint8)
    out = np.empty((n, len(pat)), np.uint8)
    alph = {ord("V"): np.frombuffer(b"ACG", np.uint8), ord("B"): np.frombuffer(b"CGT", np.uint8)}
    for j, c in enumerate(pat):
        if c in alph:
            out[:, j] = alph[c][rng.integers(0, 3, n)]
        else:
            out[:, j] = c
    return out


def _mutate_half(base: np.ndarray, rate: float, split: tuple[float, float, float], max_edits: int,
                 rng: np.random.Generator):
    """base: (R, L) uint8.  Returns (flat bytes, lengths, edits) with vectorised indels."""
    R, L = base.shape
    ev = rng.random((R, L)) < rate
    kind = rng.choice(3, size=(R, L), p=np.asarray(split) / sum(split))
    # cap edits per half: keep the first max_edits events
    cnt = np.cumsum(ev, axis=1)
    ev &= cnt <= max_edits
    edits = ev.sum(axis=1).astype(np.int8)
    sub = ev & (kind == 0)
    ins = ev & (kind == 1)
    dele = ev & (kind == 2)
    seq = base.copy()
    # substitution: a different base
    shift = rng.integers(1, 4, size=(R, L))
    idx = np.searchsorted(ACGT, seq)
    idx = np.clip(idx, 0, 3)
    subbed = ACGT[(idx + shift) % 4]
    seq = np.where(sub, subbed, seq)
    # per position emit: deleted -> 0, inserted -> 2 (base + random), else 1
    emit = np.ones((R, L), np.int64) - dele + ins
    lens = emit.sum(axis=1)
    flat_pos = np.repeat(np.arange(R * L), emit.ravel())
    out = seq.ravel()[flat_pos]
    # for inserted positions the second copy becomes a random base
    firsts = np.ones(len(flat_pos), bool)
    firsts[1:] = flat_pos[1:] != flat_pos[:-1]
    second = ~firsts
    out = out.copy()
    out[second] = ACGT[rng.integers(0, 4, int(second.sum()))]
    return out, lens, edits


def make_umis(n_molecules: int, seed: int, mean_reads: float = 20.0, dispersion: float = 2.0,
              error_rate: float = 0.015, split=(0.4, 0.3, 0.3), max_edits: int = 3,
              pattern_fwd: str = UMI_FWD, pattern_rev: str = UMI_REV, orient_mix: float = 0.0,
              max_reads: int | None = None) -> UmiSet:
    """Generate reads' combined UMIs.  `orient_mix` > 0 reverse-complements that fraction of
    UMIs (exercises the minus-strand search; the reference's own UMIs are molecule-oriented).
    `max_reads` truncates the read list (keeps input order random)."""
    rng = np.random.default_rng(seed)
    fwd = _instantiate(pattern_fwd, n_molecules, rng)
    rev = _instantiate(pattern_rev, n_molecules, rng)
    p = dispersion / (dispersion + mean_reads)
    reads = np.maximum(1, rng.negative_binomial(dispersion, p, size=n_molecules))
    mol = np.repeat(np.arange(n_molecules), reads)
    rng.shuffle(mol)
    if max_reads is not None:
        mol = mol[:max_reads]
    R = len(mol)
    f_out, f_len, f_ed = _mutate_half(fwd[mol], error_rate, split, max_edits, rng)
    r_out, r_len, r_ed = _mutate_half(rev[mol], error_rate, split, max_edits, rng)
    lens = f_len + r_len
    off = np.zeros(R + 1, np.int64)
    np.cumsum(lens, out=off[1:])
    seq = np.empty(int(off[-1]), np.uint8)
    # interleave halves: per read [fwd half][rev half]
    f_off = np.zeros(R + 1, np.int64)
    np.cumsum(f_len, out=f_off[1:])
    r_off = np.zeros(R + 1, np.int64)
    np.cumsum(r_len, out=r_off[1:])
    dst_f = np.repeat(off[:-1] - f_off[:-1], f_len) + np.arange(len(f_out))
    seq[dst_f] = f_out
    dst_r = np.repeat(off[:-1] + f_len - r_off[:-1], r_len) + np.arange(len(r_out))
    seq[dst_r] = r_out
    strand = rng.integers(0, 2, R).astype(np.uint8)
    if orient_mix > 0:
        flip = rng.random(R) < orient_mix
        for i in np.nonzero(flip)[0]:
            a, b = off[i], off[i + 1]
            seq[a:b] = _COMP[seq[a:b][::-1]]
    return UmiSet(seq=seq, off=off, molecule=mol, strand=strand, fwd_dist=f_ed, rev_dist=r_ed)


# BASELINE config -> (minseqlength, maxseqlength) of the vsearch run
CONFIG_LENGTHS = {1: (58, 68), 2: (58, 68), 3: (58, 68), 4: (58, 68), 5: (80, 110)}
# config 5 stress UMIs: each pattern concatenated x1.5 (48-nt halves, ~96-nt combined UMI)
UMI_FWD_LONG = UMI_FWD + UMI_FWD[:16]
UMI_REV_LONG = UMI_REV + UMI_REV[:16]


def config_umis(config: int, scale: float = 1.0) -> UmiSet:
    """BASELINE.json configs: 1 = 100k reads (seed 1001), 2 = 2M reads (seed 1002), 5 = the high-error
    stress bin (seed 1005): ~96-nt UMIs, 15 % indels (insertion : deletion = 1 : 1, up to 4 per half, as the UMI extraction caps edits),
    deep clusters (NegBin mean 1,500 reads per molecule), 300k reads at scale 1."""
    if config == 1:
        return make_umis(int(5000 * scale), seed=1001, max_reads=int(100_000 * scale))
    if config == 2:
        return make_umis(int(100_000 * scale), seed=1002, max_reads=int(2_000_000 * scale))
    if config == 5:
        return make_umis(max(1, int(200 * scale)), seed=1005, mean_reads=1500.0, error_rate=0.15,
                         split=(0.0, 0.5, 0.5), max_edits=4, pattern_fwd=UMI_FWD_LONG,
                         pattern_rev=UMI_REV_LONG, max_reads=int(300_000 * scale))
    raise ValueError(config)


# ---------------------------------------------------------------- multi-bin configs 3 and 4
# 24 barcodes (the SQK-NBD114-24 kit, scripts/run_basecall_pipeline_multi-gpu.sh:48-49) x
# region bins whose sizes follow Zipf(1.1) (a few 100k-read bins and a long tail); bin k of barcode b is
# shard id b * BINS_PER_BARCODE + k with seed config_seed * 1_000_003 + shard id.
N_BARCODES = 24
BINS_PER_BARCODE = 40
ZIPF_S = 1.1
CONFIG_TOTAL_READS = {3: 10_000_000, 4: 70_000_000}


@dataclasses.dataclass
class Bin:
    """One (barcode x region bin): one vsearch invocation of the reference (tcr_consensus.py:231-245)."""
    barcode: int
    region: int
    shard_id: int
    seed: int
    umis: UmiSet

    @property
    def name(self) -> str:
        return f"barcode{self.barcode + 1:02d}/region_cluster{self.region}"


@dataclasses.dataclass
class BinSet:
    """Bins concatenated in bin order (what umiclust_load_bins takes): bin b = records
    [bin_start[b], bin_start[b+1])."""
    bins: list
    seq: np.ndarray
    off: np.ndarray
    bin_start: np.ndarray

    @property
    def n(self) -> int:
        return len(self.off) - 1

    def subset(self, idx) -> "BinSet":
        return concat_bins([self.bins[i] for i in idx])


def concat_bins(bins: list) -> BinSet:
    seqs = [b.umis.seq for b in bins]
    sizes = np.array([b.umis.n for b in bins], np.int64)
    bin_start = np.zeros(len(bins) + 1, np.int64)
    np.cumsum(sizes, out=bin_start[1:])
    seq = np.concatenate(seqs) if seqs else np.zeros(0, np.uint8)
    off = np.zeros(int(bin_start[-1]) + 1, np.int64)
    base = 0
    for b, s0 in zip(bins, bin_start[:-1]):
        off[s0:s0 + b.umis.n + 1] = b.umis.off + base
        base += int(b.umis.off[-1])
    return BinSet(bins=bins, seq=seq, off=off, bin_start=bin_start)


def zipf_bin_sizes(total_reads: int, n_barcodes: int = N_BARCODES, bins_per_barcode: int = BINS_PER_BARCODE,
                   s: float = ZIPF_S) -> np.ndarray:
    """[n_barcodes, bins_per_barcode] reads per bin: every barcode gets total/n_barcodes reads, split
    over its bins with weights k^-s (k = 1 .. bins_per_barcode), at least 1 read per bin."""
    w = np.arange(1, bins_per_barcode + 1, dtype=np.float64) ** -s
    per = total_reads / n_barcodes
    sizes = np.maximum(1, np.round(per * w / w.sum())).astype(np.int64)
    return np.tile(sizes, (n_barcodes, 1))


def _make_bin(args) -> Bin:
    b, k, sid, seed, reads = args
    return Bin(barcode=b, region=k, shard_id=sid, seed=seed, umis=make_umis(max(1, reads // 20), seed=seed,
                                                                              max_reads=reads))


def config_bins(config: int, scale: float = 1.0, barcodes=None, workers: int = 1, shard_ids=None) -> list:
    """BASELINE configs 3 (10M reads, seed 1003) and 4 (70M reads, seed 1004, round 1 input): 24 barcodes
    x 40 Zipf(1.1) region bins of 64-nt dual UMIs (R10.4.1-like 1.5 % errors, NegBin(20, 2) reads per
    molecule).  `scale` multiplies every bin's read count; `barcodes` restricts the barcodes built, `shard_ids`
    the bins (shard id = barcode * 40 + region; e.g. [200] = config 4's giant-molecule bin alone).
    Every bin has its own seed, so `workers` > 1 (spawned processes) gives identical bins."""
    if config not in CONFIG_TOTAL_READS:
        raise ValueError(config)
    seed0 = 1000 + config
    sizes = zipf_bin_sizes(int(CONFIG_TOTAL_READS[config] * scale))
    jobs = []
    for b in range(N_BARCODES) if barcodes is None else barcodes:
        for k in range(BINS_PER_BARCODE):
            sid = b * BINS_PER_BARCODE + k
            if shard_ids is not None and sid not in shard_ids:
                continue
            jobs.append((b, k, sid, seed0 * 1_000_003 + sid, int(sizes[b, k])))
    if workers <= 1:
        return [_make_bin(j) for j in jobs]
    import concurrent.futures as cf
    import multiprocessing as mp
    # largest bins first so the pool stays busy; results are put back in bin order
    order = sorted(range(len(jobs)), key=lambda i: -jobs[i][4])
    out = [None] * len(jobs)
    with cf.ProcessPoolExecutor(max_workers=workers, mp_context=mp.get_context("spawn")) as ex:
        for i, r in zip(order, ex.map(_make_bin, [jobs[i] for i in order], chunksize=1)):
            out[i] = r
    return out


def mutate_ragged(seqs: list, rate: float, seed: int, split=(0.4, 0.3, 0.3)) -> UmiSet:
    """Per-base substitution / insertion / deletion errors on variable-length sequences (vectorised
    over the concatenation)."""
    rng = np.random.default_rng(seed)
    raw = np.frombuffer("".join(seqs).encode(), np.uint8) if seqs else np.zeros(0, np.uint8)
    lens = np.array([len(x) for x in seqs], np.int64)
    owner = np.repeat(np.arange(len(seqs)), lens)
    ev = rng.random(len(raw)) < rate
    kind = rng.choice(3, size=len(raw), p=np.asarray(split) / sum(split))
    idx = np.clip(np.searchsorted(ACGT, raw), 0, 3)
    out = np.where(ev & (kind == 0), ACGT[(idx + rng.integers(1, 4, len(raw))) % 4], raw)
    emit = np.ones(len(raw), np.int64) - (ev & (kind == 2)) + (ev & (kind == 1))
    pos = np.repeat(np.arange(len(raw)), emit)
    res = out[pos].copy()
    second = np.ones(len(pos), bool)
    second[0:1] = False
    second[1:] = pos[1:] == pos[:-1]
    res[second] = ACGT[rng.integers(0, 4, int(second.sum()))]
    new_lens = np.bincount(owner, weights=emit, minlength=len(seqs)).astype(np.int64)
    off = np.zeros(len(seqs) + 1, np.int64)
    np.cumsum(new_lens, out=off[1:])
    n = len(seqs)
    return UmiSet(seq=res.astype(np.uint8), off=off, molecule=np.arange(n), strand=rng.integers(0, 2, n).astype(np.uint8),
                  fwd_dist=np.zeros(n, np.int8), rev_dist=np.zeros(n, np.int8))


def round2_bin(b: Bin, consensus: list, cluster_sizes, min_reads: int = 4, residual_error: float = 0.002) -> Bin:
    """Round-2 input of a bin (tcr_consensus.py:376-446): one UMI per round-1 cluster that
    the round-1 parse writes (>= min_reads_per_cluster reads, run_config.json:17), i.e. one per polished
    consensus molecule, carrying the round-1 consensus UMI with 0.2 % residual error (standing in for
    medaka polishing + extract_umis on the consensus read, both outside the hot path)."""
    keep = [c for c, sz in enumerate(cluster_sizes) if sz >= min_reads and consensus[c]]
    u = mutate_ragged([consensus[c] for c in keep], residual_error, seed=b.seed * 7 + 2)
    return Bin(barcode=b.barcode, region=b.region, shard_id=b.shard_id, seed=b.seed * 7 + 2, umis=u)


def _rand_read(rng: np.random.Generator, n: int) -> str:
    return ACGT[rng.integers(0, 4, n)].tobytes().decode()


def write_umi_fasta(path: str, umis: UmiSet, seed: int = 7, read_len: int = 32) -> None:
    """Write the 7-field-header FASTA that extract_umis.write_fasta produces
    (/root/reference/ont_tcr_consensus/extract_umis.py:154-186).  `read_len` sizes the
    synthetic full read carried in the `seq=` field (1,500 in production; 32 isolates I/O)."""
    rng = np.random.default_rng(seed)
    raw = umis.seq.tobytes()
    with open(path, "w") as f:
        for i in range(umis.n):
            u = raw[umis.off[i]:umis.off[i + 1]].decode()
            rid = str(uuid.UUID(bytes=rng.bytes(16), version=4))
            st = "-" if umis.strand[i] else "+"
            half = len(u) // 2
            f.write(f">{rid};strand={st};umi_fwd_dist={int(umis.fwd_dist[i])};"
                    f"umi_rev_dist={int(umis.rev_dist[i])};umi_fwd_seq={u[:half]};"
                    f"umi_rev_seq={u[half:]};seq={_rand_read(rng, read_len)}\n{u}\n")


def write_umi_fasta_fast(path: str, umis: UmiSet, seed: int = 7, read_len: int = 1500,
                         chunk: int = 65536) -> None:
    """write_umi_fasta's format at benchmark scale: uuid4-shaped read ids from random bytes and `seq=` reads
    sliced from a random pool (every read is a distinct random offset), written in chunks."""
    rng = np.random.default_rng(seed)
    pool = ACGT[rng.integers(0, 4, 1 << 22)].tobytes()
    raw = umis.seq.tobytes()
    hexd = np.frombuffer(b"0123456789abcdef", np.uint8)
    with open(path, "wb") as f:
        for c0 in range(0, umis.n, chunk):
            c1 = min(umis.n, c0 + chunk)
            m = c1 - c0
            rb = rng.integers(0, 256, (m, 16), dtype=np.uint8)
            rb[:, 6] = (rb[:, 6] & 0x0F) | 0x40
            rb[:, 8] = (rb[:, 8] & 0x3F) | 0x80
            hx = np.empty((m, 32), np.uint8)
            hx[:, 0::2] = hexd[rb >> 4]
            hx[:, 1::2] = hexd[rb & 15]
            hx = hx.tobytes()
            starts = rng.integers(0, len(pool) - read_len, m)
            parts = []
            for j in range(m):
                i = c0 + j
                u = raw[umis.off[i]:umis.off[i + 1]]
                h = hx[32 * j:32 * j + 32]
                half = len(u) // 2
                parts.append(b"".join((b">", h[0:8], b"-", h[8:12], b"-", h[12:16], b"-", h[16:20], b"-", h[20:32],
                                       b";strand=", b"-" if umis.strand[i] else b"+",
                                       b";umi_fwd_dist=%d;umi_rev_dist=%d;umi_fwd_seq=" % (umis.fwd_dist[i], umis.rev_dist[i]),
                                       u[:half], b";umi_rev_seq=", u[half:], b";seq=",
                                       pool[starts[j]:starts[j] + read_len], b"\n", u, b"\n")))
            f.write(b"".join(parts))


def segment_stress(n_rand: int = 470_000, n_copy: int = 3000, seed: int = 91, length: int = 64):
    """A bin past one counter segment (> 7 x 65,536 centroids, the prefilter's LDS counter range): n_rand
    random `length`-mers (nearly all their own centroids) followed by 1-substitution copies of sequences
    from both segments.  Returns (buf uint8, off int64) in input order."""
    rng = np.random.default_rng(seed)
    base = ACGT[rng.integers(0, 4, (n_rand, length))]
    half = n_copy // 2
    src = np.concatenate([rng.integers(0, min(n_rand, 400_000), half),
                          rng.integers(max(0, n_rand - 10_000), n_rand, n_copy - half)])
    cp = base[src].copy()
    rows = np.arange(n_copy)
    pos = rng.integers(0, length, n_copy)
    cp[rows, pos] = ACGT[(np.searchsorted(ACGT, cp[rows, pos]) + rng.integers(1, 4, n_copy)) % 4]
    buf = np.ascontiguousarray(np.concatenate([base, cp])).reshape(-1)
    off = np.arange(0, (n_rand + n_copy) * length + 1, length, dtype=np.int64)
    return buf, off
