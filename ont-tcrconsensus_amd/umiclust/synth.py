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
CONFIG_LENGTHS = {1: (58, 68), 2: (58, 68), 5: (80, 110)}
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
