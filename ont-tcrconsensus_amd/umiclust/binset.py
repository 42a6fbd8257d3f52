"""Many region bins on one GPU: BASELINE configs 3 and 4.

The reference runs one `vsearch --cluster_fast` process per (library x region bin), round 1 at
/root/reference/ont_tcr_consensus/tcr_consensus.py:231-267 and round 2 at :411-446.  Here a rank keeps
all of its bins resident in HBM in one load (`umiclust_load_bins`) and clusters them one after another
(`umiclust_cluster_bin`); each bin's result is exactly its own vsearch run's.  Round 2 clusters, per
bin, the UMIs of the round-1 consensus molecules (synth.round2_bin).
"""
from __future__ import annotations

import hashlib
import json

import numpy as np

from . import _lib, synth

ROUND1 = dict(preset=_lib.PRESET_ROUND1, identity=0.93)           # run_config.json:16, vsearch_umi_cluster.py:44-52
ROUND2 = dict(preset=_lib.PRESET_VSEARCH_DEFAULT, identity=0.97)  # run_config.json:28, vsearch_umi_cluster.py:93-95
MIN_READS_PER_CLUSTER = 4                                         # run_config.json:17 (round-1 parse)


def digest(res: dict) -> dict:
    """Size-independent digest of one bin's clustering (same keys for the GPU and the oracle)."""
    h = lambda b: hashlib.sha256(b).hexdigest()  # noqa: E731
    return dict(n_clusters=int(res["n_clusters"]),
                cluster=h(np.ascontiguousarray(res["cluster"], np.int32).tobytes()),
                strand=h(np.ascontiguousarray(res["strand"], np.uint8).tobytes()),
                centroid=h(np.ascontiguousarray(res["centroid"], np.uint8).tobytes()),
                consensus=h("\n".join(res["consensus"]).encode()))


def combine(digests: list) -> str:
    """A checksum of the per-bin checksums, in bin order."""
    return hashlib.sha256("\n".join(json.dumps(d, sort_keys=True) for d in digests).encode()).hexdigest()


def cluster_sizes(res: dict) -> np.ndarray:
    cl = np.asarray(res["cluster"])
    return np.bincount(cl[cl >= 0], minlength=int(res["n_clusters"]))


class BinRunner:
    """One rank's bins of one round, resident on one device."""

    def __init__(self, ctx: _lib.Context, binset: synth.BinSet, preset: int, identity: float,
                 minlen: int = 58, maxlen: int = 68):
        self.ctx = ctx
        self.binset = binset
        self.params = _lib.params(preset, identity, minlen, maxlen)
        ctx.load_bins(self.params, binset.seq, binset.off, binset.bin_start)

    @property
    def nbins(self) -> int:
        return len(self.binset.bins)

    def cluster_all(self) -> list:
        """Cluster every bin; per-bin stats."""
        return [self.ctx.cluster_bin(b) for b in range(self.nbins)]

    def results(self) -> list:
        return [self.ctx.fetch_bin(b) for b in range(self.nbins)]


def round2_binset(binset: synth.BinSet, results: list, min_reads: int = MIN_READS_PER_CLUSTER) -> synth.BinSet:
    """Round-2 inputs of every bin from its round-1 result."""
    return synth.concat_bins([synth.round2_bin(b, r["consensus"], cluster_sizes(r), min_reads)
                              for b, r in zip(binset.bins, results)])
