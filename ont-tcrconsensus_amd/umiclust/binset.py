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

import os

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


class RunStats(list):
    """BinRunner.cluster_all's result: the stats of every call unit (bins clustered alone, then packs).  per_bin[b] is
    bin b's stats or None (clustered in a pack); packs lists the packs' stats, each with its "bins"."""

    def __init__(self, units, per_bin, packs):
        super().__init__(units)
        self.per_bin = per_bin
        self.packs = packs


class BinRunner:
    """One rank's bins of one round, resident on one device.

    Bins are independent, so a rank runs `lanes` of them at once: one device context per lane (its own
    streams and working buffers), the bins LPT-split over the lanes, one host thread per lane (the C ABI
    releases the GIL; distinct contexts are re-entrant).  Small bins are launch- and latency-bound on
    their own; lanes keep the GPU fed.  Results do not depend on the lane count."""

    def __init__(self, ctx, binset: synth.BinSet, preset: int, identity: float, minlen: int = 58,
                 maxlen: int = 68, lanes: int = 1, device: int = 0, pack_reads: int = 0, critical_priority=None,
                 threads: int = 1):
        """pack_reads > 0: a lane clusters its bins in packs (umiclust_cluster_pack) of consecutive bins holding up
        to pack_reads reads (a larger bin is a pack of its own): small bins share the GPU passes of their pack.
        critical_priority (default: UMICLUST_CRIT_PRIO, 1 -- on with several lanes; 0 turns it off): 1 / True: the lane
        holding the largest bin -- the bin that
        sets the makespan when it is far above the rest -- counts on a stream of the greatest priority
        (umiclust_set_priority) while the other lanes keep plain ones; 2: every lane holding a bin of at least half
        the largest one's cost on prioritised streams, the others on plain ones (set_priority -1).
        threads > 1: vsearch --threads `threads` (policy O4, the mode the reference runs every bin in:
        vsearch_umi_cluster.py:33-34, utils.py:56-63); 1: the sequential definition."""
        from .shard import bin_cost, lpt_assign
        self.binset = binset
        self.pack_reads = pack_reads
        self.params = _lib.params(preset, identity, minlen, maxlen, threads=threads)
        nb = len(binset.bins)
        lanes = max(1, min(lanes, nb)) if nb else 1
        plan = lpt_assign([bin_cost(b.umis.n) for b in binset.bins], lanes)
        self.ctxs = [ctx] + [_lib.Context(device) for _ in range(lanes - 1)]
        self._own = self.ctxs[1:]
        self.plan = plan
        self.where = {}  # bin -> (lane, index in the lane's load)
        for lane, idx in enumerate(plan):
            sub = binset.subset(idx) if lanes > 1 else binset
            if lanes == 1:
                idx = list(range(nb))
                self.plan = [idx]
            for j, b in enumerate(idx):
                self.where[b] = (lane, j)
            self.ctxs[lane].stage(sub.seq, sub.off, sub.bin_start)
        if critical_priority is None:
            critical_priority = int(os.environ.get("UMICLUST_CRIT_PRIO", "1") or 0)
        self.critical_lane = None
        self.critical_lanes = []
        if critical_priority and len(self.ctxs) > 1 and nb:
            big = max(range(nb), key=lambda b: binset.bins[b].umis.n)
            self.critical_lane = self.where[big][0]
            if critical_priority == 2:
                # every lane holding a bin of at least half the largest bin's cost counts and aligns on prioritised
                # streams, the other lanes on plain ones (background)
                cmax = bin_cost(binset.bins[big].umis.n)
                self.critical_lanes = sorted({self.where[b][0] for b in range(nb)
                                              if bin_cost(binset.bins[b].umis.n) >= 0.5 * cmax})
                for lane, c in enumerate(self.ctxs):
                    c.set_priority(1 if lane in self.critical_lanes else -1)
            else:
                self.critical_lanes = [self.critical_lane]
                for lane, c in enumerate(self.ctxs):
                    c.set_priority(1 if lane == self.critical_lane else 0)
        self.prepare()

    def _each_lane(self, fn) -> list:
        if len(self.ctxs) == 1:
            return [fn(0)]
        import concurrent.futures as cf
        with cf.ThreadPoolExecutor(len(self.ctxs)) as ex:
            return list(ex.map(fn, range(len(self.ctxs))))

    def prepare(self) -> None:
        """umiclust_prepare on every lane: vsearch's load-time work (length filter, DUST, sort, k-mers) of the staged
        bins (bench.py times it inside each step)."""
        self._each_lane(lambda lane: self.ctxs[lane].prepare(self.params))

    @property
    def nbins(self) -> int:
        return len(self.binset.bins)

    def packs(self, lane: int) -> list:
        """(first, count) runs of the lane's load bins clustered together."""
        idx = self.plan[lane]
        if self.pack_reads <= 0:
            return [(j, 1) for j in range(len(idx))]
        out, j = [], 0
        while j < len(idx):
            k, reads = j, 0
            while k < len(idx) and (k == j or reads + self.binset.bins[idx[k]].umis.n <= self.pack_reads):
                reads += self.binset.bins[idx[k]].umis.n
                k += 1
            out.append((j, k - j))
            j = k
        return out

    def cluster_all(self) -> "RunStats":
        """Cluster every bin.  Returns the stats of every call unit -- each bin clustered alone, then each pack (stats
        cover the pack's bins together) -- as a RunStats list, so sums over it are totals; `.per_bin[b]` holds bin b's
        own stats (None for a bin clustered inside a pack) and `.packs` the packs' (with their bins).  The list is NOT
        indexed by bin."""
        out = [None] * self.nbins
        packed = [[] for _ in self.ctxs]

        def run(lane):
            for j, m in self.packs(lane):
                if m == 1:
                    st = self.ctxs[lane].cluster_bin(j)
                    st["bins"] = [self.plan[lane][j]]
                    out[self.plan[lane][j]] = st
                else:
                    st = self.ctxs[lane].cluster_pack(j, m)
                    st["bins"] = [self.plan[lane][x] for x in range(j, j + m)]
                    packed[lane].append(st)

        self._each_lane(run)
        packs = [x for p in packed for x in p]
        return RunStats([x for x in out if x is not None] + packs, out, packs)

    def results(self) -> list:
        return [self.ctxs[self.where[b][0]].fetch_bin(self.where[b][1]) for b in range(self.nbins)]

    def close(self):
        for c in self._own:
            c.close()
        self._own = []


def round2_binset(binset: synth.BinSet, results: list, min_reads: int = MIN_READS_PER_CLUSTER) -> synth.BinSet:
    """Round-2 inputs of every bin from its round-1 result."""
    return synth.concat_bins([synth.round2_bin(b, r["consensus"], cluster_sizes(r), min_reads)
                              for b, r in zip(binset.bins, results)])
