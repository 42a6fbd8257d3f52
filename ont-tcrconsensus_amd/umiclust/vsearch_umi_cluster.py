"""Drop-in for /root/reference/ont_tcr_consensus/vsearch_umi_cluster.py.

Same function names, signatures, defaults and return value as the reference
(`vsearch_cluster` :8-56, `vsearch_cluster_consensus` :59-99).  The reference builds a vsearch
argv and runs it with `subprocess.run` (:21-54, :71-97); here the *same argv* is handed to the
MI355X library through its C ABI (`umiclust_run_argv`, include/umiclust.h), which parses it with
vsearch's option semantics and writes the same files: `<out_dir>/cluster<N>`,
`<out_dir>/umi_clusters_consensus.fasta` and the log.

Differences that cannot change a successful run's outputs:
  * `threads` does not set a CPU thread count (the work runs on the GPU); as in vsearch it selects the clustering
    definition: n > 1 is vsearch's multithreaded cluster_fast (rounds of n queries searched against the index
    frozen at the round's start, then re-checked in order: policy O4), which is what the
    reference computes since it always passes n >= 25 (utils.py:56-63); n = 1 the sequential definition.
    UMICLUST_O4=sequential forces the sequential definition;
  * failures raise `UmiclustError` (the reference silently returns the consout path even when
    vsearch fails, since `subprocess.run` has no `check=`).

When `ray` is importable both functions are `ray.remote` tasks exactly like the reference, so
call sites such as `vsearch_cluster.options(num_cpus=n).remote(...)`
(/root/reference/ont_tcr_consensus/tcr_consensus.py:237-245, :419-427) work unchanged.  Without
ray the same call syntax runs synchronously in-process.
"""
from __future__ import annotations

import os
from typing import Union

from . import _lib

_CTX: dict[int, _lib.Context] = {}


def _device() -> int:
    return int(os.environ.get("UMICLUST_DEVICE", "0"))


def context(device: int | None = None) -> _lib.Context:
    """Process-wide device context (one per process and GPU, reused across bins)."""
    d = _device() if device is None else device
    if d not in _CTX:
        _CTX[d] = _lib.Context(d)
    return _CTX[d]


def round1_argv(umi_fasta, clustering_out_dir, threads, min_umi_length, max_umi_length, identity) -> list[str]:
    """The argv of vsearch_umi_cluster.py:22-53, element for element."""
    consensus_umi_fasta = os.path.join(clustering_out_dir, "umi_clusters_consensus.fasta")
    log_file = os.path.join(clustering_out_dir, "vsearch_cluster.log")
    return ["vsearch", "--clusterout_id", "--clusters", clustering_out_dir + "/cluster", "--consout",
            consensus_umi_fasta, "--minseqlength", str(min_umi_length), "--maxseqlength", str(max_umi_length),
            "--threads", str(threads), "--cluster_fast", umi_fasta, "--strand", "both", "--log", log_file,
            "--quiet", "--no_progress", "--clusterout_sort", "--gapopen", "0E/40I", "--mismatch", "-40",
            "--match", "10", "--id", str(identity)]


def round2_argv(umi_fasta, clustering_consensus_out_dir, threads, min_umi_length, max_umi_length,
                identity) -> list[str]:
    """The argv of vsearch_umi_cluster.py:72-96, element for element."""
    consensus_umi_fasta = os.path.join(clustering_consensus_out_dir, "umi_clusters_consensus.fasta")
    log_file = os.path.join(clustering_consensus_out_dir, "vsearch_cluster_consensus.log")
    return ["vsearch", "--clusterout_id", "--clusters", clustering_consensus_out_dir + "/cluster", "--consout",
            consensus_umi_fasta, "--minseqlength", str(min_umi_length), "--maxseqlength", str(max_umi_length),
            "--threads", str(threads), "--cluster_fast", umi_fasta, "--strand", "both", "--log", log_file,
            "--quiet", "--no_progress", "--clusterout_sort", "--id", str(identity)]


def _vsearch_cluster(
    umi_fasta: Union[str, os.PathLike[str]],
    clustering_out_dir: Union[str, os.PathLike[str]],
    threads: int,
    min_umi_length: int = 50,
    max_umi_length: int = 60,
    identity: float = 0.94,
):
    consensus_umi_fasta = os.path.join(clustering_out_dir, "umi_clusters_consensus.fasta")
    argv = round1_argv(os.fspath(umi_fasta), os.fspath(clustering_out_dir), threads, min_umi_length,
                       max_umi_length, identity)
    context().run_argv(argv)
    return consensus_umi_fasta


def _vsearch_cluster_consensus(
    umi_fasta: Union[str, os.PathLike[str]],
    clustering_consensus_out_dir: Union[str, os.PathLike[str]],
    threads: int,
    min_umi_length: int = 50,
    max_umi_length: int = 60,
    identity: float = 0.97,
):
    consensus_umi_fasta = os.path.join(clustering_consensus_out_dir, "umi_clusters_consensus.fasta")
    argv = round2_argv(os.fspath(umi_fasta), os.fspath(clustering_consensus_out_dir), threads, min_umi_length,
                       max_umi_length, identity)
    context().run_argv(argv)
    return consensus_umi_fasta


class _LocalRemote:
    """`f.options(...).remote(...)` / `f.remote(...)` / `f(...)` without ray: runs in-process."""

    def __init__(self, fn):
        self._fn = fn
        self.__doc__ = fn.__doc__
        self.__name__ = fn.__name__.lstrip("_")

    def options(self, **_kw):
        return self

    def remote(self, *a, **kw):
        return self._fn(*a, **kw)

    def __call__(self, *a, **kw):
        return self._fn(*a, **kw)


try:  # pragma: no cover - ray is not installed in this image
    import ray as _ray

    vsearch_cluster = _ray.remote(_vsearch_cluster)
    vsearch_cluster_consensus = _ray.remote(_vsearch_cluster_consensus)
except ImportError:
    vsearch_cluster = _LocalRemote(_vsearch_cluster)
    vsearch_cluster_consensus = _LocalRemote(_vsearch_cluster_consensus)
