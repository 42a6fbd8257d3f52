"""ctypes binding of the C ABI declared in include/umiclust.h (libumiclust.so, built in-tree).

There is no CPU fallback: if the library or a HIP device is missing every entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libumiclust.so")

QL, TL, QI, TI, QR, TR = range(6)
PRESET_ROUND1 = 1
PRESET_VSEARCH_DEFAULT = 2
MAX_LEN = 112

ERRORS = {-22: "EINVAL", -5: "EIO", -12: "ENOMEM", -19: "EDEVICE", -77: "ESTATE", -34: "ERANGE", -17: "EEXIST",
          -74: "EFORMAT"}


class UmiclustError(RuntimeError):
    def __init__(self, code: int, msg: str = ""):
        super().__init__(f"umiclust error {code} ({ERRORS.get(code, '?')}): {msg}")
        self.code = code


class Params(C.Structure):
    _fields_ = [
        ("id", C.c_double),
        ("weak_id", C.c_double),
        ("minseqlength", C.c_int32),
        ("maxseqlength", C.c_int32),
        ("wordlength", C.c_int32),
        ("minwordmatches", C.c_int32),
        ("maxaccepts", C.c_int32),
        ("maxrejects", C.c_int32),
        ("match", C.c_int32),
        ("mismatch", C.c_int32),
        ("gap_open", C.c_int32 * 6),
        ("gap_ext", C.c_int32 * 6),
        ("strand_both", C.c_int32),
        ("qmask_dust", C.c_int32),
        ("clusterout_sort", C.c_int32),
        ("clusterout_id", C.c_int32),
        ("fasta_width", C.c_int32),
        ("policy_boundary_open", C.c_int32),
        ("threads", C.c_int32),
        ("policy_threads", C.c_int32),
    ]


class Stats(C.Structure):
    _fields_ = [
        ("n_input", C.c_int64),
        ("n_kept", C.c_int64),
        ("n_clusters", C.c_int64),
        ("n_alignments", C.c_int64),
        ("cells", C.c_int64),
        ("cells_computed", C.c_int64),
        ("kmer_postings", C.c_int64),
        ("n_blocks", C.c_int64),
        ("t_total_s", C.c_double),
        ("t_prefilter_s", C.c_double),
        ("t_align_s", C.c_double),
        ("t_consensus_s", C.c_double),
        ("t_host_s", C.c_double),
        ("n_deferred", C.c_int64),
        ("pairs_round_b", C.c_int64),
        ("pairs_peer", C.c_int64),
        ("t_index_s", C.c_double),
        ("t_sync_s", C.c_double),
        ("t_host_pass1_s", C.c_double),
        ("n_merged_walks", C.c_int64),
        ("t_merged_s", C.c_double),
        ("t_read_s", C.c_double),
        ("t_write_s", C.c_double),
        ("t_run_s", C.c_double),
        ("n_reruns", C.c_int64),
        ("n_overlap_passes", C.c_int64),
        ("n_lazy_passes", C.c_int64),
        ("t_count_s", C.c_double),
        ("n_count_launches", C.c_int64),
        ("kmer_postings_deferred", C.c_int64),
        ("counter_cells", C.c_int64),
        ("n_regrows", C.c_int64),
    ]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


class ParseParams(C.Structure):
    _fields_ = [("min_reads_per_cluster", C.c_int32), ("max_reads_per_cluster", C.c_int32),
                ("balance_strands", C.c_int32), ("max_clusters", C.c_int32)]


class ParseResult(C.Structure):
    _fields_ = [("n_clusters", C.c_int64), ("n_written", C.c_int64), ("reads_found", C.c_int64),
                ("reads_written", C.c_int64), ("empty_region", C.c_int32), ("pad", C.c_int32)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_ if k != "pad"}


# every symbol include/umiclust.h declares
EXPORTS = [
    "umiclust_abi_version", "umiclust_params_init", "umiclust_params_from_argv", "umiclust_create",
    "umiclust_destroy", "umiclust_last_error", "umiclust_run_fasta", "umiclust_run_argv", "umiclust_run_fasta_parse",
    "umiclust_load", "umiclust_stage", "umiclust_prepare", "umiclust_set_priority", "umiclust_cluster", "umiclust_fetch", "umiclust_load_bins", "umiclust_cluster_bin", "umiclust_cluster_pack",
    "umiclust_fetch_bin", "umiclust_overlap_counts", "umiclust_overlap_regions", "umiclust_extract_umis",
    "umiclust_extract_umis_file", "umiclust_region_split", "umiclust_align_pairs", "umiclust_prep",
    "umiclust_timeline", "umiclust_wait_host",
]
OVERLAP_MAX_REGIONS = 4096
ABI_VERSION = 9  # include/umiclust.h UMICLUST_ABI_VERSION: the struct layouts below

_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise UmiclustError(-19, f"{LIB_PATH} not built (run `make -C ont-tcrconsensus_amd` or "
                                 "__graft_entry__.build()); there is no CPU fallback")
    L = C.CDLL(LIB_PATH)
    P = C.POINTER
    L.umiclust_abi_version.restype = C.c_int32
    if L.umiclust_abi_version() != ABI_VERSION:  # a stale build would read the structs with the wrong layout
        raise UmiclustError(-22, f"{LIB_PATH} has ABI {L.umiclust_abi_version()}, this binding expects "
                                 f"{ABI_VERSION}: rebuild (make -C ont-tcrconsensus_amd)")
    L.umiclust_params_init.restype = C.c_int32
    L.umiclust_params_init.argtypes = [P(Params), C.c_int32, C.c_double, C.c_int32, C.c_int32]
    L.umiclust_params_from_argv.restype = C.c_int32
    L.umiclust_params_from_argv.argtypes = [P(Params), C.c_int32, P(C.c_char_p), C.c_char_p, C.c_char_p,
                                            C.c_char_p, C.c_char_p, C.c_int32]
    L.umiclust_create.restype = C.c_void_p
    L.umiclust_create.argtypes = [C.c_int32, P(C.c_int32)]
    L.umiclust_destroy.restype = None
    L.umiclust_destroy.argtypes = [C.c_void_p]
    L.umiclust_wait_host.restype = C.c_int32
    L.umiclust_wait_host.argtypes = [C.c_void_p]
    L.umiclust_last_error.restype = C.c_char_p
    L.umiclust_last_error.argtypes = [C.c_void_p]
    L.umiclust_run_fasta.restype = C.c_int64
    L.umiclust_run_fasta.argtypes = [C.c_void_p, P(Params), C.c_char_p, C.c_char_p, C.c_char_p, C.c_char_p,
                                     P(Stats)]
    L.umiclust_run_fasta_parse.restype = C.c_int64
    L.umiclust_run_fasta_parse.argtypes = [C.c_void_p, P(Params), C.c_char_p, C.c_char_p, C.c_char_p, C.c_char_p,
                                           P(ParseParams), C.c_char_p, P(ParseResult), P(Stats)]
    L.umiclust_run_argv.restype = C.c_int64
    L.umiclust_run_argv.argtypes = [C.c_void_p, C.c_int32, P(C.c_char_p), P(Stats)]
    L.umiclust_load.restype = C.c_int32
    L.umiclust_load.argtypes = [C.c_void_p, P(Params), C.c_void_p, P(C.c_int64), C.c_int64]
    L.umiclust_stage.restype = C.c_int32
    L.umiclust_stage.argtypes = [C.c_void_p, C.c_void_p, P(C.c_int64), C.c_int64, P(C.c_int64), C.c_int32]
    L.umiclust_prepare.restype = C.c_int32
    L.umiclust_prepare.argtypes = [C.c_void_p, P(Params)]
    L.umiclust_set_priority.restype = C.c_int32
    L.umiclust_set_priority.argtypes = [C.c_void_p, C.c_int32]
    L.umiclust_cluster.restype = C.c_int64
    L.umiclust_cluster.argtypes = [C.c_void_p, P(Stats)]
    L.umiclust_fetch.restype = C.c_int64
    L.umiclust_fetch.argtypes = [C.c_void_p, P(C.c_int32), P(C.c_uint8), P(C.c_uint8), C.c_void_p, C.c_int64,
                                 P(C.c_int64)]
    L.umiclust_load_bins.restype = C.c_int32
    L.umiclust_load_bins.argtypes = [C.c_void_p, P(Params), C.c_void_p, P(C.c_int64), C.c_int64, P(C.c_int64),
                                     C.c_int32]
    L.umiclust_cluster_bin.restype = C.c_int64
    L.umiclust_cluster_bin.argtypes = [C.c_void_p, C.c_int32, P(Stats)]
    L.umiclust_cluster_pack.restype = C.c_int64
    L.umiclust_cluster_pack.argtypes = [C.c_void_p, C.c_int32, C.c_int32, P(Stats)]
    L.umiclust_fetch_bin.restype = C.c_int64
    L.umiclust_fetch_bin.argtypes = [C.c_void_p, C.c_int32, P(C.c_int32), P(C.c_uint8), P(C.c_uint8), C.c_void_p,
                                     C.c_int64, P(C.c_int64)]
    L.umiclust_overlap_counts.restype = C.c_int32
    L.umiclust_overlap_counts.argtypes = [C.c_void_p, C.c_void_p, P(C.c_int64), C.c_int64, C.c_void_p, P(C.c_int64),
                                          C.c_int64, P(C.c_int64)]
    L.umiclust_overlap_regions.restype = C.c_int32
    L.umiclust_overlap_regions.argtypes = [C.c_void_p, C.c_void_p, P(C.c_int64), C.c_int64, P(C.c_int64), C.c_int32,
                                           P(C.c_int64), P(C.c_int32)]
    L.umiclust_extract_umis.restype = C.c_int32
    L.umiclust_extract_umis.argtypes = [C.c_void_p, C.c_void_p, P(C.c_int64), C.c_int64, C.c_int32, C.c_int32, C.c_int32,
                                        C.c_char_p, C.c_char_p, P(C.c_int32)]
    L.umiclust_extract_umis_file.restype = C.c_int64
    L.umiclust_extract_umis_file.argtypes = [C.c_void_p, C.c_char_p, C.c_char_p, C.c_int32, C.c_int32, C.c_int32,
                                             C.c_char_p, C.c_char_p]
    L.umiclust_region_split.restype = C.c_int64
    L.umiclust_region_split.argtypes = [C.c_void_p, C.c_char_p, C.c_int32, P(C.c_char_p), P(C.c_int64), P(C.c_int32),
                                        C.c_double, C.c_int32, C.c_int32, C.c_char_p, P(C.c_int64), P(C.c_int64),
                                        C.c_int32, P(C.c_uint8), C.c_char_p, C.c_int32]
    L.umiclust_align_pairs.restype = C.c_int32
    L.umiclust_align_pairs.argtypes = [C.c_void_p, P(Params), C.c_void_p, P(C.c_int64), C.c_void_p, P(C.c_int64),
                                       C.c_int64, P(C.c_int32), P(C.c_int32), P(C.c_int32), C.c_void_p, C.c_int32,
                                       P(C.c_int32)]
    L.umiclust_prep.restype = C.c_int32
    L.umiclust_prep.argtypes = [C.c_void_p, P(Params), C.c_void_p, P(C.c_int64), C.c_int64, C.c_void_p,
                                P(C.c_uint16), C.c_int32, P(C.c_int32)]
    L.umiclust_timeline.restype = C.c_int32
    L.umiclust_timeline.argtypes = [C.c_int32, C.c_int32, C.c_int32, P(C.c_double), P(C.c_int64)]
    _lib = L
    return L


def timeline(kind: int, reset: bool = False, device: int = 0) -> tuple[float, int]:
    """umiclust_timeline: (union of the kind's HIP-event brackets in seconds, brackets) since the last reset;
    kind 0 = counting launches, 1 = alignment chains."""
    s, n = C.c_double(0.0), C.c_int64(0)
    rc = lib().umiclust_timeline(device, kind, 1 if reset else 0, C.byref(s), C.byref(n))
    if rc != 0:
        raise UmiclustError(rc, "timeline")
    return s.value, n.value


def params(preset: int = PRESET_ROUND1, identity: float = 0.93, minlen: int = 58, maxlen: int = 68,
           threads: int = 1) -> Params:
    """A preset's parameters; threads > 1 selects vsearch's --threads mode (policy O4, rounds of `threads` queries:
    umiclust_params.policy_threads = 1), threads = 1 the sequential definition."""
    p = Params()
    rc = lib().umiclust_params_init(C.byref(p), preset, identity, minlen, maxlen)
    if rc != 0:
        raise UmiclustError(rc, "params_init")
    if threads > 1:
        p.threads, p.policy_threads = int(threads), 1
    return p


def params_from_argv(argv: list[str]) -> tuple[Params, dict]:
    p = Params()
    bufs = [C.create_string_buffer(4096) for _ in range(4)]
    arr = (C.c_char_p * len(argv))(*[str(a).encode() for a in argv])
    rc = lib().umiclust_params_from_argv(C.byref(p), len(argv), arr, *bufs, 4096)
    if rc != 0:
        raise UmiclustError(rc, f"cannot parse argv {argv!r}")
    keys = ["in_fasta", "clusters_prefix", "consout", "log"]
    return p, {k: (b.value.decode() or None) for k, b in zip(keys, bufs)}


def _i64(a):
    return a.ctypes.data_as(C.POINTER(C.c_int64))


def _pack(seqs) -> tuple[np.ndarray, np.ndarray]:
    """list of str/bytes -> (uint8 buffer, int64 offsets)."""
    bs = [s.encode() if isinstance(s, str) else bytes(s) for s in seqs]
    off = np.zeros(len(bs) + 1, np.int64)
    if bs:
        np.cumsum([len(b) for b in bs], out=off[1:])
    buf = np.frombuffer(b"".join(bs) + b"\0", np.uint8).copy()
    return buf, off


class Context:
    """One device context (one per process and GPU)."""

    def __init__(self, device: int = 0):
        err = C.c_int32(0)
        self._h = lib().umiclust_create(device, C.byref(err))
        if not self._h:
            raise UmiclustError(err.value, f"no HIP device {device} (there is no CPU backend)")

    def close(self):
        if self._h:
            lib().umiclust_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _check(self, rc: int, what: str) -> int:
        if rc < 0:
            msg = lib().umiclust_last_error(self._h)
            raise UmiclustError(int(rc), f"{what}: {msg.decode() if msg else ''}")
        return rc

    def wait_host(self) -> None:
        """Waits for the host work the last file-path call left running (its input's release)."""
        self._check(lib().umiclust_wait_host(self._h), "wait_host")

    def run_fasta(self, p: Params, in_fasta: str, clusters_prefix: str | None, consout: str | None,
                  log: str | None) -> dict:
        st = Stats()
        enc = lambda x: x.encode() if x else None  # noqa: E731
        k = lib().umiclust_run_fasta(self._h, C.byref(p), enc(in_fasta), enc(clusters_prefix), enc(consout),
                                     enc(log), C.byref(st))
        self._check(k, "run_fasta")
        return st.as_dict()

    def run_fasta_parse(self, p: Params, in_fasta: str, clusters_prefix: str | None, consout: str | None,
                        log: str | None, pp: ParseParams, work_dir: str) -> tuple[dict, dict]:
        """Clustering + parse_umi_clusters' outputs from memory (include/umiclust.h)."""
        st, pr = Stats(), ParseResult()
        enc = lambda x: x.encode() if x else None  # noqa: E731
        k = lib().umiclust_run_fasta_parse(self._h, C.byref(p), enc(in_fasta), enc(clusters_prefix), enc(consout),
                                           enc(log), C.byref(pp), work_dir.encode(), C.byref(pr), C.byref(st))
        self._check(k, "run_fasta_parse")
        return st.as_dict(), pr.as_dict()

    def run_argv(self, argv: list[str]) -> dict:
        st = Stats()
        arr = (C.c_char_p * len(argv))(*[str(a).encode() for a in argv])
        k = lib().umiclust_run_argv(self._h, len(argv), arr, C.byref(st))
        self._check(k, "run_argv")
        return st.as_dict()

    def load(self, p: Params, seqs=None, buf: np.ndarray | None = None, off: np.ndarray | None = None) -> None:
        if seqs is not None:
            buf, off = _pack(seqs)
        n = len(off) - 1
        self._check(lib().umiclust_load(self._h, C.byref(p), buf.ctypes.data, _i64(off), n), "load")
        self._n = n
        self._bins = None

    def stage(self, buf: np.ndarray, off: np.ndarray, bin_start=None) -> None:
        """umiclust_stage: the raw records into HBM (one bin, or bins [bin_start[b], bin_start[b+1]))."""
        n = len(off) - 1
        bs = None if bin_start is None else np.ascontiguousarray(bin_start, np.int64)
        self._check(lib().umiclust_stage(self._h, buf.ctypes.data, _i64(off), n, None if bs is None else _i64(bs),
                                         0 if bs is None else len(bs) - 1), "stage")
        self._n = n
        self._bins = bs

    def prepare(self, p: Params) -> None:
        """umiclust_prepare: length filter, sort, DUST, codes and k-mers of the staged records."""
        self._check(lib().umiclust_prepare(self._h, C.byref(p)), "prepare")

    def set_priority(self, level: int) -> None:
        """umiclust_set_priority: 1 = this context's counting stream at the greatest priority, 0 = plain (the
        alignment stream prioritised at both), -1 = every stream plain (background)."""
        self._check(lib().umiclust_set_priority(self._h, int(level)), "set_priority")

    def cluster(self) -> dict:
        st = Stats()
        self._check(lib().umiclust_cluster(self._h, C.byref(st)), "cluster")
        return st.as_dict()

    def fetch(self) -> dict:
        return self.fetch_bin(0) if getattr(self, "_bins", None) is not None else self._fetch(None, self._n)

    def load_bins(self, p: Params, buf: np.ndarray, off: np.ndarray, bin_start) -> None:
        """Many region bins resident at once: bin b = records [bin_start[b], bin_start[b+1])."""
        bs = np.ascontiguousarray(bin_start, np.int64)
        n = len(off) - 1
        self._check(lib().umiclust_load_bins(self._h, C.byref(p), buf.ctypes.data, _i64(off), n, _i64(bs),
                                             len(bs) - 1), "load_bins")
        self._n = n
        self._bins = bs

    def cluster_pack(self, first: int, nbins: int) -> dict:
        """Bins [first, first + nbins) of the load in one greedy order (umiclust_cluster_pack); stats of the pack."""
        st = Stats()
        self._check(lib().umiclust_cluster_pack(self._h, first, nbins, C.byref(st)), "cluster_pack")
        return st.as_dict()

    def cluster_bin(self, b: int) -> dict:
        st = Stats()
        self._check(lib().umiclust_cluster_bin(self._h, b, C.byref(st)), "cluster_bin")
        return st.as_dict()

    def fetch_bin(self, b: int) -> dict:
        bs = getattr(self, "_bins", None)
        n = int(bs[b + 1] - bs[b]) if bs is not None else self._n
        return self._fetch(b, n)

    def _fetch(self, b, n: int) -> dict:
        cl = np.empty(max(n, 1), np.int32)
        sd = np.empty(max(n, 1), np.uint8)
        ce = np.empty(max(n, 1), np.uint8)
        P = C.POINTER
        if b is None:
            f = lambda *a: lib().umiclust_fetch(self._h, *a)  # noqa: E731
        else:
            f = lambda *a: lib().umiclust_fetch_bin(self._h, b, *a)  # noqa: E731
        k = self._check(f(None, None, None, None, 0, None), "fetch")
        off = np.zeros(k + 1, np.int64)
        self._check(f(None, None, None, None, 0, _i64(off)), "fetch")
        cons = np.zeros(int(off[-1]) + 1, np.uint8)
        self._check(f(cl.ctypes.data_as(P(C.c_int32)), sd.ctypes.data_as(P(C.c_uint8)),
                      ce.ctypes.data_as(P(C.c_uint8)), cons.ctypes.data, len(cons), _i64(off)), "fetch")
        raw = cons.tobytes()
        return dict(n_clusters=int(k), cluster=cl[:n], strand=sd[:n], centroid=ce[:n],
                    consensus=[raw[off[c]:off[c + 1]].decode() for c in range(k)])

    def overlap_counts(self, seqs1, seqs2) -> np.ndarray:
        """Per set-1 sequence, the number of byte-equal set-2 sequences (umiclust_overlap_counts)."""
        b1, o1 = _pack(seqs1)
        b2, o2 = _pack(seqs2)
        n1 = len(o1) - 1
        out = np.zeros(max(n1, 1), np.int64)
        self._check(lib().umiclust_overlap_counts(self._h, b1.ctypes.data, _i64(o1), n1, b2.ctypes.data, _i64(o2),
                                                  len(o2) - 1, _i64(out)), "overlap_counts")
        return out[:n1]

    def overlap_regions(self, regions) -> tuple[np.ndarray, np.ndarray]:
        """regions: list of sequence lists.  (total, maxcount) R x R matrices, entries [a, b] for a < b."""
        flat = [s for r in regions for s in r]
        buf, off = _pack(flat)
        rs = np.zeros(len(regions) + 1, np.int64)
        np.cumsum([len(r) for r in regions], out=rs[1:])
        R = len(regions)
        tot = np.zeros(R * R, np.int64)
        mx = np.zeros(R * R, np.int32)
        self._check(lib().umiclust_overlap_regions(self._h, buf.ctypes.data, _i64(off), len(flat), _i64(rs), R,
                                                   _i64(tot), mx.ctypes.data_as(C.POINTER(C.c_int32))),
                    "overlap_regions")
        return tot.reshape(R, R), mx.reshape(R, R)

    def extract_umis(self, seqs, a5: int = 73, a3: int = 68, k: int = 3, fwd: str = "", rev: str = "") -> np.ndarray:
        """[n, 6] int32: (dist, start, end) of the 5' and 3' UMI per read (-1: none), window coordinates."""
        buf, off = _pack(seqs)
        n = len(off) - 1
        out = np.zeros(max(n, 1) * 6, np.int32)
        self._check(lib().umiclust_extract_umis(self._h, buf.ctypes.data, _i64(off), n, a5, a3, k, fwd.encode(),
                                                rev.encode(), out.ctypes.data_as(C.POINTER(C.c_int32))),
                    "extract_umis")
        return out[:n * 6].reshape(n, 6)

    def extract_umis_file(self, fastx: str, out_fasta: str, a5: int, a3: int, k: int, fwd: str, rev: str) -> int:
        return int(self._check(lib().umiclust_extract_umis_file(self._h, fastx.encode(), out_fasta.encode(), a5, a3, k,
                                                                fwd.encode(), rev.encode()), "extract_umis_file"))

    def region_split(self, bam_file: str, names, lengths, clusters, minov: float, s5: int, s3: int, out_dir: str):
        """umiclust_region_split: (counts[4], reads_per_cluster, region_detected); KeyError(name) as the
        reference raises it."""
        R = len(names)
        nm = (C.c_char_p * max(R, 1))(*[x.encode() for x in names])
        ln = np.asarray(lengths, np.int64)
        cl = np.asarray(clusters, np.int32)
        cap = int(max([0] + [k + 1 for k in clusters]))
        counts = np.zeros(4, np.int64)
        rpc = np.zeros(max(cap, 1), np.int64)
        det = np.zeros(max(R, 1), np.uint8)
        miss = C.create_string_buffer(4096)
        P = C.POINTER
        rc = lib().umiclust_region_split(self._h, bam_file.encode(), R, nm, _i64(ln), cl.ctypes.data_as(P(C.c_int32)),
                                         minov, s5, s3, out_dir.encode(), _i64(counts), _i64(rpc), cap,
                                         det.ctypes.data_as(P(C.c_uint8)), miss, 4096)
        if rc == -74 and miss.value:
            raise KeyError(miss.value.decode())
        if rc == -74 and (lib().umiclust_last_error(self._h) or b"").startswith(b"TypeError: "):
            raise TypeError(lib().umiclust_last_error(self._h).decode()[len("TypeError: "):])
        self._check(rc, "region_split")
        return counts, rpc[:cap], det[:R]

    def align_pairs(self, p: Params, queries, targets, with_ops: bool = False) -> dict:
        qb, qo = _pack(queries)
        tb, to = _pack(targets)
        n = len(qo) - 1
        P = C.POINTER
        sc = np.zeros(max(n, 1), np.int32)
        m = np.zeros(max(n, 1), np.int32)
        il = np.zeros(max(n, 1), np.int32)
        stride = 2 * MAX_LEN
        ops = np.zeros(max(n, 1) * stride, np.uint8) if with_ops else None
        nops = np.zeros(max(n, 1), np.int32) if with_ops else None
        rc = lib().umiclust_align_pairs(self._h, C.byref(p), qb.ctypes.data, _i64(qo), tb.ctypes.data, _i64(to), n,
                                        sc.ctypes.data_as(P(C.c_int32)), m.ctypes.data_as(P(C.c_int32)),
                                        il.ctypes.data_as(P(C.c_int32)), ops.ctypes.data if with_ops else None,
                                        stride, nops.ctypes.data_as(P(C.c_int32)) if with_ops else None)
        self._check(rc, "align_pairs")
        out = dict(score=sc[:n], matches=m[:n], internal_len=il[:n])
        if with_ops:
            raw = ops.tobytes()
            out["ops"] = [raw[k * stride:k * stride + nops[k]].decode() for k in range(n)]
        return out

    def prep(self, p: Params, seqs) -> dict:
        b, o = _pack(seqs)
        n = len(o) - 1
        masked = np.zeros(len(b), np.uint8)
        kst = MAX_LEN - 7  # >= unique 8-mers per strand
        km = np.zeros(max(n, 1) * 2 * kst, np.uint16)
        nk = np.zeros(max(n, 1) * 2, np.int32)
        P = C.POINTER
        rc = lib().umiclust_prep(self._h, C.byref(p), b.ctypes.data, _i64(o), n, masked.ctypes.data,
                                 km.ctypes.data_as(P(C.c_uint16)), kst, nk.ctypes.data_as(P(C.c_int32)))
        self._check(rc, "prep")
        mb = masked.tobytes()
        return dict(masked=[mb[o[i]:o[i + 1]].decode() for i in range(n)],
                    kmers=[[list(km[(2 * i + s) * kst:(2 * i + s) * kst + nk[2 * i + s]]) for s in range(2)]
                           for i in range(n)])
