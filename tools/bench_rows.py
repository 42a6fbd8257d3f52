"""Measurement of the widened rows on one MI355X, each beside its CPU restatement.

    python tools/bench_rows.py [--reads N] [--out json]          (GPU box; rocprofv3 --kernel-trace --stats
                                                                  around it gives the kernel durations)
Per row: the GPU entry point's wall time through the C ABI (host buffers in, results out: PCIe-inclusive),
a parity check of its output against the oracle on a sample, and the oracle (oracle/, test infrastructure,
used only as the checker and the CPU baseline) timed on a bounded sample on one host thread.
  f1 extract_umis   (extract_umis.py:19-267): N synthetic ~1 kb reads with both UMIs in their adapter windows
  f3 overlap        (extract_umis.py:270-369): 40 regions x 20k UMIs (64 nt, shared pool -> overlaps)
  f4 region binning (region_split.py:219-333): a BGZF BAM of N/2 records over 60 regions
Inputs are synthetic and seeded.  Prints one JSON object.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import struct
import sys
import tempfile
import time
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ont-tcrconsensus_amd"), os.path.join(ROOT, "oracle")]
from umiclust import _lib, synth  # noqa: E402

ACGT = np.frombuffer(b"ACGT", np.uint8)


def _instances(rng, pattern: str, n: int) -> np.ndarray:
    """n instances of a UMI pattern (V -> A/C/G, B -> C/G/T), 2 % substitutions, as an [n, m] u8 array."""
    m = len(pattern)
    out = np.empty((n, m), np.uint8)
    for i, ch in enumerate(pattern):
        if ch == "V":
            out[:, i] = np.frombuffer(b"ACG", np.uint8)[rng.integers(0, 3, n)]
        elif ch == "B":
            out[:, i] = np.frombuffer(b"CGT", np.uint8)[rng.integers(0, 3, n)]
        else:
            out[:, i] = ord(ch)
    sub = rng.random((n, m)) < 0.02
    out[sub] = ACGT[rng.integers(0, 4, int(sub.sum()))]
    return out


def f1_reads(n: int, seed: int = 11):
    """[n] reads of 20 + 32 + 900 + 32 + 15 nt: prefix, 5' UMI, body, 3' UMI, suffix (uniform length)."""
    rng = np.random.default_rng(seed)
    parts = [ACGT[rng.integers(0, 4, (n, 20))], _instances(rng, synth.UMI_FWD, n), ACGT[rng.integers(0, 4, (n, 900))],
             _instances(rng, synth.UMI_REV, n), ACGT[rng.integers(0, 4, (n, 15))]]
    mat = np.ascontiguousarray(np.concatenate(parts, axis=1))
    off = np.arange(n + 1, dtype=np.int64) * mat.shape[1]
    return mat.reshape(-1), off


def bench_f1(ctx, n: int, cpu_sample: int) -> dict:
    import extract as ox
    buf, off = f1_reads(n)
    out = np.zeros(n * 6, np.int32)
    L = _lib.lib()
    fwd, rev = synth.UMI_FWD.encode(), synth.UMI_REV.encode()

    def run():
        rc = L.umiclust_extract_umis(ctx._h, buf.ctypes.data, off.ctypes.data_as(C.POINTER(C.c_int64)), n, 73, 68, 3,
                                     fwd, rev, out.ctypes.data_as(C.POINTER(C.c_int32)))
        if rc < 0:
            raise RuntimeError(f"extract_umis {rc}")
    run()
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        run()
        ts.append(time.perf_counter() - t0)
    gpu_s = min(ts)
    got = out.reshape(n, 6)
    raw = buf.tobytes()
    t0 = time.perf_counter()
    bad = 0
    for i in range(cpu_sample):
        s = raw[off[i]:off[i + 1]].decode()
        for w, (win, pat) in enumerate(((s[:73], synth.UMI_FWD), (s[-68:], synth.UMI_REV))):
            r = ox.hw_locate(pat, win, 3)
            want = (-1, -1, -1) if r is None else r
            bad += tuple(int(x) for x in got[i, 3 * w:3 * w + 3]) != tuple(want)
    cpu_s = time.perf_counter() - t0
    found = int(((got[:, 0] >= 0) & (got[:, 3] >= 0)).sum())
    return dict(row="f1 extract_umis", reads=n, read_len=int(off[1]), gpu_wall_s=gpu_s, reads_per_s=n / gpu_s,
                both_umis_found=found, parity_sample=cpu_sample, parity_mismatches=bad,
                cpu_baseline=dict(value=cpu_sample / cpu_s, unit="reads/s", cores=1, kind="port",
                                  sample=f"first {cpu_sample} reads, oracle/extract.py (O(mn) Python DP restating "
                                         "edlib HW/path; edlib itself is absent, so this is not edlib's speed)"),
                h2d_bytes=int(off[-1]), note="wall through the C ABI: whole reads H2D from pageable host memory, "
                                             "kernel, results D2H")


def f3_regions(R: int, per: int, seed: int = 13):
    rng = np.random.default_rng(seed)
    pool = ACGT[rng.integers(0, 4, (per * R // 4, 64))]
    regions = []
    for r in range(R):
        pick = rng.integers(0, len(pool), per)
        own = rng.random(per) < 0.6
        mat = pool[pick].copy()
        mat[own] = ACGT[rng.integers(0, 4, (int(own.sum()), 64))]
        regions.append(mat)
    return regions


def bench_f3(ctx, R: int, per: int, cpu_pairs: int) -> dict:
    import overlap as oo
    regions = f3_regions(R, per)
    flat = np.ascontiguousarray(np.concatenate(regions)).reshape(-1)
    n = R * per
    off = np.arange(n + 1, dtype=np.int64) * 64
    rs = np.arange(R + 1, dtype=np.int64) * per
    tot = np.zeros(R * R, np.int64)
    mx = np.zeros(R * R, np.int32)
    L = _lib.lib()
    P64 = C.POINTER(C.c_int64)

    def run():
        rc = L.umiclust_overlap_regions(ctx._h, flat.ctypes.data, off.ctypes.data_as(P64), n, rs.ctypes.data_as(P64), R,
                                        tot.ctypes.data_as(P64), mx.ctypes.data_as(C.POINTER(C.c_int32)))
        if rc < 0:
            raise RuntimeError(f"overlap_regions {rc}")
    run()
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        run()
        ts.append(time.perf_counter() - t0)
    gpu_s = min(ts)
    strs = [[bytes(x).decode() for x in reg] for reg in regions]
    T, M = tot.reshape(R, R), mx.reshape(R, R)
    t0 = time.perf_counter()
    bad = 0
    done = 0
    for a in range(R):
        for b in range(a + 1, R):
            if done >= cpu_pairs:
                break
            c = oo.overlap_counts(strs[a], strs[b])
            bad += (sum(c) != T[a, b]) + (max(c) != M[a, b])
            done += 1
    cpu_s = time.perf_counter() - t0
    pairs = R * (R - 1) // 2
    return dict(row="f3 count_overlapping_umis_between_all_regions", regions=R, umis_per_region=per, umis=n,
                region_pairs=pairs, gpu_wall_s=gpu_s, region_pairs_per_s=pairs / gpu_s, umis_per_s=n / gpu_s,
                parity_pairs=done, parity_mismatches=int(bad),
                cpu_baseline=dict(value=done / cpu_s, unit="region pairs/s", cores=1, kind="port",
                                  sample=f"{done} region pairs, oracle/overlap.py multiset join (the reference scans "
                                         "O(n*m) per pair, so this is faster than the reference's CPU path)"))


def _bgzf(raw: bytes, block: int = 65000) -> bytes:
    out = []
    for i in range(0, len(raw), block):
        d = raw[i:i + block]
        c = zlib.compressobj(1, zlib.DEFLATED, -15)
        comp = c.compress(d) + c.flush()
        out.append(struct.pack("<BBBBIBBHBBHH", 31, 139, 8, 4, 0, 0, 255, 6, 66, 67, 2, len(comp) + 25) + comp +
                   struct.pack("<II", zlib.crc32(d) & 0xffffffff, len(d)))
    out.append(bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000"))
    return b"".join(out)


def f4_bam(path: str, n: int, nref: int = 60, lseq: int = 600, seed: int = 17):
    """A BAM of n fixed-layout records (name r%09d, one CIGAR op) over nref regions of length 500."""
    rng = np.random.default_rng(seed)
    refs = [(f"TRBV{r}_1", 500) for r in range(nref)]
    hdr = bytearray(b"BAM\x01") + struct.pack("<i", 11) + b"@HD\tVN:1.6\n" + struct.pack("<i", nref)
    for nm, ln in refs:
        b = nm.encode() + b"\0"
        hdr += struct.pack("<i", len(b)) + b + struct.pack("<i", ln)
    lrn = 11
    body = 32 + lrn + 4 + (lseq + 1) // 2 + lseq
    dt = np.dtype([("bs", "<i4"), ("ref", "<i4"), ("pos", "<i4"), ("lrn", "u1"), ("mq", "u1"), ("bin", "<u2"),
                   ("ncig", "<u2"), ("flag", "<u2"), ("lseq", "<i4"), ("nref", "<i4"), ("npos", "<i4"), ("tlen", "<i4"),
                   ("name", "S11"), ("cig", "<u4"), ("seq", "u1", ((lseq + 1) // 2,)), ("qual", "u1", (lseq,))])
    rec = np.zeros(n, dt)
    rec["bs"] = body
    rec["ref"] = rng.integers(0, nref, n)
    rec["lrn"] = lrn
    rec["mq"] = 60
    rec["ncig"] = 1
    u = rng.random(n)
    flag = np.where(u < 0.05, 4, np.where(u < 0.1, 256, 0)) | np.where(rng.random(n) < 0.5, 16, 0)
    rec["flag"] = flag
    rec["lseq"] = lseq
    rec["nref"] = -1
    rec["npos"] = -1
    rec["name"] = np.array([b"r%09d" % i for i in range(n)], "S11")
    aln = np.where(rng.random(n) < 0.8, 500, 400)  # 20 % too short an overlap
    rec["cig"] = (aln << 4).astype(np.uint32)
    codes = np.array([1, 2, 4, 8], np.uint8)
    s = codes[rng.integers(0, 4, (n, lseq))]
    rec["seq"] = (s[:, 0::2] << 4) | s[:, 1::2]
    rec["qual"] = 0xff
    with open(path, "wb") as fh:
        fh.write(_bgzf(bytes(hdr) + rec.tobytes()))
    return refs


def bench_f4(ctx, n: int, cpu_records: int) -> dict:
    import bam
    import region_split as ors
    tmp = tempfile.mkdtemp(prefix="rows_f4_")
    path = os.path.join(tmp, "bc.bam")
    refs = f4_bam(path, n)
    names = [r[0] for r in refs]
    lengths = [r[1] for r in refs]
    clusters = [i // 2 for i in range(len(refs))]
    ts = []
    res = None
    for it in range(3):
        od = os.path.join(tmp, f"out{it}")
        os.makedirs(od)
        t0 = time.perf_counter()
        res = ctx.region_split(path, names, lengths, clusters, 0.95, 73, 68, od)
        ts.append(time.perf_counter() - t0)
    gpu_s = min(ts)
    counts, rpc, _ = res
    small = os.path.join(tmp, "small.bam")
    f4_bam(small, cpu_records)
    _, recs = bam.read_bam(small)
    od = os.path.join(tmp, "cpu")
    os.makedirs(od)
    t0 = time.perf_counter()
    cc, pc, _, _ = ors.split_records(recs, dict(zip(names, lengths)), dict(zip(names, clusters)), out_dir=od)
    cpu_s = time.perf_counter() - t0
    gd = os.path.join(tmp, "gpu_small")
    os.makedirs(gd)
    sc, _, _ = ctx.region_split(small, names, lengths, clusters, 0.95, 73, 68, gd)
    same = sorted(os.listdir(od)) == sorted(os.listdir(gd)) and all(
        open(os.path.join(od, f), "rb").read() == open(os.path.join(gd, f), "rb").read() for f in os.listdir(od))
    same = same and [int(x) for x in sc] == [cc["unmapped"], cc["primary"], cc["short"], cc["long"]]
    bam_bytes = os.path.getsize(path)
    return dict(row="f4 filter_and_split_reads_by_region_cluster", records=n, bam_bytes=bam_bytes, read_len=600,
                gpu_wall_s=gpu_s, records_per_s=n / gpu_s, counts=[int(x) for x in counts],
                parity_sample=cpu_records, parity_files_equal=bool(same),
                cpu_baseline=dict(value=cpu_records / cpu_s, unit="records/s", cores=1, kind="port",
                                  sample=f"{cpu_records} records: oracle/region_split.py record loop with one append "
                                         "open() per kept record as the reference does (BAM decoding by oracle/bam.py "
                                         "excluded)"),
                note="wall through the C ABI: BGZF inflate on host threads, device classify/emit, files appended")


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=1_000_000)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    ctx = _lib.Context(0)
    rows = []
    for name, fn in (("f1", lambda: bench_f1(ctx, args.reads, 150)), ("f3", lambda: bench_f3(ctx, 40, 20_000, 40)),
                     ("f4", lambda: bench_f4(ctx, args.reads // 2, 20_000))):
        t0 = time.perf_counter()
        rows.append(fn())
        print(f"{name} done in {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
    res = dict(device="MI355X (cuda:0)", rows=rows)
    ctx.close()
    s = json.dumps(res, indent=1)
    if args.out:
        open(args.out, "w").write(s)
    print(s, flush=True)


if __name__ == "__main__":
    main()
