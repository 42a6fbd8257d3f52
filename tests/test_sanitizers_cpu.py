"""Host-code sanitizers: the C oracle built with AddressSanitizer + UndefinedBehaviorSanitizer
(-fno-sanitize-recover) and driven through clustering (both presets), alignment with CIGARs, DUST and k-mer
extraction on seeded structured UMIs (oracle/asan_main.c).  A sanitizer report fails the test.  (GPU code
is not sanitized: GPU ASan / XNACK runs are unavailable on the GPU pool.)"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="no gcc")
def test_oracle_under_asan_ubsan(tmp_path):
    out = str(tmp_path)
    b = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan_check", f"OUT={out}"],
                       capture_output=True, text=True, timeout=300)
    assert b.returncode == 0, b.stderr
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([os.path.join(out, "orc_asan_check"), "2500"], capture_output=True, text=True, timeout=600,
                       env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    assert r.stdout.strip().endswith("ok")
    assert "runtime error" not in r.stderr


# ---- the drop-in's HIP-free host code (ont-tcrconsensus_amd/csrc/host_io.cpp) under ASan + UBSan ----
# tools/host_asan_main.cpp drives FASTA/FASTQ reading (threaded slicing past 1 MiB), the vsearch writers, the
# in-process parse_umi_clusters (against the fixtures the reference itself produced, tests/golden/parse), the
# detected-UMI writer, BGZF inflation and the argv grammar.  A sanitizer report fails the test.
import glob
import gzip
import json
import random
import re
import struct
import zlib

SAN_ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")


@pytest.fixture(scope="module")
def host_asan(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    out = str(tmp_path_factory.mktemp("host_asan"))
    b = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "ont-tcrconsensus_amd"), "host_asan", f"SAN_OUT={out}"],
                       capture_output=True, text=True, timeout=300)
    assert b.returncode == 0, b.stderr
    exe = os.path.join(out, "host_asan")

    def run(*args):
        r = subprocess.run([exe, *map(str, args)], capture_output=True, text=True, timeout=300, env=SAN_ENV)
        assert r.returncode == 0, r.stderr[-4000:]
        assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
        return r.stdout
    return run


def _vsearch_fasta(text):
    """vsearch's reading of a FASTA: labels cut at the first whitespace, letters only, lines before the first
    '>' ignored (the semantics host_io.cpp read_fasta restates)."""
    recs, cur = [], None
    for line in text.split("\n"):
        if line.startswith(">"):
            cur = [re.split(r"[ \t\r]", line[1:])[0], []]
            recs.append(cur)
        elif cur is not None:
            cur[1].append("".join(c for c in line if c.isalpha() and c.isascii()))
    return [(a, "".join(b)) for a, b in recs]


def test_host_fasta_reader_under_asan(host_asan, tmp_path):
    rng = random.Random(3)
    parts = ["junk before the first record\n", "\n"]
    for i in range(9000):  # > 1 MiB: the threaded slicing path
        seq = "".join(rng.choice("ACGTacgtN") for _ in range(rng.randint(0, 260)))
        label = f"r{i};strand={'+-'[i % 2]};x=y" + (" trailing words" if i % 7 == 0 else "")
        eol = "\r\n" if i % 11 == 0 else "\n"
        wrapped = eol.join(seq[j:j + 60] for j in range(0, len(seq), 60)) if i % 3 else seq
        parts.append(f">{label}{eol}{wrapped}{eol}" + ("\n" if i % 13 == 0 else ""))
    text = "".join(parts)
    fa = tmp_path / "in.fa"
    fa.write_text(text)
    assert fa.stat().st_size > (1 << 20)
    host_asan("fasta", fa, tmp_path / "out.tsv")
    got = [tuple(line.split("\t")) for line in (tmp_path / "out.tsv").read_text().splitlines()]
    assert got == _vsearch_fasta(text)


def test_host_fastq_reader_under_asan(host_asan, tmp_path):
    fq = tmp_path / "in.fq"
    fq.write_text("@a;strand=+ desc\nACGT\nAC\n+\nIIII\nII\n@b;strand=-\nGGGG\n+b\n!!!!\n\n@c\n\n+\n\n")
    host_asan("fastq", fq, tmp_path / "out.tsv")
    assert (tmp_path / "out.tsv").read_text().splitlines() == ["a;strand=+\tACGTAC", "b;strand=-\tGGGG", "c\t"]


def _relabel(text, pos_of):
    """Cluster ids of a reference fixture (consout order is arbitrary there) -> consout positions, the numbering
    the in-process parse uses (vsearch --clusterout_sort writes the consout in clusterid order)."""
    text = re.sub(r"clusters_fa/cluster(\d+)\.fasta", lambda m: f"clusters_fa/cluster{pos_of[int(m.group(1))]}.fasta",
                  text)
    text = re.sub(r"(?m)^>(\d+)$", lambda m: f">{pos_of[int(m.group(1))]}", text)
    text = re.sub(r"(?m)^cluster(\d+)\t", lambda m: f"cluster{pos_of[int(m.group(1))]}\t", text)
    return re.sub(r"Cluster (\d+) skipped", lambda m: f"Cluster {pos_of[int(m.group(1))]} skipped", text)


PARSE_FIX = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "parse", "*.json")))


@pytest.fixture(params=["disk", "ram"])
def out_dir(request, tmp_path):
    """Where the writers write: tmp_path, or a RAM-backed directory (/dev/shm: tmpfs), where host_io maps the one-file
    outputs (consout, smolecule_clusters.fa) instead of pwrite-ing them (ram_backed())."""
    if request.param == "disk":
        yield tmp_path
        return
    import shutil
    import tempfile
    if not os.path.isdir("/dev/shm") or not os.access("/dev/shm", os.W_OK):
        pytest.skip("no /dev/shm")
    d = tempfile.mkdtemp(prefix="uc_asan_", dir="/dev/shm")
    try:
        yield __import__("pathlib").Path(d)
    finally:
        shutil.rmtree(d, ignore_errors=True)


@pytest.mark.parametrize("mode", ["parse", "parse_pre"])
@pytest.mark.parametrize("path", PARSE_FIX, ids=[os.path.basename(p)[:-5] for p in PARSE_FIX])
def test_host_parse_vs_reference_fixtures_under_asan(host_asan, out_dir, path, mode):
    tmp_path = out_dir
    case = json.load(open(path))
    inp, exp = case["inputs"], case["outputs"]
    ids = [int(line.split(";")[-1].split("=")[1]) for line in inp["consout"].splitlines() if line.startswith(">")]
    pos_of = {cid: k for k, cid in enumerate(ids)}
    text = "".join(inp["clusters"][f"cluster{cid}"] for cid in ids)
    sizes = [inp["clusters"][f"cluster{cid}"].count(">") for cid in ids]
    (tmp_path / "in.fa").write_text(text)
    work = tmp_path / inp["region"]
    work.mkdir()
    a = inp["args"]
    out = host_asan(mode, tmp_path / "in.fa", ",".join(map(str, sizes)), work, a.get("min_reads_per_cluster", 20),
                    a.get("max_reads_per_cluster", 60), int(a.get("balance_strands", False)),
                    a.get("max_clusters") or 0)
    got = {}
    for root, _dirs, fns in os.walk(work):
        for fn in fns:
            got[os.path.relpath(os.path.join(root, fn), work)] = \
                open(os.path.join(root, fn)).read().replace(str(work), "{DIR}")
    want = {_relabel(k, pos_of): _relabel(v, pos_of) for k, v in exp["files"].items()}
    assert got == want
    assert out.split()[3] == ("1" if exp["returned"] is None else "0")


@pytest.mark.parametrize("mode", ["parse", "parse_pre"])
def test_host_parse_errors_under_asan(host_asan, out_dir, mode):
    """The reference's failures: a missing seq= field in the middle of a written cluster (IndexError: the records
    before it written, no stats line for that cluster), a header without 7 fields, clusters_fa already present."""
    tmp_path = out_dir
    def rec(i, strand, seq=True):
        tail = f";seq=READ{i}" if seq else ";noseq"
        return f">r{i};strand={strand};umi_fwd_dist=0;umi_rev_dist=0;umi_fwd_seq=A;umi_rev_seq=C{tail}\nACGTACGT\n"
    recs = [rec(i, "+-"[i % 2]) for i in range(6)] + [rec(6, "+"), rec(7, "-", seq=False), rec(8, "+")]
    (tmp_path / "in.fa").write_text("".join(recs))
    w = tmp_path / "w1"
    w.mkdir()
    out = host_asan(mode, tmp_path / "in.fa", "6,3", w, 1, 60, 0, 0)
    assert out.startswith(f"error -74 ")
    assert sorted(os.listdir(w / "clusters_fa")) == ["cluster0.fasta", "cluster1.fasta"]
    # cluster 1 writes its '+' reads first: r6, r8, then r7 (the '-' read without seq=) raises
    assert (w / "clusters_fa" / "cluster1.fasta").read_text() == ">r6\nREAD6\n>r8\nREAD8\n"
    assert (w / "vsearch_cluster_stats.tsv").read_text().count("\n") == 2  # header + cluster0
    assert not (w / "parse_cluster.log").exists()
    (tmp_path / "bad.fa").write_text(">r0;strand=+;a;b\nACGT\n")
    w2 = tmp_path / "w2"
    w2.mkdir()
    assert host_asan(mode, tmp_path / "bad.fa", "1", w2, 1, 60, 0, 0).startswith("error -74 ")
    assert host_asan(mode, tmp_path / "bad.fa", "1", w2, 1, 60, 0, 0).startswith("error -17 ")
    # a strand other than + / - (the precomputed fields leave it to the reference's own error path)
    (tmp_path / "badstrand.fa").write_text(rec(0, "+") + rec(1, "x"))
    w3 = tmp_path / "w3"
    w3.mkdir()
    out = host_asan(mode, tmp_path / "badstrand.fa", "2", w3, 1, 60, 0, 0)
    assert out.startswith("error -74 ") and "Strand annotation is x but only - or + are allowed!" in out


def test_host_writers_under_asan(host_asan, out_dir):
    tmp_path = out_dir
    rng = random.Random(5)
    seqs = ["".join(rng.choice("ACGT") for _ in range(rng.randint(1, 170))) for _ in range(700)]
    sizes = []
    left = len(seqs)
    while left:
        sizes.append(min(left, rng.randint(1, 9)))
        left -= sizes[-1]
    (tmp_path / "in.fa").write_text("".join(f">s{i};x\n{s}\n" for i, s in enumerate(seqs)))
    host_asan("write", tmp_path / "in.fa", ",".join(map(str, sizes)), tmp_path / "cluster", tmp_path / "cons.fa")

    def wrap(s):
        return "".join(s[i:i + 80] + "\n" for i in range(0, len(s), 80)) or "\n"
    want, i = [], 0
    for k, m in enumerate(sizes):
        want.append(f">centroid=s{i};x;seqs={m};clusterid={k}\n" + wrap(seqs[i]))
        assert (tmp_path / f"cluster{k}").read_text() == "".join(f">s{j};x\n" + wrap(seqs[j][:128])
                                                                for j in range(i, i + m))
        i += m
    assert (tmp_path / "cons.fa").read_text() == "".join(want)
    # no sequence changed by masking: the writer prints the input's own bytes (no masked download)
    host_asan("write_input", tmp_path / "in.fa", ",".join(map(str, sizes)), tmp_path / "icluster", tmp_path / "icons.fa")
    i = 0
    for k, m in enumerate(sizes):
        assert (tmp_path / f"icluster{k}").read_text() == "".join(f">s{j};x\n" + wrap(seqs[j]) for j in range(i, i + m))
        i += m


def test_host_detected_umis_writer_under_asan(host_asan, tmp_path):
    recs = [("r0;strand=+", "AAAACCCCGGGGTTTT"), ("r1;strand=-", "ACGTACGTACGTACGT"), ("r2;strand=+", "GGGGGGGG")]
    (tmp_path / "in.fa").write_text("".join(f">{a}\n{b}\n" for a, b in recs))
    res = [[0, 0, 3, 1, 1, 4], [2, 4, 7, 0, 0, 2], [-1, 0, 0, 0, 0, 1]]
    (tmp_path / "res.txt").write_text("\n".join(" ".join(map(str, r)) for r in res))
    assert host_asan("umis", tmp_path / "in.fa", tmp_path / "res.txt", tmp_path / "out.fa", 6).strip() == "2"
    rc = lambda s: s[::-1].translate(str.maketrans("ACGT", "TGCA"))  # noqa: E731
    # r0: 5' window [0, 3], 3' window = the last 6 bases, UMI at [1, 4] of it
    s0, s1 = recs[0][1], recs[1][1]
    u5, u3 = s0[0:4], s0[-6:][1:5]
    v5, v3 = s1[4:8], s1[-6:][0:3]
    assert (tmp_path / "out.fa").read_text() == (
        f">r0;strand=+;umi_fwd_dist=0;umi_rev_dist=1;umi_fwd_seq={u5};umi_rev_seq={u3};seq={s0}\n{u5}{u3}\n"
        f">r1;strand=-;umi_fwd_dist=2;umi_rev_dist=0;umi_fwd_seq={v5};umi_rev_seq={v3};seq={s1}\n{rc(v3)}{rc(v5)}\n")


def _bgzf(data: bytes, block: int = 20000) -> bytes:
    out = b""
    for i in range(0, len(data), block):
        chunk = data[i:i + block]
        c = zlib.compressobj(6, zlib.DEFLATED, -15)
        comp = c.compress(chunk) + c.flush()
        bsize = 18 + len(comp) + 8
        out += (b"\x1f\x8b\x08\x04" + b"\x00" * 4 + b"\x00\xff" + struct.pack("<H", 6) + b"BC" +
                struct.pack("<HH", 2, bsize - 1) + comp + struct.pack("<II", zlib.crc32(chunk) & 0xffffffff, len(chunk)))
    c = zlib.compressobj(6, zlib.DEFLATED, -15)  # the BGZF EOF block
    comp = c.compress(b"") + c.flush()
    return out + (b"\x1f\x8b\x08\x04" + b"\x00" * 4 + b"\x00\xff" + struct.pack("<H", 6) + b"BC" +
                  struct.pack("<HH", 2, 18 + len(comp) + 8 - 1) + comp + struct.pack("<II", 0, 0))


def test_host_bgzf_under_asan(host_asan, tmp_path):
    rng = random.Random(9)
    data = bytes(rng.getrandbits(8) if i % 5 else 65 for i in range(300_000))
    (tmp_path / "a.bgzf").write_bytes(_bgzf(data))
    host_asan("bgzf", tmp_path / "a.bgzf", tmp_path / "a.raw")
    assert (tmp_path / "a.raw").read_bytes() == data
    assert gzip.decompress((tmp_path / "a.bgzf").read_bytes()) == data  # a valid multi-member gzip too
    blob = _bgzf(data)
    (tmp_path / "t.bgzf").write_bytes(blob[:len(blob) // 2])  # truncated mid-block
    assert host_asan("bgzf", tmp_path / "t.bgzf", tmp_path / "t.raw").strip() == "error bgzf"
    (tmp_path / "g.bgzf").write_bytes(gzip.compress(data))  # plain gzip: no BC field
    assert host_asan("bgzf", tmp_path / "g.bgzf", tmp_path / "g.raw").strip() == "error bgzf"


def test_host_argv_under_asan(host_asan):
    argv = json.load(open(os.path.join(ROOT, "tests", "golden", "argv.json")))["calls"][0]["argv"]
    out = host_asan("argv", *argv)
    assert "id 0.9300 len 58 68 match 10 mismatch -40 open 0 0 40 40 0 0 ext 1 1 2 2 1 1 strand 1 sort 1 id 1" in out
    assert "threads 25" in out and "in in.fa clusters /tmp/out/cluster" in out
    assert host_asan("argv", "vsearch", "--gapopen", "4X", "--cluster_fast", "a").strip() == "rc -22"
    assert host_asan("argv", "vsearch", "--cluster_fast").strip() == "rc -22"
    assert host_asan("argv", "vsearch", "--cluster_fast", "x" * 300).strip() == "rc -22"  # longer than the buffer


# ---- the host resolve (ont-tcrconsensus_amd/csrc/resolve.cpp) under ThreadSanitizer ----
# resolve_block's classify phase runs on a worker pool over the window's states and the pass's records while the
# in-order phase writes the block's states; tools/resolve_tsan_main.cpp replays resolve_block calls recorded from
# GPU clustering runs (tests/golden/make_resolve_dumps.py: a config-2-like bin, lazy peers with round B, deep
# clusters, batched O4 rounds) with 1, 3 and 8 threads -- and with the in-order phase forced onto 3 and 8 pool threads
# (its dependency-ordered parallel form) -- and checks every output against the recorded one.
RESOLVE_DUMPS = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "resolve", "*.bin.gz")))


@pytest.fixture(scope="module")
def resolve_tsan(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    out = str(tmp_path_factory.mktemp("resolve_tsan"))
    exe = os.path.join(out, "resolve_tsan")
    src = os.path.join(ROOT, "ont-tcrconsensus_amd", "csrc")
    b = subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-fsanitize=thread", "-o", exe,
                        os.path.join(ROOT, "tools", "resolve_tsan_main.cpp"), os.path.join(src, "resolve.cpp"),
                        "-lpthread"], capture_output=True, text=True, timeout=300)
    assert b.returncode == 0, b.stderr
    return exe, out


@pytest.mark.skipif(not RESOLVE_DUMPS, reason="no recorded resolve dumps")
@pytest.mark.parametrize("path", RESOLVE_DUMPS, ids=[os.path.basename(p)[:-7] for p in RESOLVE_DUMPS])
def test_host_resolve_under_tsan(resolve_tsan, path):
    exe, out = resolve_tsan
    raw = os.path.join(out, os.path.basename(path)[:-3])
    with gzip.open(path, "rb") as fi, open(raw, "wb") as fo:
        fo.write(fi.read())
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1")
    r = subprocess.run([exe, raw], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "ThreadSanitizer" not in r.stderr, r.stderr[-4000:]
    assert r.stdout.count(": equal") == 5, r.stdout
