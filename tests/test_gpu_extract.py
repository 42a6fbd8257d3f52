"""§8f row f1 on the GPU: the Myers kernel (umiclust_extract_umis) and the file-level drop-in
(umiclust.extract_umis) against the CPU restatement of edlib's HW/path semantics (oracle/extract.py) on
seeded reads.  Parity against edlib itself is unpinned (not installed; the reference has no fixture)."""
import os
import random

import extract as ox
import pytest
from umiclust import extract_umis as ge
from umiclust import synth

pytestmark = pytest.mark.gpu

FWD, REV = synth.UMI_FWD, synth.UMI_REV


def _mut(rng, s, n):
    s = list(s)
    for _ in range(n):
        x = rng.randrange(len(s))
        u = rng.random()
        if u < 0.4:
            s[x] = rng.choice("ACGT")
        elif u < 0.7:
            s.insert(x, rng.choice("ACGT"))
        elif len(s) > 1:
            del s[x]
    return "".join(s)


def _inst(rng, pat):
    return "".join(rng.choice("ACG") if c == "V" else rng.choice("CGT") if c == "B" else c for c in pat)


def _reads(seed, n):
    rng = random.Random(seed)
    out = []
    for i in range(n):
        body = "".join(rng.choice("ACGT") for _ in range(rng.randint(150, 400)))
        kind = rng.random()
        u5 = _mut(rng, _inst(rng, FWD), rng.choice([0, 0, 1, 2, 3, 4]))
        u3 = _mut(rng, _inst(rng, REV), rng.choice([0, 0, 1, 2, 3, 5]))
        pre = "".join(rng.choice("ACGT") for _ in range(rng.randint(0, 40)))
        suf = "".join(rng.choice("ACGT") for _ in range(rng.randint(0, 30)))
        if kind < 0.1:
            seq = body  # no UMI
        elif kind < 0.15:
            seq = (pre + u5 + "TTTTT" + body + "AAAAA" + u3 + suf).lower()  # lowercase read
        elif kind < 0.2:
            seq = pre + u5[:20]  # short read: windows overlap / truncated
        else:
            seq = pre + u5 + body + u3 + suf
        if rng.random() < 0.05:
            x = rng.randrange(len(seq))
            seq = seq[:x] + "N" + seq[x + 1:]
        out.append((f"read{i};strand={'+' if rng.random() < 0.5 else '-'}", seq))
    return out


@pytest.mark.parametrize("seed,k", [(1, 3), (2, 0), (3, 6)])
def test_windows_vs_oracle(gpu_ctx, seed, k):
    recs = _reads(seed, 600)
    seqs = [s for _, s in recs]
    got = gpu_ctx.extract_umis(seqs, 73, 68, k, FWD, REV)
    for i, s in enumerate(seqs):
        for w, (pat, win) in enumerate(((FWD, s[:73]), (REV, s[-68:]))):
            want = ox.hw_locate(pat, win, k)
            g = tuple(int(x) for x in got[i, 3 * w:3 * w + 3])
            assert g == (want if want else (-1, -1, -1)), (i, w, win)


@pytest.mark.parametrize("a5,a3", [(73, 68), (81, 76), (0, 40), (250, 0), (400, 300), (5, 255)])
def test_window_sizes_vs_oracle(gpu_ctx, a5, a3):
    """Both device paths: host-gathered windows (short windows) and whole reads (a3 == 0: the whole read as
    Python's seq[-0:] gives; windows past the gather limit), against Python slicing semantics."""
    seqs = [s for _, s in _reads(8, 250)]
    got = gpu_ctx.extract_umis(seqs, a5, a3, 3, FWD, REV)
    for i, s in enumerate(seqs):
        for w, (pat, win) in enumerate(((FWD, s[:a5]), (REV, s[-a3:]))):
            want = ox.hw_locate(pat, win, 3)
            g = tuple(int(x) for x in got[i, 3 * w:3 * w + 3])
            assert g == (want if want else (-1, -1, -1)), (i, w, a5, a3)


def test_single_window_helper(gpu_ctx):
    for name, s in _reads(4, 50):
        assert ge.extract_umi(s[:73], FWD, 3) == ox.extract_umi(s[:73], FWD, 3)


@pytest.mark.parametrize("fmt", ["fasta", "fastq"])
def test_file_dropin_vs_oracle(tmp_path, fmt):
    recs = _reads(5, 3000)
    src = tmp_path / f"region_cluster12.{fmt}"
    with open(src, "w") as fh:
        for name, s in recs:
            if fmt == "fasta":
                fh.write(f">{name} extra comment\n{s[:70]}\n{s[70:]}\n" if len(s) > 70 else f">{name}\n{s}\n")
            else:
                fh.write(f"@{name}\n{s}\n+\n{'I' * len(s)}\n")
    out = ge.extract_umis.remote(str(src), str(tmp_path), True, 73, 68, 3, FWD, REV)
    want, n = ox.extract_records(recs, 73, 68, 3, FWD, REV)
    assert out == os.path.join(str(tmp_path), "region_cluster12_detected_umis.fasta")
    assert open(out).read() == want and n > 0


def test_missing_strand_writes_earlier_records_then_raises(tmp_path):
    from umiclust import _lib
    recs = _reads(6, 20)
    recs[12] = ("read12", recs[12][1])
    src = tmp_path / "r.fasta"
    src.write_text("".join(f">{n}\n{s}\n" for n, s in recs))
    with pytest.raises(_lib.UmiclustError):
        ge.extract_umis(str(src), str(tmp_path), False)
    want, _ = ox.extract_records(recs[:12], 73, 68, 3, ge.UMI_FWD_DEFAULT, ge.UMI_REV_DEFAULT)
    assert open(tmp_path / "_detected_umis.fasta").read() == want


def test_no_umi_returns_none(tmp_path):
    src = tmp_path / "r.fasta"
    src.write_text(">a;strand=+\n" + "ACGT" * 50 + "\n")
    assert ge.extract_umis(str(src), str(tmp_path), True) is None
    assert (tmp_path / "r_detected_umis.fasta").read_text() == ""


# ---- pinned by the reference itself: tests/golden/extract (make_golden_extract.py ran extract_umis.py here) ----
import glob as _glob
import json as _json

_EXTRACT_FIX = sorted(_glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "extract",
                                              "*.json")))


@pytest.mark.parametrize("path", _EXTRACT_FIX, ids=[os.path.basename(p)[:-5] for p in _EXTRACT_FIX])
def test_extract_umis_vs_reference_fixtures(tmp_path, path):
    """umiclust.extract_umis byte for byte against the reference's extract_umis outputs: FASTA and multi-line
    FASTQ input, write_region True/False (the output-path rule), a zero 3' window (`seq[-0:]` = the whole read),
    a zero 5' window, the run_config.json patterns at k = 0 and 3, extra `;` fields after strand=, lowercase
    reads, `N`s, no read with both UMIs (returns None, empty file), and a record without `strand=` (the records
    before it written, then the exception)."""
    case = _json.load(open(path))
    src = tmp_path / case["file_name"]
    src.write_text(case["input"])
    out = tmp_path / "out"
    out.mkdir()
    if case["error"]:
        with pytest.raises(Exception):
            ge.extract_umis(str(src), str(out), **case["args"])
    else:
        ret = ge.extract_umis(str(src), str(out), **case["args"])
        assert (None if ret is None else os.path.relpath(ret, out)) == case["returned"]
    assert {f: open(os.path.join(out, f)).read() for f in sorted(os.listdir(out))} == case["files"]
