"""Host-side checks of the drop-in boundary that need no GPU: library load + exports, argv parity
with the reference (golden argv captured from vsearch_umi_cluster.py), parameter decoding."""
import ctypes
import json
import os
import re

import pytest
from umiclust import _lib
from umiclust.vsearch_umi_cluster import round1_argv, round2_argv

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGV = json.load(open(os.path.join(ROOT, "tests", "golden", "argv.json")))


def test_library_exports_every_declared_symbol():
    hdr = open(os.path.join(ROOT, "include", "umiclust.h")).read()
    declared = set(re.findall(r"\b(umiclust_[a-z_]+)\s*\(", hdr))
    assert declared == set(_lib.EXPORTS)
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for name in declared:
        assert hasattr(lib, name), name
    assert _lib.lib().umiclust_abi_version() == 9


def test_argv_matches_reference():
    for call in ARGV["calls"]:
        a = call["args"] + [None] * (6 - len(call["args"]))
        fn = round1_argv if call["fn"] == "vsearch_cluster" else round2_argv
        defaults = (50, 60, 0.94 if call["fn"] == "vsearch_cluster" else 0.97)
        args = [x if x is not None else defaults[i - 3] for i, x in enumerate(a)]
        assert fn(*args) == call["argv"]


def test_params_from_round1_argv():
    p, paths = _lib.params_from_argv(ARGV["calls"][0]["argv"])
    assert (p.match, p.mismatch, p.id, p.minseqlength, p.maxseqlength) == (10, -40, 0.93, 58, 68)
    assert list(p.gap_open) == [0, 0, 40, 40, 0, 0] and list(p.gap_ext) == [1, 1, 2, 2, 1, 1]
    assert (p.strand_both, p.clusterout_sort, p.clusterout_id, p.qmask_dust) == (1, 1, 1, 1)
    assert paths == {"in_fasta": "in.fa", "clusters_prefix": "/tmp/out/cluster",
                     "consout": "/tmp/out/umi_clusters_consensus.fasta", "log": "/tmp/out/vsearch_cluster.log"}


def test_params_from_round2_argv():
    p, paths = _lib.params_from_argv(ARGV["calls"][1]["argv"])
    assert (p.match, p.mismatch, p.id) == (2, -4, 0.97)
    assert list(p.gap_open) == [2, 2, 20, 20, 2, 2] and list(p.gap_ext) == [1, 1, 2, 2, 1, 1]
    assert paths["log"] == "/tmp/out2/vsearch_cluster_consensus.log"


def test_presets_equal_argv_decoding(monkeypatch):
    monkeypatch.delenv("UMICLUST_O4", raising=False)
    a, _ = _lib.params_from_argv(ARGV["calls"][0]["argv"])
    b = _lib.params(_lib.PRESET_ROUND1, 0.93, 58, 68, threads=25)  # the captured argv's --threads 25: policy O4
    assert bytes(a) == bytes(b)
    a, _ = _lib.params_from_argv(ARGV["calls"][1]["argv"])
    b = _lib.params(_lib.PRESET_VSEARCH_DEFAULT, 0.97, 58, 68, threads=25)
    assert bytes(a) == bytes(b)


@pytest.mark.parametrize("env,policy", [(None, 1), ("sequential", 0), ("batched", 1)])
def test_o4_policy_from_argv_threads(monkeypatch, env, policy):
    """the reference's argv carries --threads 25, so by default the drop-in computes vsearch's
    multithreaded clustering (the batched restatement, rounds of 25 queries); UMICLUST_O4=sequential opts out."""
    if env is None:
        monkeypatch.delenv("UMICLUST_O4", raising=False)
    else:
        monkeypatch.setenv("UMICLUST_O4", env)
    p, _ = _lib.params_from_argv(ARGV["calls"][0]["argv"])
    assert (p.threads, p.policy_threads) == (25, policy)


@pytest.mark.parametrize("threads,policy", [("1", 0), ("2", 1), ("64", 1)])
def test_o4_policy_follows_threads(monkeypatch, threads, policy):
    """--threads 1 is vsearch's sequential clustering (cluster_core_serial); any n > 1 its rounds of n queries."""
    monkeypatch.delenv("UMICLUST_O4", raising=False)
    argv = list(ARGV["calls"][0]["argv"])
    argv[argv.index("--threads") + 1] = threads
    p, _ = _lib.params_from_argv(argv)
    assert (p.threads, p.policy_threads) == (int(threads), policy)


def test_o4_policy_bad_environment(monkeypatch):
    monkeypatch.setenv("UMICLUST_O4", "sometimes")
    with pytest.raises(_lib.UmiclustError):
        _lib.params_from_argv(ARGV["calls"][0]["argv"])


@pytest.mark.parametrize("bad", [["vsearch", "--cluster_fast"], ["vsearch", "--bogus", "--cluster_fast", "a"],
                                 ["vsearch", "--gapopen", "4X", "--cluster_fast", "a"], ["vsearch"]])
def test_bad_argv_rejected(bad):
    with pytest.raises(_lib.UmiclustError):
        _lib.params_from_argv(bad)


def test_gap_string_grammar():
    p, _ = _lib.params_from_argv(["vsearch", "--cluster_fast", "a", "--gapopen", "20I/2E/5QL", "--gapext", "3"])
    assert list(p.gap_open) == [5, 2, 20, 20, 2, 2]
    assert list(p.gap_ext) == [3] * 6


def test_no_device_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(_lib.UmiclustError):
        _lib.Context(0)
