"""Generate tests/golden/overlap/*.json from the REFERENCE itself (run here, not on the GPU box): inputs and
outputs of count_overlapping_umis_between_all_regions / count_overlapping_umis_between_2_regions
(/root/reference/ont_tcr_consensus/extract_umis.py:270-369).

`ray`, `pysam` and `edlib` are not installed (ordinary ModuleNotFoundError).  They are
replaced by stand-ins that execute nothing from the data: ray.remote(...) returns an object whose .remote()
calls the function directly and returns a future holding its value or its exception, and ray.get() of a list
of futures returns their values or, after every task has run, raises the first exception in list order --
Ray's semantics: one failing task does not stop the others from appending their TSV rows (TSV rows come in
itertools.combinations order); pysam.FastxFile is the FASTA iterator of make_golden.py; edlib.align is never
called (its call is commented out upstream) and raises if it were.  Only data is written to the fixtures.

Usage: python tests/golden/make_golden_overlap.py  (requires /root/reference)
"""
from __future__ import annotations

import json
import os
import random
import shutil
import sys
import tempfile
import types

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden  # noqa: E402  (the pysam stand-in and the module loader)


def _stubs():
    make_golden._stub_modules()  # pysam + a pass-through ray, replaced below

    class _Future:
        def __init__(self, f, a, k):
            try:
                self.value, self.exc = f(*a, **k), None
            except Exception as e:  # noqa: BLE001 -- held until ray.get, as Ray does
                self.value, self.exc = None, e

    class _Remote:
        def __init__(self, f):
            self.f = f

        def remote(self, *a, **k):
            return _Future(self.f, a, k)

        def options(self, **_k):
            return self

        def __call__(self, *a, **k):
            return self.f(*a, **k)

    ray = types.ModuleType("ray")
    ray.remote = lambda *a, **k: (_Remote(a[0]) if a and callable(a[0]) else (lambda f: _Remote(f)))
    def _get(x):
        if isinstance(x, list):
            vals = [_get(y) if not isinstance(y, _Future) or y.exc is None else y for y in x]
            for y in vals:
                if isinstance(y, _Future):
                    raise y.exc
            return vals
        if isinstance(x, _Future):
            if x.exc is not None:
                raise x.exc
            return x.value
        return x

    ray.get = _get
    sys.modules["ray"] = ray
    edlib = types.ModuleType("edlib")

    def _align(*a, **k):
        raise RuntimeError("edlib.align is not called by the reference's overlap count")

    edlib.align = _align
    sys.modules["edlib"] = edlib


def _consout(d, seqs, width):
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "umi_clusters_consensus.fasta"), "w") as fh:
        for i, s in enumerate(seqs):
            fh.write(f">centroid=r{i};strand=+;seqs={1 + i % 5};clusterid={i}\n")
            for j in range(0, max(1, len(s)), width):
                fh.write(s[j:j + width] + "\n")


def _case(rng, name, n_regions, sizes, pool_size, dup_frac, width=80, long_frac=0.0, empty=()):
    pool = []
    for _ in range(pool_size):
        n = rng.randint(81, 110) if rng.random() < long_frac else rng.randint(56, 70)
        pool.append("".join(rng.choice("ACGT") for _ in range(n)))
    regions = []
    for r in range(n_regions):
        n = 0 if r in empty else rng.choice(sizes)
        seqs = [rng.choice(pool) if rng.random() < dup_frac else
                "".join(rng.choice("ACGTN" if rng.random() < 0.05 else "ACGT") for _ in range(rng.randint(56, 70)))
                for _ in range(n)]
        regions.append(dict(name=f"region_cluster{rng.randint(0, 999)}_{r}", seqs=seqs))
    return dict(name=name, width=width, regions=regions)


def run_case(mod, case):
    tmp = tempfile.mkdtemp(prefix="ovl_")
    try:
        dirs = []
        for reg in case["regions"]:
            d = os.path.join(tmp, reg["name"])
            _consout(d, reg["seqs"], case["width"])
            dirs.append(d)
        logs = os.path.join(tmp, "logs")
        os.mkdir(logs)
        fas = [os.path.join(d, "smolecule_filtered.fa") for d in dirs]
        out = dict(case)
        try:
            out["result"] = mod.count_overlapping_umis_between_all_regions(
                smolecule_filtered_fa_list=fas, overlapping_umi_edit_threshold=2, logs_dir=logs)
            out["error"] = None
        except ValueError as e:  # max() of an empty region 1
            out["result"] = None
            out["error"] = f"ValueError: {e}"
        files = {}
        for fn in sorted(os.listdir(logs)):
            files[fn] = open(os.path.join(logs, fn)).read()
        out["files"] = files
        return out
    finally:
        shutil.rmtree(tmp)


def main():
    _stubs()
    mod = make_golden._load("extract_umis")
    rng = random.Random(20261016)
    cases = [
        _case(rng, "small_shared_pool", 4, [5, 12, 30], 20, 0.8),
        _case(rng, "duplicates_warning", 5, [40, 60], 15, 0.95),
        _case(rng, "disjoint", 3, [50], 100, 0.0),
        _case(rng, "long_multiline", 4, [20, 35], 25, 0.7, width=80, long_frac=0.6),
        _case(rng, "narrow_wrap", 3, [25], 10, 0.9, width=7),
        _case(rng, "empty_region_2", 3, [20], 10, 0.9, empty=(2,)),
        _case(rng, "empty_region_1", 3, [20], 10, 0.9, empty=(0,)),
        _case(rng, "many_regions", 12, [10, 50, 120], 200, 0.6),
        _case(rng, "empty_region_mid", 5, [20, 30], 10, 0.9, empty=(2,)),
    ]
    od = os.path.join(HERE, "overlap")
    os.makedirs(od, exist_ok=True)
    for c in cases:
        res = run_case(mod, c)
        with open(os.path.join(od, c["name"] + ".json"), "w") as fh:
            json.dump(res, fh, indent=0, sort_keys=True)
        print(c["name"], res["result"], res["error"], list(res["files"]))


if __name__ == "__main__":
    main()
