"""Debug aid: traceback ops of random pairs through umiclust_align_pairs (with_ops) in this process; prints a digest
per query length so two runs (UMICLUST_TRACE=step vs default) can be compared.  Usage: python tools/trace_ab.py out.json"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ont-tcrconsensus_amd")]
from umiclust import _lib  # noqa: E402


def main():
    rng = np.random.default_rng(5)
    qs, ts = [], []
    for _ in range(4000):
        ql = int(rng.integers(56, 112))
        q = "".join(rng.choice(list("ACGT"), ql))
        t = list(q)
        for _e in range(int(rng.integers(0, 5))):
            k = int(rng.integers(0, len(t)))
            r = rng.random()
            if r < 0.4:
                t[k] = str(rng.choice(list("ACGT")))
            elif r < 0.7:
                del t[k]
            else:
                t.insert(k, str(rng.choice(list("ACGT"))))
        qs.append(q)
        ts.append("".join(t)[:112])
    p = _lib.params(1, 0.9, 32, 112)
    with _lib.Context(0) as ctx:
        r = ctx.align_pairs(p, qs, ts, with_ops=True)
    out = {"ops": list(r["ops"]), "q": qs, "t": ts}
    json.dump(out, open(sys.argv[1], "w"))


if __name__ == "__main__":
    main()
