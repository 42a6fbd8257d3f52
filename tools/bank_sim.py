"""LDS bank load of k_pf_count's counting atomics under two posting layouts (measurement aid, not product code).

Index proxy as tools/posting_hist.py (every 20th read of the synthetic config-2 bin as centroids).  For sampled
query-strands of part 0, the stream of the query's posting lists (padded to 8-posting chunks) is counted as the
kernel does: lane l of a 64-chunk window takes chunk l, instruction e adds posting e of every lane's chunk; an
instruction costs the largest number of lanes on one LDS bank (u8 counters, dword = counter >> 2).  Layouts: `sorted`
(a chunk holds 8 consecutive postings of its list, as built today) and `transposed` (slot e of chunk i holds posting
e * C + i of a C-chunk list: consecutive lanes take consecutive postings of a list).

    python tools/bank_sim.py [banks]
"""
import json
import os
import sys
from collections import defaultdict

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ont-tcrconsensus_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from umiclust import synth  # noqa: E402
from posting_hist import kmers, rc  # noqa: E402

K_CENT_BASE = 3392
K_DUMMY = 3072


def chunks(lst, layout):
    n = len(lst)
    C = (n + 7) // 8
    pad = [-(1 + (i % 64)) for i in range(8 * C - n)]  # padding postings: spare counters
    full = list(lst) + pad
    if layout == "sorted":
        return [full[8 * i:8 * i + 8] for i in range(C)]
    return [[full[e * C + i] for e in range(8)] for i in range(C)]


def main():
    banks = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    u = synth.make_umis(100_000, seed=1002, max_reads=2_000_000)
    seqs = u.as_list()
    cents = seqs[::20][:100_000]
    post = defaultdict(list)
    for ci, s in enumerate(cents):
        if ci % 8:
            continue  # part 0
        for k in kmers(s):
            post[k].append(ci // 8)
    rng = np.random.default_rng(1)
    out = {}
    for layout in ("sorted", "transposed"):
        cyc, ninst = 0, 0
        for qi in rng.choice(len(seqs), 300, replace=False):
            for s in (seqs[qi], rc(seqs[qi])):
                stream = []
                for k in sorted(kmers(s)):
                    stream += chunks(post.get(k, []), layout)
                for w0 in range(0, len(stream), 64):
                    win = stream[w0:w0 + 64]
                    for e in range(8):
                        load = np.zeros(banks, np.int64)
                        for ch in win:
                            c = ch[e]
                            dw = (K_DUMMY + (-c - 1)) // 4 if c < 0 else (K_CENT_BASE + c) // 4
                            load[dw % banks] += 1
                        cyc += int(load.max())
                        ninst += 1
        out[layout] = dict(instructions=ninst, mean_busiest_bank=cyc / ninst)
    out["banks"] = banks
    print(json.dumps(out))


if __name__ == "__main__":
    main()
