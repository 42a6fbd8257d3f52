"""Posting-list lengths by query k-mer rank on config-2 data, and what exact frequent-k-mer deferral would save
(measurement only).  Writes profiles/r03/posting_hist.json.

Index proxy: every 20th read of the synthetic config-2 bin (synth.make_umis, seed 1002; about one centroid per
molecule at 0.90 identity: the GPU run keeps ~100k centroids of 2M reads).  For 2,000 sampled queries the unique
8-mers (vsearch's k-mer set) are ranked by the length of their posting list.  Deferral with f k-mers: count the
other lists with threshold T - f (T = min(minwordmatches 12, k-mers)); the survivors are the centroids that could
still reach T once the f deferred k-mers are looked up in their own k-mer sets -- exact, as a centroid gains at
most f from them.  Reported per f: fraction of postings not streamed, survivors and true candidates per
query-strand.
"""
import json
import os
import sys
from collections import defaultdict

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ont-tcrconsensus_amd"))
from umiclust import synth  # noqa: E402

CODE = {"A": 0, "C": 1, "G": 2, "T": 3}


def kmers(s):
    out, x = set(), 0
    for i, ch in enumerate(s):
        x = ((x << 2) | CODE.get(ch, 0)) & 0xFFFF
        if i >= 7:
            out.add(x)
    return out


def rc(s):
    return s[::-1].translate(str.maketrans("ACGT", "TGCA"))


def main():
    u = synth.make_umis(100_000, seed=1002, max_reads=2_000_000)
    seqs = u.as_list()
    cents = seqs[::20][:100_000]
    cnt = np.zeros(65536, np.int64)
    post = defaultdict(list)
    for ci, s in enumerate(cents):
        for k in kmers(s):
            cnt[k] += 1
            post[k].append(ci)
    C = len(cents)
    rng = np.random.default_rng(0)
    qs = [seqs[i] for i in rng.choice(len(seqs), 2000, replace=False)]
    nr = 64
    ranked, tot = [], []
    for s in qs:
        ks = sorted((int(cnt[k]) for k in kmers(s)), reverse=True)
        ranked.append(ks[:nr] + [0] * (nr - len(ks[:nr])))
        tot.append(sum(ks))
    ranked = np.array(ranked, np.float64)
    tot = np.array(tot, np.float64)
    by_rank = [dict(rank=r, mean_list=float(ranked[:, r].mean()), p50=float(np.median(ranked[:, r])),
                    p99=float(np.percentile(ranked[:, r], 99)),
                    cum_share=float(ranked[:, :r + 1].sum(1).mean() / tot.mean())) for r in range(nr)]
    defer = []
    for strand in (0, 1):
        for f in (0, 1, 2, 3, 5, 8):
            surv, cand, saved = [], [], []
            for s in qs[:300]:
                q = s if strand == 0 else rc(s)
                ks = sorted(kmers(q), key=lambda k: -cnt[k])
                F, R = ks[:f], ks[f:]
                thr = min(12, len(ks))
                c = np.zeros(C, np.int32)
                for k in R:
                    if post[k]:
                        c[post[k]] += 1
                full = c.copy()
                for k in F:
                    if post[k]:
                        full[post[k]] += 1
                t_r, t_all = sum(cnt[k] for k in R), sum(cnt[k] for k in ks)
                surv.append(int((c >= max(1, thr - f)).sum()))
                cand.append(int((full >= thr).sum()))
                saved.append(1.0 - t_r / max(1, t_all))
            defer.append(dict(strand="+" if strand == 0 else "-", f=f, postings_saved=float(np.mean(saved)),
                              survivors_per_qs=float(np.mean(surv)), candidates_per_qs=float(np.mean(cand))))
            print(defer[-1], flush=True)
    out = dict(source="tools/posting_hist.py", index_proxy_centroids=C, queries=len(qs),
               mean_postings_per_query_strand=float(tot.mean()), by_rank=by_rank, deferral=defer)
    path = os.path.join(ROOT, "profiles", "r03", "posting_hist.json")
    json.dump(out, open(path, "w"), indent=1)
    print("mean postings", tot.mean(), "top-3 share", by_rank[2]["cum_share"], "->", path)


if __name__ == "__main__":
    main()
