"""Pure-Python restatement of vsearch `--cluster_fast` + `--consout` for TINY inputs.

TEST INFRASTRUCTURE ONLY (see umiclust_oracle.h): a second, independently written restatement
of SURVEY.md Appendix A, used to cross-check the C oracle (umiclust_oracle.c) on small cases.
It works on CIGAR strings and explicit candidate heaps the way vsearch's own code does
(searchcore.cc search_onequery/align_delayed, align_simd.cc backtrack16, msa.cc), instead of the
C oracle's loops, so the two share no code.  PARITY UNPINNED against vsearch itself.
"""
from __future__ import annotations

import heapq
import re

NEG = -10 ** 8
_C4 = {c: v for c, v in zip("ACGTURYSWKMBDHVN", [1, 2, 4, 8, 8, 5, 10, 6, 9, 12, 3, 14, 13, 11, 7, 15])}
_COMP = dict(zip("ACGTURYSWKMBDHVNacgturyswkmbdhvn", "TGCAAYRSWMKVHDBNtgcaayrswmkvhdbn"))
QL, TL, QI, TI, QR, TR = range(6)


def c4(ch):
    return _C4.get(ch.upper(), 0)


def revcomp(s):
    return "".join(_COMP.get(c, c) for c in reversed(s))


class P:
    def __init__(self, preset=1, identity=0.93, minlen=58, maxlen=68):
        self.id, self.minlen, self.maxlen = identity, minlen, maxlen
        self.k, self.minwm, self.maxaccepts, self.maxrejects = 8, 12, 1, 32
        self.ge = [1, 1, 2, 2, 1, 1]
        if preset == 1:
            self.match, self.mismatch, self.go = 10, -40, [0, 0, 40, 40, 0, 0]
        else:
            self.match, self.mismatch, self.go = 2, -4, [2, 2, 20, 20, 2, 2]
        self.dust = True
        self.boundary_open = True


def _sub(p, a, b):
    x, y = c4(a), c4(b)
    if x not in (1, 2, 4, 8) or y not in (1, 2, 4, 8):
        return 0
    return p.match if x == y else p.mismatch


def nw(p, q, t):
    """Gotoh DP with vsearch's path bits, then backtrack16. Returns (score, cigar, matches)."""
    n, m = len(q), len(t)
    H = [[0] * (m + 1) for _ in range(n + 1)]  # H[i+1][j+1]
    for j in range(m):
        H[0][j + 1] = -(p.go[QL] + (j + 1) * p.ge[QL])
    for i in range(n):
        H[i + 1][0] = -(p.go[TL] + (i + 1) * p.ge[TL])
    D = {}
    Fcol = []
    for j in range(m):
        r = TR if j == m - 1 else TI
        Fcol.append(H[0][j + 1] - (p.go[r] + p.ge[r]) if p.boundary_open else NEG)
    for i in range(n):
        rq = QR if i == n - 1 else QI
        E = H[i + 1][0] - (p.go[rq] + p.ge[rq]) if p.boundary_open else NEG
        for j in range(m):
            rt = TR if j == m - 1 else TI
            diag = H[i][j] + _sub(p, q[i], t[j])
            F = Fcol[j]
            best, up, left = diag, F > diag, False
            if up:
                best = F
            if E > best:
                best, left = E, True
            H[i + 1][j + 1] = best
            fo, fe = best - (p.go[rt] + p.ge[rt]), F - p.ge[rt]
            extup = fe > fo
            Fcol[j] = fe if extup else fo
            eo, ee = best - (p.go[rq] + p.ge[rq]), E - p.ge[rq]
            extleft = ee > eo
            E = ee if extleft else eo
            D[(i, j)] = (up, left, extup, extleft)
    ops = []
    i, j, op, matches = n - 1, m - 1, None, 0
    while i >= 0 and j >= 0:
        up, left, extup, extleft = D[(i, j)]
        if op == "I" and extleft:
            j -= 1
        elif op == "D" and extup:
            i -= 1
        elif left:
            op = "I"
            j -= 1
        elif up:
            op = "D"
            i -= 1
        else:
            matches += 1 if c4(q[i]) & c4(t[j]) else 0
            op = "M"
            i -= 1
            j -= 1
        ops.append(op)
    ops += ["D"] * (i + 1) + ["I"] * (j + 1)
    ops.reverse()
    cigar = "".join((f"{len(g.group(0))}" if len(g.group(0)) > 1 else "") + g.group(0)[0]
                    for g in re.finditer(r"M+|D+|I+", "".join(ops)))
    return H[n][m], cigar, matches


def trim_id(cigar, matches):
    """align_trim + iddef 2 on a vsearch CIGAR string."""
    runs = [(int(n) if n else 1, o) for n, o in re.findall(r"(\d*)([MDI])", cigar)]
    cols = sum(r for r, _ in runs)
    left = runs[0][0] if runs[0][1] != "M" else 0
    right = runs[-1][0] if runs[-1][1] != "M" else 0
    if left >= cols:
        right = 0
    internal = cols - left - right
    return (100.0 * matches / internal if internal > 0 else 0.0), internal


def dust(seq):
    s = seq
    m = list(seq.upper())
    c2 = [("ACGT".index(ch.upper()) if ch.upper() in "ACGT" else (3 if ch.upper() == "U" else 0)) for ch in s]
    for i0 in range(0, len(s), 32):
        L = min(64, len(s) - i0)
        l1 = L - 3 + 1 - 5
        if l1 < 0:
            continue
        words = []
        w = 0
        for j in range(L):
            w = ((w << 2) | c2[i0 + j]) & 63
            words.append(w)
        bestv = besti = bestj = 0
        for i in range(l1):
            counts = [0] * 64
            tot = 0
            for j in range(2, L - i):
                x = words[i + j]
                if counts[x]:
                    tot += counts[x]
                    v = 10 * tot // j
                    if v > bestv:
                        bestv, besti, bestj = v, i, j
                counts[x] += 1
        if bestv > 20:
            for j in range(besti + i0, besti + bestj + i0 + 1):
                m[j] = s[j].lower()
    return "".join(m)


def kmers(seq, k=8, mask=True):
    out = set()
    for x in range(len(seq) - k + 1):
        w = seq[x:x + k]
        if mask and any(ch.islower() for ch in w):
            continue
        code = 0
        for ch in w:
            code = code * 4 + ({"C": 1, "G": 2, "T": 3, "U": 3}.get(ch.upper(), 0))
        out.add(code)
    return out


def cluster(p, seqs):
    """Returns (cluster number per input (-1 filtered), strand per input, consensus list)."""
    keep = [i for i, s in enumerate(seqs) if p.minlen <= len(s) <= p.maxlen]
    order = sorted(keep, key=lambda i: -len(seqs[i]))  # Python sort is stable: ties keep input order
    db = [dust(seqs[i]) if p.dust else seqs[i] for i in order]
    kdb = [kmers(s, p.k, p.dust) for s in db]
    cents, cno, strand, cig, ncl = [], {}, {}, {}, 0
    for s, qseq in enumerate(db):
        hits = []
        for st, qs in ((0, qseq), (1, revcomp(qseq))):
            qk = kmers(qs, p.k, p.dust)
            thr = min(p.minwm, len(qk))
            cands = [(-len(qk & kdb[c]), len(db[c]), c) for c in cents if len(qk & kdb[c]) >= thr]
            top = heapq.nsmallest(p.maxaccepts + p.maxrejects + 8, cands)
            acc = rej = fin = 0
            pos = 0
            while pos < len(top) and fin < p.maxaccepts + p.maxrejects - 1 and acc < p.maxaccepts and \
                    rej < p.maxrejects:
                batch = top[pos:pos + min(8, p.maxaccepts + p.maxrejects - 1 - fin)]
                pos += len(batch)
                for _cnt, _len, c in batch:
                    _sc, cg, mt = nw(p, qs, db[c])
                    idv, _ = trim_id(cg, mt)
                    ok = idv >= 100.0 * p.id
                    hits.append((idv, c, st, cg, ok))
                    acc += ok
                    rej += not ok
                    fin += 1
        best = None
        for h in hits:  # plus-strand hits first, so ties keep the plus strand
            if h[4] and (best is None or h[0] > best[0] or (h[0] == best[0] and h[1] < best[1])):
                best = h
        if best:
            cno[s], strand[s], cig[s] = cno[best[1]], best[2], best[3]
        else:
            cno[s], strand[s] = ncl, 0
            ncl += 1
            cents.append(s)
    sizes = [0] * ncl
    for s in range(len(db)):
        sizes[cno[s]] += 1
    rank = {c: r for r, c in enumerate(sorted(range(ncl), key=lambda c: (-sizes[c], c)))}
    members = [[] for _ in range(ncl)]
    for s in range(len(db)):
        members[rank[cno[s]]].append(s)
    cons = [msa(db, m, strand, cig) for m in members]
    out_c = [-1] * len(seqs)
    out_s = [0] * len(seqs)
    for s, i in enumerate(order):
        out_c[i] = rank[cno[s]]
        out_s[i] = strand[s]
    return out_c, out_s, cons


def msa(db, mem, strand, cig):
    cen = mem[0]
    L = len(db[cen])
    maxi = [0] * (L + 1)
    parsed = {}
    for s in mem[1:]:
        runs = [(int(n) if n else 1, o) for n, o in re.findall(r"(\d*)([MDI])", cig[s])]
        parsed[s] = runs
        pos = 0
        for r, o in runs:
            if o == "D":
                maxi[pos] = max(maxi[pos], r)
            else:
                pos += r
    cols = []
    for k, s in enumerate(mem):
        seq = db[s] if (k == 0 or not strand[s]) else revcomp(db[s])
        row, t = [], 0
        if k == 0:
            for pos in range(L):
                row += ["-"] * maxi[pos] + [seq[pos]]
            row += ["-"] * maxi[L]
        else:
            pos, inserted = 0, False
            for r, o in parsed[s]:
                if o == "D":
                    row += [seq[t + x] if x < r else "-" for x in range(maxi[pos])]
                    t += r
                    inserted = True
                else:
                    for _ in range(r):
                        if not inserted:
                            row += ["-"] * maxi[pos]
                        row.append(seq[t] if o == "M" else "-")
                        t += o == "M"
                        pos += 1
                        inserted = False
            if not inserted:
                row += ["-"] * maxi[pos]
        cols.append(row)
    alen = len(cols[0])
    out = []
    for x in range(maxi[0], alen - maxi[L]):
        cnt = {"A": 0, "C": 0, "G": 0, "T": 0, "N": 0, "-": 0}
        for row in cols:
            ch = row[x].upper()
            key = "T" if ch == "U" else (ch if ch in cnt else "N")
            cnt[key] += 1
        best, bc = "A", 0
        for b in "ACGT":
            if cnt[b] > bc:
                best, bc = b, cnt[b]
        if bc == 0 and cnt["N"] > 0:
            best, bc = "N", cnt["N"]
        if bc >= cnt["-"]:
            out.append(best)
    return "".join(out)
