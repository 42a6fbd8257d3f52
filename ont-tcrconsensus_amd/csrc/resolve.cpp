// resolve.cpp -- the host's in-order resolution of one greedy block (resolve.h), host-only C++ (no HIP).
//
// vsearch's greedy assignment is sequential (cluster.cc cluster_core_serial; cluster_core_parallel under policy O4,
// SURVEY App. A.6 and App. C); the reference runs it inside `vsearch --cluster_fast` (vsearch_umi_cluster.py:21-54).
// The device has walked every (query, strand) of the block against T_old (the index before the peer window) and
// aligned the relevant in-window peers speculatively; this decides, in sorted order, which queries become
// centroids and which centroid each member joins:
//
// A (query, strand) without a record (no relevant peer: k_pack) takes the device walk.  With one, its outcome
// depends on the peers' states: a relevant peer still undetermined blocks it; a relevant peer that is a centroid
// makes the host run the exact merged walk over T_old u (peers that are centroids) -- every such peer now matters,
// so an undetermined one blocks too.  A merged walk that needs an alignment the pass did not compute (a T_old entry
// past the device walk, or a peer that was not aligned) is deferred to round B, and so are queries blocked by
// deferred ones.  Classification runs on the worker pool (every strand whose outcome needs no in-order state is
// resolved there); the in-order phase and round B run on the calling thread.
#include "resolve.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <memory>
#include <thread>

namespace uc {

namespace {

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

inline unsigned long long cand_key(uint32_t count, uint32_t len, uint32_t seqno) {
  return ((unsigned long long)(127u - count) << 56) | ((unsigned long long)len << 48) | seqno;
}

// One candidate of a merged walk.
struct MCand {
  unsigned long long key;
  uint32_t seqno;
  uint32_t res;  // alignment result (matches | internal << 8), valid if have
  bool have;
};

// vsearch search_onequery over a merged, sorted candidate list (maxaccepts 1, maxrejects 32).
// Returns false if an alignment result is missing.
bool merged_walk(const ResolveEnv& env, std::vector<MCand>& L, int ql, Outcome& o) {
  const int n = std::min<int>((int)L.size(), kTopHits);
  int w = 0;
  o = Outcome();
  while (w < n && w < kWalk && !o.acc) {
    const int b1 = std::min(std::min(n, w + kBatch), kWalk);
    for (int x = w; x < b1; x++) {
      if (!L[x].have) return false;
      const uint32_t m = L[x].res & 0xffu, Li = (L[x].res >> 8) & 0xffu;
      o.cells += (int64_t)ql * env.hlen[L[x].seqno];
      if (env.acc[(size_t)Li * kTabM + m]) {
        const uint16_t rk = env.rank[(size_t)Li * kTabM + m];
        if (!o.acc || rk > o.rank || (rk == o.rank && L[x].seqno < o.t)) {
          o.rank = rk;
          o.t = L[x].seqno;
        }
        o.acc = true;
      }
    }
    w = b1;
  }
  o.walked = w;
  return true;
}

// search_findbest2_byid: max id, then lower target seqno, plus strand first.
inline bool better(const Outcome& a, const Outcome& b) {
  if (!a.acc) return false;
  if (!b.acc) return true;
  if (a.rank != b.rank) return a.rank > b.rank;
  return a.t < b.t;
}

inline int32_t round_start(const ResolveEnv& env, int32_t s0, int32_t q) {
  return o4_round_start(env.o4_T, env.hqbin, env.bin_s, s0, q);
}

}  // namespace

int resolve_block(const ResolveEnv& env, int32_t q0, int32_t nq, int32_t w0, const HostQs* hq, const uint32_t* recs,
                  const StateView& state, ResolveScratch& rsx, WorkPool& pool, std::vector<int32_t>& new_cents,
                  ResolveStats& rst, const RoundB& round_b) {
  const int both = env.both;
  const int32_t nqs = nq * both;
  for (int32_t qs = 0; qs < nqs; qs++)
    if (hq[qs].flags & 2u) return kResolveOverflow;
  new_cents.clear();
  constexpr int kSlots = kWalk + kPeerCap;  // round-B result slots per query-strand: T_old, peers
  std::vector<int32_t> deferred;
  std::vector<uint32_t> extra_res;   // [row*kSlots + slot] results of round B (valid if flag)
  std::vector<uint8_t> extra_have;
  std::vector<int32_t> extra_row;    // qs -> row of the round-B arrays (-1: none)
  struct Rec {
    int nt, np;
    const uint32_t *seq, *res, *cw, *peer, *pres;
    uint32_t count(int x) const { return (cw[x >> 2] >> ((x & 3) * 8)) & 0xffu; }
  };
  auto rec_of = [&](const HostQs& h) {
    const uint32_t* r = recs + h.rec;
    Rec R;
    R.nt = (int)(r[0] & 0xffu);
    R.np = (int)((r[0] >> 8) & 0xffu);
    R.seq = r + 1;
    R.res = R.seq + R.nt;
    R.cw = R.res + R.nt;
    R.peer = R.cw + ((R.nt + 3) >> 2);
    R.pres = R.peer + R.np;
    return R;
  };
  auto device_outcome = [](const HostQs& h, Outcome& o) {
    o.acc = (h.flags & 1u) != 0;
    o.rank = h.best_rank;
    o.t = h.best_t;
    o.walked = h.w;
    o.cells = h.cells;
  };
  // Membership can be certain while the walk's outcome is not: a device walk that accepted within its first w
  // candidates still accepts when at most nrel relevant peers are inserted before them (w + nrel <= kWalk).
  // Such a query is a member whichever centroid it ends up joining, so later queries that only need to
  // know "centroid or not" are not held up by it.
  auto cert_device = [](const HostQs& h) { return (h.flags & 1u) && (int)h.w + (int)h.nrel <= kWalk; };
  struct Scratch {
    std::vector<std::pair<unsigned long long, int>> cp, cx;
    std::vector<MCand> L;
    int64_t merged = 0;
    double t_merged = 0;  // merged-walk time off the sequential path (summed into rst.t_merged_s by phase 2)
  };
  // seq: the in-order phase (debug counters, merged-walk timer); otherwise a classify thread resolving a strand
  // whose peers' states are all final, with its own scratch
  auto strand_outcome_s = [&](int32_t qs, int32_t q, bool allow_extra, Outcome& o, bool& cert, Scratch& scr,
                              bool seq, uint32_t ib_lim = UINT32_MAX) -> int {
    // returns 0 resolved, 1 blocked by an undetermined peer, 2 needs alignments not computed; peers with a window id
    // >= ib_lim are taken as non-centroids (the classify phase's speculative resolution, kind 5)
    auto& cp = scr.cp;
    auto& L = scr.L;
    const HostQs& h = hq[qs];
    cert = false;
    if (h.rec == 0xffffffffu) {
      device_outcome(h, o);
      return 0;
    }
    if (seq && env.debug) rst.dbg_p[h.nrel <= (uint32_t)kInlineRel ? 0 : 1]++;
    if (h.nrel <= (uint32_t)kInlineRel) {
      bool cent = false;
      for (uint32_t i = 0; i < h.nrel; i++) {
        if (h.rel[i] >= ib_lim) continue;
        const uint8_t st = state[(uint32_t)w0 + h.rel[i]];
        if (st == ST_UNDET) {
          cert = cert_device(h);
          return 1;
        }
        cent |= st == ST_CENT;
      }
      if (!cent) {
        device_outcome(h, o);
        return 0;
      }
    }
    if (seq && env.debug) rst.dbg_p[2]++;
    const Rec R = rec_of(h);
    if (seq && env.debug) rst.dbg_p[3] += R.np;
    bool affects = false, undet = false;
    for (int y = 0; y < R.np; y++) {
      const uint32_t pw = R.peer[y];
      if ((pw & 0xffffu) >= ib_lim) continue;
      const uint8_t st = state[(uint32_t)w0 + (pw & 0xffffu)];
      if ((pw >> 24) & 1u) {
        if (st == ST_UNDET) {
          if (seq) rst.dbg[2]++;
          cert = cert_device(h);
          return 1;
        }
        affects |= st == ST_CENT;
        if (seq && !((pw >> 25) & 1u)) rst.dbg[st == ST_CENT ? 0 : 1]++;  // mispredicted / saved
      } else {
        undet |= st == ST_UNDET;
      }
    }
    if (!affects) {
      device_outcome(h, o);
      return 0;
    }
    if (undet) {
      cert = cert_device(h);
      return 1;
    }
    scr.merged++;
    struct TAcc { double* p; double t0; ~TAcc() { *p += now_s() - t0; } } tacc{seq ? &rst.t_merged_s : &scr.t_merged,
                                                                               now_s()};
    // exact merged walk: T_old (sorted by the prefilter) and the centroid peers (sorted here;
    // usually one or two) are merged linearly; only the first kWalk entries can ever be aligned
    const int32_t row = allow_extra ? extra_row[qs] : -1;
    // O4 batched rounds: centroids created before q's round join its search (the merged walk); those of its
    // own round are the extras of the re-check below.  Sequential: every centroid peer joins the walk.
    const uint32_t rb = env.o4_T ? (uint32_t)round_start(env, state.s0, q) : UINT32_MAX;
    auto& cx = scr.cx;
    cp.clear();
    cx.clear();
    for (int y = 0; y < R.np; y++) {
      const uint32_t pw = R.peer[y];
      if ((pw & 0xffffu) >= ib_lim) continue;
      const uint32_t ps = (uint32_t)w0 + (pw & 0xffffu);
      if (state[ps] == ST_CENT) (ps < rb ? cp : cx).push_back({cand_key((pw >> 16) & 0xffu, env.hlen[ps], ps), y});
    }
    std::sort(cp.begin(), cp.end());
    L.clear();
    int i = 0;
    size_t x = 0;
    while ((int)L.size() < kWalk && (i < R.nt || x < cp.size())) {
      const unsigned long long kt = (i < R.nt) ? cand_key(R.count(i), env.hlen[R.seq[i]], R.seq[i]) : ~0ull;
      const unsigned long long kp = (x < cp.size()) ? cp[x].first : ~0ull;
      MCand m;
      if (kt < kp) {
        m.key = kt;
        m.seqno = R.seq[i];
        if (i < h.e) {
          m.res = R.res[i];
          m.have = true;
        } else if (row >= 0 && extra_have[(size_t)row * kSlots + i]) {
          m.res = extra_res[(size_t)row * kSlots + i];
          m.have = true;
        } else {
          m.res = 0;
          m.have = false;
        }
        i++;
      } else {
        const int y = cp[x].second;
        m.key = kp;
        m.seqno = (uint32_t)w0 + (R.peer[y] & 0xffffu);
        if ((R.peer[y] >> 25) & 1u) {  // aligned by the pass
          m.res = R.pres[y];
          m.have = true;
        } else if (row >= 0 && extra_have[(size_t)row * kSlots + kWalk + y]) {
          m.res = extra_res[(size_t)row * kSlots + kWalk + y];
          m.have = true;
        } else {
          m.res = 0;
          m.have = false;
        }
        x++;
      }
      L.push_back(m);
    }
    if (merged_walk(env, L, env.hlen[q], o)) {
      if (cx.empty()) return 0;
      // cluster_core_parallel's re-check (policy O4): the round's new centroids over the k-mer threshold are
      // inserted into the hit list (the walked candidates, all aligned) by (count desc, shorter first, then
      // seqno), and the list is walked again one alignment at a time from the top until an accept or
      // maxrejects rejects; the best hit is then the best accepted one of every aligned hit
      std::sort(cx.begin(), cx.end());
      int acc = 0, rej = 0;
      size_t a = 0, b = 0;
      const size_t w = (size_t)o.walked;
      while (acc < env.maxaccepts && rej < env.maxrejects && (a < w || b < cx.size())) {
        uint32_t res, t;
        if (a < w && (b >= cx.size() || L[a].key < cx[b].first)) {
          res = L[a].res;
          t = L[a].seqno;
          a++;
        } else {
          const int y = cx[b].second;
          t = (uint32_t)w0 + (R.peer[y] & 0xffffu);
          if ((R.peer[y] >> 25) & 1u) {
            res = R.pres[y];
          } else if (row >= 0 && extra_have[(size_t)row * kSlots + kWalk + y]) {
            res = extra_res[(size_t)row * kSlots + kWalk + y];
          } else {
            cert = o.acc;  // an accepted hit of the search stays a candidate whatever the re-check finds
            return 2;
          }
          b++;
          o.walked++;
          o.cells += (int64_t)env.hlen[q] * env.hlen[t];
        }
        const uint32_t m = res & 0xffu, Li = (res >> 8) & 0xffu;
        if (env.acc[(size_t)Li * kTabM + m]) {
          acc++;
          const uint16_t rk = env.rank[(size_t)Li * kTabM + m];
          if (!o.acc || rk > o.rank || (rk == o.rank && t < o.t)) {
            o.rank = rk;
            o.t = t;
          }
          o.acc = true;
        } else {
          rej++;
        }
      }
      return 0;
    }
    // an accept already known within the first kWalk candidates ends the walk by its batch at the latest
    for (int x = 0; x < std::min<int>((int)L.size(), kWalk) && !cert; x++)
      if (L[x].have) {
        const uint32_t m = L[x].res & 0xffu, Li = (L[x].res >> 8) & 0xffu;
        cert = env.acc[(size_t)Li * kTabM + m] != 0;
      }
    return 2;
  };
  Scratch scr0;
  auto strand_outcome = [&](int32_t qs, int32_t q, bool allow_extra, Outcome& o, bool& cert) -> int {
    return strand_outcome_s(qs, q, allow_extra, o, cert, scr0, true);
  };
  struct Acc {
    int64_t aln = 0, cells = 0;
  };
  // par: a phase-2 worker (its own accumulators; new centroids are collected afterwards, in order)
  auto resolve = [&](int32_t ql, bool allow_extra, auto&& strand_fn, Acc* par = nullptr) -> bool {
    const int32_t q = q0 + ql;
    Outcome best, os[2];
    int bs = 0;
    bool open = false, member = false;
    for (int s = 0; s < both; s++) {
      bool cert = false;
      if (strand_fn(ql * both + s, q, allow_extra, os[s], cert) != 0) {
        open = true;
        member |= cert;
      } else {
        member |= os[s].acc;
      }
    }
    if (open) {
      // deferred; a certain member is marked so already (its centroid is settled in round B)
      if (member) state[q] = ST_MEMBER;
      return false;
    }
    for (int s = 0; s < both; s++) {
      (par ? par->aln : rst.n_alignments) += os[s].walked;
      (par ? par->cells : rst.cells) += os[s].cells;
      if (env.walk_dump) {
        env.walk_dump[(size_t)(q - state.s0) * 4 + s] = (int16_t)os[s].walked;
        env.walk_dump[(size_t)(q - state.s0) * 4 + 2 + s] = allow_extra ? 3 : 2;
      }
      if (better(os[s], best)) {
        best = os[s];
        bs = s;
      }
    }
    if (best.acc) {
      state[q] = ST_MEMBER;
      env.target[q] = (int32_t)best.t;
      env.strand[q] = (uint8_t)bs;
    } else {
      state[q] = ST_CENT;
      if (!par) new_cents.push_back(q);
    }
    return true;
  };
  if (env.debug) {
    const uint32_t inb = (uint32_t)(q0 - w0);
    for (int32_t ql = 0; ql < nq; ql++) {
      int cls = 0;
      for (int s = 0; s < both; s++) {
        const HostQs& h = hq[ql * both + s];
        if (h.rec == 0xffffffffu) continue;
        cls = std::max(cls, 1);
        const Rec R = rec_of(h);
        for (int y = 0; y < R.np; y++)
          if (((R.peer[y] >> 24) & 1u) && (R.peer[y] & 0xffffu) >= inb) cls = 2;
      }
      rst.dbg_q[cls]++;
    }
  }
  const double tp0 = now_s();
  // Phase 1 (host threads): classify every query-strand.  Peers in earlier blocks are final, so a strand
  // whose relevant peers there include a centroid needs the full (sequential) resolution, and one whose
  // relevant peers are all earlier-block members and in-block peers keeps its device outcome unless one of
  // those in-block peers becomes a centroid or is deferred -- checked in order in phase 2.
  constexpr int kDeps = 8;
  const uint32_t inb = (uint32_t)(q0 - w0);
  rsx.kind.resize((size_t)nqs);
  rsx.ndeps.resize((size_t)nqs);
  rsx.deps.resize((size_t)nqs * kDeps);
  rsx.pre.resize((size_t)nqs);
  rsx.pre_cert.resize((size_t)nqs);
  // kind 0: the device outcome is final; 1: final unless an in-block dependency becomes a centroid or is
  // deferred; 2: full resolution in order; 3 / 4: every peer lies in an earlier (resolved) block, so the
  // full resolution needs no in-order state and ran here: resolved (3) or needing round B (4)
  auto classify = [&](int32_t qs, Scratch& scr) {
    const HostQs& h = hq[qs];
    uint8_t& kd = rsx.kind[qs];
    if (h.rec == 0xffffffffu) {
      kd = 0;
      return;
    }
    if (env.o4_T) {  // O4 batched rounds: every strand with a record resolves in order (strand_outcome_s)
      kd = 2;
      return;
    }
    int nd = 0;
    uint16_t* d = rsx.deps.data() + (size_t)qs * kDeps;
    auto rel_peer = [&](uint32_t id) -> bool {  // false: needs the full resolution
      if (id >= inb) {
        if (nd == kDeps) return false;
        d[nd++] = (uint16_t)id;
        return true;
      }
      return state[(uint32_t)w0 + id] != ST_CENT;
    };
    bool ok = true;
    if (h.nrel <= (uint32_t)kInlineRel) {
      for (uint32_t i = 0; i < h.nrel && ok; i++) ok = rel_peer(h.rel[i]);
    } else {
      const Rec R = rec_of(h);
      for (int y = 0; y < R.np && ok; y++)
        if ((R.peer[y] >> 24) & 1u) ok = rel_peer(R.peer[y] & 0xffffu);
    }
    kd = !ok ? 2 : nd ? 1 : 0;
    rsx.ndeps[qs] = (uint8_t)nd;
    if (kd == 2 && env.pre_resolve) {
      const Rec R = rec_of(h);
      int nib = 0;  // in-block peers (any relevance)
      for (int y = 0; y < R.np; y++) nib += (R.peer[y] & 0xffffu) >= inb;
      if (nib == 0) {
        bool cert = false;
        const int r = strand_outcome_s(qs, q0 + qs / both, false, rsx.pre[qs], cert, scr, false);
        if (r != 1) {
          kd = r == 0 ? 3 : 4;
          rsx.pre_cert[qs] = cert;
        }
      } else if (nib <= kDeps && env.pre_spec) {
        // kind 5: resolved here as if no in-block peer were a centroid (earlier-block peers are final); phase 2
        // keeps this outcome if every in-block peer -- relevant or not: once a centroid peer joins the walk, any
        // peer can -- turns out a member, and otherwise runs the full resolution
        bool cert = false;
        const int r = strand_outcome_s(qs, q0 + qs / both, false, rsx.pre[qs], cert, scr, false, inb);
        if (r == 0) {
          kd = 5;
          nd = 0;
          for (int y = 0; y < R.np; y++)
            if ((R.peer[y] & 0xffffu) >= inb) d[nd++] = (uint16_t)(R.peer[y] & 0xffffu);
          rsx.ndeps[qs] = (uint8_t)nd;
        }
      }
    }
  };
  // A query whose strands are all final here (kinds 0 and 3: no in-block dependency) is resolved here too: its
  // outcome needs no in-order state, and only in-block queries ever read its state, in phase 2, after this
  // phase.  rsx.done: 0 pending (phase 2), 1 member, 2 centroid.
  rsx.done.resize((size_t)nq);
  auto classify_query = [&](int32_t ql, Scratch& scr, Acc& acc) {
    bool det = true;
    for (int s = 0; s < both; s++) {
      const int32_t qs = ql * both + s;
      classify(qs, scr);
      det &= rsx.kind[qs] == 0 || rsx.kind[qs] == 3;
    }
    if (!det) {
      rsx.done[ql] = 0;
      return;
    }
    Outcome best, os[2];
    int bs = 0;
    for (int s = 0; s < both; s++) {
      const int32_t qs = ql * both + s;
      if (rsx.kind[qs] == 0) device_outcome(hq[qs], os[s]);
      else os[s] = rsx.pre[qs];
      acc.aln += os[s].walked;
      acc.cells += os[s].cells;
      if (env.walk_dump) {
        env.walk_dump[(size_t)(q0 + ql - state.s0) * 4 + s] = (int16_t)os[s].walked;
        env.walk_dump[(size_t)(q0 + ql - state.s0) * 4 + 2 + s] = rsx.kind[qs] == 0 ? 0 : 1;
      }
      if (better(os[s], best)) {
        best = os[s];
        bs = s;
      }
    }
    const int32_t q = q0 + ql;
    if (best.acc) {
      state[q] = ST_MEMBER;
      env.target[q] = (int32_t)best.t;
      env.strand[q] = (uint8_t)bs;
      rsx.done[ql] = 1;
    } else {
      state[q] = ST_CENT;
      rsx.done[ql] = 2;
    }
  };
  const int T = nqs < 2048 ? 1 : pool.size();
  std::vector<Scratch> scr_t((size_t)T);
  std::vector<Acc> acc_t((size_t)T);
  if (T == 1) {
    for (int32_t ql = 0; ql < nq; ql++) classify_query(ql, scr_t[0], acc_t[0]);
  } else {
    pool.run([&](int t) {
      const int32_t lo = (int32_t)((int64_t)nq * t / T), hi = (int32_t)((int64_t)nq * (t + 1) / T);
      for (int32_t ql = lo; ql < hi; ql++) classify_query(ql, scr_t[(size_t)t], acc_t[(size_t)t]);
    });
  }
  for (const Scratch& x : scr_t) rst.n_merged_walks += x.merged;
  for (const Acc& x : acc_t) {
    rst.n_alignments += x.aln;
    rst.cells += x.cells;
  }
  const double tp1 = now_s();
  rst.t_classify_s += tp1 - tp0;
  // Phase 2 (sequential, sorted order): confirm the device outcomes against the in-block peers' states
  auto strand_fast_s = [&](int32_t qs, int32_t q, Outcome& o, bool& cert, Scratch& scr, bool seq) -> int {
    const HostQs& h = hq[qs];
    cert = false;
    if (rsx.kind[qs] == 0) {
      device_outcome(h, o);
      return 0;
    }
    if (rsx.kind[qs] == 3) {
      o = rsx.pre[qs];
      return 0;
    }
    if (rsx.kind[qs] == 4) {
      cert = rsx.pre_cert[qs] != 0;
      return 2;
    }
    if (rsx.kind[qs] == 5) {
      const uint16_t* d = rsx.deps.data() + (size_t)qs * kDeps;
      bool member_peers = true;
      for (int i = 0; i < rsx.ndeps[qs] && member_peers; i++) member_peers = state[(uint32_t)w0 + d[i]] == ST_MEMBER;
      if (member_peers) {
        o = rsx.pre[qs];
        return 0;
      }
      return strand_outcome_s(qs, q, false, o, cert, scr, seq);
    }
    if (rsx.kind[qs] == 1) {
      const uint16_t* d = rsx.deps.data() + (size_t)qs * kDeps;
      bool cent = false;
      for (int i = 0; i < rsx.ndeps[qs]; i++) {
        const uint8_t st = state[(uint32_t)w0 + d[i]];
        if (st == ST_UNDET) {
          cert = cert_device(h);
          return 1;
        }
        cent |= st == ST_CENT;
      }
      if (!cent) {
        device_outcome(h, o);
        return 0;
      }
    }
    return strand_outcome_s(qs, q, false, o, cert, scr, seq);
  };
  auto strand_fast = [&](int32_t qs, int32_t q, bool, Outcome& o, bool& cert) -> int {
    return strand_fast_s(qs, q, o, cert, scr0, true);
  };
  std::vector<int32_t> pend;  // queries phase 1 left open, in sorted order
  for (int32_t ql = 0; ql < nq; ql++)
    if (rsx.done[ql] == 0) pend.push_back(ql);
  const int TP = pool.size();
  if (env.par_inorder && TP > 1 && (int)pend.size() >= env.par_min && !env.debug) {
    // Phase 2 on the pool, with the sequential result: a query reads the states of its in-window peers only (every
    // peer is an earlier query), so it may run once each of its in-block peers has been processed -- resolved or
    // deferred -- as it would have been in sorted order.  Workers take the open queries in sorted order, so the
    // earliest one in progress always has its peers done (no deadlock).  Under O4 as well: the re-check's extras
    // (the round's earlier centroids) are peers of the same record, waited on like the others.
    const int32_t np = (int32_t)pend.size();
    std::unique_ptr<std::atomic<uint8_t>[]> proc(new std::atomic<uint8_t>[(size_t)nq]);
    for (int32_t ql = 0; ql < nq; ql++) proc[ql].store(rsx.done[ql] != 0 ? 1 : 0, std::memory_order_relaxed);
    std::vector<uint8_t> ok((size_t)np);
    std::atomic<int32_t> next{0};
    std::atomic<bool> bad_peer{false};
    std::vector<Scratch> scr_p((size_t)TP);
    std::vector<Acc> acc_p((size_t)TP);
    pool.run([&](int t) {
      Scratch& scr = scr_p[(size_t)t];
      Acc& acc = acc_p[(size_t)t];
      auto fast = [&](int32_t qs, int32_t q, bool, Outcome& o, bool& cert) -> int {
        return strand_fast_s(qs, q, o, cert, scr, false);
      };
      // chunks of consecutive open queries (each worker writes runs of neighbouring flags and states); the earliest
      // unprocessed query is always the one its chunk's worker is on
      for (;;) {
       const int32_t i0 = next.fetch_add(kParChunk, std::memory_order_relaxed);
       if (i0 >= np) break;
       for (int32_t i = i0; i < std::min(np, i0 + kParChunk); i++) {
        const int32_t ql = pend[(size_t)i];
        for (int s = 0; s < both; s++) {
          const HostQs& h = hq[ql * both + s];
          if (h.rec == 0xffffffffu) continue;
          const Rec R = rec_of(h);
          for (int y = 0; y < R.np; y++) {
            const uint32_t id = R.peer[y] & 0xffffu;
            if (id < inb) continue;
            if (id - inb >= (uint32_t)ql) {  // not an earlier query: waiting on it would never end
              bad_peer.store(true, std::memory_order_relaxed);
              continue;
            }
            for (int spin = 0; !proc[id - inb].load(std::memory_order_acquire); spin++)
              if (spin > 64) std::this_thread::yield();
          }
        }
        ok[(size_t)i] = resolve(ql, false, fast, &acc) ? 1 : 0;
        proc[ql].store(1, std::memory_order_release);
       }
      }
    });
    if (bad_peer.load()) return kResolveBadPeer;
    for (const Acc& x : acc_p) {
      rst.n_alignments += x.aln;
      rst.cells += x.cells;
    }
    for (const Scratch& x : scr_p) {
      rst.n_merged_walks += x.merged;
      rst.t_merged_s += x.t_merged;
    }
    for (int32_t ql = 0; ql < nq; ql++)
      if (rsx.done[ql] == 2) new_cents.push_back(q0 + ql);
    for (int32_t i = 0; i < np; i++) {
      const int32_t ql = pend[(size_t)i];
      if (!ok[(size_t)i]) deferred.push_back(ql);
      else if (state[q0 + ql] == ST_CENT) new_cents.push_back(q0 + ql);
    }
    std::sort(new_cents.begin(), new_cents.end());
  } else {
    for (int32_t ql = 0; ql < nq; ql++) {
      const uint8_t d = rsx.done[ql];
      if (d == 2) new_cents.push_back(q0 + ql);
      else if (d == 0 && !resolve(ql, false, strand_fast)) deferred.push_back(ql);
    }
  }
  rst.t_inorder_s += now_s() - tp1;
  rst.n_deferred += (int64_t)deferred.size();
  // --- round B (side stream, so the queued pass keeps the device busy): align every T_old entry and
  // every peer a deferred query could still need, then resolve the deferred queries in order
  if (!deferred.empty()) {
    std::vector<uint32_t> bpq, bpt, bidx;
    for (int32_t ql : deferred)
      for (int s = 0; s < both; s++) {
        const int32_t qs = ql * both + s;
        const HostQs& h = hq[qs];
        if (h.rec == 0xffffffffu) continue;
        const Rec R = rec_of(h);
        const uint32_t qv = ((uint32_t)(q0 + ql) << 1) | (uint32_t)s;
        for (int x = h.e; x < R.nt; x++) {
          bpq.push_back(qv);
          bpt.push_back(R.seq[x]);
          bidx.push_back((uint32_t)(qs * kSlots + x));
        }
        for (int y = 0; y < R.np; y++)
          // a peer that is a member never enters the merged walk (only centroids are candidates)
          if (!((R.peer[y] >> 25) & 1u) && state[(uint32_t)w0 + (R.peer[y] & 0xffffu)] != ST_MEMBER) {
            bpq.push_back(qv);
            bpt.push_back((uint32_t)w0 + (R.peer[y] & 0xffffu));
            bidx.push_back((uint32_t)(qs * kSlots + kWalk + y));
          }
      }
    const int32_t nb = (int32_t)bpq.size();
    rst.pairs_round_b += nb;
    for (int32_t x = 0; x < nb; x++) rst.cells_round_b += (int64_t)env.hlen[bpq[x] >> 1] * env.hlen[bpt[x]];
    std::vector<uint32_t> bres(nb);
    if (nb > 0) {
      const double tb0 = now_s();
      round_b(bpq, bpt, bres);
      rst.t_round_b_s += now_s() - tb0;
    }
    extra_row.assign((size_t)nqs, -1);
    for (size_t r = 0; r < deferred.size(); r++)
      for (int s = 0; s < both; s++) extra_row[(size_t)deferred[r] * both + s] = (int32_t)(r * both + s);
    extra_res.assign(deferred.size() * both * kSlots, 0);
    extra_have.assign(deferred.size() * both * kSlots, 0);
    for (int32_t x = 0; x < nb; x++) {
      const int32_t qs = (int32_t)(bidx[x] / kSlots), e = (int32_t)(bidx[x] % kSlots);
      extra_res[(size_t)extra_row[qs] * kSlots + e] = bres[x];
      extra_have[(size_t)extra_row[qs] * kSlots + e] = 1;
    }
    for (int32_t ql : deferred)
      if (!resolve(ql, true, strand_outcome)) return kResolveStuck;
    std::sort(new_cents.begin(), new_cents.end());
  }
  rst.n_merged_walks += scr0.merged;
  return kResolveOk;
}


}  // namespace uc
