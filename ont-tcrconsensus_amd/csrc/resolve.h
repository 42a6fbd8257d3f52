// resolve.h -- the host's in-order resolution of one greedy block (vsearch's sequential assignment,
// cluster.cc cluster_core_serial / cluster_core_parallel, behind vsearch_umi_cluster.py:21-54), host-only C++:
// no HIP, so the ThreadSanitizer harness (tools/resolve_tsan_main.cpp, tests/test_sanitizers_cpu.py) builds it
// with g++ and replays recorded passes through it.  driver.cpp's resolve_pass waits for a pass on the device and
// calls resolve_block with the pass's per-query-strand outcomes (HostQs) and records; round B (alignments the
// device did not compute) is a callback.
#pragma once
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <mutex>
#include <pthread.h>
#include <sched.h>
#include <thread>
#include <vector>

#include "umiclust_consts.h"

namespace uc {

// Outcome of one strand's walk.
struct Outcome {
  bool acc = false;
  uint16_t rank = 0;
  uint32_t t = 0xffffffffu;
  int walked = 0;
  int64_t cells = 0;
};

enum : uint8_t { ST_UNDET = 0, ST_CENT = 1, ST_MEMBER = 2 };

// greedy state of the sorted seqnos [s0, s0 + n) of the bin being clustered, indexed by absolute seqno
constexpr int kParChunk = 8;        // open queries a worker takes at a time
constexpr int kParInorderMin = 4096;  // open queries below which the in-order phase stays on the calling thread
struct StateView {
  uint8_t* p = nullptr;
  int32_t s0 = 0;
  uint8_t& operator[](int64_t i) const { return p[i - s0]; }
};

// A small persistent worker pool: run(f) calls f(t) for t in [0, size()) on the workers and the caller (t = 0).
class WorkPool {
 public:
  explicit WorkPool(int n) {
    for (int i = 1; i < n; i++) th_.emplace_back([this, i] { loop(i); });
  }
  ~WorkPool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  int size() const { return (int)th_.size() + 1; }
  void set_affinity(const cpu_set_t& set) {
    for (auto& t : th_) pthread_setaffinity_np(t.native_handle(), sizeof set, &set);
  }
  void run(const std::function<void(int)>& f) {
    if (th_.empty()) {
      f(0);
      return;
    }
    {
      std::lock_guard<std::mutex> g(m_);
      job_ = &f;
      pending_ = (int)th_.size();
      gen_++;
    }
    cv_.notify_all();
    f(0);
    std::unique_lock<std::mutex> g(m_);
    done_.wait(g, [this] { return pending_ == 0; });
    job_ = nullptr;
  }

 private:
  void loop(int i) {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(int)>* f;
      {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        f = job_;
      }
      (*f)(i);
      {
        std::lock_guard<std::mutex> g(m_);
        if (--pending_ == 0) done_.notify_one();
      }
    }
  }
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_, done_;
  const std::function<void(int)>* job_ = nullptr;
  uint64_t gen_ = 0;
  int pending_ = 0;
  bool stop_ = false;
};

// What the resolution reads of the context (stable over a bin) and writes besides the block's states.
struct ResolveEnv {
  const uint8_t* hlen = nullptr;     // sorted lengths, absolute seqno
  const uint8_t* acc = nullptr;      // [kTabL * kTabM] acceptance: 100.0*m/L >= 100.0*id (IEEE double, exact)
  const uint16_t* rank = nullptr;    // [kTabL * kTabM] rank of the id value
  int both = 2;
  int32_t o4_T = 0;                  // policy O4: rounds of o4_T queries; 0 = sequential
  int maxaccepts = 1, maxrejects = 32;
  const int32_t* hqbin = nullptr;    // packs: sorted seqno -> load bin (nullptr: the block's bin starts at s0)
  const int32_t* bin_s = nullptr;    // packs: each load bin's first sorted seqno
  bool pre_resolve = true;           // classify threads resolve strands whose peers are all final (kinds 3 / 4)
  bool pre_spec = true;              // ... and speculatively those whose in-block peers all turn out members (kind 5)
  bool par_inorder = true;           // the in-order phase on the pool, peer by peer (UMICLUST_PAR_INORDER=0: one thread)
  int par_min = kParInorderMin;      // ... from this many open queries on
  bool debug = false;
  int32_t* target = nullptr;         // absolute seqno -> centroid seqno a member joins (written)
  uint8_t* strand = nullptr;         // absolute seqno -> strand of that hit (written)
  int16_t* walk_dump = nullptr;      // UMICLUST_WALK_DUMP: [(q - s0) * 4 + {0, 1, 2, 3}] walked, path (or nullptr)
};

// per pass scratch of the classification (kept across passes: no reallocation per block)
struct ResolveScratch {
  std::vector<uint8_t> kind, ndeps, pre_cert, done;
  std::vector<uint16_t> deps;
  std::vector<Outcome> pre;
};

struct ResolveStats {
  int64_t n_alignments = 0, cells = 0, n_merged_walks = 0, n_deferred = 0, pairs_round_b = 0, cells_round_b = 0;
  double t_merged_s = 0, t_classify_s = 0, t_inorder_s = 0, t_round_b_s = 0;
  int64_t dbg[4] = {0, 0, 0, 0}, dbg_p[4] = {0, 0, 0, 0}, dbg_q[4] = {0, 0, 0, 0};
};

// Round B: align (query seqno << 1 | strand, target seqno) pairs, results as the device aligner writes them.
using RoundB = std::function<void(const std::vector<uint32_t>& pq, const std::vector<uint32_t>& pt,
                                  std::vector<uint32_t>& res)>;

enum : int { kResolveOk = 0, kResolveOverflow = 1, kResolveStuck = 2, kResolveBadPeer = 3 };

// Policy O4 (batched rounds of o4_T queries): the first query of q's round.  Rounds are counted from the first
// sorted query of q's own bin -- in a pack of bins (one greedy order over several bins, hqbin / bin_s given) from
// the bin's first seqno, so every bin's rounds are the ones its own vsearch run would have.  Sequential: q itself.
inline int32_t o4_round_start(int32_t o4_T, const int32_t* hqbin, const int32_t* bin_s, int32_t s0, int32_t q) {
  if (!o4_T) return q;
  const int32_t b0 = hqbin ? bin_s[hqbin[q]] : s0;
  return b0 + (q - b0) / o4_T * o4_T;
}

// Resolve block [q0, q0 + nq) (peer window [w0, q0 + nq)) in sorted order from the pass's outcomes hq[nq * both]
// and records (word array, HostQs::rec offsets).  Every query of the window before the block is resolved.
// new_cents: the block's new centroids, sorted.  Returns kResolveOverflow (a peer list overflowed: the caller
// re-runs the block in pieces), kResolveStuck (a deferred query still unresolved after round B: an internal error)
// or kResolveBadPeer (a record names an in-block peer that is not an earlier query -- the kernels' window bound
// lim = min(npeer, q - base) rules it out; checked because the parallel in-order phase would wait on it forever).
int resolve_block(const ResolveEnv& env, int32_t q0, int32_t nq, int32_t w0, const HostQs* hq, const uint32_t* recs,
                  const StateView& state, ResolveScratch& scr, WorkPool& pool, std::vector<int32_t>& new_cents,
                  ResolveStats& st, const RoundB& round_b);

}  // namespace uc
