// driver.cpp -- host side of the MI355X UMI clustering hot path and the C ABI (include/umiclust.h).
//
// Replaces the `vsearch --cluster_fast` subprocess of
// /root/reference/ont_tcr_consensus/vsearch_umi_cluster.py:21-54 (round 1) and :71-97 (round 2).
// vsearch's greedy is sequential: query k (length-sorted) is compared with the centroids created
// by queries 0..k-1.  This driver keeps that definition exactly while batching on the GPU:
//
//   for each block of B consecutive sorted queries of one length:
//     K2  prefilter every (query, strand) against C_old (the index: centroids of the blocks before
//         the peer window) -> exact top-41 list T_old, and against the earlier queries of the peer
//         window (previous block + this block) -> peer list P (count >= threshold)
//     K3W walk T_old on the device in batches of 8 (vsearch's pop loop), aligning with K3, and
//         align every (query, peer) pair speculatively
//     host pass 1: in sorted order, a query whose centroid peers cannot change its walk takes the
//         device outcome; otherwise it runs the exact merged walk over T_old u centroid peers,
//         deferred only if that walk needs a T_old entry the device did not align
//     round B (side stream): align what deferred queries need; host pass 2 resolves them
//     new centroids are appended to the LSM index (sealed / base / delta tiles)
//
// The passes form a software pipeline: pass k+1 is queued before the host resolves block k, so
// the host work hides behind device work.  Pass k+1's index lacks block k, which is why its peer
// window includes block k.  top-41 of (C_old u N) = top-41 of (top-41(C_old) u N), and a walk
// touches at most 32 entries, so every alignment a query can need exists: the result is
// identical to the sequential definition (vsearch --threads 1).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fcntl.h>
#include <string>
#include <sys/mman.h>
#include <sys/stat.h>
#include <condition_variable>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <pthread.h>
#include <sched.h>
#include <thread>
#include <unistd.h>
#include <unordered_map>
#include <vector>
#include <zlib.h>

#include "../../include/umiclust.h"
#include "host_io.h"
#include "resolve.h"
#include "umiclust_internal.h"

using namespace uc;
using uc::io::Fasta;
using uc::io::io_threads;
using uc::io::parallel_for;
using uc::io::pjoin;
using uc::io::Sv;
using uc::io::split1;

namespace {

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

template <typename T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
  hipError_t ensure(size_t count) {
    if (count <= n && p) return hipSuccess;
    release();
    size_t c = count ? count : 1;
    hipError_t e = hipMalloc(reinterpret_cast<void**>(&p), c * sizeof(T));
    if (e == hipSuccess) n = c;
    return e;
  }
};

template <typename T>
struct PinBuf {
  T* p = nullptr;
  size_t n = 0;
  PinBuf() = default;
  PinBuf(const PinBuf&) = delete;
  PinBuf& operator=(const PinBuf&) = delete;
  ~PinBuf() { release(); }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    n = 0;
  }
  // Kernels write these buffers directly (pinned host memory is device-accessible); the host reads
  // them only after the writing kernel's completion event, and copies what it scans into pageable
  // vectors first.
  hipError_t ensure(size_t count) {
    if (count <= n && p) return hipSuccess;
    release();
    size_t c = count ? count : 1;
    const unsigned flags = hipHostMallocDefault;
    hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&p), c * sizeof(T), flags);
    if (e == hipSuccess) n = c;
    return e;
  }
};

constexpr int32_t kDelta = 8192;  // centroids in the per-block delta tile before folding into base

struct Tile {
  DevBuf<uint32_t> hist;      // [kBins], all zero between builds (the scan re-zeroes it)
  DevBuf<uint32_t> off;       // [kBins + 1] padded list offsets, tile-relative
  DevBuf<uint32_t> cursor;    // [kBins]
  DevBuf<uint32_t> partial;   // [kScanBlocks]
  uint64_t post_base = 0;     // the tile's slot in the postings arena
  size_t post_cap = 0;        // slot capacity (postings)
  int32_t n = 0;              // sequences
  int32_t base = 0;           // first centroid ordinal / first seqno (peer tiles)
  int32_t seg = 0;            // counter segment / peer region
  int32_t len = 0;            // peer tiles: the block's query length
  int32_t built_n = -1;       // n at last build
  bool prebuilt = false;      // peer tile built ahead of its pass (for the block [base, base + n))
};

// postings a tile slot of nseq sequences can need: every k-mer plus up to 7 padding postings per
// non-empty list
inline size_t tile_cap(int64_t nseq) {
  const int64_t raw = nseq * kMaxKmers;
  return (size_t)((raw + 7 * std::min<int64_t>(kBins, raw) + 64) & ~int64_t(7));
}

struct Fail {
  int code;
};

// One greedy block in flight: its own peer tile, device outputs and pinned mirrors, so the device
// runs block k+1 while the host resolves block k.
struct Pass {
  int32_t q0 = 0, nq = 0, w0 = 0;  // block [q0, q0+nq), peer window [w0, q0+nq)
  bool live = false;
  bool rec_direct = false;  // this pass's outcomes and records written by k_pack into pinned host memory
  PinBuf<TileView> h_tiles;
  DevBuf<TileView> d_tiles;
  DevBuf<uint32_t> d_top_seqno;
  DevBuf<uint8_t> d_top_count, d_ntop;
  DevBuf<uint32_t> d_pcand, d_units;  // per-(query-strand, part) prefilter candidates, overflowed units
  DevBuf<uint8_t> d_pncand, d_ppeer_count, d_pnpeer;
  DevBuf<uint32_t> d_ppost;  // postings touched per (query-strand, part), summed by k_pf_merge
  DevBuf<uint16_t> d_ppeer_id;
  DevBuf<uint16_t> d_peer_id;
  DevBuf<uint8_t> d_peer_count, d_npeer;
  bool ctr_zeroed = false;      // d_counters re-zeroed by the last k_pack on this buffer set
  DevBuf<uint32_t> d_counters;  // [0] postings, [1..5] npairs per walk round, [8] peer pairs,
                                // [9] target residues of walk pairs, [10] of peer pairs
  DevBuf<uint32_t> d_pq, d_pt, d_outidx, d_res;
  DevBuf<WalkState> d_ws;
  DevBuf<HostQs> d_hq;              // k_pack's per query-strand outcomes, copied to h_hq by DMA
  DevBuf<unsigned long long> d_paligned;  // per query-strand: the peers k_peer_pairs aligned
  DevBuf<uint32_t> d_reccount;
  DevBuf<uint32_t> d_rec;           // k_pack's records, copied to h_rec by DMA (a prefix of rec_est words;
                                    // the host fetches the rest in the rare pass that used more)
  uint32_t rec_est = 1u << 16;
  // host side: per query-strand outcomes and records (DMA), counters (written by k_pack), record words used
  PinBuf<HostQs> h_hq;
  PinBuf<uint32_t> h_rec, h_counters, h_reccount;
  std::vector<HostQs> hq_copy;
  std::vector<uint32_t> rec_copy;
  ResolveScratch rsx;  // resolve_block's classification scratch (resolve.h)
  hipEvent_t ev[5] = {};  // prefilter begin/end, align begin/end, results in host memory
  // split passes: the counting half (enqueue_count) of the block this buffer set serves next
  PinBuf<TileView> h_tiles_a;
  DevBuf<TileView> d_tiles_a;
  DevBuf<uint32_t> d_anunits;  // overflowed units of the lean kernel (the merge resets it)
  hipEvent_t ev_a = nullptr;   // after the counting half's view upload (h_tiles_a may be rewritten)
  hipEvent_t ev_c[2] = {};     // whole passes: the counting kernel alone
  bool c_timed = false;
  bool a_live = false, a_timed = false;
  int32_t a_q0 = -1, a_base = 0, a_slot = 0, t_slot = 0;
  ~Pass() {
    for (hipEvent_t e : ev)
      if (e) (void)hipEventDestroy(e);
    if (ev_a) (void)hipEventDestroy(ev_a);
    for (hipEvent_t e : ev_c)
      if (e) (void)hipEventDestroy(e);
  }
};

}  // namespace

static std::atomic<int> g_live_ctx{0};  // contexts alive in this process (L3Pin)
struct umiclust_ctx;

// Process-wide timeline of the counting launches (kind 0) and the alignment chains (kind 1), for
// umiclust_timeline: with several contexts (lanes) on one device their HIP-event brackets overlap, so the sum of
// the brackets overstates the time the kernel held the device; the union of the intervals, each taken against
// one reference event, does not.
struct Timeline {
  std::mutex m;
  hipEvent_t ref = nullptr;
  int dev = -1;
  std::vector<std::pair<float, float>> iv[2];
  // intervals ending below fold_hi[kind] are folded into folded_ms[kind] (their union's measure) once iv[kind] grows
  // past kTlCap, so that a long run does not grow the vectors without bound; later intervals are clipped at fold_hi
  double folded_ms[2] = {0.0, 0.0};
  float fold_hi[2] = {-1e30f, -1e30f};
  int64_t n[2] = {0, 0};
};
static Timeline g_tl;
constexpr size_t kTlCap = 1 << 16, kTlKeep = 4096;  // keep the latest kTlKeep merged intervals unfolded (late arrivals)

// union of sorted intervals: merges v in place, returns the measure
static double tl_merge(std::vector<std::pair<float, float>>& v) {
  std::sort(v.begin(), v.end());
  size_t w = 0;
  double tot = 0.0;
  for (size_t i = 0; i < v.size(); i++) {
    if (w > 0 && v[i].first <= v[w - 1].second) {
      v[w - 1].second = std::max(v[w - 1].second, v[i].second);
    } else {
      v[w++] = v[i];
    }
  }
  v.resize(w);
  for (const auto& x : v) tot += x.second - x.first;
  return tot;
}

static void tl_add(int dev, int kind, hipEvent_t a, hipEvent_t b) {
  std::lock_guard<std::mutex> lk(g_tl.m);
  if (!g_tl.ref || dev != g_tl.dev) return;  // events of another device than the reference's: not comparable
  float t0 = 0.f, t1 = 0.f;
  if (hipEventElapsedTime(&t0, g_tl.ref, a) != hipSuccess || hipEventElapsedTime(&t1, g_tl.ref, b) != hipSuccess) {
    (void)hipGetLastError();  // measurement only: never leave a sticky error for the caller's next launch check
    return;
  }
  g_tl.n[kind]++;
  t0 = std::max(t0, g_tl.fold_hi[kind]);
  if (t1 <= t0) return;
  auto& v = g_tl.iv[kind];
  v.emplace_back(t0, t1);
  if (v.size() > kTlCap) {
    tl_merge(v);
    if (v.size() > kTlKeep) {
      const size_t f = v.size() - kTlKeep;
      for (size_t i = 0; i < f; i++) g_tl.folded_ms[kind] += v[i].second - v[i].first;
      g_tl.fold_hi[kind] = v[f - 1].second;
      v.erase(v.begin(), v.begin() + (ptrdiff_t)f);
    }
  }
}

struct umiclust_ctx {
  int dev = 0;
  hipStream_t st = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  std::string err;

  umiclust_params p{};
  Scoring sc{};
  int both = 2;
  bool ambig = false;             // some kept sequence holds a non-ACGT (IUPAC) symbol
  bool loaded = false;
  bool clustered = false;
  DevBuf<unsigned long long> pf_prof;  // prefilter phase clocks (UMICLUST_PFPROF)
  // UMI extraction (f1): gathered adapter windows, kept across calls
  PinBuf<char> ex_win;
  PinBuf<uint8_t> ex_len;
  DevBuf<char> ex_dwin;
  DevBuf<uint8_t> ex_dlen;
  DevBuf<int32_t> ex_dout;
  DevBuf<ExtractPatterns> ex_dpat;

  // input (host copies kept only for the file path outputs).  A load holds one or more independent
  // region bins (umiclust_load_bins): bin b is input records [bin_in[b], bin_in[b+1]) and sorted
  // seqnos [bin_s[b], bin_s[b+1]) -- every bin is length-sorted on its own and clustered on its own,
  // with absolute seqnos on the device.
  int64_t n_input = 0;
  int32_t n = 0;                  // kept sequences (all bins)
  std::vector<int32_t> perm;      // sorted -> input index
  std::vector<uint8_t> hlen;      // sorted lengths
  std::vector<int64_t> bin_in;    // [nbins + 1] input record boundaries
  std::vector<int32_t> bin_s;     // [nbins + 1] sorted seqno boundaries
  int32_t cur_bin = -1;           // bin of the last umiclust_cluster* call

  // device: sequences
  DevBuf<char> d_ascii;
  DevBuf<int64_t> d_offs;
  DevBuf<int32_t> d_perm;
  DevBuf<uint32_t> d_codes;
  DevBuf<uint8_t> d_lens;
  DevBuf<uint16_t> d_kmers;
  DevBuf<uint8_t> d_nk;
  DevBuf<char> d_masked;
  DevBuf<int32_t> d_iota;
  size_t iota_n = 0;               // d_iota holds 0 .. iota_n - 1
  // staged raw records (umiclust_stage): ASCII + offsets in HBM (d_ascii, d_offs), lengths on the host
  bool staged = false;
  std::vector<uint32_t> rec_len;
  PinBuf<int32_t> h_perm;          // the sorted order's pinned mirror (perm upload)
  DevBuf<uint32_t> d_amb;    // [0] an ambiguous code was seen, [1] sequences whose masked output differs from the input
  PinBuf<uint32_t> h_amb;
  int64_t n_changed = 0;     // h_amb[1] of the last prepare: 0 -> the cluster files print the input bytes
  DevBuf<uint8_t> d_mchg;    // [sorted seqno] 1: its masked output differs from its input (the writer needs that row)
  PinBuf<uint16_t> h_xm;
  DevBuf<uint16_t> d_xm;
  // packs (umiclust_cluster_pack, multi-bin loads): sorted seqno -> load bin, each bin's first seqno and its first
  // centroid ordinal in the pack being clustered (INT32_MAX until indexed), the per-bin k-mer XOR masks
  std::vector<int32_t> hqbin;
  DevBuf<int32_t> d_qbin, d_bin_seq0, d_bin_ord0;
  PinBuf<int32_t> h_bin_ord0;
  bool pack_on = false;            // the current cluster_all call clusters a pack of several bins
  // device: tables
  DevBuf<uint8_t> d_acc;
  DevBuf<uint16_t> d_rank;
  std::vector<uint8_t> h_acc;
  std::vector<uint16_t> h_rank;
  // device: index = sealed tiles (kTile centroids each, built once) + an open base tile (rebuilt
  // every kDelta new centroids) + a delta tile (rebuilt every block): an LSM layout, so a block
  // only rebuilds postings of at most kDelta centroids
  std::vector<Tile*> tiles;       // sealed
  Tile base_tile, delta_tile[2];  // the delta alternates: a counting half may still read the previous one
  int32_t delta_cur = 0;
  int32_t sealed_end = 0, base_end = 0;
  DevBuf<int32_t> d_cent;         // ordinal -> seqno
  DevBuf<uint8_t> d_cent_len;     // ordinal -> length
  std::vector<uint8_t> cent_len;
  int32_t cnt_ge[kMaxLen + 1] = {};  // centroids of length >= L
  // two passes in flight (software pipeline over blocks) + round B on a side stream
  Pass pass[kPeerTiles];          // passes in flight (the pipeline depth: UMICLUST_DEPTH, <= kPeerTiles)
  Tile blk_tile[kPeerTiles + 1], solo_tile;  // per-block peer tiles (ring of depth + 1), overflow re-runs
  Tile round_tile[2];             // O4 batched rounds: a pass's window from its first query's round start
  // passes in flight: 2; 3 (window of three blocks) hides more host time but its extra peers cost more than that
  // on configs 2/3/5 (profiles/r02/pipeline_depth_sweep.json)
  static constexpr int32_t depth = 2;
  // split passes (depth 2, UMICLUST_SPLIT=0 turns them off): a block's counting runs against the index
  // before the block two ahead is resolved, that block's hits flagged; only the merge and the alignment
  // wait for its resolution, so the counting leaves the host <-> device critical cycle
  int32_t split_env = -1;         // UMICLUST_SPLIT (-1: single-bin loads split, multi-bin sets do not)
  bool pin = true;                 // UMICLUST_PIN=0: host resolve threads not kept in the caller's L3 domain (L3Pin;
                                   // config 2 on two boxes: 3.41-3.90 M unpinned, 3.84-3.93 M pinned, profiles/r02/pin_ab.json);
                                   // off by default when LOCAL_WORLD_SIZE > 1
  bool pin_forced = false;         // UMICLUST_PIN=1: pinned even beside other contexts / ranks
  int par_min = kParInorderMin;    // UMICLUST_PAR_MIN: open queries from which it runs on the pool
  int32_t band_pairs = 140000;     // UMICLUST_BAND: alignment launches of at most this many pairs run banded
                                   // (launch bound: a few one-lane waves per SIMD); 70,000 before the faster
                                   // k_align_pk (profiles/r03/band_ab.json)
  DevBuf<int32_t> d_seq2ord;      // [seqno - bin start] centroid ordinal or -1 (the merge's flagged hits)
  PinBuf<int32_t> h_seq2ord;
  hipEvent_t a_ev[4][3] = {};     // counting halves, ring by block: begin / end / spare
  // split passes: index appends and peer-tile builds run on st_b beside the counting on the main stream;
  // they start after the latest second half (every earlier reader of the slots they rebuild precedes it)
  // and the main stream's next pass waits for ix_done
  hipStream_t ix_st = nullptr;     // null: the main stream
  hipEvent_t ix_done = nullptr, last_r_ev = nullptr;
  std::unique_ptr<WorkPool> pool;  // host threads of resolve_pass (UMICLUST_RESOLVE_THREADS)
  // the file path's input (a multi-GB mapping: ~0.11 s of page-table teardown for config 2's 3.5 GB FASTA) is released
  // on this thread after the call has written its outputs; joined by the context's next file-path call and by
  // umiclust_destroy
  std::thread in_release;
  void join_release() {
    if (in_release.joinable()) in_release.join();
  }
  // host threads of resolve_pass (caller included); 0: 8 while this is the process's only context (config 2: host
  // resolve 0.22 -> 0.14 s per step, profiles/r03/resolve_threads_ab.json), 4 beside other contexts (bin-set lanes)
  int32_t resolve_threads = 0;
  DevBuf<uint16_t> arena;         // postings of every tile (one buffer, one descriptor per pass)
  uint64_t sealed_slot0 = 0;      // arena index of sealed tile 0's slot
  int32_t index_end = 0;          // centroid ordinals [0, index_end) are indexed
  int32_t pass_B = 0;
  hipStream_t st_b = nullptr, st_copy = nullptr;
  PinBuf<uint32_t> h_bpq, h_bpt, h_bres;  // round B's pairs and results (pinned: no staged copies on the host's path)
  hipStream_t st_al = nullptr;    // walk / alignment rounds / packing of the passes
  int32_t last_a_slot = -1;       // a_ev slot of the latest counting half
  hipEvent_t evb[2] = {nullptr, nullptr};
  DevBuf<uint32_t> d_bpq, d_bpt, d_bres;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ix_events;  // index rebuild timing
  size_t nix = 0;

  // results (sorted order, absolute seqnos; each bin's range is rewritten when it is clustered)
  std::vector<int32_t> cno;       // creation cluster number (within the bin)
  std::vector<uint8_t> strand;
  std::vector<int32_t> target;    // centroid seqno a member aligned to (-1 for centroids)
  std::vector<int32_t> ocl;       // output cluster number (within the bin)
  std::vector<int32_t> cent;      // ordinal -> seqno (current bin)
  // pinned mirrors of cent / cent_len: every ordinal is uploaded once per bin from here (asynchronous DMA)
  PinBuf<int32_t> h_cent;
  PinBuf<uint8_t> h_cent_len;
  int32_t nclusters = 0;          // current bin
  // outputs of the current bin (output-cluster numbering)
  std::vector<int32_t> rank_of;   // creation number -> output number
  std::vector<int32_t> ostart, omemb;  // members per output cluster (centroid first)
  std::vector<char> cons;
  std::vector<int64_t> cons_off;
  // per-bin results kept for umiclust_fetch_bin
  struct BinOut {
    bool done = false;
    int32_t K = 0;
    std::vector<char> cons;
    std::vector<int64_t> cons_off;
  };
  std::vector<BinOut> bout;
  umiclust_stats stats{};
  int32_t block_size = 8192;
  // UMICLUST_BLOCK unset: a bin of n queries uses blocks of about n / block_div (>= block_min): a small bin's
  // window then holds fewer same-molecule peers (fewer speculative peer alignments and overflows)
  int32_t block_div = 16;
  static constexpr int32_t block_min = 2048;
  // UMICLUST_MIXLEN=0: blocks end at every query-length change (one alignment launch per round); =1: a block spans
  // up to kSegLens lengths (one launch per length and round): a small bin is then a few passes, not one per length
  // k_pack writes the outcomes and records straight into pinned host memory (true) or into device buffers copied by
  // DMA (false).  Set per clustering call: DMA with one context in the process (config 2: 4.33-4.36 vs 4.21-4.22 M
  // UMIs/s, the direct PCIe writes held k_pack at 133 us on the pass chain), direct with several (config 3, 8 lanes:
  // 7.56-7.60 vs 6.42-6.47 M: the lanes' copy dispatches contend for the hardware queues).
  bool rec_direct = false;
  static constexpr int32_t kDirectRecQ = 4096;  // blocks of at most this many queries write their records directly
  int32_t mix_len = -1;  // -1: bins whose default block is below kMaxBlock (the bin has < 16 x kMaxBlock queries)
  // speculative walk below this best k-mer count (20 and 30 equal, 45 slower: profiles/r03/spec_ab)
  static constexpr int32_t spec_thr = 30;
  // relevant peers certain to become members are not aligned speculatively (config 2 4.02 -> 4.14 M, round 4)
  static constexpr bool peer_cert = true;
  int32_t pf1_lds = 10240;  // UMICLUST_PF1: one-wave counting units up to this LDS per unit (0: never)
  int32_t regrow_depth = kPeerCap / 4;  // UMICLUST_REGROW_DEPTH: a block whose deepest peer list reaches this is not clean
  int32_t pt_side = 1;       // UMICLUST_PT_SIDE: whole passes build the next peer tiles on st_b beside the counting
                             // (1: single-bin loads; 2: always; 0: on the main stream, as before round 6)
  hipEvent_t pt_ev = nullptr;
  bool pt_pending = false;   // pt_ev recorded since the main stream last waited for it
  int32_t arrange = 1;       // UMICLUST_ARRANGE: bank-aware posting order in large tiles (1) / small tiles (2)
  int32_t regrow = 8;        // UMICLUST_REGROW: clean shallow blocks before a halved block size doubles (0: never)
  int32_t last_max_npeer = 0;
  bool pf_probe = getenv("UMICLUST_PFPROBE") != nullptr;  // the counting kernel's phases without the count loop
  DevBuf<uint32_t> d_probe;
  // lazy peers below this new-centroid rate (per mille; higher rates lose: profiles/r02/lazy_peer_sweep.json)
  int32_t lazy_permille = 5;  // UMICLUST_LAZY (0: never lazy)
  int32_t rb_wprio = 0;       // round B's alignment waves at raised issue priority (UMICLUST_RB_WPRIO)
  int32_t rb_direct = 4096;   // round B: at most this many pairs read / written in pinned memory (UMICLUST_RB_DIRECT)
  int32_t o4_T = 0;               // policy O4 (umiclust_params.policy_threads): rounds of o4_T queries; 0 = sequential
  int32_t b_hint = 1 << 30;       // block size the last bin ended with (peer overflows halve it)
  int al_level = 0;                 // the alignment stream: 0 prioritised (al_priority), -1 plain (set_priority -1)
  int st_level = 0, prio_user = 0;  // the main stream's priority now / as umiclust_set_priority left it
  int64_t dbg[4] = {0, 0, 0, 0};  // UMICLUST_DEBUG: mispredicted peers, saved peers, blocked, -
  // UMICLUST_DEBUG: per-block lines and sequential in-order resolution; UMICLUST_DEBUG=2: the per-bin summary only (the
  // production code path, with its parallel in-order phase)
  bool debug = getenv("UMICLUST_DEBUG") != nullptr && strcmp(getenv("UMICLUST_DEBUG"), "2") != 0;
  int64_t dbg_q[4] = {0, 0, 0, 0};
  // UMICLUST_WALK_DUMP=<file>: per sorted seqno of the bin, the alignments each strand's walk counted and the
  // path that resolved it (0 device, 1 classify thread, 2 in order, 3 round B) -- a parity-debugging aid
  const char* walk_dump = getenv("UMICLUST_WALK_DUMP");
  // UMICLUST_RESOLVE_DUMP=<prefix>[:i,j,...]: record resolve_block's inputs and outputs of the i-th, j-th, ... passes
  // of the context (default 10, 40, 80) to <prefix>.<i>.bin (single-bin clustering only)
  const char* resolve_dump = getenv("UMICLUST_RESOLVE_DUMP");
  int64_t n_resolved = 0;
  bool dump_want(int64_t k) const {
    const char* c = strchr(resolve_dump, ':');
    if (!c) return k == 10 || k == 40 || k == 80;
    for (const char* p = c + 1; *p;) {
      char* e;
      const long v = strtol(p, &e, 10);
      if (e == p) break;
      if (v == k) return true;
      p = *e == ',' ? e + 1 : e;
    }
    return false;
  }
  std::vector<int16_t> wd;
  double dbg_rb[4] = {};  // UMICLUST_DEBUG: round B device time (s), round trips, launches, pairs
  double dbg_t[10] = {};  // UMICLUST_DEBUG: resolve_pass phases (s): event wait, outcome copy, record copy, classify,
                          // in-order resolve, enqueue, total, appends, round B round trips, resolve_block
  int64_t dbg_p[4] = {0, 0, 0, 0};  // UMICLUST_DEBUG: strands on the inline path / with > kInlineRel relevant
                                    // peers / reading their record / peers scanned there  // UMICLUST_DEBUG: queries without records / records with only earlier-block
                                    // relevant peers / with an in-block relevant peer / host ns in pass 1
  // traceback / consensus buffers, kept across calls (a bin set clusters hundreds of small bins)
  DevBuf<uint32_t> t_mpq, t_mpt, t_mout;
  PinBuf<uint32_t> h_mpq, h_mpt;     // the member pairs' pinned staging (traceback launch)
  PinBuf<int32_t> h_mseq, h_mops, h_cstart;
  PinBuf<uint8_t> h_mstr;
  PinBuf<uint16_t> h_clen;           // consensus lengths / sequences / overflow flag (pinned downloads)
  PinBuf<char> h_craw;
  PinBuf<int32_t> h_over;
  std::vector<int32_t> t_opsidx;
  DevBuf<uint8_t> t_ops, t_mstrand;
  DevBuf<uint16_t> t_nops, t_conslen;
  DevBuf<int32_t> t_cstart, t_mseq, t_mops, t_over;
  DevBuf<char> t_cons;
  hipEvent_t tev[2] = {nullptr, nullptr};

  void fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    err = buf;
    throw Fail{code};
  }
  void hip(hipError_t e, const char* what) {
    if (e != hipSuccess) fail(UMICLUST_EDEVICE, "%s: %s", what, hipGetErrorString(e));
  }
};

namespace {

// Keep the host resolve -- the calling thread and the resolve pool -- inside the L3 domain the caller runs on,
// for the duration of one call; the caller's and the pool's affinity are restored afterwards.  Only while this
// is the process's one live context and the process is its node's only rank (LOCAL_WORLD_SIZE <= 1): several
// contexts (bin-set lanes) or ranks pinned by where their callers happen to run could all land on one CCD.
// UMICLUST_PIN=0 turns it off, UMICLUST_PIN=1 forces it on.
// CPUs the calling thread may run on (its affinity mask: taskset, cgroup cpusets, L3Pin's narrowing), bounded by
// the process's cgroup CPU quota
int affinity_cpus() {
  cpu_set_t set;
  if (sched_getaffinity(0, sizeof set, &set) != 0) return io::host_cpus();
  return std::max(1, std::min(CPU_COUNT(&set), io::host_cpus()));
}

// 8 resolve threads (4 beside other contexts), never more than the caller's affinity mask holds: the in-order
// phase's workers spin on each other's flags, so more threads than CPUs would only take slices from the worker
// the others wait on
int pool_threads(const umiclust_ctx* c) {
  const int want = c->resolve_threads > 0 ? c->resolve_threads : (g_live_ctx.load() > 1 ? 4 : 8);
  return std::max(1, std::min(want, affinity_cpus()));
}

struct L3Pin {
  cpu_set_t saved;
  bool on = false;
  umiclust_ctx* c = nullptr;
  explicit L3Pin(umiclust_ctx* ctx) : c(ctx) {
    if (!c->pin || (g_live_ctx.load() > 1 && !c->pin_forced) || sched_getaffinity(0, sizeof saved, &saved) != 0)
      return;
    // the pool is created with the caller's own mask before the caller is narrowed, so restoring `saved` on
    // both undoes the call's pinning completely
    if (!c->pool) c->pool.reset(new WorkPool(pool_threads(c)));
    const int cpu = sched_getcpu();
    char path[96], buf[256];
    snprintf(path, sizeof path, "/sys/devices/system/cpu/cpu%d/cache/index3/shared_cpu_list", cpu);
    FILE* f = cpu >= 0 ? fopen(path, "r") : nullptr;
    if (!f) return;
    const bool got = fgets(buf, sizeof buf, f) != nullptr;
    fclose(f);
    if (!got) return;
    cpu_set_t want;
    CPU_ZERO(&want);
    for (char* p = buf; *p;) {  // "a-b,c,d-e"
      char* e;
      const long a = strtol(p, &e, 10);
      if (e == p) break;
      long b = a;
      if (*e == '-') b = strtol(e + 1, &e, 10);
      for (long x = a; x <= b && x < CPU_SETSIZE; x++)
        if (CPU_ISSET((int)x, &saved)) CPU_SET((int)x, &want);
      p = *e == ',' ? e + 1 : e;
      if (*p == '\n') break;
    }
    if (CPU_COUNT(&want) == 0 || sched_setaffinity(0, sizeof want, &want) != 0) return;
    c->pool->set_affinity(want);
    on = true;
  }
  ~L3Pin() {
    if (!on) return;
    sched_setaffinity(0, sizeof saved, &saved);
    c->pool->set_affinity(saved);
  }
};

Scoring to_scoring(const umiclust_params& p) {
  Scoring s{};
  s.match = p.match;
  s.mismatch = p.mismatch;
  for (int k = 0; k < 6; k++) {
    s.go[k] = p.gap_open[k];
    s.ge[k] = p.gap_ext[k];
  }
  s.boundary_open = p.policy_boundary_open;
  return s;
}

void validate(umiclust_ctx* c, const umiclust_params& p) {
  if (p.wordlength != 8) c->fail(UMICLUST_EINVAL, "wordlength %d unsupported (8 required)", p.wordlength);
  if (p.maxaccepts != 1 || p.maxrejects != 32)
    c->fail(UMICLUST_EINVAL, "maxaccepts/maxrejects must be 1/32 (got %d/%d)", p.maxaccepts, p.maxrejects);
  if (p.minseqlength < 1 || p.minseqlength > p.maxseqlength)
    c->fail(UMICLUST_EINVAL, "bad length window [%d,%d]", p.minseqlength, p.maxseqlength);
  if (!(p.id > 0.0 && p.id <= 1.0)) c->fail(UMICLUST_EINVAL, "--id must be in (0,1]");
  if (p.minwordmatches < 0) c->fail(UMICLUST_EINVAL, "minwordmatches < 0");
  if (p.policy_threads != 0 && p.policy_threads != 1) c->fail(UMICLUST_EINVAL, "policy_threads must be 0 or 1");
  if (p.policy_threads && (p.threads < 1 || p.threads > kMaxBlock))
    c->fail(UMICLUST_EINVAL, "policy_threads = 1 needs 1 <= threads <= %d", kMaxBlock);
  int mx = std::abs(p.match) + std::abs(p.mismatch);
  for (int k = 0; k < 6; k++) mx = std::max(mx, p.gap_open[k] + p.gap_ext[k]);
  if (mx * 2 * kMaxLen > 15000) c->fail(UMICLUST_EINVAL, "scores too large for 16-bit DP");
}

// exact acceptance / id-order tables: id2 = 100.0*m/L (align_trim, iddef 2),
// accept iff id2 >= 100.0*opt_id, both in IEEE double exactly as vsearch evaluates them.
void build_tables(umiclust_ctx* c) {
  const int NL = kTabL, NM = kTabM;
  c->h_acc.assign((size_t)NL * NM, 0);
  c->h_rank.assign((size_t)NL * NM, 0);
  std::vector<std::pair<double, int>> v;
  v.reserve((size_t)NL * NM);
  const double thr = 100.0 * c->p.id;
  for (int L = 0; L < NL; L++)
    for (int m = 0; m < NM; m++) {
      const double id = L > 0 ? 100.0 * m / L : 0.0;
      c->h_acc[(size_t)L * NM + m] = (L > 0 && m <= L && id >= thr) ? 1 : 0;
      v.push_back({id, L * NM + m});
    }
  std::sort(v.begin(), v.end());
  uint16_t r = 0;
  for (size_t i = 0; i < v.size(); i++) {
    if (i > 0 && v[i].first != v[i - 1].first) r++;
    c->h_rank[(size_t)v[i].second] = r;
  }
  c->hip(c->d_acc.ensure(c->h_acc.size()), "alloc acc");
  c->hip(c->d_rank.ensure(c->h_rank.size()), "alloc rank");
  c->hip(hipMemcpyAsync(c->d_acc.p, c->h_acc.data(), c->h_acc.size(), hipMemcpyHostToDevice, c->st), "acc");
  c->hip(hipMemcpyAsync(c->d_rank.p, c->h_rank.data(), c->h_rank.size() * 2, hipMemcpyHostToDevice, c->st),
         "rank");
}

DevSeqs dev_seqs(umiclust_ctx* c) {
  DevSeqs s;
  s.codes = c->d_codes.p;
  s.lens = c->d_lens.p;
  s.kmers = c->d_kmers.p;
  s.nk = c->d_nk.p;
  return s;
}

// (re)build one index tile over sequences map[first .. first+n) with ordinals xoff + c; postings
// vbase + ((xoff + c) % seg_mod) / kParts (umiclust_internal.h), in the tile's arena slot
void build_tile(umiclust_ctx* c, Tile& t, const int32_t* map, int32_t first, int32_t n, int32_t xoff, int32_t vbase,
                int32_t seg_mod, hipStream_t st = nullptr) {
  if (!st) st = c->st;
  if (!t.hist.p) {
    c->hip(t.hist.ensure(kBins), "tile alloc");
    c->hip(hipMemsetAsync(t.hist.p, 0, (size_t)kBins * 4, st), "tile memset");
  }
  c->hip(t.off.ensure(kBins + 1), "tile alloc");
  c->hip(t.cursor.ensure(kBins), "tile alloc");
  c->hip(t.partial.ensure(kScanBlocks), "tile alloc");
  if (tile_cap(n) > t.post_cap) c->fail(UMICLUST_EDEVICE, "internal: index tile slot too small");
  uint16_t* post = c->arena.p + t.post_base;
  c->hip(launch_index_count(c->d_kmers.p, c->d_nk.p, map, first, n, xoff, t.hist.p, st), "index count");
  c->hip(launch_index_scan(t.hist.p, t.partial.p, t.off.p, t.cursor.p, post, st), "index scan");
  c->hip(launch_index_fill(c->d_kmers.p, c->d_nk.p, map, first, n, xoff, vbase, seg_mod, t.cursor.p, post, st),
         "index fill");
  // bank-aware posting order (kernels.hip k_list_arrange): large tiles (bit 0: the base tile and sealed tiles, built
  // once per fold / seal) and small ones (bit 1: delta, peer and round tiles, rebuilt every block)
  if (n > 0 && (c->arrange & (n >= 2 * kDelta ? 1 : 2)))
    c->hip(launch_index_arrange(t.off.p, post, st), "index arrange");
  t.n = n;
  t.built_n = n;
}

TileView view_of(const Tile& t) {
  TileView v;
  v.off = t.off.p;
  v.post_base = t.post_base;
  v.n = t.n;
  v.base = t.base;
  v.seg = t.seg;
  v.len = t.len;
  return v;
}

inline int32_t round_start(const umiclust_ctx* c, int32_t s0, int32_t q) {
  return o4_round_start(c->o4_T, c->pack_on ? c->hqbin.data() : nullptr, c->bin_s.data(), s0, q);
}

void ensure_pass_buffers(umiclust_ctx* c, Pass& P, int32_t B) {
  const size_t nqs = (size_t)B * c->both;
  c->hip(P.d_top_seqno.ensure(nqs * kTopHits), "alloc");
  c->hip(P.d_top_count.ensure(nqs * kTopHits), "alloc");
  c->hip(P.d_ntop.ensure(nqs), "alloc");
  c->hip(P.d_pcand.ensure(nqs * kParts * kPartCand), "alloc");
  c->hip(P.d_pncand.ensure(nqs * kParts), "alloc");
  c->hip(P.d_units.ensure(nqs * kParts), "alloc");
  c->hip(P.d_ppeer_id.ensure(nqs * kParts * kPeerCap), "alloc");
  c->hip(P.d_ppeer_count.ensure(nqs * kParts * kPeerCap), "alloc");
  c->hip(P.d_pnpeer.ensure(nqs * kParts), "alloc");
  c->hip(P.d_ppost.ensure(nqs * kParts), "alloc");
  c->hip(P.d_peer_id.ensure(nqs * kPeerCap), "alloc");
  c->hip(P.d_peer_count.ensure(nqs * kPeerCap), "alloc");
  c->hip(P.d_npeer.ensure(nqs), "alloc");
  c->hip(P.d_counters.ensure(kCountersLen), "alloc");
  P.ctr_zeroed = false;  // (a new bin or a grown buffer set: the next pass memsets them)
  // pair lists: a launch aligns up to kWalk walk pairs plus kPeerCap peer pairs per query-strand; results
  // land in d_res: walk candidate x of qs at [qs * kWalk + x], peer y at [nqs * kWalk + qs * kPeerCap + y]
  c->hip(P.d_pq.ensure(nqs * (kWalk + kPeerCap)), "alloc");
  c->hip(P.d_pt.ensure(nqs * (kWalk + kPeerCap)), "alloc");
  c->hip(P.d_outidx.ensure(nqs * (kWalk + kPeerCap)), "alloc");
  c->hip(P.d_res.ensure(nqs * (kWalk + kPeerCap)), "alloc");
  c->hip(P.d_hq.ensure(nqs), "alloc");
  c->hip(P.d_paligned.ensure((size_t)nqs * (kPeerCap / 64)), "alloc");  // 64-bit aligned-peer masks per query-strand
  c->hip(P.d_ws.ensure(nqs), "alloc");
  if (!P.d_reccount.p) {  // [0] record words allocated, [1] k_pack's workgroup tickets; k_pack leaves both zero
    c->hip(P.d_reccount.ensure(2), "alloc");
    c->hip(hipMemsetAsync(P.d_reccount.p, 0, 8, c->st), "memset");
  }
  c->hip(P.h_hq.ensure(nqs), "pin");
  c->hip(P.h_rec.ensure(nqs * kRecWords), "pin");
  c->hip(P.d_rec.ensure(nqs * kRecWords), "alloc");
  c->hip(P.h_counters.ensure(16), "pin");
  c->hip(P.h_reccount.ensure(1), "pin");
  // fixed capacities, so a pass never frees memory a queued pass still reads
  c->hip(P.h_tiles.ensure(64), "pin");
  c->hip(P.d_tiles.ensure(64), "alloc");
  c->hip(P.h_tiles_a.ensure(64), "pin");
  c->hip(P.d_tiles_a.ensure(64), "alloc");
  if (!P.d_anunits.p) {
    c->hip(P.d_anunits.ensure(1), "alloc");
    c->hip(hipMemsetAsync(P.d_anunits.p, 0, 4, c->st), "memset");
  }
  if (!P.ev_a) c->hip(hipEventCreate(&P.ev_a), "event");
}

// Enqueue the device pass of block [q0, q0+nq) against the index as it stands (centroids of the
// blocks before the peer window), with no host synchronisation: the block's own peer tile (kept
// for the next block's window), prefilter, the batch-of-8 walk over T_old (up to 4 align rounds),
// the speculative alignment of every (query, earlier window query) pair passing the k-mer
// threshold, and one download of the walk states, top lists, walked results and peer results.
// The peer window is [prev->base, q0+nq) with prev = the previous block's tile, or the block
// alone (prev == nullptr).
// the longest / shortest query of a block (sorted within a bin, but a pack's lengths restart at every bin)
int32_t block_maxlen(const umiclust_ctx* c, int32_t q0, int32_t nq) {
  int32_t m = 0;
  for (int32_t q = q0; q < q0 + nq; q++) m = std::max<int32_t>(m, c->hlen[q]);
  return m;
}
int32_t block_minlen(const umiclust_ctx* c, int32_t q0, int32_t nq) {
  int32_t m = kMaxLen;
  for (int32_t q = q0; q < q0 + nq; q++) m = std::min<int32_t>(m, c->hlen[q]);
  return m;
}

// the packs' bin bounds of the prefilter (PrefilterArgs::qbin) and the centroid length table
void set_bins(umiclust_ctx* c, PrefilterArgs& a) {
  a.qbin = c->pack_on ? c->d_qbin.p : nullptr;
  a.bin_seq0 = c->d_bin_seq0.p;
  a.bin_ord0 = c->d_bin_ord0.p;
  a.cent_len = c->d_cent_len.p;
}

// UMICLUST_PFPROBE=1 (measurement only): after every counting launch, the same launch without its count loop
// (k_pf_count<2>) into scratch outputs, so a kernel trace shows what the table, zeroing, scan and output phases cost
// on their own beside the full kernel
void launch_pf_probe(umiclust_ctx* c, const PrefilterArgs& a, hipStream_t st) {
  const size_t U = (size_t)a.nq * a.both * kParts;
  const size_t words = U * kPartCand + U * (kPeerCap / 2) + 8 * U + 16 + U * (kPeerCap / 4);
  c->hip(c->d_probe.ensure(words), "alloc probe");
  uint32_t* p = c->d_probe.p;
  PrefilterArgs b = a;
  b.pcand = p;
  p += U * kPartCand;
  b.ppeer_id = reinterpret_cast<uint16_t*>(p);
  p += U * (kPeerCap / 2);
  b.ppost = p;
  b.units = p + 3 * U;
  b.pncand = reinterpret_cast<uint8_t*>(p + 4 * U);
  b.pnpeer = reinterpret_cast<uint8_t*>(p + 5 * U);
  b.nunits = p + 7 * U + 8;
  b.ppeer_count = reinterpret_cast<uint8_t*>(p + 8 * U + 16);  // U * kPeerCap bytes
  b.prof = nullptr;
  c->hip(hipMemsetAsync(b.nunits, 0, 4, st), "memset");
  c->hip(launch_prefilter(b, st, 3), "prefilter probe");
}

void enqueue_pass(umiclust_ctx* c, Pass& P, int32_t q0, int32_t nq, const Tile* const* prevs, int nprev, Tile& own,
                  int32_t region, bool lazy_peers = false, bool after_count = false) {
  const int32_t w0 = nprev > 0 ? prevs[0]->base : q0;
  const int both = c->both;
  const int32_t nqs = nq * both;
  hipStream_t st = c->st;
  if (c->ix_st && c->ix_done) c->hip(hipStreamWaitEvent(st, c->ix_done, 0), "wait");  // index / peer tiles
  if (c->pt_pending) {  // whole passes: the peer tiles built ahead on the side stream (cluster_all)
    c->hip(hipStreamWaitEvent(st, c->pt_ev, 0), "wait");
    c->pt_pending = false;
  }
  P.q0 = q0;
  P.nq = nq;
  P.w0 = w0;
  P.live = true;
  const bool built_now = !(own.prebuilt && own.base == q0 && own.n == nq && own.seg == region);
  if (built_now) build_tile(c, own, c->d_iota.p, q0, nq, 0, region * kPeerRegion, 1 << 30);
  own.prebuilt = false;
  own.base = q0;
  own.seg = region;
  own.len = block_maxlen(c, q0, nq);  // the block's longest query
  const bool second_half = after_count && P.a_live && P.a_q0 == q0;
  // a second half's prefilter (full kernel + merge) runs on the align stream ahead of its walk, so the
  // main stream's next counting half does not queue behind it.  It needs its counting half (a_ev) and the
  // index / tiles (ix_done; index appends on the side stream wait for the latest second half, last_r_ev)
  if (second_half && c->ix_st && !built_now) {
    st = c->st_al;
    if (c->ix_done) c->hip(hipStreamWaitEvent(st, c->ix_done, 0), "wait");
  }
  int32_t nv = 0;
  const size_t need = c->tiles.size() + 2;
  if (need > P.h_tiles.n) {
    c->hip(hipStreamSynchronize(st), "sync");  // rare: the views array grows
    c->hip(P.h_tiles.ensure(need * 2), "pin");
    c->hip(P.d_tiles.ensure(need * 2), "alloc");
  }
  for (Tile* t : c->tiles)
    if (t->n > 0) P.h_tiles.p[nv++] = view_of(*t);
  if (c->base_tile.n > 0) P.h_tiles.p[nv++] = view_of(c->base_tile);
  if (c->delta_tile[c->delta_cur].n > 0) P.h_tiles.p[nv++] = view_of(c->delta_tile[c->delta_cur]);
  if (nv > kArgTiles)
    c->hip(hipMemcpyAsync(P.d_tiles.p, P.h_tiles.p, (size_t)nv * sizeof(TileView), hipMemcpyHostToDevice, st),
           "tiles");
  // the counters are zero unless this buffer set's last pass launched no k_pack (which re-zeroes them at its end)
  if (!P.ctr_zeroed) c->hip(hipMemsetAsync(P.d_counters.p, 0, kCountersLen * 4, st), "memset");
  P.ctr_zeroed = false;
  PrefilterArgs a{};
  for (int32_t i = 0; i < nv && nv <= kArgTiles; i++) a.tv[i] = P.h_tiles.p[i];
  a.seqs = dev_seqs(c);
  a.arena = c->arena.p;
  a.tiles = P.d_tiles.p;
  a.ntiles = nv;
  // centroid tiles are in segment order (sealed tiles, then base and delta); each pass addresses its
  // postings from the lowest arena slot it reads
  a.ncent = c->index_end;
  a.nseg = (c->index_end + kSegCentroids - 1) / kSegCentroids;
  if (a.nseg > kMaxSegs) c->fail(UMICLUST_ERANGE, "more than %d centroids in one bin", kMaxSegs * kSegCentroids);
  for (int s = 0, vi = 0; s <= a.nseg; s++) {
    while (vi < nv && P.h_tiles.p[vi].seg < s) vi++;
    a.seg_tile[s] = s == a.nseg ? nv : vi;
  }
  {
    uint64_t peer_lo = own.post_base;
    for (int i = 0; i < nprev; i++) peer_lo = std::min(peer_lo, prevs[i]->post_base);
    for (int s = 0; s < std::max(a.nseg, 1); s++) {
      uint64_t lo = (s == std::max(a.nseg, 1) - 1) ? peer_lo : UINT64_MAX;
      if (a.nseg > 0)
        for (int v = a.seg_tile[s]; v < a.seg_tile[s + 1]; v++) lo = std::min(lo, P.h_tiles.p[v].post_base);
      a.seg_base[s] = lo;
    }
  }
  a.cent_seqno = c->d_cent.p;
  for (int L = 0; L <= kMaxLen; L++) a.cnt_ge[L] = c->cnt_ge[L];
  a.q0 = q0;
  a.nq = nq;
  a.both = both;
  a.minwordmatches = c->p.minwordmatches;
  // peer slots oldest first, the own tile last; missing earlier blocks leave n = 0 slots in front
  for (int i = 0; i < kPeerTiles - 1; i++) {
    const int j = i - (kPeerTiles - 1 - nprev);
    a.peer[i] = j >= 0 ? view_of(*prevs[j]) : TileView{};
  }
  a.peer[kPeerTiles - 1] = view_of(own);
  a.peer_base = w0;
  a.pcand = P.d_pcand.p;
  a.pncand = P.d_pncand.p;
  a.units = P.d_units.p;
  a.nunits = P.d_anunits.p;
  a.flag_tile = -1;
  a.cand_base = w0;
  a.peer_shift = 0;
  a.peer_id_add = 0;
  a.seq2ord = c->d_seq2ord.p - c->bin_s[c->cur_bin];
  if (second_half) {
    // the counting half ran with the window one block wider (oldest first): its peer ids are relative to
    // that window's start
    a.cand_base = P.a_base;
    a.peer_shift = w0 - P.a_base;
    a.peer_id_add = a.peer_shift;
  }
  // list table of the lean kernel: every k-mer of the block's length in every tile it reads
  a.nlist_cap = std::min(kMaxKmers * 12, std::max(1, block_maxlen(c, q0, nq) - 7) *
                                              ((a.nseg > 0 ? a.seg_tile[1] - a.seg_tile[0] : 0) + kPeerTiles));
  a.pf1_lds = c->pf1_lds;
  a.ppeer_id = P.d_ppeer_id.p;
  a.ppeer_count = P.d_ppeer_count.p;
  a.pnpeer = P.d_pnpeer.p;
  a.ppost = P.d_ppost.p;
  a.top_seqno = P.d_top_seqno.p;
  a.top_count = P.d_top_count.p;
  a.ntop = P.d_ntop.p;
  a.peer_id = P.d_peer_id.p;
  a.peer_count = P.d_peer_count.p;
  a.npeer = P.d_npeer.p;
  a.postings_touched = P.d_counters.p;
  a.prof = c->pf_prof.p;  // null unless UMICLUST_PFPROF is set
  set_bins(c, a);
  if (second_half) c->hip(hipStreamWaitEvent(st, c->a_ev[P.a_slot][1], 0), "wait");
  c->hip(hipEventRecord(P.ev[0], st), "event");
  P.c_timed = false;
  if (second_half) {
    c->hip(launch_prefilter(a, st, 2), "prefilter");
  } else if (a.nseg <= 1) {
    // whole pass: the lean counting (timed alone), then the full kernel over its overflowed units + merge
    for (auto& e : P.ev_c)
      if (!e) c->hip(hipEventCreate(&e), "event");
    c->hip(hipEventRecord(P.ev_c[0], st), "event");
    c->hip(launch_prefilter(a, st, 1), "prefilter (count)");
    c->hip(hipEventRecord(P.ev_c[1], st), "event");
    c->stats.counter_cells += (int64_t)nq * c->both * a.ncent;
    if (c->pf_probe) launch_pf_probe(c, a, st);
    c->hip(launch_prefilter(a, st, 2), "prefilter");
    P.c_timed = true;
  } else {
    c->hip(launch_prefilter(a, st, 0), "prefilter");
  }
  c->hip(hipEventRecord(P.ev[1], st), "event");
  c->last_r_ev = P.ev[1];
  P.a_timed = second_half;
  P.t_slot = P.a_slot;
  P.a_live = false;
  // The walk, its alignment rounds and the packing run on the align stream: they read only this
  // pass's buffers and the sequences, so the main stream goes on with the index append of the block
  // being resolved and the next pass's prefilter while these small launches run.
  c->hip(hipStreamWaitEvent(c->st_al, P.ev[1], 0), "wait");
  st = c->st_al;
  DevSeqs ds = dev_seqs(c);
  // the block's query lengths (sorted, non-increasing): one pair segment and one alignment launch per length
  const int32_t lmax = block_maxlen(c, q0, nq), nsg = lmax - block_minlen(c, q0, nq) + 1;
  if (nsg > kSegLens) c->fail(UMICLUST_EINVAL, "block spans %d query lengths (> %d)", nsg, kSegLens);
  int32_t nql[kSegLens] = {};
  for (int32_t q = q0; q < q0 + nq; q++) nql[lmax - c->hlen[q]]++;
  SegTab sg0{}, sg1{};
  sg0.lmax = sg1.lmax = lmax;
  sg0.nseg = sg1.nseg = nsg;
  for (int32_t i = 0, b0 = 0, b1 = 0; i < nsg; i++) {
    sg0.base[i] = (uint32_t)b0;
    sg1.base[i] = (uint32_t)b1;
    b0 += nql[i] * both * kWalk;
    b1 += nql[i] * both * (kWalk + kPeerCap);
  }
  uint32_t* segc = P.d_counters.p + kSegSlot;  // [walk round][segment]
  unsigned long long* cells_w = reinterpret_cast<unsigned long long*>(P.d_counters.p + 12);
  unsigned long long* cells_p = reinterpret_cast<unsigned long long*>(P.d_counters.p + 14);
  auto align_round = [&](const SegTab& sg, int per_qs, uint32_t* cnt, const char* what) {
    for (int32_t i = 0; i < nsg; i++)
      if (nql[i])
        c->hip(launch_align(ds, lmax - i, c->ambig, P.d_pq.p + sg.base[i], P.d_pt.p + sg.base[i], nql[i] * both * per_qs,
                            cnt + i, P.d_outidx.p + sg.base[i], c->sc, P.d_res.p, st, c->band_pairs),
               what);
  };
  c->hip(launch_walk(-1, q0, nqs, both, c->spec_thr, P.d_top_seqno.p, P.d_top_count.p, P.d_ntop.p, c->d_lens.p, P.d_res.p,
                     c->d_acc.p, c->d_rank.p, P.d_ws.p, P.d_pq.p, P.d_pt.p, P.d_outidx.p, sg0, segc, cells_w, st),
         "walk");
  c->hip(hipEventRecord(P.ev[2], st), "event");
  // two dependent alignment launches: batch 0 (or a speculative whole walk), then the rest of every
  // unfinished walk together with the relevant in-window peers (their relevance is taken from the walk
  // state after round 0, which only widens it: a superset of what the final state needs)
  const uint32_t peer_out0 = (uint32_t)nqs * kWalk;
  // small passes (deep clusters cut blocks small) spread every pair over a lane group
  align_round(sg0, kWalk, segc, "align 0");
  c->hip(launch_walk(0, q0, nqs, both, c->spec_thr, P.d_top_seqno.p, P.d_top_count.p, P.d_ntop.p, c->d_lens.p,
                     P.d_res.p, c->d_acc.p, c->d_rank.p, P.d_ws.p, P.d_pq.p, P.d_pt.p, P.d_outidx.p, sg1, segc + kSegLens,
                     cells_w, st),
         "walk 0");
  // the previous block's pass (its walk states are final and stay until that buffer set's next walk, which is
  // queued after this one on the align stream): peers there whose device walk accepted are certain members
  const Pass* prev = nullptr;
  if (c->peer_cert)
    for (const Pass& Q : c->pass)
      if (&Q != &P && Q.nq > 0 && Q.q0 + Q.nq == q0) prev = &Q;
  c->hip(launch_peer_pairs(q0, w0, nqs, both, c->d_lens.p, P.d_ws.p, P.d_peer_id.p, P.d_peer_count.p, P.d_npeer.p,
                           P.d_pq.p, P.d_pt.p, P.d_outidx.p, sg1, segc + kSegLens, cells_p, P.d_counters.p + 8,
                           peer_out0, P.d_paligned.p, lazy_peers ? 0 : 1,
                           prev ? prev->d_ws.p : nullptr, prev ? prev->d_npeer.p : nullptr, prev ? prev->q0 : 0,
                           prev ? prev->nq : 0, st),
         "peer pairs");
  align_round(sg1, kWalk + kPeerCap, segc + kSegLens, "align 1");
  c->hip(launch_walk(1, q0, nqs, both, c->spec_thr, P.d_top_seqno.p, P.d_top_count.p, P.d_ntop.p, c->d_lens.p,
                     P.d_res.p, c->d_acc.p, c->d_rank.p, P.d_ws.p, P.d_pq.p, P.d_pt.p, P.d_outidx.p, sg1,
                     segc + 2 * kSegLens, cells_w, st),
         "walk 1");
  c->hip(hipEventRecord(P.ev[3], st), "event");
  // what the host needs goes straight to pinned host memory; the pass that next reuses these
  // buffers is enqueued only after the host has waited for ev[4]
  // small blocks (deep clusters: config 5's ~2k-query blocks) write directly too: their copies are dispatch-bound
  // (`profiles/r05/recdirect_small_ab/`: config 5 3.52 -> 3.64 M UMIs/s, config 2's 8k-query blocks lose with it)
  P.rec_direct = c->rec_direct || nq <= umiclust_ctx::kDirectRecQ;
  // rec_direct: k_pack writes the outcomes and records straight into the pinned host buffers (no DMA copies on the
  // chain the host waits for: a 3 MB record copy was 0.14 ms per config-2 block); otherwise device buffers + copies
  c->hip(launch_pack(nqs, w0, c->d_lens.p, P.d_ws.p, P.d_ntop.p, P.d_top_seqno.p, P.d_top_count.p, P.d_res.p,
                     P.d_npeer.p, P.d_peer_id.p, P.d_peer_count.p, P.d_res.p + peer_out0, P.d_paligned.p, P.d_reccount.p,
                     P.rec_direct ? P.h_hq.p : P.d_hq.p,
                     P.rec_direct ? P.h_rec.p : P.d_rec.p, P.d_counters.p, P.h_counters.p, P.h_reccount.p, st),
         "pack");
  P.ctr_zeroed = nqs > 0;
  if (!P.rec_direct)
    c->hip(hipMemcpyAsync(P.h_hq.p, P.d_hq.p, (size_t)nqs * sizeof(HostQs), hipMemcpyDeviceToHost, st), "d2h outcomes");
  if (!P.rec_direct) {
    const size_t est = std::min<size_t>(P.rec_est, P.d_rec.n);
    c->hip(hipMemcpyAsync(P.h_rec.p, P.d_rec.p, est * 4, hipMemcpyDeviceToHost, st), "d2h records");
  }
  c->hip(hipEventRecord(P.ev[4], st), "event");
}

// The counting half of a split pass (block [q0, q0+nq), launch_prefilter mode 1): the lean kernel against
// the index as it stands and the window's peer tiles `wins` (oldest first, the block's own -- built -- last);
// the hits of wins[flag] (a block not yet resolved) become flagged candidates.  The second half is
// enqueue_pass(..., after_count = true) once that block is resolved and appended.  Bins past one counter
// segment are not split (a_live stays false and the second half runs the whole prefilter).
void enqueue_count(umiclust_ctx* c, Pass& P, int32_t q0, int32_t nq, const Tile* const* wins, int nwin, int flag,
                   int32_t slot) {
  P.a_live = false;
  const int32_t nseg = (c->index_end + kSegCentroids - 1) / kSegCentroids;
  if (nseg > 1) return;
  for (auto& e : c->a_ev[slot])
    if (!e) c->hip(hipEventCreate(&e), "event");
  // on its own stream, gated by the main stream's work so far (index append, peer tiles, this buffer set's
  // last merge): the main stream's next append and second half do not queue behind it
  hipStream_t st = c->st;
  if (c->ix_st && c->ix_done) c->hip(hipStreamWaitEvent(st, c->ix_done, 0), "wait");  // index / peer tiles
  if (c->pt_pending) {  // whole passes: the peer tiles built ahead on the side stream (cluster_all)
    c->hip(hipStreamWaitEvent(st, c->pt_ev, 0), "wait");
    c->pt_pending = false;
  }
  // this buffer set's last second half (full kernel + merge on the align stream) has read what
  // the counting half overwrites
  if (c->ix_st) c->hip(hipStreamWaitEvent(st, P.ev[1], 0), "wait");
  c->hip(hipEventSynchronize(P.ev_a), "sync");  // the last upload from h_tiles_a is done
  int32_t nv = 0;
  const size_t need = c->tiles.size() + 2;
  if (need > P.h_tiles_a.n) {
    c->hip(hipStreamSynchronize(st), "sync");  // rare: the views array grows
    c->hip(P.h_tiles_a.ensure(need * 2), "pin");
    c->hip(P.d_tiles_a.ensure(need * 2), "alloc");
  }
  for (Tile* t : c->tiles)
    if (t->n > 0) P.h_tiles_a.p[nv++] = view_of(*t);
  if (c->base_tile.n > 0) P.h_tiles_a.p[nv++] = view_of(c->base_tile);
  if (c->delta_tile[c->delta_cur].n > 0) P.h_tiles_a.p[nv++] = view_of(c->delta_tile[c->delta_cur]);
  if (nv > kArgTiles)
    c->hip(hipMemcpyAsync(P.d_tiles_a.p, P.h_tiles_a.p, (size_t)nv * sizeof(TileView), hipMemcpyHostToDevice, st),
           "tiles");
  c->hip(hipEventRecord(P.ev_a, st), "event");
  PrefilterArgs a{};
  for (int32_t i = 0; i < nv && nv <= kArgTiles; i++) a.tv[i] = P.h_tiles_a.p[i];
  a.seqs = dev_seqs(c);
  a.arena = c->arena.p;
  a.tiles = P.d_tiles_a.p;
  a.ntiles = nv;
  a.ncent = c->index_end;
  a.nseg = nseg;
  a.seg_tile[0] = 0;
  a.seg_tile[1] = nv;
  uint64_t lo = UINT64_MAX;
  for (int i = 0; i < nwin; i++) lo = std::min(lo, wins[i]->post_base);
  for (int v = 0; v < nv; v++) lo = std::min(lo, P.h_tiles_a.p[v].post_base);
  a.seg_base[0] = lo;
  a.cent_seqno = c->d_cent.p;
  for (int L = 0; L <= kMaxLen; L++) a.cnt_ge[L] = c->cnt_ge[L];
  a.q0 = q0;
  a.nq = nq;
  a.both = c->both;
  a.minwordmatches = c->p.minwordmatches;
  for (int i = 0; i < kPeerTiles; i++) {
    const int j = i - (kPeerTiles - nwin);
    a.peer[i] = j >= 0 ? view_of(*wins[j]) : TileView{};
  }
  a.flag_tile = flag >= 0 ? (kPeerTiles - nwin) + flag : -1;
  a.peer_base = a.cand_base = wins[0]->base;
  a.seq2ord = c->d_seq2ord.p - c->bin_s[c->cur_bin];
  a.pcand = P.d_pcand.p;
  a.pncand = P.d_pncand.p;
  a.units = P.d_units.p;
  a.nunits = P.d_anunits.p;
  a.nlist_cap = std::min(kMaxKmers * 12, std::max(1, block_maxlen(c, q0, nq) - 7) * (nv + kPeerTiles));
  a.pf1_lds = c->pf1_lds;
  a.ppeer_id = P.d_ppeer_id.p;
  a.ppeer_count = P.d_ppeer_count.p;
  a.pnpeer = P.d_pnpeer.p;
  a.ppost = P.d_ppost.p;
  a.prof = c->pf_prof.p;  // null unless UMICLUST_PFPROF is set
  set_bins(c, a);
  c->hip(hipEventRecord(c->a_ev[slot][0], st), "event");
  c->hip(launch_prefilter(a, st, 1), "prefilter (count)");
  c->hip(hipEventRecord(c->a_ev[slot][1], st), "event");
  c->stats.counter_cells += (int64_t)nq * c->both * a.ncent;
  if (c->pf_probe) launch_pf_probe(c, a, st);
  c->last_a_slot = slot;
  P.a_live = true;
  P.a_q0 = q0;
  P.a_base = wins[0]->base;
  P.a_slot = slot;
}

// One resolve_block call, replayable without a GPU (format read by tools/resolve_tsan_main.cpp): little-endian,
// "UCRD" v1, the parameters, hlen of the bin up to the block's end, the acceptance / rank tables, the window's states
// before, the pass's HostQs and records, round B's pairs and results, then the outputs (the block's states, targets
// and strands, the new centroids, alignments and cells).
void write_resolve_dump(const umiclust_ctx* c, const ResolveEnv& env, int32_t q0, int32_t nq, int32_t w0,
                        const StateView& state, const std::vector<uint8_t>& state_in, const HostQs* hq,
                        const uint32_t* recs, uint32_t nrec, const std::vector<uint32_t>& bpq,
                        const std::vector<uint32_t>& bpt, const std::vector<uint32_t>& bres,
                        const std::vector<int32_t>& new_cents, const ResolveStats& rs) {
  const std::string path = std::string(c->resolve_dump, strcspn(c->resolve_dump, ":")) + "." +
                           std::to_string(c->n_resolved - 1) + ".bin";
  FILE* f = fopen(path.c_str(), "wb");
  if (!f) return;
  auto w = [&](const void* p, size_t n) { fwrite(p, 1, n, f); };
  auto wi = [&](int64_t v) { w(&v, 8); };
  w("UCRD", 4);
  const int32_t s0 = state.s0;
  const int32_t hdr[12] = {1, q0, nq, w0, env.both, env.o4_T, env.maxaccepts, env.maxrejects, env.pre_resolve ? 1 : 0,
                           env.pre_spec ? 1 : 0, s0, 0};
  w(hdr, sizeof hdr);
  wi(q0 + nq - s0);
  w(env.hlen + s0, (size_t)(q0 + nq - s0));
  w(env.acc, (size_t)kTabL * kTabM);
  w(env.rank, (size_t)kTabL * kTabM * 2);
  wi((int64_t)state_in.size());
  w(state_in.data(), state_in.size());
  const int64_t nqs = (int64_t)nq * env.both;
  wi(nqs);
  w(hq, (size_t)nqs * sizeof(HostQs));
  wi(nrec);
  w(recs, (size_t)nrec * 4);
  wi((int64_t)bpq.size());
  w(bpq.data(), bpq.size() * 4);
  w(bpt.data(), bpt.size() * 4);
  w(bres.data(), bres.size() * 4);
  w(&state[q0], (size_t)nq);
  w(env.target + q0, (size_t)nq * 4);
  w(env.strand + q0, (size_t)nq);
  wi((int64_t)new_cents.size());
  w(new_cents.data(), new_cents.size() * 4);
  wi(rs.n_alignments);
  wi(rs.cells);
  fclose(f);
}

// Wait for a pass and resolve its block on the host in sorted order (resolve.cpp resolve_block).  Returns false if a
// peer list overflowed (the caller re-runs the block in smaller pieces).
bool resolve_pass(umiclust_ctx* c, Pass& P, const StateView& state, std::vector<int32_t>& new_cents,
                  double& t_pf, double& t_al, double& t_host, int32_t* resolved) {
  const int both = c->both;
  const int32_t q0 = P.q0, w0 = P.w0;
  int32_t nq = P.nq;
  int32_t nqs = nq * both;
  if (resolved) *resolved = 0;
  const double tsync0 = now_s();
  c->hip(hipEventSynchronize(P.ev[4]), "sync");
  c->stats.t_sync_s += now_s() - tsync0;
  c->dbg_t[0] += now_s() - tsync0;
  struct DAcc { double* p; double t0; ~DAcc() { *p += now_s() - t0; } } dtot{&c->dbg_t[6], tsync0};
  P.live = false;
  float ms = 0;
  c->hip(hipEventElapsedTime(&ms, P.ev[0], P.ev[1]), "elapsed");
  t_pf += ms * 1e-3;
  if (P.a_timed) {
    c->hip(hipEventElapsedTime(&ms, c->a_ev[P.t_slot][0], c->a_ev[P.t_slot][1]), "elapsed");
    t_pf += ms * 1e-3;
    c->stats.t_count_s += ms * 1e-3;
    c->stats.n_count_launches++;
    tl_add(c->dev, 0, c->a_ev[P.t_slot][0], c->a_ev[P.t_slot][1]);
  } else if (P.c_timed) {
    c->hip(hipEventElapsedTime(&ms, P.ev_c[0], P.ev_c[1]), "elapsed");
    c->stats.t_count_s += ms * 1e-3;
    c->stats.n_count_launches++;
    tl_add(c->dev, 0, P.ev_c[0], P.ev_c[1]);
  }
  c->hip(hipEventElapsedTime(&ms, P.ev[2], P.ev[3]), "elapsed");
  t_al += ms * 1e-3;
  tl_add(c->dev, 1, P.ev[2], P.ev[3]);
  {
    // records past the DMA'd prefix (a pass that used more than the estimate): fetch the rest now
    const size_t used = *P.h_reccount.p, est = std::min<size_t>(P.rec_est, P.d_rec.n);
    if (used > est && !P.rec_direct) {
      c->hip(hipMemcpyAsync(P.h_rec.p + est, P.d_rec.p + est, (used - est) * 4, hipMemcpyDeviceToHost, c->st_copy),
             "d2h records");
      c->hip(hipStreamSynchronize(c->st_copy), "sync");
    }
    P.rec_est = (uint32_t)std::max<size_t>(1u << 16, used + used / 2 + 4096);
  }
  c->stats.kmer_postings += P.h_counters.p[0];
  c->stats.pairs_peer += P.h_counters.p[8];
  // every alignment the device computed for this pass (walk rounds + speculative peers)
  {
    unsigned long long cw = 0, cp = 0;  // u64 cells of the walk pairs / the peer pairs (counters 12-13 / 14-15)
    memcpy(&cw, P.h_counters.p + 12, 8);
    memcpy(&cp, P.h_counters.p + 14, 8);
    c->stats.cells_computed += (int64_t)(cw + cp);
  }
  // a pageable copy of the per-query-strand outcomes (sequential, revisited below); the records
  // are read in place, only for the query-strands whose relevant peers include a centroid
  const double tc0 = now_s();
  P.hq_copy.assign(P.h_hq.p, P.h_hq.p + nqs);
  {
    uint32_t mx = 0;  // the block's deepest peer list (regrowth: a window far from the cap may double)
    for (int32_t qs = 0; qs < nqs; qs++) mx = std::max<uint32_t>(mx, P.hq_copy[qs].npeer);
    c->last_max_npeer = (int32_t)mx;
  }
  c->stats.t_sync_s += now_s() - tc0;
  c->dbg_t[1] += now_s() - tc0;
  const HostQs* hq = P.hq_copy.data();
  if (!c->pool) c->pool.reset(new WorkPool(pool_threads(c)));
  // the records are copied into pageable memory first (one streaming read; scattered reads of the DMA'd
  // pinned buffer are slow): config 2 +2-3 %
  const uint32_t* recs = P.h_rec.p;
  {
    const double tc1 = now_s();
    // on the resolve threads: one core's streaming read of pinned memory is the limit (0.05 s per config-2 step)
    const size_t nw = *P.h_reccount.p;
    if (P.rec_copy.size() < nw) P.rec_copy.resize(nw + nw / 4);
    const int TC = nw < (1u << 18) ? 1 : c->pool->size();
    if (TC == 1) {
      memcpy(P.rec_copy.data(), P.h_rec.p, nw * 4);
    } else {
      c->pool->run([&](int t) {
        const size_t lo = nw * (size_t)t / (size_t)TC, hi = nw * (size_t)(t + 1) / (size_t)TC;
        memcpy(P.rec_copy.data() + lo, P.h_rec.p + lo, (hi - lo) * 4);
      });
    }
    recs = P.rec_copy.data();
    c->stats.t_sync_s += now_s() - tc1;
    c->dbg_t[2] += now_s() - tc1;
  }
  ResolveEnv env;
  env.hlen = c->hlen.data();
  env.acc = c->h_acc.data();
  env.rank = c->h_rank.data();
  env.both = both;
  env.o4_T = c->o4_T;
  env.maxaccepts = c->p.maxaccepts;
  env.maxrejects = c->p.maxrejects;
  env.hqbin = c->pack_on ? c->hqbin.data() : nullptr;
  env.bin_s = c->bin_s.data();

  // (one context only: several lanes' pools already share the host's cores, config 3 7.59 -> 7.40 M UMIs/s with it)
  // (and only when every pool thread has a CPU of its own under the caller's current mask, L3Pin's included: its
  // workers spin-wait on each other)
  env.par_inorder = g_live_ctx.load() <= 1 && c->pool->size() <= affinity_cpus();
  env.par_min = c->par_min;
  env.debug = c->debug;
  env.target = c->target.data();
  env.strand = c->strand.data();
  env.walk_dump = c->wd.empty() ? nullptr : c->wd.data();
  // round B on the copy stream (a hardware queue of its own, otherwise idle): on st_b it queued behind the split
  // passes' index appends and peer-tile builds, which wait for the next counting half -- about one counting launch of
  // latency on the host's critical path per block with deferred queries
  auto round_b = [&](const std::vector<uint32_t>& bpq, const std::vector<uint32_t>& bpt, std::vector<uint32_t>& bres) {
    const int32_t nb = (int32_t)bpq.size();
    hipStream_t sb = c->st_copy;
    c->hip(c->h_bpq.ensure(nb), "pin");
    c->hip(c->h_bpt.ensure(nb), "pin");
    c->hip(c->h_bres.ensure(nb), "pin");
    memcpy(c->h_bpq.p, bpq.data(), (size_t)nb * 4);
    memcpy(c->h_bpt.p, bpt.data(), (size_t)nb * 4);
    // small rounds (the usual: tens of pairs) read their pairs from and write their scores to the pinned buffers
    // directly: one dispatch per query length and no copies on the host's critical path (two uploads and a download
    // were ~70 us of dispatch latency per block with deferred queries); large ones go through device buffers
    const bool direct = nb <= c->rb_direct;
    const uint32_t *pq = c->h_bpq.p, *pt = c->h_bpt.p;
    uint32_t* pres = c->h_bres.p;
    if (!direct) {
      c->hip(c->d_bpq.ensure(nb), "alloc");
      c->hip(c->d_bpt.ensure(nb), "alloc");
      c->hip(c->d_bres.ensure(nb), "alloc");
      c->hip(hipMemcpyAsync(c->d_bpq.p, c->h_bpq.p, (size_t)nb * 4, hipMemcpyHostToDevice, sb), "h2d");
      c->hip(hipMemcpyAsync(c->d_bpt.p, c->h_bpt.p, (size_t)nb * 4, hipMemcpyHostToDevice, sb), "h2d");
      pq = c->d_bpq.p;
      pt = c->d_bpt.p;
      pres = c->d_bres.p;
    }
    c->hip(hipEventRecord(c->evb[0], sb), "event");
    Scoring scb = c->sc;
    scb.wave_prio = c->rb_wprio;
    // the pairs are in query order: one launch per run of one query length
    int nl = 0;
    for (int32_t x0 = 0; x0 < nb; nl++) {
      const int32_t L = c->hlen[bpq[x0] >> 1];
      int32_t x1 = x0 + 1;
      while (x1 < nb && c->hlen[bpq[x1] >> 1] == L) x1++;
      c->hip(launch_align(dev_seqs(c), L, c->ambig, pq + x0, pt + x0, x1 - x0, nullptr, nullptr, scb, pres + x0, sb,
                          c->band_pairs),
             "align B");
      x0 = x1;
    }
    c->hip(hipEventRecord(c->evb[1], sb), "event");
    if (!direct)
      c->hip(hipMemcpyAsync(c->h_bres.p, c->d_bres.p, (size_t)nb * 4, hipMemcpyDeviceToHost, sb), "d2h");
    c->hip(hipStreamSynchronize(sb), "sync");
    memcpy(bres.data(), c->h_bres.p, (size_t)nb * 4);
    float bms = 0;
    c->hip(hipEventElapsedTime(&bms, c->evb[0], c->evb[1]), "elapsed");
    t_al += bms * 1e-3;
    c->dbg_rb[0] += bms * 1e-3;
    c->dbg_rb[1] += 1;
    c->dbg_rb[2] += nl;
    c->dbg_rb[3] += nb;
  };
  // UMICLUST_RESOLVE_DUMP: the pass's inputs, round-B pairs / results and outputs, for the host-only replay
  // (tools/resolve_tsan_main.cpp: the ThreadSanitizer harness of the CPU suite)
  const bool dump = c->resolve_dump && !c->pack_on && c->dump_want(c->n_resolved);
  c->n_resolved++;
  std::vector<uint32_t> dpq, dpt, dres;
  std::vector<uint8_t> state_in;
  if (dump) state_in.assign(&state[w0], &state[w0] + (q0 + nq - w0));
  RoundB round_b_rec = [&](const std::vector<uint32_t>& bpq, const std::vector<uint32_t>& bpt, std::vector<uint32_t>& bres) {
    round_b(bpq, bpt, bres);
    dpq.insert(dpq.end(), bpq.begin(), bpq.end());
    dpt.insert(dpt.end(), bpt.begin(), bpt.end());
    dres.insert(dres.end(), bres.begin(), bres.end());
  };
  ResolveStats rs;
  const double th0 = now_s();
  // partial resolution (resolved != nullptr): the queries before the block's first overflowing one depend on earlier
  // queries only, so they are resolved now and only the rest is re-run
  bool partial = false;
  if (resolved)
    for (int32_t qs = 0; qs < nqs; qs++)
      if (hq[qs].flags & 2u) {
        if (qs / both == 0) return false;
        nq = qs / both;
        nqs = nq * both;
        partial = true;
        break;
      }
  const int r = resolve_block(env, q0, nq, w0, hq, recs, state, P.rsx, *c->pool, new_cents, rs,
                              dump ? round_b_rec : RoundB(round_b));
  const double th = now_s() - th0;
  if (r == kResolveOverflow) return false;
  if (r == kResolveStuck) c->fail(UMICLUST_EDEVICE, "internal: a deferred query of block %d is still unresolved", q0);
  if (r == kResolveBadPeer) c->fail(UMICLUST_EDEVICE, "internal: a peer of block %d is not an earlier query", q0);
  if (dump)
    write_resolve_dump(c, env, q0, nq, w0, state, state_in, hq, recs, *P.h_reccount.p, dpq, dpt, dres, new_cents, rs);
  t_host += th - rs.t_round_b_s;
  // UMICLUST_DEBUG: one line per resolved block (where the host's time goes, block by block)
  if (c->debug)
    fprintf(stderr, "blk q0 %d nq %d new %zu wait %.3f classify %.3f inorder %.3f roundB %.3f (%lld pairs) merged %lld "
            "deferred %lld ms-since-wait %.3f\n", q0, nq, new_cents.size(), 1e3 * (tc0 - tsync0), 1e3 * rs.t_classify_s,
            1e3 * rs.t_inorder_s, 1e3 * rs.t_round_b_s, (long long)rs.pairs_round_b, (long long)rs.n_merged_walks,
            (long long)rs.n_deferred, 1e3 * (now_s() - tsync0));
  c->stats.t_host_pass1_s += rs.t_classify_s + rs.t_inorder_s;
  c->dbg_t[3] += rs.t_classify_s;
  c->dbg_t[4] += rs.t_inorder_s;
  c->dbg_t[8] += rs.t_round_b_s;
  c->dbg_t[9] += th;
  c->stats.n_alignments += rs.n_alignments;
  c->stats.cells += rs.cells;
  c->stats.n_merged_walks += rs.n_merged_walks;
  c->stats.t_merged_s += rs.t_merged_s;
  c->stats.n_deferred += rs.n_deferred;
  c->stats.pairs_round_b += rs.pairs_round_b;
  c->stats.cells_computed += rs.cells_round_b;
  for (int i = 0; i < 4; i++) {
    c->dbg[i] += rs.dbg[i];
    c->dbg_p[i] += rs.dbg_p[i];
    c->dbg_q[i] += rs.dbg_q[i];
  }
  if (resolved) *resolved = nq;
  return !partial;
}

// Append a block's new centroids (sorted seqnos) to the LSM index, enqueued on the main stream
// behind any queued pass (which keeps reading the tiles as they were when it was enqueued).
void append_centroids(umiclust_ctx* c, const std::vector<int32_t>& new_cents) {
  if (new_cents.empty()) return;
  hipStream_t st = c->ix_st ? c->ix_st : c->st;
  if (c->ix_st && c->last_r_ev) c->hip(hipStreamWaitEvent(st, c->last_r_ev, 0), "wait");
  const int32_t ord0 = (int32_t)c->cent.size();
  int32_t s2o_lo = 0, s2o_n = 0, bo_lo = 0, bo_n = 0;
  for (int32_t q : new_cents) {  // capacity reserved: no reallocation
    c->cent.push_back(q);
    c->cent_len.push_back(c->hlen[q]);
    for (int L = 0; L <= c->hlen[q]; L++) c->cnt_ge[L]++;
  }
  {
    // seqno -> ordinal for the merge's flagged hits (the new centroids are in sorted order)
    const int32_t s0 = c->bin_s[c->cur_bin];
    for (size_t i = 0; i < new_cents.size(); i++) c->h_seq2ord.p[new_cents[i] - s0] = ord0 + (int32_t)i;
    s2o_lo = new_cents.front() - s0;
    s2o_n = std::max(0, new_cents.back() - s0 - s2o_lo + 1);
  }
  if (c->pack_on) {
    // a bin's first query is always a centroid (nothing of its bin precedes it): its ordinal opens the bin's range
    // (the bins starting inside this append are consecutive: one copy)
    int32_t blo = INT32_MAX, bhi = -1;
    for (size_t i = 0; i < new_cents.size(); i++) {
      const int32_t q = new_cents[i], b = c->hqbin[q];
      if (q == c->bin_s[b]) {
        c->h_bin_ord0.p[b] = ord0 + (int32_t)i;
        blo = std::min(blo, b);
        bhi = std::max(bhi, b);
      }
    }
    if (bhi >= blo) {
      bo_lo = blo;
      bo_n = bhi - blo + 1;
    }
  }
  memcpy(c->h_cent.p + ord0, c->cent.data() + ord0, new_cents.size() * 4);
  memcpy(c->h_cent_len.p + ord0, c->cent_len.data() + ord0, new_cents.size());
  // one dispatch reads the pinned ranges (as the copies it replaces, at its execution time)
  c->hip(launch_append_stage(c->h_cent.p + ord0, c->h_cent_len.p + ord0, (int32_t)new_cents.size(), c->d_cent.p + ord0,
                             c->d_cent_len.p + ord0, c->h_seq2ord.p + s2o_lo, c->d_seq2ord.p + s2o_lo, s2o_n,
                             bo_n ? c->h_bin_ord0.p + bo_lo : nullptr, bo_n ? c->d_bin_ord0.p + bo_lo : nullptr, bo_n,
                             st),
         "append stage");
  const int32_t ordend = (int32_t)c->cent.size();
  if (c->nix >= c->ix_events.size()) {
    hipEvent_t e0, e1;
    c->hip(hipEventCreate(&e0), "event");
    c->hip(hipEventCreate(&e1), "event");
    c->ix_events.push_back({e0, e1});
  }
  const auto& ev = c->ix_events[c->nix++];
  c->hip(hipEventRecord(ev.first, st), "event");
  while (ordend - c->sealed_end >= kTile) {  // seal a full tile
    Tile* t = new Tile();
    t->base = c->sealed_end;
    t->seg = t->base / kSegCentroids;
    t->post_cap = tile_cap(kTile);
    t->post_base = c->sealed_slot0 + (uint64_t)c->tiles.size() * t->post_cap;
    build_tile(c, *t, c->d_cent.p, t->base, kTile, t->base, kCentBase, kSegCentroids, st);
    c->tiles.push_back(t);
    c->sealed_end += kTile;
    c->base_end = std::max(c->base_end, c->sealed_end);
    c->base_tile.n = 0;
  }
  if (ordend - c->base_end > kDelta) {  // fold the delta into the base tile
    // the base is rebuilt in place: the latest counting half may still read it
    if (c->last_a_slot >= 0) c->hip(hipStreamWaitEvent(st, c->a_ev[c->last_a_slot][1], 0), "wait");
    c->base_tile.base = c->sealed_end;
    c->base_tile.seg = c->sealed_end / kSegCentroids;
    build_tile(c, c->base_tile, c->d_cent.p, c->sealed_end, ordend - c->sealed_end, c->sealed_end, kCentBase,
               kSegCentroids, st);
    c->base_end = ordend;
  }
  // the other delta slot was last read by a counting half the main stream has already waited for (the
  // second half of its pass precedes this append)
  c->delta_cur ^= 1;
  Tile& dt = c->delta_tile[c->delta_cur];
  dt.base = c->base_end;
  dt.seg = c->base_end / kSegCentroids;
  if (ordend > c->base_end)
    build_tile(c, dt, c->d_cent.p, c->base_end, ordend - c->base_end, c->base_end, kCentBase, kSegCentroids, st);
  else
    dt.n = 0;
  c->index_end = ordend;
  c->hip(hipEventRecord(ev.second, st), "event");
  if (c->ix_st) {
    if (!c->ix_done) c->hip(hipEventCreate(&c->ix_done), "event");
    c->hip(hipEventRecord(c->ix_done, st), "event");
  }
}

// Cluster bin `bin` -- or, npk > 1, the pack of bins [bin, bin + npk) in one greedy order (each bin's queries in
// its own sorted order, the bins one after another: bins never interact, so this is every bin's own vsearch run):
// blocks then span bin boundaries and small bins share passes; the prefilter keeps only a query's own bin
// (PrefilterArgs::qbin) and the results are split per bin.
// The main (counting) stream re-created at the greatest priority (level 1) or as a plain stream (0), after its queued
// work; no other handle of it is kept (ix_st is st_b or null, events recorded on it have completed).
hipError_t main_stream_priority(umiclust_ctx* c, int level) {
  if (c->st_level == level) return hipSuccess;
  int lo = 0, hi = 0;
  hipError_t e = hipDeviceGetStreamPriorityRange(&lo, &hi);
  hipStream_t s = nullptr;
  if (e == hipSuccess) e = hipStreamSynchronize(c->st);  // work queued since the caller's drain (memsets) first
  if (e == hipSuccess)
    e = level ? hipStreamCreateWithPriority(&s, hipStreamNonBlocking, hi) : hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  if (e != hipSuccess) return e;
  (void)hipStreamDestroy(c->st);
  c->st = s;
  c->st_level = level;
  return hipSuccess;
}

void cluster_all(umiclust_ctx* c, int32_t bin, bool multi_bin = false, int32_t npk = 1) {
  static const int rec_env = [] {
    const char* e = getenv("UMICLUST_REC_DIRECT");
    return e ? atoi(e) : -1;
  }();
  c->rec_direct = rec_env >= 0 ? rec_env > 0 : g_live_ctx.load() > 1;
  const double t0 = now_s();
  if (bin < 0 || npk < 1 || bin + npk >= (int32_t)c->bin_s.size())
    c->fail(UMICLUST_EINVAL, "bins [%d, %d) out of range", bin, bin + npk);
  c->pack_on = npk > 1;
  // one bin (or pack) = the sorted seqnos [s0, s1); seqnos stay absolute everywhere
  const int32_t s0 = c->bin_s[bin], s1 = c->bin_s[bin + npk];
  const int32_t n = s1 - s0;
  c->cur_bin = bin;
  std::fill(c->cno.begin() + s0, c->cno.begin() + s1, -1);
  std::fill(c->strand.begin() + s0, c->strand.begin() + s1, 0);
  std::fill(c->target.begin() + s0, c->target.begin() + s1, -1);
  c->cent.clear();
  c->cent.reserve((size_t)n + 1);
  c->cent_len.clear();
  std::fill(c->cnt_ge, c->cnt_ge + kMaxLen + 1, 0);
  c->cent_len.reserve((size_t)n + 1);
  c->nclusters = 0;
  c->hip(hipStreamSynchronize(c->st), "sync");  // no queued work may still read the old tiles
  for (Tile* t : c->tiles) delete t;
  c->tiles.clear();
  c->base_tile.n = c->delta_tile[0].n = c->delta_tile[1].n = 0;
  c->last_a_slot = -1;
  c->sealed_end = c->base_end = 0;
  c->index_end = 0;
  c->nix = 0;
  c->stats = umiclust_stats{};
  c->stats.n_input = c->bin_in[bin + npk] - c->bin_in[bin];
  if (c->pack_on) {
    for (int32_t b = bin; b < bin + npk; b++) c->h_bin_ord0.p[b] = INT32_MAX;  // no centroid of the bin indexed yet
    c->hip(hipMemcpyAsync(c->d_bin_ord0.p + bin, c->h_bin_ord0.p + bin, (size_t)npk * 4, hipMemcpyHostToDevice, c->st),
           "h2d bin ord0");
  }
  c->stats.n_kept = n;
  c->hip(c->d_cent.ensure((size_t)n + 1), "alloc cent");
  c->hip(c->d_cent_len.ensure((size_t)n + 1), "alloc cent");
  c->hip(c->h_cent.ensure((size_t)n + 1), "pin cent");
  c->hip(c->h_cent_len.ensure((size_t)n + 1), "pin cent");
  c->hip(c->d_seq2ord.ensure((size_t)n + 1), "alloc seq2ord");
  c->hip(c->h_seq2ord.ensure((size_t)n + 1), "pin seq2ord");
  std::fill(c->h_seq2ord.p, c->h_seq2ord.p + n, -1);
  c->hip(hipMemsetAsync(c->d_seq2ord.p, 0xff, (size_t)n * 4, c->st), "memset");
  std::vector<uint8_t> state_buf((size_t)n, ST_UNDET);
  StateView state{state_buf.data(), s0};
  if (c->walk_dump) c->wd.assign((size_t)n * 4, -1);
  double t_pf = 0, t_al = 0, t_host = 0;
  // blocks of at most B queries of one length (the aligner is compiled per query length); a block's
  // peer tile fills one kPeerRegion of the prefilter counters, so B <= kMaxBlock
  int32_t B = std::max(1, std::min<int32_t>(c->block_size, kMaxBlock));
  if (c->block_div > 0) B = std::min<int32_t>(B, std::max<int32_t>(c->block_min, ((s1 - s0) / c->block_div + 255) & ~255));
  c->pass_B = B;
  for (Pass& P : c->pass) ensure_pass_buffers(c, P, B);
  // postings arena: the base, delta, peer-ring and solo slots, then the sealed tile slots in creation
  // order (n / kTile of them at most); a prefilter pass reads the slots of one counter segment (plus
  // the unsealed ones in its last pass), which keeps its 32-bit buffer offsets in range
  {
    uint64_t off = 0;
    auto slot = [&](Tile& t, int64_t nseq) {
      t.post_base = off;
      t.post_cap = tile_cap(nseq);
      off += t.post_cap;
    };
    slot(c->base_tile, kTile);
    slot(c->delta_tile[0], kDelta);
    slot(c->delta_tile[1], kDelta);
    for (Tile& t : c->blk_tile) slot(t, kMaxBlock);
    slot(c->solo_tile, kMaxBlock);
    if (c->o4_T)
      for (Tile& t : c->round_tile) slot(t, c->o4_T);
    c->sealed_slot0 = off;
    off += (uint64_t)(n / kTile) * tile_cap(kTile);
    c->hip(c->arena.ensure((size_t)off + 64), "alloc arena");
  }
  std::vector<std::pair<int32_t, int32_t>> blocks;
  // blocks across length changes: bins below the full block size (config 3: 4.15 vs 3.61 M UMIs/s; a 2M-read bin
  // gains nothing, its length runs are many blocks long: profiles/r03/mixlen_ab.json)
  const bool mix = c->mix_len > 0 || (c->mix_len < 0 && (B < kMaxBlock || c->pack_on));
  // the blocks from query `from` on, at most `bmax` queries (of one length each unless mix)
  auto split_blocks = [&](int32_t from, int32_t bmax) {
    // packs: bmax (a deep cluster's halved size) holds until the end of `from`'s bin, the next bins start at B
    const int32_t until = c->pack_on ? c->bin_s[c->hqbin[from] + 1] : s1;
    for (int32_t q0 = from; q0 < s1;) {
      int32_t same = 1;
      const int32_t bcap = q0 < until ? bmax : B;
      if (mix) {  // across length changes, at most kSegLens lengths (one pair segment each)
        const int32_t lim = std::min<int32_t>(bcap, s1 - q0);
        int32_t lo = c->hlen[q0], hi = lo;  // (a pack's lengths restart at every bin)
        while (same < lim && std::max<int32_t>(hi, c->hlen[q0 + same]) - std::min<int32_t>(lo, c->hlen[q0 + same]) < kSegLens) {
          lo = std::min<int32_t>(lo, c->hlen[q0 + same]);
          hi = std::max<int32_t>(hi, c->hlen[q0 + same]);
          same++;
        }
      } else {
        while (q0 + same < s1 && same < bcap && c->hlen[q0 + same] == c->hlen[q0]) same++;
      }
      // O4: a block cut by the size cap ends at a round start (trimmed by < 1 round), so the next block's window needs
      // no round tile: only blocks starting at a length change (or a bin start in a pack) still begin mid-round
      // (same-box A/B: config 3 +2.2 %, config 5 +1.8 %, config 2 unchanged; profiles/r05/round_align_ab/)
      if (c->o4_T && same == bcap && q0 + same < s1) {
        const int32_t r = round_start(c, s0, q0 + same);
        if (r > q0 + same / 2) same = r - q0;
      }
      blocks.push_back({q0, same});
      q0 += same;
    }
  };
  // Policy O4 batched rounds (c->o4_T queries each, counted from the first sorted query of q's bin): query q's search
  // sees only the centroids before its round start rstart(q), and the centroids of its round before it are the
  // re-check's extras -- both must be in its pass's peer window, and the index must hold nothing from the round.
  // Every pass that may still run or re-run counts: a queued pass is re-run alone when its block overflows a peer
  // list (run_alone), against the index as it stands then.  So the index only ever holds the centroids before
  // W = rstart(first query of the earliest block not yet resolved) -- the oldest window tile's first query -- and a
  // *round tile* over [W, that query) joins the window in front of the nominal tiles; resolved centroids wait in
  // `pending` until W has passed them.  (Round 4 synced the index to min(nominal window start, round start of the
  // pass's own first query): when block k overflowed after pass k+1 had been queued, block k's re-run met centroids
  // of its own first round in the index -- config 5 under --threads 25 aligned 15-50 more pairs than the oracle and
  // moved reads between clusters, tests/test_gpu_o4.py::test_o4_config_vs_oracle_golden.)
  const int32_t T4 = c->o4_T;
  auto rstart = [&](int32_t q) { return round_start(c, s0, q); };
  std::vector<int32_t> pending;
  auto sync_index = [&](int32_t X) {  // the index gets the pending centroids before seqno X
    size_t m = 0;
    while (m < pending.size() && pending[m] < X) m++;
    if (!m) return;
    std::vector<int32_t> a(pending.begin(), pending.begin() + (ptrdiff_t)m);
    append_centroids(c, a);
    pending.erase(pending.begin(), pending.begin() + (ptrdiff_t)m);
  };
  // the window of a pass starting at query q with the nprev tiles prevs (oldest first), adjusted for the rounds:
  // the round tile (counter region 2; the block tiles of the D = 2 ring use 0 and 1) goes in front
  auto round_window = [&](int32_t q, const Tile** prevs, int& nprev, int slot) {
    const int32_t first = nprev ? prevs[0]->base : q;
    const int32_t W = rstart(first);
    if (W < first) {
      Tile& rt = c->round_tile[slot & 1];
      build_tile(c, rt, c->d_iota.p, W, first - W, 0, (kPeerTiles - 1) * kPeerRegion, 1 << 30);
      rt.base = W;
      rt.seg = kPeerTiles - 1;
      rt.len = 0;  // several lengths
      rt.prebuilt = false;
      for (int i = nprev; i > 0; i--) prevs[i] = prevs[i - 1];
      prevs[0] = &rt;
      nprev++;
    }
    sync_index(W);
  };
  // a bin starts at the block size the previous one ended with, doubled (deep bins tend to follow deep bins)
  int32_t b_eff = c->pack_on ? B : std::min<int64_t>(B, std::max<int64_t>(256, (int64_t)c->b_hint * 2));
  int32_t eff_bin = -1;  // packs: the bin b_eff was last halved in (a deep cluster of one bin does not shrink the next)
  // Halving stops at 256 queries (a floor of kPeerCap / 4 = 32, at which no window can overflow, ran config 4's
  // giant-molecule bin 200 in 8,578 blocks: 1.44 s alone against 0.6 s at 256; a peer-load feedback that re-cut the
  // queued blocks from each block's largest peer list lost on config 5: profiles/r04/block_policy)
  constexpr int32_t kMinBlock = 256;
  auto halve = [&](int32_t q) -> bool {  // false: already at the smallest block
    if (c->pack_on && c->hqbin[q] != eff_bin) {
      eff_bin = c->hqbin[q];
      b_eff = B;
    }
    if (b_eff <= kMinBlock) return false;
    b_eff = std::max(kMinBlock, b_eff / 2);
    return true;
  };
  split_blocks(s0, b_eff);
  int32_t nb = (int32_t)blocks.size();
  int32_t clean = 0;  // blocks resolved since the last overflow (regrowth)
  std::vector<int32_t> new_cents;
  // Member tracebacks: tw_launch(lo, hi, stream) traces the members among seqnos [lo, hi) (their targets are final),
  // queries of <= 64 nt in a launch of their own (a one-stripe direction store: more waves per CU), appending to the
  // pair arrays at tw_n; opsidx maps a member to its traceback slot.  (Tracing the first blocks' members early on a
  // least-priority stream while later blocks are clustered measured no faster: round 4 cumask_early_ab/.)
  std::vector<int32_t>& opsidx = c->t_opsidx;
  opsidx.assign(n, -1);
  int32_t tw_n = 0;
  c->hip(c->h_mpq.ensure((size_t)std::max(n, 1)), "pin");
  c->hip(c->h_mpt.ensure((size_t)std::max(n, 1)), "pin");
  c->hip(c->t_mpq.ensure(n), "alloc");
  c->hip(c->t_mpt.ensure(n), "alloc");
  c->hip(c->t_mout.ensure(n), "alloc");
  c->hip(c->t_ops.ensure((size_t)std::max(n, 1) * kOpsStride), "alloc");
  c->hip(c->t_nops.ensure(n), "alloc");
  const DevSeqs ds = dev_seqs(c);
  const int32_t tw_maxl = s1 > s0 ? *std::max_element(c->hlen.begin() + s0, c->hlen.begin() + s1) : kMaxLen;
  // members of <= 64-nt queries in a launch of their own (one launch for all measured equal: round 4 twsplit_ab/)
  constexpr int tw_split = 64;
  auto tw_launch = [&](int32_t lo, int32_t hi, hipStream_t stq) {
    const int32_t x0 = tw_n;
    int32_t x = x0, nm1 = 0, maxq1 = 0, maxq2 = 0;
    for (int pass = 0; pass < 2; pass++) {
      for (int32_t s = lo; s < hi; s++)
        if (c->target[s] >= 0 && (((int)c->hlen[s] <= tw_split) == (pass == 0))) {
          opsidx[s - s0] = x;
          c->h_mpq.p[x] = ((uint32_t)s << 1) | c->strand[s];
          c->h_mpt.p[x] = (uint32_t)c->target[s];
          (pass ? maxq2 : maxq1) = std::max(pass ? maxq2 : maxq1, (int32_t)c->hlen[s]);
          x++;
        }
      if (pass == 0) nm1 = x;
    }
    tw_n = x;
    if (x == x0) return;
    c->hip(hipMemcpyAsync(c->t_mpq.p + x0, c->h_mpq.p + x0, (size_t)(x - x0) * 4, hipMemcpyHostToDevice, stq), "h2d");
    c->hip(hipMemcpyAsync(c->t_mpt.p + x0, c->h_mpt.p + x0, (size_t)(x - x0) * 4, hipMemcpyHostToDevice, stq), "h2d");
    c->hip(launch_traceback(ds, c->t_mpq.p + x0, c->t_mpt.p + x0, nm1 - x0, c->sc, c->t_ops.p + (size_t)x0 * kOpsStride,
                            c->t_nops.p + x0, c->t_mout.p + x0, stq, tw_maxl, maxq1),
           "traceback");
    c->hip(launch_traceback(ds, c->t_mpq.p + nm1, c->t_mpt.p + nm1, x - nm1, c->sc, c->t_ops.p + (size_t)nm1 * kOpsStride,
                            c->t_nops.p + nm1, c->t_mout.p + nm1, stq, tw_maxl, maxq2),
           "traceback");
  };
  // A block whose peer list overflowed: re-run it alone (window = itself, index complete up to it)
  // in halving pieces, synchronously.
  auto run_alone = [&](int32_t q0, int32_t nq) {
    Pass& P = c->pass[0];
    int32_t piece = nq;
    for (int32_t q = q0; q < q0 + nq;) {
      const int32_t m = std::min(piece, q0 + nq - q);
      const Tile* prevs[kPeerTiles];
      int nprev = 0;
      if (T4) round_window(q, prevs, nprev, 0);
      enqueue_pass(c, P, q, m, prevs, nprev, c->solo_tile, 0);
      c->stats.n_reruns++;
      int32_t done = 0;
      const bool all = resolve_pass(c, P, state, new_cents, t_pf, t_al, t_host, &done);
      if (done > 0) {  // the whole piece, or its prefix before the first overflowing query
        if (T4) pending.insert(pending.end(), new_cents.begin(), new_cents.end());
        else append_centroids(c, new_cents);
        c->stats.n_blocks++;
        q += done;
      }
      if (!all && done == 0) {
        if (m == 1) c->fail(UMICLUST_EDEVICE, "peer overflow with block of 1");
        piece = std::max(1, m / 2);
      }
    }
  };
  // Software pipeline over blocks, D = c->depth passes in flight: passes k+1 .. k+D-1 are queued before
  // the host resolves block k.  Pass j runs against the index of the blocks before its peer window (blocks
  // j-D+1 .. j), and the window covers every later query before block j's, so C_old u window = all queries
  // before j: the merged walk is exact.  Invariant at the top of iteration k: passes k .. k+D-1 (those that
  // exist) are queued, the index holds blocks < k.  Block k's peer tile lives in blk_tile[k % (D + 1)]
  // (read by passes k .. k+D-1) and counts into peer region k % D of the prefilter counters.
  const int D = T4 ? 2 : c->depth;
  auto tile_of = [&](int32_t k) -> Tile& { return c->blk_tile[k % (D + 1)]; };
  // Lazy peers: once new centroids have become rare (the last resolved block created fewer than
  // lazy_permille per mille), in-window peers are not aligned speculatively; a query whose relevant peer
  // turns out to be a centroid is deferred and round B aligns what it needs (deep clusters: config 5)
  bool lazy = false;
  // enqueue block k's pass with the nprev blocks before it in its peer window
  auto enqueue = [&](int32_t k, int nprev) {
    const Tile* prevs[kPeerTiles];
    for (int i = 0; i < nprev; i++) prevs[i] = &tile_of(k - nprev + i);
    if (T4) round_window(blocks[k].first, prevs, nprev, k);
    enqueue_pass(c, c->pass[k % D], blocks[k].first, blocks[k].second, prevs, nprev, tile_of(k), k % D, lazy);
  };
  // split passes shorten the host <-> device cycle of one bin at the price of a wider counting window;
  // multi-bin sets run several lanes on one GPU, which is throughput-bound: there the whole passes win
  // (configs 2 / 5: +12 % / +2 %, config 3: -6 %; profiles/r02/split_ab.json)
  const bool split = !T4 && (c->split_env >= 0 ? c->split_env != 0 : !multi_bin);
  c->ix_st = (split && D == 2) ? c->st_b : nullptr;
  c->last_r_ev = nullptr;
  if (split && D == 2) {
    // Split passes.  Pass j = counting half A(j) (index of blocks <= j-3, window j-2 .. j with block j-2
    // flagged) enqueued after block j-3 is resolved, and second half R(j) (the full kernel over A's
    // overflowed units against index <= j-2 / window j-1 .. j, the merge keeping the flagged hits that are
    // centroids, then walk / align / pack) after block j-2 is.  Block j's peer tile: blk_tile[j % 4],
    // counter region j % 3 (three consecutive blocks share a counting window).
    auto stile = [&](int32_t j) -> Tile& { return c->blk_tile[j % (kPeerTiles + 1)]; };
    auto build_peer = [&](int32_t j, bool side) {
      Tile& t = stile(j);
      const int32_t region = j % kPeerTiles;
      if (!(t.prebuilt && t.base == blocks[j].first && t.n == blocks[j].second && t.seg == region)) {
        hipStream_t bs = c->st;
        if (side && c->ix_st) {
          bs = c->ix_st;
          if (c->last_r_ev) c->hip(hipStreamWaitEvent(bs, c->last_r_ev, 0), "wait");
        }
        build_tile(c, t, c->d_iota.p, blocks[j].first, blocks[j].second, 0, region * kPeerRegion, 1 << 30, bs);
        if (bs != c->st) {
          if (!c->ix_done) c->hip(hipEventCreate(&c->ix_done), "event");
          c->hip(hipEventRecord(c->ix_done, bs), "event");
        }
      }
      t.base = blocks[j].first;
      t.seg = region;
      t.len = c->hlen[blocks[j].first];
      t.prebuilt = true;
    };
    // R(j) with the window's blocks from `first` (first = j - 1 in the steady state)
    auto second_half = [&](int32_t j, int32_t first, bool after_count) {
      const Tile* prevs[kPeerTiles];
      int np = 0;
      for (int32_t i = first; i < j; i++) prevs[np++] = &stile(i);
      enqueue_pass(c, c->pass[j % 2], blocks[j].first, blocks[j].second, prevs, np, stile(j), j % kPeerTiles, lazy,
                   after_count);
    };
    auto count_half = [&](int32_t j, int32_t first, int flag) {
      const Tile* wins[kPeerTiles];
      int nw = 0;
      for (int32_t i = first; i <= j; i++) wins[nw++] = &stile(i);
      enqueue_count(c, c->pass[j % 2], blocks[j].first, blocks[j].second, wins, nw, flag, j % 4);
    };
    // the index holds the blocks before r and nothing is queued: classic passes r (window r) and r+1 (window
    // r, r+1), then A(r+2) with block r flagged
    auto prime = [&](int32_t r) {
      for (int32_t j = r; j < r + 3 && j < nb; j++) build_peer(j, false);
      if (r < nb) second_half(r, r, false);
      if (r + 1 < nb) second_half(r + 1, r, false);
      if (r + 2 < nb) count_half(r + 2, r, 0);
    };
    prime(0);
    for (int32_t k = 0; k < nb; k++) {
      Pass& P = c->pass[k % 2];
      const double tb0 = now_s();
      if (k + 3 < nb) build_peer(k + 3, true);  // queries only: built while the host resolves block k
      c->dbg_t[5] += now_s() - tb0;
      if (!resolve_pass(c, P, state, new_cents, t_pf, t_al, t_host, nullptr)) {
        // drain everything queued (its windows include block k) and restart the pipeline after block k
        c->hip(hipStreamSynchronize(c->st_al), "sync");
        c->hip(hipStreamSynchronize(c->st_b), "sync");
        c->hip(hipStreamSynchronize(c->st), "sync");
        for (Pass& Q : c->pass) {
          Q.live = false;
          Q.a_live = false;
          c->hip(hipMemsetAsync(Q.d_anunits.p, 0, 4, c->st), "memset");
        }
      run_alone(blocks[k].first, blocks[k].second);
        if (k + 1 < nb && halve(blocks[k].first)) {
          const int32_t from = blocks[k].first + blocks[k].second;
          blocks.resize((size_t)k + 1);
          split_blocks(from, b_eff);
          nb = (int32_t)blocks.size();
        }
        for (Tile& t : c->blk_tile) t.prebuilt = false;
        prime(k + 1);
        continue;
      }
      const double ta0 = now_s();
      append_centroids(c, new_cents);
      const double ta1 = now_s();
      c->stats.n_blocks++;
      lazy = c->lazy_permille > 0 && (int64_t)new_cents.size() * 1000 < (int64_t)blocks[k].second * c->lazy_permille;
      c->stats.n_lazy_passes += (lazy && k + 2 < nb) ? 1 : 0;
      if (k + 2 < nb) second_half(k + 2, k + 1, true);
      if (k + 3 < nb) count_half(k + 3, k + 1, 0);
      c->dbg_t[7] += ta1 - ta0;           // UMICLUST_DEBUG: index appends (host side)
      c->dbg_t[5] += now_s() - ta1;       // and the next passes' enqueue
    }
  } else {
  for (int32_t i = 0; i < D && i < nb; i++) enqueue(i, i);
  for (int32_t k = 0; k < nb; k++) {
    Pass& P = c->pass[k % D];
    const double te0 = now_s();
    if (k + D < nb) {
      // block k+D's peer tile depends on its queries only: build it now, while the host resolves block k (its ring
      // slot was last read by pass k's prefilter).  Since round 6 on the side stream (after pass k's prefilter), so
      // the build runs beside the main stream's counting instead of between two counting launches; the pass that
      // next enqueues on the main stream waits for it (enqueue_pass, pt_ev).  Before, it sat on the main stream.
      Tile& t = tile_of(k + D);
      hipStream_t bst = nullptr;
      if (c->pt_side == 2 || (c->pt_side == 1 && !multi_bin)) {  // config 2 +1.6 %, multi-lane config 3 -2 %
        bst = c->st_b;
        c->hip(hipStreamWaitEvent(bst, P.ev[1], 0), "wait");
        if (!c->pt_ev) c->hip(hipEventCreateWithFlags(&c->pt_ev, hipEventDisableTiming), "event");
      }
      build_tile(c, t, c->d_iota.p, blocks[k + D].first, blocks[k + D].second, 0, ((k + D) % D) * kPeerRegion,
                 1 << 30, bst);
      if (bst) {
        c->hip(hipEventRecord(c->pt_ev, bst), "event");
        c->pt_pending = true;
      }
      t.base = blocks[k + D].first;
      t.seg = (k + D) % D;
      t.prebuilt = true;
    }
    c->dbg_t[5] += now_s() - te0;
    int32_t done = 0;
    if (!resolve_pass(c, P, state, new_cents, t_pf, t_al, t_host, &done)) {
      // drain the queued passes k+1 .. k+D-1 (their windows include block k) and restart the pipeline
      for (int i = 1; i < D; i++) {
        Pass& Q = c->pass[(k + i) % D];
        if (Q.live) {
          c->hip(hipEventSynchronize(Q.ev[4]), "sync");
          Q.live = false;
        }
      }
      // the block's prefix before its first overflowing query is resolved (its queries' peers are all earlier)
      if (done > 0) {
        if (T4) pending.insert(pending.end(), new_cents.begin(), new_cents.end());
        else append_centroids(c, new_cents);
        c->stats.n_blocks++;
      }
      // an overflowing bin runs synchronous re-runs from here on: with other lanes sharing the GPU they queue behind
      // every lane's work unless its main stream goes first (config 4: a 792k-read bin with a giant molecule took
      // 7.2 s among 8 lanes, 0.6 s alone)
      run_alone(blocks[k].first + done, blocks[k].second - done);
      clean = 0;
      // deep clusters flood the peer window: later blocks are cut smaller (a smaller window holds fewer
      // same-molecule peers), so the overflow re-runs do not repeat block after block
      if (k + 1 < nb && halve(blocks[k].first)) {
        const int32_t from = blocks[k].first + blocks[k].second;
        blocks.resize((size_t)k + 1);
        split_blocks(from, b_eff);
        nb = (int32_t)blocks.size();
      }
      for (int i = 1; i <= D; i++)
        if (k + i < nb) enqueue(k + i, i - 1);
      continue;
    }
    if (T4) pending.insert(pending.end(), new_cents.begin(), new_cents.end());
    else append_centroids(c, new_cents);
    c->stats.n_blocks++;
    lazy = c->lazy_permille > 0 && (int64_t)new_cents.size() * 1000 < (int64_t)blocks[k].second * c->lazy_permille;
    c->stats.n_lazy_passes += (lazy && k + D < nb) ? 1 : 0;
    // Regrowth: after `regrow` consecutive blocks without an overflow whose deepest peer list stayed below a quarter of
    // the cap, the blocks not yet queued are cut at twice the size.  With overflowing blocks resolved up to their first
    // overflowing query (resolve_pass), a giant molecule's stretch no longer pins a bin at 256-query blocks: config 4's
    // bin 200 7.0 -> 1.6 s among 8 lanes, config 4 6.51 -> 7.59 M UMIs/s; config 5's windows stay deep, so its blocks
    // do not grow (3.33 / 3.36 M; ungated regrowth after 4 clean blocks: 2.47 M) -- profiles/r05/regrow_ab/.
    if (c->last_max_npeer >= c->regrow_depth) {
      clean = 0;  // a deep window: no regrowth yet, and it does not count as a clean block
    } else if (c->regrow > 0 && b_eff < B && ++clean >= c->regrow && k + D < nb) {
      b_eff = std::min<int32_t>(B, b_eff * 2);
      c->stats.n_regrows++;
      clean = 0;
      const int32_t from = blocks[k + D].first;
      blocks.resize((size_t)k + D);
      split_blocks(from, b_eff);
      nb = (int32_t)blocks.size();
      tile_of(k + D).prebuilt = false;
    }
    const double te1 = now_s();
    if (k + D < nb) enqueue(k + D, D - 1);
    c->dbg_t[5] += now_s() - te1;
  }
  }
  c->b_hint = b_eff;
  // centroids still pending (O4): creation numbers only, no index is needed any more
  c->cent.insert(c->cent.end(), pending.begin(), pending.end());
  c->hip(hipStreamSynchronize(c->st_b), "sync");
  c->ix_st = nullptr;
  c->hip(hipStreamSynchronize(c->st_al), "sync");
  c->hip(hipStreamSynchronize(c->st), "sync");
  c->hip(main_stream_priority(c, c->prio_user), "stream priority");
  for (size_t i = 0; i < c->nix; i++) {
    float ms = 0;
    c->hip(hipEventElapsedTime(&ms, c->ix_events[i].first, c->ix_events[i].second), "elapsed");
    c->stats.t_index_s += ms * 1e-3;
  }
  // --- member tracebacks first: their pairs (sorted seqno order) need only the targets, so the launch goes out
  // before the host numbers the clusters, which then overlaps the traceback (round 4: the numbering and the
  // pageable pair uploads were ~16 ms of idle GPU before the traceback of a 2M-read bin).  The members before
  tw_launch(s0, s1, c->st);
  const int32_t nm = tw_n;
  if (!c->tev[0]) {
    c->hip(hipEventCreate(&c->tev[0]), "event");
    c->hip(hipEventCreate(&c->tev[1]), "event");
  }
  c->hip(hipEventRecord(c->tev[0], c->st), "event");
  (void)nm;
  // creation numbers: centroids in creation (= sorted seqno) order, members inherit their centroid's
  c->nclusters = (int32_t)c->cent.size();
  for (int32_t k = 0; k < c->nclusters; k++) c->cno[c->cent[k]] = k;
  for (int32_t s = s0; s < s1; s++)
    if (c->target[s] >= 0) c->cno[s] = c->cno[c->target[s]];
  // --- output numbering: --clusterout_sort orders clusters by size desc, creation order
  const int32_t K = c->nclusters;
  std::vector<int32_t> size(K, 0);
  for (int32_t s = s0; s < s1; s++) size[c->cno[s]]++;
  std::vector<int32_t> order(K);
  for (int32_t k = 0; k < K; k++) order[k] = k;
  // (a pack's clusters stay grouped by bin -- creation order already is -- and are sorted within their bin)
  auto cbin = [&](int32_t k) { return c->pack_on ? c->hqbin[c->cent[k]] : 0; };
  if (c->p.clusterout_sort)
    std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) {
      const int32_t ba = cbin(a), bb = cbin(b);
      return ba != bb ? ba < bb : size[a] > size[b];
    });
  c->rank_of.assign(K, 0);
  for (int32_t k = 0; k < K; k++) c->rank_of[order[k]] = k;
  c->ostart.assign((size_t)K + 1, 0);
  for (int32_t s = s0; s < s1; s++) {
    c->ocl[s] = c->rank_of[c->cno[s]];
    c->ostart[c->ocl[s] + 1]++;
  }
  for (int32_t k = 0; k < K; k++) c->ostart[k + 1] += c->ostart[k];
  c->omemb.assign(n, 0);
  {
    std::vector<int32_t> fill(c->ostart.begin(), c->ostart.end() - 1);
    for (int32_t s = s0; s < s1; s++) c->omemb[fill[c->ocl[s]]++] = s;
  }
  // --- consensus (behind the traceback on the same stream)
  double t_cons = 0;
  {
    // consensus inputs in output-cluster order (pinned: the uploads are queued, not staged)
    c->hip(c->h_mseq.ensure((size_t)std::max(n, 1)), "pin");
    c->hip(c->h_mops.ensure((size_t)std::max(n, 1)), "pin");
    c->hip(c->h_mstr.ensure((size_t)std::max(n, 1)), "pin");
    c->hip(c->h_cstart.ensure((size_t)K + 1), "pin");
    for (int32_t x = 0; x < n; x++) {
      const int32_t s = c->omemb[x];
      c->h_mseq.p[x] = s;
      c->h_mops.p[x] = opsidx[s - s0];
      c->h_mstr.p[x] = c->strand[s];
    }
    std::copy(c->ostart.begin(), c->ostart.end(), c->h_cstart.p);
    c->hip(c->t_cstart.ensure((size_t)K + 1), "alloc");
    c->hip(c->t_mseq.ensure(n), "alloc");
    c->hip(c->t_mops.ensure(n), "alloc");
    c->hip(c->t_mstrand.ensure(n), "alloc");
    c->hip(c->t_cons.ensure((size_t)std::max(K, 1) * kConsCap), "alloc");
    c->hip(c->t_conslen.ensure((size_t)std::max(K, 1)), "alloc");
    c->hip(c->t_over.ensure(1), "alloc");
    c->hip(hipMemsetAsync(c->t_over.p, 0, 4, c->st), "memset");
    c->hip(hipMemcpyAsync(c->t_cstart.p, c->h_cstart.p, ((size_t)K + 1) * 4, hipMemcpyHostToDevice, c->st), "h2d");
    if (n > 0) {
      c->hip(hipMemcpyAsync(c->t_mseq.p, c->h_mseq.p, (size_t)n * 4, hipMemcpyHostToDevice, c->st), "h2d");
      c->hip(hipMemcpyAsync(c->t_mops.p, c->h_mops.p, (size_t)n * 4, hipMemcpyHostToDevice, c->st), "h2d");
      c->hip(hipMemcpyAsync(c->t_mstrand.p, c->h_mstr.p, (size_t)n, hipMemcpyHostToDevice, c->st), "h2d");
    }
    c->hip(launch_consensus(ds, c->t_cstart.p, K, c->t_mseq.p, c->t_mops.p, c->t_mstrand.p, c->t_ops.p, c->t_nops.p,
                            c->t_cons.p, c->t_conslen.p, c->t_over.p, c->st),
           "consensus");
    c->hip(hipEventRecord(c->tev[1], c->st), "event");
    c->hip(c->h_clen.ensure((size_t)std::max(K, 1)), "pin");
    c->hip(c->h_craw.ensure((size_t)std::max(K, 1) * kConsCap), "pin");
    c->hip(c->h_over.ensure(1), "pin");
    const uint16_t* clen = c->h_clen.p;
    const char* craw = c->h_craw.p;
    if (K > 0) {
      c->hip(hipMemcpyAsync(c->h_clen.p, c->t_conslen.p, (size_t)K * 2, hipMemcpyDeviceToHost, c->st), "d2h");
      c->hip(hipMemcpyAsync(c->h_craw.p, c->t_cons.p, (size_t)K * kConsCap, hipMemcpyDeviceToHost, c->st), "d2h");
    }
    c->hip(hipMemcpyAsync(c->h_over.p, c->t_over.p, 4, hipMemcpyDeviceToHost, c->st), "d2h");
    c->hip(hipStreamSynchronize(c->st), "sync");
    const int32_t over = *c->h_over.p;
    float ms = 0;
    c->hip(hipEventElapsedTime(&ms, c->tev[0], c->tev[1]), "elapsed");
    t_cons = ms * 1e-3;
    if (over) c->fail(UMICLUST_ERANGE, "consensus: %d clusters exceed the MSA column budget", over);
    c->cons_off.assign((size_t)K + 1, 0);
    for (int32_t k = 0; k < K; k++) c->cons_off[k + 1] = c->cons_off[k] + clen[k];
    c->cons.resize((size_t)c->cons_off[K]);
    for (int32_t k = 0; k < K; k++)
      memcpy(c->cons.data() + c->cons_off[k], craw + (size_t)k * kConsCap, clen[k]);
  }
  if (!c->pack_on) {
    auto& bo = c->bout[bin];
    bo.done = true;
    bo.K = K;
    bo.cons = c->cons;
    bo.cons_off = c->cons_off;
  } else {
    // per bin: its output clusters are the consecutive output numbers [k0, k1); numbers within the bin
    int32_t k0 = 0;
    for (int32_t b = bin; b < bin + npk; b++) {
      int32_t k1 = k0;
      while (k1 < K && cbin(order[k1]) == b) k1++;
      auto& bo = c->bout[b];
      bo.done = true;
      bo.K = k1 - k0;
      bo.cons_off.assign((size_t)bo.K + 1, 0);
      for (int32_t k = 0; k <= bo.K; k++) bo.cons_off[k] = c->cons_off[k0 + k] - c->cons_off[k0];
      bo.cons.assign(c->cons.begin() + c->cons_off[k0], c->cons.begin() + c->cons_off[k1]);
      for (int32_t s = c->bin_s[b]; s < c->bin_s[b + 1]; s++) c->ocl[s] -= k0;
      k0 = k1;
    }
  }
  c->stats.n_clusters = K;
  c->stats.t_prefilter_s = t_pf;
  c->stats.t_align_s = t_al;
  c->stats.t_consensus_s = t_cons;
  c->stats.t_host_s = t_host;
  if (c->pf_prof.p) {
    unsigned long long h[24];
    c->hip(hipMemcpy(h, c->pf_prof.p, sizeof(h), hipMemcpyDeviceToHost), "d2h");
    const double nwg = h[8] ? (double)h[8] : 1.0;
    fprintf(stderr,
            "prefilter phase clocks per workgroup (%llu): query %.0f views %.0f offsets %.0f table %.0f count %.0f "
            "scan %.0f select %.0f out %.0f\n",
            h[8], h[5] / nwg, h[6] / nwg, h[7] / nwg, h[0] / nwg, h[1] / nwg, h[2] / nwg, h[3] / nwg, h[4] / nwg);
    const double nc = h[14] ? (double)h[14] : 1.0;
    fprintf(stderr,
            "k_pf_count phase clocks per workgroup (%llu sampled): zero %.0f table %.0f count %.0f scan %.0f "
            "peers+out %.0f; chunks per workgroup %.1f; table = offsets %.0f + block scan %.0f + writes\n",
            h[14], h[9] / nc, h[10] / nc, h[11] / nc, h[12] / nc, h[13] / nc, h[15] / nc, h[16] / nc, h[17] / nc);
    if (h[19])
      fprintf(stderr, "k_pf_count sampled workgroups: %.0f shader cycles in %.2f us real time = %.2f GHz in the pipeline\n",
              h[18] / nc, h[19] / nc / 100.0, (double)h[18] / ((double)h[19] / 100e6) / 1e9);
    c->hip(hipMemset(c->pf_prof.p, 0, 24 * sizeof(unsigned long long)), "memset");
  }
  c->stats.t_total_s = now_s() - t0;
  c->clustered = true;
  if (c->walk_dump && !c->wd.empty()) {
    if (FILE* f = fopen(c->walk_dump, "wb")) {
      fwrite(c->wd.data(), 2, c->wd.size(), f);
      fclose(f);
    }
    c->wd.clear();
  }
  if (getenv("UMICLUST_DEBUG"))
    fprintf(stderr, "bin %d: n %d mispredicted %lld saved(seen) %lld blocked %lld deferred %lld\n", bin, n,
            (long long)c->dbg[0], (long long)c->dbg[1], (long long)c->dbg[2], (long long)c->stats.n_deferred);
  if (getenv("UMICLUST_DEBUG"))
    fprintf(stderr, "bin %d: queries no-record %lld earlier-block-only %lld in-block %lld; pass-1 host %.3f s\n", bin,
            (long long)c->dbg_q[0], (long long)c->dbg_q[1], (long long)c->dbg_q[2], c->dbg_q[3] * 1e-9);
  if (getenv("UMICLUST_DEBUG"))
    fprintf(stderr, "bin %d: strands inline %lld many-relevant %lld record-read %lld peers-scanned %lld\n", bin,
            (long long)c->dbg_p[0], (long long)c->dbg_p[1], (long long)c->dbg_p[2], (long long)c->dbg_p[3]);
  if (getenv("UMICLUST_DEBUG"))
    fprintf(stderr, "bin %d: resolve wait %.3f hq-copy %.3f rec-copy %.3f classify %.3f in-order %.3f total %.3f s "
            "(round B and the rest %.3f: round-B round trips %.3f, rest of resolve_block %.3f, outside it %.3f)\n", bin,
            c->dbg_t[0], c->dbg_t[1], c->dbg_t[2], c->dbg_t[3], c->dbg_t[4], c->dbg_t[6],
            c->dbg_t[6] - c->dbg_t[0] - c->dbg_t[1] - c->dbg_t[2] - c->dbg_t[3] - c->dbg_t[4], c->dbg_t[8],
            c->dbg_t[9] - c->dbg_t[3] - c->dbg_t[4] - c->dbg_t[8],
            c->dbg_t[6] - c->dbg_t[0] - c->dbg_t[1] - c->dbg_t[2] - c->dbg_t[9]);
  if (getenv("UMICLUST_DEBUG"))
    fprintf(stderr, "bin %d: host: split-pass appends %.3f, enqueue (peer tiles, appends, launches) %.3f s; bin %.3f s\n",
            bin, c->dbg_t[7], c->dbg_t[5], now_s() - t0);
  if (getenv("UMICLUST_DEBUG"))
    fprintf(stderr, "bin %d: round B: %.0f round trips, %.0f launches, %.0f pairs, %.4f s between its first and last "
            "launch's events\n", bin, c->dbg_rb[1], c->dbg_rb[2], c->dbg_rb[3], c->dbg_rb[0]);
  for (double& x : c->dbg_rb) x = 0;
  for (double& x : c->dbg_t) x = 0;
  c->dbg_q[0] = c->dbg_q[1] = c->dbg_q[2] = c->dbg_q[3] = 0;
  c->dbg_p[0] = c->dbg_p[1] = c->dbg_p[2] = c->dbg_p[3] = 0;
  c->dbg[0] = c->dbg[1] = c->dbg[2] = 0;
}

// ---------------------------------------------------------------- load
// bin_in: nbins + 1 input record boundaries (NULL: one bin of all n records)
// Stage the raw records of a load in HBM (umiclust_stage): the ASCII bytes and record offsets, and the record lengths
// and bin boundaries on the host.  Nothing of A3 (length filter, sort, DUST, k-mers) happens here: that is
// prepare_impl's, from these resident records.
void stage_impl(umiclust_ctx* c, const char* seqs, const int64_t* offs, int64_t n, const int64_t* bin_in = nullptr,
                int32_t nbins = 1) {
  if ((!seqs && n > 0) || !offs || n < 0 || nbins < 1) c->fail(UMICLUST_EINVAL, "null argument");
  c->staged = false;
  c->loaded = false;
  c->clustered = false;
  c->n_input = n;
  c->bin_in.assign((size_t)nbins + 1, 0);
  if (bin_in) {
    if (bin_in[0] != 0 || bin_in[nbins] != n) c->fail(UMICLUST_EINVAL, "bin boundaries must span [0, n]");
    for (int32_t b = 0; b < nbins; b++)
      if (bin_in[b + 1] < bin_in[b]) c->fail(UMICLUST_EINVAL, "bin boundaries must not decrease");
    for (int32_t b = 0; b <= nbins; b++) c->bin_in[b] = bin_in[b];
  } else {
    c->bin_in[1] = n;
  }
  c->rec_len.resize((size_t)n);
  for (int64_t i = 0; i < n; i++) {
    const int64_t L = offs[i + 1] - offs[i];
    if (L < 0) c->fail(UMICLUST_EINVAL, "record offsets must not decrease");
    c->rec_len[i] = (uint32_t)std::min<int64_t>(L, UINT32_MAX);
  }
  const int64_t bytes = n > 0 ? offs[n] - offs[0] : 0;
  c->hip(c->d_ascii.ensure((size_t)bytes + 1), "alloc ascii");
  c->hip(c->d_offs.ensure((size_t)n + 1), "alloc offs");
  std::vector<int64_t> rel((size_t)n + 1);
  for (int64_t i = 0; i <= n; i++) rel[i] = offs[i] - offs[0];
  if (bytes > 0)
    c->hip(hipMemcpyAsync(c->d_ascii.p, seqs + offs[0], (size_t)bytes, hipMemcpyHostToDevice, c->st), "h2d");
  c->hip(hipMemcpyAsync(c->d_offs.p, rel.data(), ((size_t)n + 1) * 8, hipMemcpyHostToDevice, c->st), "h2d");
  c->hip(hipStreamSynchronize(c->st), "sync stage");  // `rel` goes out of scope
  c->staged = true;
}

// vsearch's load, length filter, DUST and length sort over the staged records
// (umiclust_prepare): the stable counting sort by length on the host (perm, hlen: the host's resolve and writers
// use them), then K1 k_prep on the device (DUST, 4-bit codes, unique 8-mers of both strands) from the resident
// ASCII.  One stream synchronisation at the end.
void prepare_impl(umiclust_ctx* c, const umiclust_params* p) {
  if (!p) c->fail(UMICLUST_EINVAL, "null argument");
  if (!c->staged) c->fail(UMICLUST_ESTATE, "umiclust_prepare before umiclust_stage");
  validate(c, *p);
  c->loaded = false;
  c->clustered = false;
  c->p = *p;
  c->sc = to_scoring(*p);
  c->both = p->strand_both ? 2 : 1;
  c->o4_T = (p->policy_threads && p->threads > 1) ? p->threads : 0;
  const double tp0 = now_s();
  build_tables(c);
  const int64_t n = c->n_input;
  const int32_t nbins = (int32_t)c->bin_in.size() - 1;
  const uint32_t* rl = c->rec_len.data();
  // length filter + stable sort by length desc within every bin (db_sortbylength; ties keep input
  // order, O1): one counting sort per bin, bins laid out one after another.  A bin of >= 256k records is sorted on
  // io_threads() threads (per-thread histograms over consecutive chunks, offsets laid out key-major then chunk-major,
  // so ties keep input order): 6.2 ms of a config-2 step's prepare on one thread
  const int64_t maxlen = std::min<int64_t>(p->maxseqlength, kMaxLen);
  if (n > (int64_t)INT32_MAX) c->fail(UMICLUST_ERANGE, "too many sequences in one load");  // perm holds int32
  c->hip(c->h_perm.ensure((size_t)n + 1), "pin perm");
  c->hlen.resize((size_t)n);
  c->bin_s.assign((size_t)nbins + 1, 0);
  int64_t kept = 0, bad = INT64_MAX;  // bad: the first input record whose length is out of range
  {
    int32_t* perm = c->h_perm.p;
    uint8_t* hl = c->hlen.data();
    const int64_t minlen = p->minseqlength, maxseq = p->maxseqlength;
    constexpr int K = kMaxLen + 1;  // key kMaxLen - L: longest first
    const int T = io_threads();
    std::vector<int64_t> hist((size_t)T * K), tbad((size_t)T);
    for (int32_t b = 0; b < nbins && bad == INT64_MAX; b++) {
      c->bin_s[b] = (int32_t)kept;
      const int64_t i0 = c->bin_in[b], m = c->bin_in[b + 1] - i0;
      const int Tb = m >= (1 << 18) ? T : 1;
      auto lo = [&](int t) { return i0 + m * t / Tb; };
      parallel_for(Tb, [&](int t) {
        int64_t* h = &hist[(size_t)t * K];
        std::fill(h, h + K, 0);
        int64_t fb = INT64_MAX;
        for (int64_t i = lo(t), e = lo(t + 1); i < e; i++) {
          const int64_t L = rl[i];
          const bool k = L >= minlen && L <= maxlen;
          if (((L > kMaxLen && L <= maxseq) || (k && L < kMinTplLen)) && fb == INT64_MAX) fb = i;
          if (k) h[kMaxLen - L]++;
        }
        tbad[t] = fb;
      });
      for (int t = 0; t < Tb; t++) bad = std::min(bad, tbad[t]);
      if (bad != INT64_MAX) break;
      for (int k = 0; k < K; k++)
        for (int t = 0; t < Tb; t++) {
          int64_t& h = hist[(size_t)t * K + k];
          const int64_t x = h;
          h = kept;
          kept += x;
        }
      parallel_for(Tb, [&](int t) {
        int64_t* h = &hist[(size_t)t * K];
        for (int64_t i = lo(t), e = lo(t + 1); i < e; i++) {
          const int64_t L = rl[i];
          if (L >= minlen && L <= maxlen) {
            const int64_t s = h[kMaxLen - L]++;
            perm[s] = (int32_t)i;
            hl[s] = (uint8_t)L;
          }
        }
      });
    }
    c->bin_s[nbins] = (int32_t)kept;
  }
  if (bad != INT64_MAX) {
    if (rl[bad] > kMaxLen) c->fail(UMICLUST_ERANGE, "sequence longer than %d", kMaxLen);
    c->fail(UMICLUST_ERANGE, "sequence shorter than %d (minseqlength)", kMinTplLen);
  }
  if (kept > (int64_t)INT32_MAX / 2) c->fail(UMICLUST_ERANGE, "too many sequences in one load");
  c->n = (int32_t)kept;
  c->hlen.resize((size_t)kept);
  const size_t ns = (size_t)c->n + 1;
  c->hip(c->d_perm.ensure(ns), "alloc perm");
  if (c->n > 0)
    c->hip(hipMemcpyAsync(c->d_perm.p, c->h_perm.p, (size_t)c->n * 4, hipMemcpyHostToDevice, c->st), "h2d");
  c->hip(c->d_codes.ensure(ns * 2 * kCodeWords), "alloc");
  c->hip(c->d_lens.ensure(ns), "alloc");
  c->hip(c->d_kmers.ensure(ns * 2 * kKmerStride), "alloc");
  c->hip(c->d_nk.ensure(ns * 2), "alloc");
  c->hip(c->d_masked.ensure(ns * kMaxLen), "alloc");
  if (c->iota_n < ns) {  // 0, 1, 2, ... (peer tiles index sequences by seqno); the same for every load
    c->hip(c->d_iota.ensure(ns), "alloc");
    c->hip(launch_iota(c->d_iota.p, (int32_t)ns, c->st), "iota");
    c->iota_n = ns;
  }
  c->hip(c->d_amb.ensure(2), "alloc");
  c->hip(c->h_amb.ensure(2), "pin");
  c->hip(hipMemsetAsync(c->d_amb.p, 0, 8, c->st), "memset");
  c->hip(c->d_mchg.ensure((size_t)std::max(c->n, 1)), "alloc");
  const double tp1 = now_s();
  c->hip(launch_prep(c->d_ascii.p, c->d_offs.p, c->d_perm.p, c->n, p->qmask_dust, c->d_codes.p,
                     c->d_lens.p, c->d_kmers.p, c->d_nk.p, c->d_masked.p, c->d_amb.p, c->st, c->d_mchg.p),
         "prep");
  c->hip(hipMemcpyAsync(c->h_amb.p, c->d_amb.p, 8, hipMemcpyDeviceToHost, c->st), "d2h");
  // the host's per-sequence state is filled while K1 runs
  c->perm.assign(c->h_perm.p, c->h_perm.p + c->n);
  c->cno.assign(c->n, -1);
  c->strand.assign(c->n, 0);
  c->target.assign(c->n, -1);
  c->ocl.assign(c->n, -1);
  c->bout.assign(nbins, umiclust_ctx::BinOut());
  c->cur_bin = -1;
  c->hqbin.clear();
  if (nbins > 1 && c->n > 0) {
    // packs: per-bin XOR masks on the k-mers (a bijection within a bin: counts within a bin are unchanged; other
    // bins' structured k-mers land on unrelated lists), sorted seqno -> bin, each bin's first seqno
    c->hqbin.resize(c->n);
    c->hip(c->h_xm.ensure((size_t)nbins), "pin");
    for (int32_t b = 0; b < nbins; b++) {
      for (int32_t s = c->bin_s[b]; s < c->bin_s[b + 1]; s++) c->hqbin[s] = b;
      uint32_t h = (uint32_t)b * 0x9E3779B1u + 0x7F4A7C15u;  // murmur3 finaliser
      h ^= h >> 16;
      h *= 0x85EBCA6Bu;
      h ^= h >> 13;
      h *= 0xC2B2AE35u;
      h ^= h >> 16;
      c->h_xm.p[b] = (uint16_t)(h ^ (h >> 16));
    }
    c->hip(c->d_qbin.ensure(c->n), "alloc");
    c->hip(c->d_bin_seq0.ensure(nbins), "alloc");
    c->hip(c->d_bin_ord0.ensure(nbins), "alloc");
    c->hip(c->h_bin_ord0.ensure(nbins), "pin");
    c->hip(c->d_xm.ensure(nbins), "alloc");
    c->hip(hipMemcpyAsync(c->d_qbin.p, c->hqbin.data(), (size_t)c->n * 4, hipMemcpyHostToDevice, c->st), "h2d");
    c->hip(hipMemcpyAsync(c->d_bin_seq0.p, c->bin_s.data(), (size_t)nbins * 4, hipMemcpyHostToDevice, c->st), "h2d");
    c->hip(hipMemcpyAsync(c->d_xm.p, c->h_xm.p, (size_t)nbins * 2, hipMemcpyHostToDevice, c->st), "h2d");
    c->hip(launch_kmer_xor(c->d_kmers.p, c->d_nk.p, c->n, c->d_qbin.p, c->d_xm.p, c->st), "k-mer masks");
  }
  const double tp2 = now_s();
  c->hip(hipStreamSynchronize(c->st), "sync load");
  if (getenv("UMICLUST_DEBUG"))
    fprintf(stderr, "umiclust: prepare: host sort %.4f s, after the K1 launch %.4f s, sync %.4f s\n", tp1 - tp0,
            tp2 - tp1, now_s() - tp2);
  c->ambig = c->h_amb.p[0] != 0;
  c->n_changed = (int64_t)c->h_amb.p[1];
  c->loaded = true;
  c->clustered = false;
}

void load_impl(umiclust_ctx* c, const umiclust_params* p, const char* seqs, const int64_t* offs, int64_t n,
               const int64_t* bin_in = nullptr, int32_t nbins = 1) {
  if (!p) c->fail(UMICLUST_EINVAL, "null argument");
  validate(c, *p);
  stage_impl(c, seqs, offs, n, bin_in, nbins);
  prepare_impl(c, p);
}

int64_t run_fasta_impl(umiclust_ctx* c, const umiclust_params* p, const char* in_fasta,
                       const char* clusters_prefix, const char* consout, const char* log_path,
                       umiclust_stats* stats, const umiclust_parse_params* pp = nullptr,
                       const char* work_dir = nullptr, umiclust_parse_result* pr = nullptr) {
  const double t0 = now_s();
  c->join_release();
  std::unique_ptr<Fasta> fin(new Fasta());
  Fasta& f = *fin;
  // output mappings handed over by the writers (released with the input; at once if the call fails)
  struct Unmaps {
    std::vector<std::pair<void*, size_t>> v;
    ~Unmaps() {
      for (auto& m : v) munmap(m.first, m.second);
    }
  } unmaps;
  if (!in_fasta || !io::read_fasta(in_fasta, f)) c->fail(UMICLUST_EIO, "cannot read %s", in_fasta ? in_fasta : "(null)");
  const int64_t n = (int64_t)f.hdr_off.size();
  for (int64_t i = 0; i < n; i++) {
    const int64_t L = f.seq_off[i + 1] - f.seq_off[i];
    if (L > kMaxLen && L <= p->maxseqlength) c->fail(UMICLUST_ERANGE, "sequence longer than %d", kMaxLen);
  }
  const double t_read = now_s() - t0;
  // the fused drop-in: the headers' fields parse_clusters needs, computed on a few host threads while the GPU
  // clusters (the resolve pool keeps the rest of the CPUs)
  std::vector<io::RecFields> pre;
  struct PreJoin {
    std::thread t;
    ~PreJoin() {
      if (t.joinable()) t.join();
    }
  } pre_th;
  if (pp) pre_th.t = std::thread([&] { io::precompute_fields(f, pre, std::max(1, std::min(4, io::host_cpus() / 4))); });
  load_impl(c, p, f.seq.data(), f.seq_off.data(), n);
  if (c->bin_s.size() != 2) c->fail(UMICLUST_EINVAL, "file path: one bin per load");
  {
    L3Pin pin(c);  // the same host placement as the session API (umiclust_cluster)
    cluster_all(c, 0);
  }
  const double t1 = now_s();
  const int32_t K = c->nclusters;
  const int width = p->fasta_width;
  const io::ClusterView cv{K, c->ostart.data(), c->omemb.data(), c->perm.data()};
  // both writers build and write disjoint cluster ranges on io_threads() threads; the consout (one file: bound by its
  // page allocation or inode lock, 0.12 s of a config-2 bin on the GPU box) is written beside the cluster<N> files
  double t_cons = 0.0;
  std::exception_ptr cons_err;
  struct Joiner {
    std::thread t;
    ~Joiner() {
      if (t.joinable()) t.join();
    }
  } cons_th;
  if (consout)
    cons_th.t = std::thread([&] {
      try {
        io::write_consout(consout, f, cv, c->cons.data(), c->cons_off.data(), p->clusterout_id != 0, width);
      } catch (...) {
        cons_err = std::current_exception();
      }
      t_cons = now_s() - t1;
    });
  double t_mask = 0.0;
  if (clusters_prefix) {
    // vsearch prints the DUST-masked (upper-cased) db sequence.  Where no sequence changed (prepare counted them:
    // nothing masked, input already upper case) that is the input's own bytes, so the 112 B-per-UMI masked
    // buffer is downloaded only when some sequence changed
    std::vector<char> masked;
    std::vector<int32_t> mrow;
    if (c->n > 0 && c->n_changed > 0) {
      const double tm = now_s();
      if (c->n_changed * 16 < c->n) {  // a few changed rows (config 2: one): their flags, then those rows alone
        std::vector<uint8_t> chg((size_t)c->n);
        c->hip(hipMemcpy(chg.data(), c->d_mchg.p, chg.size(), hipMemcpyDeviceToHost), "d2h masked flags");
        mrow.assign((size_t)c->n, -1);
        int32_t r = 0;
        for (int32_t s = 0; s < c->n; s++)
          if (chg[s]) mrow[s] = r++;
        masked.resize((size_t)r * kMaxLen);
        for (int32_t s = 0; s < c->n; s++)
          if (mrow[s] >= 0)
            c->hip(hipMemcpyAsync(masked.data() + (size_t)mrow[s] * kMaxLen, c->d_masked.p + (size_t)s * kMaxLen,
                                  kMaxLen, hipMemcpyDeviceToHost, c->st), "d2h masked row");
        c->hip(hipStreamSynchronize(c->st), "sync");
      } else {
        masked.resize((size_t)c->n * kMaxLen);
        c->hip(hipMemcpy(masked.data(), c->d_masked.p, masked.size(), hipMemcpyDeviceToHost), "d2h masked");
      }
      t_mask = now_s() - tm;
    }
    io::write_cluster_files(clusters_prefix, f, cv, masked.empty() ? nullptr : masked.data(), kMaxLen,
                            c->hlen.data(), width, mrow.empty() ? nullptr : mrow.data());
  }
  const double t_files = now_s() - t1;
  if (cons_th.t.joinable()) cons_th.t.join();
  if (cons_err) std::rethrow_exception(cons_err);
  const double t_write = now_s() - t1;
  if (getenv("UMICLUST_DEBUG"))
    fprintf(stderr, "umiclust: file path: read %.3f s, cluster %.3f s, masked download %.3f s (%lld changed), "
                    "cluster files done at %.3f s, consout (beside them) at %.3f s\n", t_read, t1 - t0 - t_read, t_mask,
            (long long)c->n_changed, t_files, t_cons);
  if (log_path) {
    const umiclust_stats& s = c->stats;
    int64_t nt = 0, singles = 0;
    int32_t smin = 0, smax = 0;
    for (int32_t x = 0; x < c->n; x++) nt += c->hlen[x];
    for (int32_t k = 0; k < K; k++) {
      const int32_t sz = c->ostart[k + 1] - c->ostart[k];
      singles += sz == 1;
      smin = k ? std::min(smin, sz) : sz;
      smax = std::max(smax, sz);
    }
    char buf[2048];
    snprintf(buf, sizeof(buf),
             "umiclust-mi355x (vsearch --cluster_fast drop-in, ABI %d)\n"
             "Reading file %s\n"
             "%lld nt in %lld seqs, min %d, max %d, avg %.0f\n"
             "%lld sequences discarded by the length window [%d, %d]\n"
             "Masking (dust), sorting by length, clustering (id %.4f, strand %s)\n"
             "Clusters: %d Size min %d, max %d, avg %.1f\n"
             "Singletons: %lld, %.1f%% of seqs, %.1f%% of clusters\n"
             "Alignments: %lld, cells: %lld, k-mer postings: %lld, blocks: %lld\n"
             "Time: read %.3f s, cluster %.3f s (prefilter %.3f, align %.3f, consensus %.3f, host %.3f), write %.3f s\n",
             UMICLUST_ABI_VERSION, in_fasta, (long long)nt, (long long)c->n,
             c->n ? (int)c->hlen[c->n - 1] : 0, c->n ? (int)c->hlen[0] : 0, c->n ? (double)nt / c->n : 0.0,
             (long long)(n - c->n), p->minseqlength, p->maxseqlength, p->id, p->strand_both ? "both" : "plus",
             K, smin, smax, K ? (double)c->n / K : 0.0, (long long)singles,
             c->n ? 100.0 * singles / c->n : 0.0, K ? 100.0 * singles / K : 0.0,
             (long long)s.n_alignments, (long long)s.cells, (long long)s.kmer_postings, (long long)s.n_blocks,
             t_read, s.t_total_s, s.t_prefilter_s, s.t_align_s, s.t_consensus_s, s.t_host_s, t_write);
    io::write_text(log_path, buf);
  }
  if (pp) {
    if (!c->p.clusterout_sort || !c->p.clusterout_id)
      c->fail(UMICLUST_EINVAL, "in-process parse needs --clusterout_sort and --clusterout_id numbering");
    const double tj = now_s();
    if (pre_th.t.joinable()) pre_th.t.join();
    if (c->debug) fprintf(stderr, "umiclust: fused: waited %.3f s for the header fields\n", now_s() - tj);
    io::parse_clusters(f, cv, pp, work_dir, pr, pre.empty() ? nullptr : pre.data(), &unmaps.v);
  }
  c->stats.t_read_s = t_read;
  c->stats.t_write_s = t_write + (pp ? now_s() - t1 - t_write : 0.0);
  // the outputs are written: the input goes on a thread of its own (UMICLUST_DEBUG prints how long it takes)
  {
    Fasta* in = fin.release();
    std::vector<std::pair<void*, size_t>> outs;
    outs.swap(unmaps.v);
    c->in_release = std::thread([in, outs] {
      const double tr = now_s();
      for (auto& m : outs) munmap(m.first, m.second);
      delete in;
      if (getenv("UMICLUST_DEBUG")) fprintf(stderr, "umiclust: file path: input released in %.3f s\n", now_s() - tr);
    });
  }
  c->stats.t_run_s = now_s() - t0;
  if (stats) *stats = c->stats;
  return K;
}

}  // namespace

// ====================================================================== C ABI
// Retired or misspelled UMICLUST_* switches fail loudly (once per process, on stderr) instead of being ignored in
// silence: every switch the library or its Python binding reads is listed here.
extern char** environ;
static void warn_unknown_env() {
  static std::once_flag once;
  std::call_once(once, [] {
    static const char* const known[] = {
        "ARRANGE", "BAND", "BAND_WPRIO", "BLOCK", "DEBUG", "IO_THREADS", "LAZY", "MIXLEN", "O4", "OVERLAP_TEST_COLLIDE", "PAR_MIN", "PF1", "PFPROBE",
        "PFPROF", "PIN", "PT_SIDE", "REC_DIRECT", "RB_DIRECT", "RB_PRIO", "RB_WPRIO", "REGROW", "REGROW_DEPTH", "RESOLVE_DUMP", "RESOLVE_THREADS", "SPLIT", "WALK_DUMP",
        // read by the Python side (umiclust/, bench.py)
        "DEVICE", "CRIT_PRIO", "PACK_READS", "BENCH_THREADS", "E2E_DIR"};
    for (char** e = environ; e && *e; e++) {
      if (strncmp(*e, "UMICLUST_", 9) != 0) continue;
      const char* name = *e + 9;
      const char* eq = strchr(name, '=');
      const size_t len = eq ? (size_t)(eq - name) : strlen(name);
      bool ok = false;
      for (const char* k : known) ok = ok || (strlen(k) == len && strncmp(k, name, len) == 0);
      if (!ok)
        fprintf(stderr, "umiclust: warning: unknown environment variable UMICLUST_%.*s ignored (retired or misspelled)\n",
                (int)len, name);
    }
  });
}

extern "C" {

int32_t umiclust_abi_version(void) { return UMICLUST_ABI_VERSION; }

int32_t umiclust_timeline(int32_t device_id, int32_t kind, int32_t reset, double* busy_s, int64_t* launches) {
  if (kind < 0 || kind > 1) return UMICLUST_EINVAL;
  std::lock_guard<std::mutex> lk(g_tl.m);
  if (reset) {
    int prev = -1;
    (void)hipGetDevice(&prev);  // the reset must not move the caller's thread to another device
    if (hipSetDevice(device_id) != hipSuccess) return UMICLUST_EDEVICE;
    if (g_tl.ref && g_tl.dev != device_id) {
      (void)hipEventDestroy(g_tl.ref);
      g_tl.ref = nullptr;
    }
    int32_t rc = 0;
    if (!g_tl.ref && hipEventCreate(&g_tl.ref) != hipSuccess) {
      g_tl.ref = nullptr;
      rc = UMICLUST_EDEVICE;
    }
    if (rc == 0 && (hipEventRecord(g_tl.ref, nullptr) != hipSuccess || hipEventSynchronize(g_tl.ref) != hipSuccess))
      rc = UMICLUST_EDEVICE;
    if (prev >= 0) (void)hipSetDevice(prev);
    if (rc) return rc;
    g_tl.dev = device_id;
    for (int k = 0; k < 2; k++) {
      g_tl.iv[k].clear();
      g_tl.folded_ms[k] = 0.0;
      g_tl.fold_hi[k] = -1e30f;
      g_tl.n[k] = 0;
    }
  }
  std::vector<std::pair<float, float>> v = g_tl.iv[kind];
  const double tot = g_tl.folded_ms[kind] + tl_merge(v);
  if (busy_s) *busy_s = tot * 1e-3;
  if (launches) *launches = g_tl.n[kind];
  return 0;
}


// The alignment stream is created with the device's greatest stream priority: a pass's walk/align/pack chain gates
// the host's resolution of its block and through it the next passes.  A prioritised stream also gets a hardware
// queue of its own class instead of sharing the normal-priority queues with the other lanes' streams (config 3, 4
// lanes on one MI355X: 1.73 -> 3.1 M UMIs/s; least priority or a plain stream measured no better, round 4
// al_prio_ab/; a CU-masked stream slower, cumask_early_ab/).
static int al_priority() {
  int lo = 0, hi = 0;
  if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) return 0;
  if (getenv("UMICLUST_DEBUG")) fprintf(stderr, "stream priorities: least %d greatest %d\n", lo, hi);
  return hi;
}

// the copy stream carries round B (the host waits for it): at the greatest priority with UMICLUST_RB_PRIO=1
static hipError_t create_copy_stream(umiclust_ctx* c) {
  const char* e = getenv("UMICLUST_RB_PRIO");
  if (e && atoi(e) > 0) return hipStreamCreateWithPriority(&c->st_copy, hipStreamNonBlocking, al_priority());
  return hipStreamCreateWithFlags(&c->st_copy, hipStreamNonBlocking);
}

static hipError_t create_al_stream(umiclust_ctx* c) {
  return hipStreamCreateWithPriority(&c->st_al, hipStreamNonBlocking, al_priority());
}

umiclust_ctx* umiclust_create(int32_t device_id, int32_t* err) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || device_id < 0 || device_id >= ndev) {
    if (err) *err = UMICLUST_EDEVICE;
    return nullptr;
  }
  umiclust_ctx* c = new (std::nothrow) umiclust_ctx();
  if (!c) {
    if (err) *err = UMICLUST_ENOMEM;
    return nullptr;
  }
  c->dev = device_id;
  if (hipSetDevice(device_id) != hipSuccess || hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&c->st_b, hipStreamNonBlocking) != hipSuccess ||
      create_copy_stream(c) != hipSuccess || create_al_stream(c) != hipSuccess ||
      hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess ||
      hipEventCreate(&c->evb[0]) != hipSuccess || hipEventCreate(&c->evb[1]) != hipSuccess || [&] {
        for (Pass& P : c->pass)
          for (hipEvent_t& e : P.ev)
            if (hipEventCreate(&e) != hipSuccess) return true;
        return false;
      }()) {
    delete c;
    if (err) *err = UMICLUST_EDEVICE;
    return nullptr;
  }
  warn_unknown_env();
  if (const char* e = getenv("UMICLUST_BAND")) c->band_pairs = std::max(0, atoi(e));
  if (const char* e = getenv("UMICLUST_MIXLEN")) c->mix_len = atoi(e) != 0 ? 1 : 0;
  if (const char* e = getenv("UMICLUST_PAR_MIN")) c->par_min = std::max(1, atoi(e));
  if (const char* e = getenv("UMICLUST_PF1")) c->pf1_lds = std::max(0, atoi(e));
  if (const char* e = getenv("UMICLUST_REGROW")) c->regrow = std::max(0, atoi(e));
  if (const char* e = getenv("UMICLUST_ARRANGE")) c->arrange = atoi(e) & 3;
  if (const char* e = getenv("UMICLUST_PT_SIDE")) c->pt_side = std::max(0, std::min(2, atoi(e)));
  if (const char* e = getenv("UMICLUST_LAZY")) c->lazy_permille = std::max(0, std::min(1000, atoi(e)));
  if (const char* e = getenv("UMICLUST_RB_DIRECT")) c->rb_direct = std::max(0, atoi(e));
  if (const char* e = getenv("UMICLUST_RB_WPRIO")) c->rb_wprio = atoi(e) > 0 ? 1 : 0;
  if (const char* e = getenv("UMICLUST_REGROW_DEPTH")) c->regrow_depth = std::max(1, std::min(kPeerCap + 1, atoi(e)));
  if (const char* e = getenv("LOCAL_WORLD_SIZE")) c->pin = atoi(e) <= 1;
  if (const char* e = getenv("UMICLUST_PIN")) {
    c->pin = atoi(e) != 0;
    c->pin_forced = atoi(e) == 1;
  }
  io::set_live_contexts(++g_live_ctx);
  if (const char* e = getenv("UMICLUST_SPLIT")) c->split_env = atoi(e) != 0 ? 1 : 0;
  if (const char* e = getenv("UMICLUST_RESOLVE_THREADS")) c->resolve_threads = std::max(1, std::min(16, atoi(e)));
  if (const char* b = getenv("UMICLUST_BLOCK")) {
    c->block_size = std::max(1, std::min(kTile, atoi(b)));
    c->block_div = 0;
  }
  if (getenv("UMICLUST_PFPROF")) {
    if (c->pf_prof.ensure(24) != hipSuccess || hipMemset(c->pf_prof.p, 0, 24 * sizeof(unsigned long long)) != hipSuccess) {
      delete c;
      if (err) *err = UMICLUST_EDEVICE;
      return nullptr;
    }
  }
  if (err) *err = UMICLUST_OK;
  return c;
}

int32_t umiclust_set_priority(umiclust_ctx* c, int32_t level) {
  if (!c || level < -1 || level > 1) return UMICLUST_EINVAL;
  if (hipSetDevice(c->dev) != hipSuccess || hipStreamSynchronize(c->st) != hipSuccess) return UMICLUST_EDEVICE;
  // level -1 (background): the alignment stream loses its priority too; 0 / 1 give it back
  const int al = level < 0 ? -1 : 0;
  if (al != c->al_level) {
    hipStream_t s = nullptr;
    if (hipStreamSynchronize(c->st_al) != hipSuccess ||
        (al < 0 ? hipStreamCreateWithFlags(&s, hipStreamNonBlocking)
                : hipStreamCreateWithPriority(&s, hipStreamNonBlocking, al_priority())) != hipSuccess)
      return UMICLUST_EDEVICE;
    (void)hipStreamDestroy(c->st_al);
    c->st_al = s;
    c->al_level = al;
  }
  c->prio_user = level < 0 ? 0 : level;
  return main_stream_priority(c, c->prio_user) == hipSuccess ? UMICLUST_OK : UMICLUST_EDEVICE;
}

int32_t umiclust_wait_host(umiclust_ctx* c) {
  if (!c) return UMICLUST_EINVAL;
  c->join_release();
  return UMICLUST_OK;
}

void umiclust_destroy(umiclust_ctx* c) {
  if (!c) return;
  c->join_release();
  io::set_live_contexts(--g_live_ctx);
  (void)hipSetDevice(c->dev);
  for (Tile* t : c->tiles) delete t;
  c->tiles.clear();
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  for (hipEvent_t e : c->evb)
    if (e) (void)hipEventDestroy(e);
  for (auto& e : c->ix_events) {
    (void)hipEventDestroy(e.first);
    (void)hipEventDestroy(e.second);
  }
  if (c->st_b) (void)hipStreamDestroy(c->st_b);
  if (c->pt_ev) (void)hipEventDestroy(c->pt_ev);
  if (c->st_copy) (void)hipStreamDestroy(c->st_copy);
  if (c->st_al) (void)hipStreamDestroy(c->st_al);
  if (c->ix_done) (void)hipEventDestroy(c->ix_done);
  for (auto& r : c->a_ev)
    for (hipEvent_t e : r)
      if (e) (void)hipEventDestroy(e);
  if (c->st) (void)hipStreamDestroy(c->st);
  delete c;
}

const char* umiclust_last_error(const umiclust_ctx* c) { return c ? c->err.c_str() : "null context"; }

#define UC_GUARD(c, ...)                                \
  do {                                                  \
    if (!(c)) return UMICLUST_EINVAL;                   \
    try {                                               \
      (void)hipSetDevice((c)->dev);                     \
      __VA_ARGS__                                       \
    } catch (const Fail& f__) {                         \
      return f__.code;                                  \
    } catch (const uc::io::IoError& e__) {              \
      (c)->err = e__.msg;                               \
      return e__.code;                                  \
    } catch (const std::bad_alloc&) {                   \
      (c)->err = "host allocation failed";              \
      return UMICLUST_ENOMEM;                           \
    } catch (...) {                                     \
      (c)->err = "unexpected exception";                \
      return UMICLUST_EDEVICE;                          \
    }                                                   \
  } while (0)

int64_t umiclust_run_fasta(umiclust_ctx* c, const umiclust_params* p, const char* in_fasta,
                           const char* clusters_prefix, const char* consout, const char* log_path,
                           umiclust_stats* stats) {
  UC_GUARD(c, {
    if (!p) c->fail(UMICLUST_EINVAL, "null params");
    return run_fasta_impl(c, p, in_fasta, clusters_prefix, consout, log_path, stats);
  });
}

int64_t umiclust_run_fasta_parse(umiclust_ctx* c, const umiclust_params* p, const char* in_fasta,
                                 const char* clusters_prefix, const char* consout, const char* log_path,
                                 const umiclust_parse_params* pp, const char* work_dir,
                                 umiclust_parse_result* result, umiclust_stats* stats) {
  UC_GUARD(c, {
    if (!p || !pp || !result) c->fail(UMICLUST_EINVAL, "null params");
    if (!p->clusterout_sort || !p->clusterout_id)
      c->fail(UMICLUST_EINVAL, "in-process parse needs --clusterout_sort and --clusterout_id numbering");
    if (pp->max_reads_per_cluster < 0 || pp->min_reads_per_cluster < 0) c->fail(UMICLUST_EINVAL, "read caps");
    return run_fasta_impl(c, p, in_fasta, clusters_prefix, consout, log_path, stats, pp, work_dir, result);
  });
}

int64_t umiclust_run_argv(umiclust_ctx* c, int32_t argc, const char* const* argv, umiclust_stats* stats) {
  UC_GUARD(c, {
    umiclust_params p;
    std::vector<char> in(4096), cl(4096), co(4096), lg(4096);
    int32_t rc = umiclust_params_from_argv(&p, argc, argv, in.data(), cl.data(), co.data(), lg.data(), 4096);
    if (rc != UMICLUST_OK) c->fail(rc, "cannot parse vsearch argv");
    return run_fasta_impl(c, &p, in.data(), cl[0] ? cl.data() : nullptr, co[0] ? co.data() : nullptr,
                          lg[0] ? lg.data() : nullptr, stats);
  });
}

int32_t umiclust_load(umiclust_ctx* c, const umiclust_params* p, const char* seqs, const int64_t* offs,
                      int64_t n) {
  UC_GUARD(c, {
    for (int64_t i = 0; i < n; i++) {
      const int64_t L = offs[i + 1] - offs[i];
      if (p && L > kMaxLen && L <= p->maxseqlength) c->fail(UMICLUST_ERANGE, "sequence longer than %d", kMaxLen);
    }
    load_impl(c, p, seqs, offs, n);
    return UMICLUST_OK;
  });
}


int64_t umiclust_cluster(umiclust_ctx* c, umiclust_stats* stats) {
  UC_GUARD(c, {
    if (!c->loaded) c->fail(UMICLUST_ESTATE, "umiclust_cluster before umiclust_load");
    if (c->bin_s.size() != 2) c->fail(UMICLUST_EINVAL, "umiclust_cluster: the load holds several bins");
    L3Pin pin(c);
    cluster_all(c, 0);
    if (stats) *stats = c->stats;
    return c->nclusters;
  });
}

int64_t umiclust_fetch(umiclust_ctx* c, int32_t* cluster, uint8_t* strand, uint8_t* centroid, char* cons,
                       int64_t cons_cap, int64_t* cons_off) {
  if (!c) return UMICLUST_EINVAL;
  if (c->bin_s.size() != 2) {
    c->err = "umiclust_fetch: the load holds several bins (umiclust_fetch_bin)";
    return UMICLUST_EINVAL;
  }
  return umiclust_fetch_bin(c, 0, cluster, strand, centroid, cons, cons_cap, cons_off);
}

int64_t umiclust_fetch_bin(umiclust_ctx* c, int32_t bin, int32_t* cluster, uint8_t* strand, uint8_t* centroid,
                           char* cons, int64_t cons_cap, int64_t* cons_off) {
  UC_GUARD(c, {
    if (!c->loaded || bin < 0 || bin >= (int32_t)c->bout.size())
      c->fail(c->loaded ? UMICLUST_EINVAL : UMICLUST_ESTATE, "umiclust_fetch_bin: no such bin");
    const auto& bo = c->bout[bin];
    if (!bo.done) c->fail(UMICLUST_ESTATE, "umiclust_fetch_bin before the bin was clustered");
    const int64_t i0 = c->bin_in[bin], n = c->bin_in[bin + 1] - i0;
    if (cluster)
      for (int64_t i = 0; i < n; i++) cluster[i] = -1;
    if (strand) memset(strand, 0, (size_t)n);
    if (centroid) memset(centroid, 0, (size_t)n);
    for (int32_t s = c->bin_s[bin]; s < c->bin_s[bin + 1]; s++) {
      const int64_t i = c->perm[s] - i0;
      if (cluster) cluster[i] = c->ocl[s];
      if (strand) strand[i] = c->strand[s];
      if (centroid) centroid[i] = c->target[s] < 0 ? 1 : 0;
    }
    const int32_t K = bo.K;
    if (cons_off)
      for (int32_t k = 0; k <= K; k++) cons_off[k] = bo.cons_off[k];
    if (cons) {
      if ((int64_t)bo.cons.size() > cons_cap) c->fail(UMICLUST_EINVAL, "consensus buffer too small");
      memcpy(cons, bo.cons.data(), bo.cons.size());
    }
    return K;
  });
}

int32_t umiclust_stage(umiclust_ctx* c, const char* seqs, const int64_t* offs, int64_t n, const int64_t* bin_start,
                       int32_t nbins) {
  UC_GUARD(c, {
    stage_impl(c, seqs, offs, n, bin_start, bin_start ? nbins : 1);
    return UMICLUST_OK;
  });
}

int32_t umiclust_prepare(umiclust_ctx* c, const umiclust_params* p) {
  UC_GUARD(c, {
    prepare_impl(c, p);
    return UMICLUST_OK;
  });
}

int32_t umiclust_load_bins(umiclust_ctx* c, const umiclust_params* p, const char* seqs, const int64_t* offs,
                           int64_t n, const int64_t* bin_start, int32_t nbins) {
  UC_GUARD(c, {
    if (!bin_start || nbins < 1) c->fail(UMICLUST_EINVAL, "bin boundaries");
    load_impl(c, p, seqs, offs, n, bin_start, nbins);
    return UMICLUST_OK;
  });
}

int64_t umiclust_cluster_bin(umiclust_ctx* c, int32_t bin, umiclust_stats* stats) {
  UC_GUARD(c, {
    if (!c->loaded) c->fail(UMICLUST_ESTATE, "umiclust_cluster_bin before umiclust_load_bins");
    L3Pin pin(c);  // only with one live context (a bin-set runner's lanes each own one: then it stays off)
    cluster_all(c, bin, true);
    if (stats) *stats = c->stats;
    return c->nclusters;
  });
}

int64_t umiclust_cluster_pack(umiclust_ctx* c, int32_t first, int32_t nbins, umiclust_stats* stats) {
  UC_GUARD(c, {
    if (!c->loaded) c->fail(UMICLUST_ESTATE, "umiclust_cluster_pack before umiclust_load_bins");
    L3Pin pin(c);
    cluster_all(c, first, true, nbins);
    if (stats) *stats = c->stats;
    return c->nclusters;
  });
}

int32_t umiclust_align_pairs(umiclust_ctx* c, const umiclust_params* p, const char* q, const int64_t* q_off,
                             const char* t, const int64_t* t_off, int64_t npairs, int32_t* score,
                             int32_t* matches, int32_t* internal_len, char* cigar_ops, int32_t ops_stride,
                             int32_t* ops_len) {
  UC_GUARD(c, {
    if (!p || npairs < 0 || (npairs > 0 && (!q || !q_off || !t || !t_off))) c->fail(UMICLUST_EINVAL, "null argument");
    umiclust_params pp = *p;
    pp.minseqlength = 1;
    pp.maxseqlength = kMaxLen;
    validate(c, pp);
    // load queries then targets as one sequence set without filtering/sorting
    std::vector<char> all;
    std::vector<int64_t> off;
    off.push_back(0);
    for (int64_t k = 0; k < npairs; k++) {
      all.insert(all.end(), q + q_off[k], q + q_off[k + 1]);
      off.push_back((int64_t)all.size());
    }
    for (int64_t k = 0; k < npairs; k++) {
      all.insert(all.end(), t + t_off[k], t + t_off[k + 1]);
      off.push_back((int64_t)all.size());
    }
    const int64_t ns = 2 * npairs;
    for (int64_t i = 0; i < ns; i++)
      if (off[i + 1] - off[i] < 1 || off[i + 1] - off[i] > kMaxLen) c->fail(UMICLUST_ERANGE, "pair sequence length");
    Scoring sc = to_scoring(pp);
    DevBuf<char> d_a;
    DevBuf<int64_t> d_o;
    DevBuf<uint32_t> d_codes, d_pq, d_pt, d_out;
    DevBuf<uint8_t> d_lens, d_nk, d_ops;
    DevBuf<uint16_t> d_km, d_nops;
    c->hip(d_a.ensure(all.size() + 1), "alloc");
    c->hip(d_o.ensure(off.size()), "alloc");
    c->hip(d_codes.ensure((size_t)ns * 2 * kCodeWords + 1), "alloc");
    c->hip(d_lens.ensure((size_t)ns + 1), "alloc");
    c->hip(d_km.ensure((size_t)ns * 2 * kKmerStride + 1), "alloc");
    c->hip(d_nk.ensure((size_t)ns * 2 + 1), "alloc");
    if (!all.empty()) c->hip(hipMemcpy(d_a.p, all.data(), all.size(), hipMemcpyHostToDevice), "h2d");
    c->hip(hipMemcpy(d_o.p, off.data(), off.size() * 8, hipMemcpyHostToDevice), "h2d");
    DevBuf<uint32_t> d_amb;
    c->hip(d_amb.ensure(1), "alloc");
    c->hip(hipMemsetAsync(d_amb.p, 0, 4, c->st), "memset");
    c->hip(launch_prep(d_a.p, d_o.p, nullptr, (int32_t)ns, 0, d_codes.p, d_lens.p, d_km.p, d_nk.p, nullptr,
                       d_amb.p, c->st),
           "prep");
    uint32_t amb = 0;
    c->hip(hipMemcpyAsync(&amb, d_amb.p, 4, hipMemcpyDeviceToHost, c->st), "d2h");
    c->hip(hipStreamSynchronize(c->st), "sync");
    // pairs grouped by query length (the aligner is compiled per query length)
    std::vector<int64_t> ord(npairs);
    for (int64_t k = 0; k < npairs; k++) {
      ord[k] = k;
      const int64_t ql = off[k + 1] - off[k];
      if (ql < kMinTplLen) c->fail(UMICLUST_ERANGE, "query shorter than %d", kMinTplLen);
    }
    std::stable_sort(ord.begin(), ord.end(), [&](int64_t a, int64_t b) {
      return (off[a + 1] - off[a]) < (off[b + 1] - off[b]);
    });
    std::vector<uint32_t> pq(npairs), pt(npairs);
    for (int64_t x = 0; x < npairs; x++) {
      pq[x] = (uint32_t)ord[x] << 1;
      pt[x] = (uint32_t)(npairs + ord[x]);
    }
    c->hip(d_pq.ensure(npairs + 1), "alloc");
    c->hip(d_pt.ensure(npairs + 1), "alloc");
    c->hip(d_out.ensure(npairs + 1), "alloc");
    if (npairs > 0) {
      c->hip(hipMemcpyAsync(d_pq.p, pq.data(), npairs * 4, hipMemcpyHostToDevice, c->st), "h2d");
      c->hip(hipMemcpyAsync(d_pt.p, pt.data(), npairs * 4, hipMemcpyHostToDevice, c->st), "h2d");
    }
    DevSeqs ds{d_codes.p, d_lens.p, d_km.p, d_nk.p};
    std::vector<uint32_t> sres(npairs);
    std::vector<uint8_t> ops;
    std::vector<uint16_t> nops;
    if (cigar_ops) {
      if (ops_stride < kOpsStride) c->fail(UMICLUST_EINVAL, "ops_stride < %d", kOpsStride);
      c->hip(d_ops.ensure((size_t)npairs * kOpsStride + 1), "alloc");
      c->hip(d_nops.ensure(npairs + 1), "alloc");
    }
    for (int64_t b0 = 0; b0 < npairs;) {
      const int32_t ql = (int32_t)(off[ord[b0] + 1] - off[ord[b0]]);
      int64_t e = b0 + 1;
      while (e < npairs && off[ord[e] + 1] - off[ord[e]] == ql) e++;
      if (cigar_ops)
        c->hip(launch_traceback(ds, d_pq.p + b0, d_pt.p + b0, (int32_t)(e - b0), sc, d_ops.p + (size_t)b0 * kOpsStride,
                                d_nops.p + b0, d_out.p + b0, c->st, kMaxLen),
               "traceback");
      else
        c->hip(launch_align(ds, ql, amb != 0, d_pq.p + b0, d_pt.p + b0, (int32_t)(e - b0), nullptr, nullptr, sc,
                            d_out.p + b0, c->st, c->band_pairs),
               "align");
      b0 = e;
    }
    if (npairs > 0)
      c->hip(hipMemcpyAsync(sres.data(), d_out.p, (size_t)npairs * 4, hipMemcpyDeviceToHost, c->st), "d2h");
    if (cigar_ops) {
      ops.resize((size_t)npairs * kOpsStride);
      nops.resize(npairs);
      c->hip(hipMemcpyAsync(ops.data(), d_ops.p, ops.size(), hipMemcpyDeviceToHost, c->st), "d2h");
      c->hip(hipMemcpyAsync(nops.data(), d_nops.p, (size_t)npairs * 2, hipMemcpyDeviceToHost, c->st), "d2h");
    }
    c->hip(hipStreamSynchronize(c->st), "sync");
    std::vector<uint32_t> res(npairs);
    for (int64_t x = 0; x < npairs; x++) {
      const int64_t k = ord[x];
      res[k] = sres[x];
      if (cigar_ops) {
        const int n = nops[x];
        memcpy(cigar_ops + (size_t)k * ops_stride, ops.data() + (size_t)x * kOpsStride + kOpsStride - n, (size_t)n);
        if (ops_len) ops_len[k] = n;
      }
    }
    for (int64_t k = 0; k < npairs; k++) {
      if (matches) matches[k] = (int32_t)(res[k] & 0xffu);
      if (internal_len) internal_len[k] = (int32_t)((res[k] >> 8) & 0xffu);
      if (score) score[k] = (int32_t)(int16_t)(res[k] >> 16);
    }
    return UMICLUST_OK;
  });
}

// ---------------------------------------------------------------- region overlap (§8f f3)
namespace {
// n sequences of nreg regions on the device, one table pass (re-seeded on a 64-bit hash collision)
struct OvRun {
  DevBuf<char> d_seq;
  DevBuf<int64_t> d_off, d_rs, d_slot;
  DevBuf<uint64_t> d_hash;
  DevBuf<int32_t> d_reg;
  DevBuf<unsigned long long> d_keys, d_rep;
  DevBuf<uint32_t> d_cnt, d_start, d_cursor, d_bsum, d_members, d_coll, d_big, d_nbig;
  OvBuffers B{};
  uint64_t mask = 0;
};

void overlap_table(umiclust_ctx* c, OvRun& R, const char* seqs, const int64_t* offs, int64_t n,
                   const int64_t* rstart, int32_t nreg, bool csr) {
  if (n < 0 || nreg < 1 || (n > 0 && (!seqs || !offs)) || !rstart) c->fail(UMICLUST_EINVAL, "null argument");
  if (rstart[0] != 0 || rstart[nreg] != n) c->fail(UMICLUST_EINVAL, "region boundaries must span [0, n]");
  for (int32_t r = 0; r < nreg; r++)
    if (rstart[r + 1] < rstart[r]) c->fail(UMICLUST_EINVAL, "region boundaries must not decrease");
  if (n > (int64_t)UINT32_MAX / 2) c->fail(UMICLUST_ERANGE, "too many sequences");
  uint64_t m = 1024;
  while (m < (uint64_t)(2 * n)) m <<= 1;
  R.mask = m - 1;
  const int64_t bytes = n > 0 ? offs[n] - offs[0] : 0;
  std::vector<int64_t> rel((size_t)n + 1);
  for (int64_t i = 0; i <= n; i++) rel[i] = n > 0 ? offs[i] - offs[0] : 0;
  c->hip(R.d_seq.ensure((size_t)bytes + 1), "alloc");
  c->hip(R.d_off.ensure((size_t)n + 1), "alloc");
  c->hip(R.d_rs.ensure((size_t)nreg + 1), "alloc");
  c->hip(R.d_slot.ensure((size_t)n + 1), "alloc");
  c->hip(R.d_hash.ensure((size_t)n + 1), "alloc");
  c->hip(R.d_reg.ensure((size_t)n + 1), "alloc");
  c->hip(R.d_keys.ensure(m), "alloc");
  c->hip(R.d_rep.ensure(m), "alloc");
  c->hip(R.d_cnt.ensure(m), "alloc");
  c->hip(R.d_start.ensure(m + 1), "alloc");
  c->hip(R.d_cursor.ensure(m), "alloc");
  c->hip(R.d_bsum.ensure(m / 1024 + 1), "alloc");
  c->hip(R.d_members.ensure((size_t)n + 1), "alloc");
  c->hip(R.d_coll.ensure(1), "alloc");
  c->hip(R.d_big.ensure((size_t)n / (kOvSmallBucket + 1) + 1), "alloc");
  c->hip(R.d_nbig.ensure(1), "alloc");
  if (bytes > 0) c->hip(hipMemcpyAsync(R.d_seq.p, seqs + offs[0], (size_t)bytes, hipMemcpyHostToDevice, c->st), "h2d");
  c->hip(hipMemcpyAsync(R.d_off.p, rel.data(), rel.size() * 8, hipMemcpyHostToDevice, c->st), "h2d");
  c->hip(hipMemcpyAsync(R.d_rs.p, rstart, ((size_t)nreg + 1) * 8, hipMemcpyHostToDevice, c->st), "h2d");
  R.B = OvBuffers{R.d_hash.p, R.d_reg.p, R.d_keys.p, R.d_rep.p, R.d_slot.p, R.d_cnt.p, R.d_start.p, R.d_cursor.p,
                  R.d_bsum.p, R.d_members.p, R.d_coll.p, R.d_big.p, R.d_nbig.p};
  // a 64-bit collision between two different sequences is detected exactly; the next seed is tried
  const uint64_t seeds[4] = {0x243f6a8885a308d3ull, 0x13198a2e03707344ull, 0xa4093822299f31d0ull,
                             0x082efa98ec4e6c89ull};
  const bool test_collide = getenv("UMICLUST_OVERLAP_TEST_COLLIDE") != nullptr;  // first pass: 8-bit hashes
  for (int k = 0; k < 4; k++) {
    uint32_t coll = 0;
    const uint64_t hmask = (test_collide && k == 0) ? 0xffull : ~0ull;
    c->hip(launch_overlap_table(R.d_seq.p, R.d_off.p, n, R.d_rs.p, nreg, seeds[k], hmask, R.mask, R.B, csr, &coll,
                                c->st),
           "overlap table");
    c->stats.n_overlap_passes++;
    if (!coll) return;
  }
  c->fail(UMICLUST_EDEVICE, "overlap: 64-bit hash collisions under four seeds");
}
}  // namespace

int32_t umiclust_overlap_counts(umiclust_ctx* c, const char* s1, const int64_t* off1, int64_t n1, const char* s2,
                                const int64_t* off2, int64_t n2, int64_t* counts) {
  UC_GUARD(c, {
    if (n1 < 0 || n2 < 0 || (n1 > 0 && (!s1 || !off1 || !counts)) || (n2 > 0 && (!s2 || !off2)))
      c->fail(UMICLUST_EINVAL, "null argument");
    // one buffer: set 1 then set 2
    std::vector<char> all;
    std::vector<int64_t> off{0};
    for (int64_t i = 0; i < n1; i++) {
      all.insert(all.end(), s1 + off1[i], s1 + off1[i + 1]);
      off.push_back((int64_t)all.size());
    }
    for (int64_t i = 0; i < n2; i++) {
      all.insert(all.end(), s2 + off2[i], s2 + off2[i + 1]);
      off.push_back((int64_t)all.size());
    }
    const int64_t n = n1 + n2, rs[3] = {0, n1, n};
    OvRun R;
    overlap_table(c, R, all.data(), off.data(), n, rs, 2, false);
    DevBuf<int64_t> d_counts;
    c->hip(d_counts.ensure((size_t)n1 + 1), "alloc");
    c->hip(launch_overlap_two(R.B, R.mask, n, n1, d_counts.p, c->st), "overlap counts");
    if (n1 > 0) c->hip(hipMemcpyAsync(counts, d_counts.p, (size_t)n1 * 8, hipMemcpyDeviceToHost, c->st), "d2h");
    c->hip(hipStreamSynchronize(c->st), "sync");
    return UMICLUST_OK;
  });
}

int32_t umiclust_overlap_regions(umiclust_ctx* c, const char* seqs, const int64_t* offs, int64_t n,
                                 const int64_t* region_start, int32_t nregions, int64_t* total, int32_t* maxcount) {
  UC_GUARD(c, {
    if (nregions < 1 || nregions > UMICLUST_OVERLAP_MAX_REGIONS || !total || !maxcount)
      c->fail(UMICLUST_EINVAL, "1..%d regions and both outputs required", UMICLUST_OVERLAP_MAX_REGIONS);
    OvRun R;
    overlap_table(c, R, seqs, offs, n, region_start, nregions, true);
    const size_t cells = (size_t)nregions * nregions;
    DevBuf<unsigned long long> d_total;
    DevBuf<uint32_t> d_max;
    c->hip(d_total.ensure(cells), "alloc");
    c->hip(d_max.ensure(cells), "alloc");
    c->hip(hipMemsetAsync(d_total.p, 0, cells * 8, c->st), "memset");
    c->hip(hipMemsetAsync(d_max.p, 0, cells * 4, c->st), "memset");
    if (n > 0) c->hip(launch_overlap_pairs(R.B, R.mask, nregions, d_total.p, d_max.p, c->st), "overlap pairs");
    std::vector<uint32_t> mx(cells);
    c->hip(hipMemcpyAsync(total, d_total.p, cells * 8, hipMemcpyDeviceToHost, c->st), "d2h");
    c->hip(hipMemcpyAsync(mx.data(), d_max.p, cells * 4, hipMemcpyDeviceToHost, c->st), "d2h");
    c->hip(hipStreamSynchronize(c->st), "sync");
    for (size_t x = 0; x < cells; x++) maxcount[x] = (int32_t)mx[x];
    return UMICLUST_OK;
  });
}

// ---------------------------------------------------------------- UMI extraction (§8f f1)
namespace {
// additionalEqualities of extract_umis.py:26-87 (either order), plus identity
constexpr const char* kIupacEq[] = {"MA", "MC", "RA", "RG", "WA", "WT", "SC", "SG", "YC", "YT", "KG", "KT", "VA", "VC",
                                "VG", "HA", "HC", "HT", "DA", "DG", "DT", "BC", "BG", "BT", "NA", "NC", "NG", "NT",
                                "ma", "mc", "ra", "rg", "wa", "wt", "sc", "sg", "yc", "yt", "kg", "kt", "va", "vc",
                                "vg", "ha", "hc", "ht", "da", "dg", "dt", "bc", "bg", "bt", "na", "nc", "ng", "nt",
                                "aA", "cC", "tT", "gG"};

// symbol equality of edlib with the reference's additionalEqualities, built at compile time (constant
// initialisation: contexts on different threads share it without a lazy first-use race)
struct EqTable {
  bool eq[256][256];
};
constexpr EqTable make_eq_table() {
  EqTable t{};
  for (int a = 0; a < 256; a++)
    for (int b = 0; b < 256; b++) t.eq[a][b] = a == b;
  for (const char* e : kIupacEq) {
    t.eq[(uint8_t)e[0]][(uint8_t)e[1]] = true;
    t.eq[(uint8_t)e[1]][(uint8_t)e[0]] = true;
  }
  return t;
}
constexpr EqTable kEqTable = make_eq_table();

void build_patterns(umiclust_ctx* c, const char* fwd, const char* rev, ExtractPatterns& P) {
  const auto& eqt = kEqTable.eq;
  memset(&P, 0, sizeof(P));
  const char* pats[2] = {fwd, rev};
  for (int w = 0; w < 2; w++) {
    if (!pats[w]) c->fail(UMICLUST_EINVAL, "null pattern");
    const int m = (int)strlen(pats[w]);
    if (m < 1 || m > 64) c->fail(UMICLUST_EINVAL, "UMI patterns of 1..64 symbols are supported (got %d)", m);
    P.m[w] = m;
    for (int ch = 0; ch < 256; ch++)
      for (int i = 0; i < m; i++) {
        if (eqt[(uint8_t)pats[w][i]][ch]) P.peq[w][ch] |= 1ull << i;
        if (eqt[(uint8_t)pats[w][m - 1 - i]][ch]) P.peqr[w][ch] |= 1ull << i;
      }
  }
}

void extract_device(umiclust_ctx* c, const char* seqs, const int64_t* offs, int64_t n, int32_t a5, int32_t a3,
                    int32_t k, const char* fwd, const char* rev, int32_t* out) {
  if (n < 0 || (n > 0 && (!seqs || !offs || !out)) || a5 < 0 || a3 < 0 || k < 0)
    c->fail(UMICLUST_EINVAL, "bad argument");
  ExtractPatterns P;
  build_patterns(c, fwd, rev, P);
  if (n == 0) return;
  // Only the adapter windows are read: with short windows the host gathers them (its threads, into pinned
  // memory) and the device gets ~141 B per read instead of the whole read
  const int32_t S = (a5 + a3 + 3) & ~3;
  if (a3 > 0 && a5 + a3 > 0 && S <= kExMaxSlot && a5 <= 255 && a3 <= 255) {
    PinBuf<char>& hw = c->ex_win;
    PinBuf<uint8_t>& hl = c->ex_len;
    c->hip(hw.ensure((size_t)n * S + 16), "alloc pinned");
    c->hip(hl.ensure((size_t)n * 2), "alloc pinned");
    const int T = n < 65536 ? 1 : io_threads();
    parallel_for(T, [&](int t) {
      const int64_t lo = n * t / T, hi = n * (t + 1) / T;
      for (int64_t i = lo; i < hi; i++) {
        const char* b = seqs + offs[i];
        const int64_t len = offs[i + 1] - offs[i];
        // Python slicing: seq[:a5] and seq[-a3:]
        const int64_t l5 = a5 < len ? a5 : len, l3 = a3 < len ? a3 : len;
        char* d = hw.p + i * S;
        memcpy(d, b, (size_t)l5);
        memcpy(d + a5, b + len - l3, (size_t)l3);
        hl.p[2 * i] = (uint8_t)l5;
        hl.p[2 * i + 1] = (uint8_t)l3;
      }
    });
    DevBuf<char>& d_w = c->ex_dwin;
    DevBuf<uint8_t>& d_l = c->ex_dlen;
    DevBuf<int32_t>& d_out = c->ex_dout;
    DevBuf<ExtractPatterns>& d_p = c->ex_dpat;
    c->hip(d_w.ensure((size_t)n * S + 16), "alloc");
    c->hip(d_l.ensure((size_t)n * 2), "alloc");
    c->hip(d_out.ensure((size_t)n * 6), "alloc");
    c->hip(d_p.ensure(1), "alloc");
    c->hip(hipMemcpyAsync(d_w.p, hw.p, (size_t)n * S, hipMemcpyHostToDevice, c->st), "h2d");
    c->hip(hipMemcpyAsync(d_l.p, hl.p, (size_t)n * 2, hipMemcpyHostToDevice, c->st), "h2d");
    c->hip(hipMemcpyAsync(d_p.p, &P, sizeof(P), hipMemcpyHostToDevice, c->st), "h2d");
    c->hip(launch_extract_win(d_w.p, d_l.p, n, S, a5, k, d_p.p, d_out.p, c->st), "extract");
    c->hip(hipMemcpyAsync(out, d_out.p, (size_t)n * 6 * 4, hipMemcpyDeviceToHost, c->st), "d2h");
    c->hip(hipStreamSynchronize(c->st), "sync");
    return;
  }
  const int64_t bytes = offs[n] - offs[0];
  std::vector<int64_t> rel((size_t)n + 1);
  for (int64_t i = 0; i <= n; i++) rel[i] = offs[i] - offs[0];
  DevBuf<char> d_s;
  DevBuf<int64_t> d_o;
  DevBuf<ExtractPatterns> d_p;
  DevBuf<int32_t> d_out;
  c->hip(d_s.ensure((size_t)bytes + 1), "alloc");
  c->hip(d_o.ensure((size_t)n + 1), "alloc");
  c->hip(d_p.ensure(1), "alloc");
  c->hip(d_out.ensure((size_t)n * 6), "alloc");
  if (bytes > 0) c->hip(hipMemcpyAsync(d_s.p, seqs + offs[0], (size_t)bytes, hipMemcpyHostToDevice, c->st), "h2d");
  c->hip(hipMemcpyAsync(d_o.p, rel.data(), rel.size() * 8, hipMemcpyHostToDevice, c->st), "h2d");
  c->hip(hipMemcpyAsync(d_p.p, &P, sizeof(P), hipMemcpyHostToDevice, c->st), "h2d");
  c->hip(launch_extract(d_s.p, d_o.p, n, a5, a3, k, d_p.p, d_out.p, c->st), "extract");
  c->hip(hipMemcpyAsync(out, d_out.p, (size_t)n * 6 * 4, hipMemcpyDeviceToHost, c->st), "d2h");
  c->hip(hipStreamSynchronize(c->st), "sync");
}

}  // namespace

int32_t umiclust_extract_umis(umiclust_ctx* c, const char* seqs, const int64_t* offsets, int64_t n,
                              int32_t adapter_length_5_end, int32_t adapter_length_3_end, int32_t max_pattern_dist,
                              const char* umi_fwd, const char* umi_rev, int32_t* out) {
  UC_GUARD(c, {
    extract_device(c, seqs, offsets, n, adapter_length_5_end, adapter_length_3_end, max_pattern_dist, umi_fwd,
                   umi_rev, out);
    return UMICLUST_OK;
  });
}

int64_t umiclust_extract_umis_file(umiclust_ctx* c, const char* fastx_file, const char* out_fasta,
                                   int32_t adapter_length_5_end, int32_t adapter_length_3_end,
                                   int32_t max_pattern_dist, const char* umi_fwd, const char* umi_rev) {
  UC_GUARD(c, {
    if (!fastx_file || !out_fasta) c->fail(UMICLUST_EINVAL, "null path");
    Fasta f;
    bool fastq = false;
    {
      FILE* fp = fopen(fastx_file, "rb");
      if (!fp) c->fail(UMICLUST_EIO, "cannot read %s", fastx_file);
      int ch;
      while ((ch = fgetc(fp)) == '\n' || ch == '\r') {}
      fastq = ch == '@';
      fclose(fp);
    }
    if (!(fastq ? io::read_fastq(fastx_file, f) : io::read_fasta(fastx_file, f)))
      c->fail(UMICLUST_EIO, "cannot parse %s", fastx_file);
    const int64_t n = (int64_t)f.hdr_off.size();
    std::vector<int32_t> res((size_t)std::max<int64_t>(n, 1) * 6);
    extract_device(c, f.seq.data(), f.seq_off.data(), n, adapter_length_5_end, adapter_length_3_end, max_pattern_dist,
                   umi_fwd, umi_rev, res.data());
    // records in input order; the reference raises at the first record without a strand annotation, after
    // writing the records before it: those are written, then the error is returned
    int64_t ngood = n;
    for (int64_t i = 0; i < n && ngood == n; i++) {
      Sv st;
      if (!split1(Sv{f.data + f.hdr_off[i], (size_t)f.hdr_len[i]}, "strand=", st)) ngood = i;
    }
    const int64_t tot = io::write_detected_umis(out_fasta, f, res.data(), ngood, adapter_length_3_end);
    if (ngood < n) c->fail(UMICLUST_EFORMAT, "Read strand not annotated!");
    return tot;
  });
}

// ---------------------------------------------------------------- region binning (§8f f4)
namespace {
int32_t rd_i32(const uint8_t* p) { int32_t v; memcpy(&v, p, 4); return v; }
}  // namespace

int64_t umiclust_region_split(umiclust_ctx* c, const char* bam_file, int32_t nregions, const char* const* region_names,
                              const int64_t* region_lengths, const int32_t* region_clusters,
                              double minimal_region_overlap, int32_t max_softclip_5_end, int32_t max_softclip_3_end,
                              const char* out_dir, int64_t* counts, int64_t* reads_per_cluster, int32_t ncluster_cap,
                              uint8_t* region_detected, char* missing_name, int32_t missing_cap) {
  UC_GUARD(c, {
    if (!bam_file || !out_dir || nregions < 0 || (nregions > 0 && (!region_names || !region_lengths || !region_clusters)) ||
        !counts || ncluster_cap < 0 || (ncluster_cap > 0 && !reads_per_cluster))
      c->fail(UMICLUST_EINVAL, "bad argument");
    std::vector<uint8_t> raw;
    if (!io::inflate_bgzf(bam_file, raw)) c->fail(UMICLUST_EIO, "cannot read BGZF/BAM %s", bam_file);
    if (raw.size() < 12 || memcmp(raw.data(), "BAM\1", 4) != 0) c->fail(UMICLUST_EFORMAT, "%s is not BAM", bam_file);
    // header: text, then the reference names, matched to the regions of the reference FASTA
    std::unordered_map<std::string, int32_t> rid;
    for (int32_t r = 0; r < nregions; r++) rid.emplace(region_names[r], r);
    size_t o = 4;
    const int32_t lt = rd_i32(raw.data() + o);
    o += 4 + (size_t)lt;
    const int32_t nref = rd_i32(raw.data() + o);
    o += 4;
    std::vector<std::string> refname(nref);
    std::vector<int64_t> rlen(nref, -1);
    std::vector<int32_t> rclu(nref, -1), rreg(nref, -1);
    for (int32_t r = 0; r < nref; r++) {
      const int32_t ln = rd_i32(raw.data() + o);
      refname[r] = std::string((const char*)raw.data() + o + 4, (size_t)std::max(0, ln - 1));
      o += 4 + (size_t)ln + 4;
      auto it = rid.find(refname[r]);
      if (it != rid.end()) {
        rreg[r] = it->second;
        rlen[r] = region_lengths[it->second];
        rclu[r] = region_clusters[it->second];
      }
    }
    std::vector<int64_t> roff;
    while (o + 4 <= raw.size()) {
      roff.push_back((int64_t)o);
      o += 4 + (size_t)rd_i32(raw.data() + o);
    }
    if (o != raw.size()) c->fail(UMICLUST_EFORMAT, "truncated BAM record");
    const int64_t n = (int64_t)roff.size();
    // device: classify every record
    DevBuf<uint8_t> d_raw;
    DevBuf<int64_t> d_roff, d_rlen, d_outlen, d_pos;
    DevBuf<int32_t> d_rclu, d_clu;
    DevBuf<int8_t> d_cls;
    c->hip(d_raw.ensure(raw.size() + 1), "alloc");
    c->hip(d_roff.ensure((size_t)n + 1), "alloc");
    c->hip(d_rlen.ensure((size_t)nref + 1), "alloc");
    c->hip(d_rclu.ensure((size_t)nref + 1), "alloc");
    c->hip(d_cls.ensure((size_t)n + 1), "alloc");
    c->hip(d_clu.ensure((size_t)n + 1), "alloc");
    c->hip(d_outlen.ensure((size_t)n + 1), "alloc");
    c->hip(d_pos.ensure((size_t)n + 1), "alloc");
    c->hip(hipMemcpyAsync(d_raw.p, raw.data(), raw.size(), hipMemcpyHostToDevice, c->st), "h2d");
    if (n) c->hip(hipMemcpyAsync(d_roff.p, roff.data(), (size_t)n * 8, hipMemcpyHostToDevice, c->st), "h2d");
    if (nref) {
      c->hip(hipMemcpyAsync(d_rlen.p, rlen.data(), (size_t)nref * 8, hipMemcpyHostToDevice, c->st), "h2d");
      c->hip(hipMemcpyAsync(d_rclu.p, rclu.data(), (size_t)nref * 4, hipMemcpyHostToDevice, c->st), "h2d");
    }
    c->hip(launch_bam_classify(d_raw.p, d_roff.p, n, nref, d_rlen.p, d_rclu.p, minimal_region_overlap,
                               max_softclip_5_end, max_softclip_3_end, d_cls.p, d_clu.p, d_outlen.p, c->st),
           "bam classify");
    std::vector<int8_t> cls(n);
    std::vector<int32_t> clu(n);
    std::vector<int64_t> olen(n);
    if (n) {
      c->hip(hipMemcpyAsync(cls.data(), d_cls.p, (size_t)n, hipMemcpyDeviceToHost, c->st), "d2h");
      c->hip(hipMemcpyAsync(clu.data(), d_clu.p, (size_t)n * 4, hipMemcpyDeviceToHost, c->st), "d2h");
      c->hip(hipMemcpyAsync(olen.data(), d_outlen.p, (size_t)n * 8, hipMemcpyDeviceToHost, c->st), "d2h");
    }
    c->hip(hipStreamSynchronize(c->st), "sync");
    // the reference raises KeyError at the first record whose region is unknown, after the records before it
    int64_t stop = n;
    for (int64_t r = 0; r < n && stop == n; r++)
      if (cls[r] == kBamNoRegion || cls[r] == kBamNoCluster) stop = r;
    int32_t ncl = 0;
    for (int64_t r = 0; r < stop; r++)
      if (cls[r] == kBamKept) ncl = std::max(ncl, clu[r] + 1);
    // output grouped by cluster, records in BAM order within a cluster
    std::vector<int64_t> cbase((size_t)ncl + 1, 0), pos(n, -1);
    for (int64_t r = 0; r < stop; r++)
      if (cls[r] == kBamKept) cbase[clu[r] + 1] += olen[r];
    for (int32_t k = 0; k < ncl; k++) cbase[k + 1] += cbase[k];
    {
      std::vector<int64_t> cur(cbase.begin(), cbase.end() - 1);
      for (int64_t r = 0; r < stop; r++)
        if (cls[r] == kBamKept) {
          pos[r] = cur[clu[r]];
          cur[clu[r]] += olen[r];
        }
    }
    std::vector<char> outb((size_t)cbase[ncl] + 1);
    DevBuf<char> d_out;
    c->hip(d_out.ensure(outb.size()), "alloc");
    if (stop) {
      c->hip(hipMemcpyAsync(d_pos.p, pos.data(), (size_t)stop * 8, hipMemcpyHostToDevice, c->st), "h2d");
      c->hip(launch_bam_emit(d_raw.p, d_roff.p, stop, d_cls.p, d_pos.p, d_out.p, c->st), "bam emit");
      c->hip(hipMemcpyAsync(outb.data(), d_out.p, (size_t)cbase[ncl], hipMemcpyDeviceToHost, c->st), "d2h");
    }
    c->hip(hipStreamSynchronize(c->st), "sync");
    // append per cluster (the reference opens region_cluster<k>.fasta with "a" for every record)
    std::vector<int32_t> used;
    for (int32_t k = 0; k < ncl; k++)
      if (cbase[k + 1] > cbase[k]) used.push_back(k);
    const int T = std::max(1, std::min<int>(io_threads(), (int)used.size()));
    std::vector<int32_t> bad(T, -1);
    parallel_for(T, [&](int t) {
      for (size_t u = (size_t)t; u < used.size(); u += (size_t)T) {
        const int32_t k = used[u];
        const std::string fn = pjoin(out_dir, "region_cluster" + std::to_string(k) + ".fasta");
        const int fd = open(fn.c_str(), O_WRONLY | O_CREAT | O_APPEND, 0666);
        bool ok = fd >= 0 && io::write_all(fd, outb.data() + cbase[k], (size_t)(cbase[k + 1] - cbase[k]));
        if (fd >= 0) ok = (close(fd) == 0) && ok;
        if (!ok) bad[t] = k;
      }
    });
    for (int32_t v : bad)
      if (v >= 0) c->fail(UMICLUST_EIO, "cannot append region_cluster%d.fasta", v);
    // counters of the records the reference reached
    int64_t cnt[4] = {0, 0, 0, 0};  // unmapped, primary mapped, short, long
    if (reads_per_cluster) memset(reads_per_cluster, 0, sizeof(int64_t) * (size_t)ncluster_cap);
    if (region_detected) memset(region_detected, 0, (size_t)nregions);
    const int64_t last = stop < n ? stop + 1 : n;  // the failing record counts as a primary alignment too
    for (int64_t r = 0; r < last; r++) {
      const int8_t k = cls[r];
      if (k == kBamUnmapped) cnt[0]++;
      if (k >= kBamShort) cnt[1]++;
      if (k == kBamShort) cnt[2]++;
      if (k == kBamLong) cnt[3]++;
      if (k == kBamKept && r < stop) {
        if (clu[r] < ncluster_cap) reads_per_cluster[clu[r]]++;
        const int32_t ref = rd_i32(raw.data() + roff[r] + 4);
        if (region_detected && rreg[ref] >= 0) region_detected[rreg[ref]] = 1;
      }
    }
    for (int x = 0; x < 4; x++) counts[x] = cnt[x];
    if (stop < n) {
      const int32_t ref = rd_i32(raw.data() + roff[stop] + 4);
      const std::string nm = ref >= 0 && ref < nref ? refname[ref] : std::string("None");
      if (missing_name && missing_cap > 0) snprintf(missing_name, (size_t)missing_cap, "%s", nm.c_str());
      c->fail(UMICLUST_EFORMAT, "KeyError: '%s'", nm.c_str());
    }
    if (ncl > ncluster_cap) c->fail(UMICLUST_ERANGE, "cluster ids up to %d exceed the counter capacity", ncl - 1);
    return (int64_t)used.size();
  });
}

int32_t umiclust_prep(umiclust_ctx* c, const umiclust_params* p, const char* seqs, const int64_t* offsets,
                      int64_t n, char* masked, uint16_t* kmers, int32_t kstride, int32_t* nk) {
  UC_GUARD(c, {
    if (!p || n < 0 || (n > 0 && (!seqs || !offsets))) c->fail(UMICLUST_EINVAL, "null argument");
    for (int64_t i = 0; i < n; i++)
      if (offsets[i + 1] - offsets[i] > kMaxLen) c->fail(UMICLUST_ERANGE, "sequence longer than %d", kMaxLen);
    DevBuf<char> d_a, d_m;
    DevBuf<int64_t> d_o;
    DevBuf<uint32_t> d_codes;
    DevBuf<uint8_t> d_lens, d_nk;
    DevBuf<uint16_t> d_km;
    const int64_t bytes = n > 0 ? offsets[n] - offsets[0] : 0;
    std::vector<int64_t> rel((size_t)n + 1);
    for (int64_t i = 0; i <= n; i++) rel[i] = offsets[i] - offsets[0];
    c->hip(d_a.ensure((size_t)bytes + 1), "alloc");
    c->hip(d_o.ensure((size_t)n + 1), "alloc");
    c->hip(d_codes.ensure((size_t)n * 2 * kCodeWords + 1), "alloc");
    c->hip(d_lens.ensure((size_t)n + 1), "alloc");
    c->hip(d_nk.ensure((size_t)n * 2 + 1), "alloc");
    c->hip(d_km.ensure((size_t)n * 2 * kKmerStride + 1), "alloc");
    c->hip(d_m.ensure((size_t)n * kMaxLen + 1), "alloc");
    if (bytes > 0) c->hip(hipMemcpy(d_a.p, seqs + offsets[0], (size_t)bytes, hipMemcpyHostToDevice), "h2d");
    c->hip(hipMemcpy(d_o.p, rel.data(), rel.size() * 8, hipMemcpyHostToDevice), "h2d");
    c->hip(launch_prep(d_a.p, d_o.p, nullptr, (int32_t)n, p->qmask_dust, d_codes.p, d_lens.p, d_km.p, d_nk.p, d_m.p,
                       nullptr, c->st),
           "prep");
    std::vector<char> m((size_t)n * kMaxLen);
    std::vector<uint16_t> km((size_t)n * 2 * kKmerStride);
    std::vector<uint8_t> nkv((size_t)n * 2);
    if (n > 0) {
      c->hip(hipMemcpyAsync(m.data(), d_m.p, m.size(), hipMemcpyDeviceToHost, c->st), "d2h");
      c->hip(hipMemcpyAsync(km.data(), d_km.p, km.size() * 2, hipMemcpyDeviceToHost, c->st), "d2h");
      c->hip(hipMemcpyAsync(nkv.data(), d_nk.p, nkv.size(), hipMemcpyDeviceToHost, c->st), "d2h");
    }
    c->hip(hipStreamSynchronize(c->st), "sync");
    for (int64_t i = 0; i < n; i++) {
      const int64_t L = offsets[i + 1] - offsets[i];
      if (masked) memcpy(masked + (offsets[i] - offsets[0]), m.data() + (size_t)i * kMaxLen, (size_t)L);
      for (int s = 0; s < 2; s++) {
        if (nk) nk[2 * i + s] = nkv[(size_t)2 * i + s];
        if (kmers)
          for (int x = 0; x < nkv[(size_t)2 * i + s] && x < kstride; x++)
            kmers[(size_t)(2 * i + s) * kstride + x] = km[(size_t)(2 * i + s) * kKmerStride + x];
      }
    }
    return UMICLUST_OK;
  });
}

}  // extern "C"
