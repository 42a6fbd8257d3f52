// kernels.hip -- MI355X (gfx950) kernels of the UMI clustering hot path.
//
// The reference delegates this arithmetic to vsearch (`--cluster_fast`, invoked at
// /root/reference/ont_tcr_consensus/vsearch_umi_cluster.py:21-54 and :71-97).  Kernels:
//   K1 k_prep        DUST soft-mask (vsearch mask.cc) + unique 8-mers both strands (unique.cc)
//   KI k_index_*     CSR inverted index tile over centroid k-mers (dbindex.cc analogue)
//   K2 k_prefilter   shared-unique-k-mer counting against every centroid + top-41 selection
//                    (searchcore.cc search_topscores / minheap.cc order), LDS u8 counters
//   K3 k_align       Gotoh global alignment, one alignment per lane, with the vsearch
//                    traceback's path statistics carried FORWARD through the DP so that no
//                    direction matrix is stored (align_simd.cc search16/backtrack16 + align_trim)
//   K3T k_traceback  same DP with a 4-bit direction matrix in HBM + explicit traceback, for
//                    the one chosen hit per member (the CIGAR feeding the consensus)
//   K4 k_consensus   star MSA + column majority vote per cluster (msa.cc)
// All integer/byte work: VALU + LDS, no MFMA (not a dense contraction).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "umiclust_internal.h"

namespace uc {

// ------------------------------------------------------------------ character maps
// 4-bit IUPAC code (vsearch chrmap_4bit): A1 C2 G4 T/U8, ambiguity codes OR-ed, N15.
__constant__ uint8_t c_map4[256];

static uint8_t h_map4[256];
static bool h_maps_init = false;

static void host_maps() {
  if (h_maps_init) return;
  const char* iupac = "ACGTURYSWKMBDHVN";
  const uint8_t v4[] = {1, 2, 4, 8, 8, 5, 10, 6, 9, 12, 3, 14, 13, 11, 7, 15};
  for (int i = 0; i < 256; i++) h_map4[i] = 0;
  for (int i = 0; iupac[i]; i++) {
    h_map4[(uint8_t)iupac[i]] = v4[i];
    h_map4[(uint8_t)(iupac[i] | 0x20)] = v4[i];
  }
  h_maps_init = true;
}

static hipError_t ensure_maps(hipStream_t st) {
  host_maps();
  return hipMemcpyToSymbolAsync(HIP_SYMBOL(c_map4), h_map4, 256, 0, hipMemcpyHostToDevice, st);
}

__device__ __forceinline__ uint32_t code2_of4(uint32_t c4) {
  // chrmap_2bit: A0 C1 G2 T3, anything else 0
  return c4 == 2 ? 1u : (c4 == 4 ? 2u : (c4 == 8 ? 3u : 0u));
}
__device__ __forceinline__ uint32_t comp4(uint32_t c4) {
  // complement of an IUPAC bitmask = nibble bit reversal (A<->T, C<->G, R<->Y, ...)
  return ((c4 & 1u) << 3) | ((c4 & 2u) << 1) | ((c4 & 4u) >> 1) | ((c4 & 8u) >> 3);
}

// ------------------------------------------------------------------ K1: prep
// One thread per (sorted) sequence.  LDS scratch per thread: residues, DUST words/counts and
// the k-mer sort buffer (runtime-indexed arrays must not live in VGPRs).
constexpr int kPrepThreads = 64;
struct PrepScratch {
  uint8_t ch[kMaxLen];     // original characters
  uint8_t words[64];
  uint8_t counts[64];
  uint16_t km[kMaxKmers + 3];
};

__device__ int dust_wo(const uint8_t* s2, int len, int* beg, int* end, uint8_t* words,
                       uint8_t* counts) {
  // vsearch mask.cc wo(): smallest region is 8 => l1 = len - 3 + 1 - 5
  int l1 = len - 3 + 1 - 5;
  if (l1 < 0) {
    *beg = 0;
    *end = len - 1;
    return 0;
  }
  int w = 0;
  for (int j = 0; j < len; j++) {
    w = ((w << 2) | s2[j]) & 63;
    words[j] = (uint8_t)w;
  }
  int bestv = 0, besti = 0, bestj = 0;
  for (int i = 0; i < l1; i++) {
    for (int x = 0; x < 64; x++) counts[x] = 0;
    int sum = 0;
    for (int j = 2; j < len - i; j++) {
      int x = words[i + j];
      int c = counts[x];
      if (c) {
        sum += c;
        // v = 10*sum/j (integer); v > bestv  <=>  10*sum >= (bestv+1)*j
        if (10 * sum >= (bestv + 1) * j) {
          bestv = (10 * sum) / j;
          besti = i;
          bestj = j;
        }
      }
      counts[x] = (uint8_t)(c + 1);
    }
  }
  *beg = besti;
  *end = besti + bestj;
  return bestv;
}

__global__ __launch_bounds__(kPrepThreads) void k_prep(const char* __restrict__ ascii,
                                                       const int64_t* __restrict__ offs,
                                                       const int32_t* __restrict__ perm, int32_t n,
                                                       int dust, uint32_t* __restrict__ codes,
                                                       uint8_t* __restrict__ lens,
                                                       uint16_t* __restrict__ kmers,
                                                       uint8_t* __restrict__ nk,
                                                       char* __restrict__ masked,
                                                       uint32_t* __restrict__ ambig) {
  __shared__ PrepScratch scr[kPrepThreads];
  int s = blockIdx.x * kPrepThreads + threadIdx.x;
  if (s >= n) return;
  PrepScratch& P = scr[threadIdx.x];
  int r = perm ? perm[s] : s;
  int64_t b = offs[r];
  int len = (int)(offs[r + 1] - b);
  for (int x = 0; x < len; x++) P.ch[x] = (uint8_t)ascii[b + x];
  // lower-case mask bits (bit x set = masked), 3 words
  uint32_t mk0 = 0, mk1 = 0, mk2 = 0;
  if (dust) {
    // dust(): the whole sequence upper-cased, masked intervals lower-cased
    uint8_t* codes2 = reinterpret_cast<uint8_t*>(P.km);  // >= 72 bytes available (136)
    for (int x = 0; x < len; x++) codes2[x] = (uint8_t)code2_of4(c_map4[P.ch[x]]);
    for (int i = 0; i < len; i += 32) {
      int l = (len > i + 64) ? 64 : len - i;
      int a = 0, e = 0;
      int v = dust_wo(codes2 + i, l, &a, &e, P.words, P.counts);
      if (v > 20) {
        for (int j = a + i; j <= e + i; j++) {
          if (j < 32) mk0 |= 1u << j;
          else if (j < 64) mk1 |= 1u << (j - 32);
          else mk2 |= 1u << (j - 64);
        }
      }
    }
  }
  auto masked_at = [&](int x) -> uint32_t {
    return x < 32 ? (mk0 >> x) & 1u : (x < 64 ? (mk1 >> (x - 32)) & 1u : (mk2 >> (x - 64)) & 1u);
  };
  lens[s] = (uint8_t)len;
  // masked ASCII (what vsearch prints) and 4-bit codes for both strands
  uint32_t w0[kCodeWords], w1[kCodeWords];
#pragma unroll
  for (int w = 0; w < kCodeWords; w++) { w0[w] = 0; w1[w] = 0; }
  for (int x = 0; x < len; x++) {
    uint8_t c = P.ch[x];
    uint8_t up = (c >= 'a' && c <= 'z') ? (uint8_t)(c - 32) : c;
    if (dust) c = masked_at(x) ? (uint8_t)(up | 0x20) : up;
    if (masked) masked[(int64_t)s * kMaxLen + x] = (char)c;
    P.ch[x] = c;
  }
  uint32_t any_amb = 0;
  for (int x = 0; x < len; x++) {
    uint32_t c4 = c_map4[P.ch[x]];
    any_amb |= (c4 != 1u && c4 != 2u && c4 != 4u && c4 != 8u) ? 1u : 0u;
    int xr = len - 1 - x;
#pragma unroll
    for (int w = 0; w < kCodeWords; w++) {
      if ((x >> 3) == w) w0[w] |= c4 << ((x & 7) * 4);
      if ((xr >> 3) == w) w1[w] |= comp4(c4) << ((xr & 7) * 4);
    }
  }
#pragma unroll
  for (int w = 0; w < kCodeWords; w++) {
    codes[((int64_t)s * 2 + 0) * kCodeWords + w] = w0[w];
    codes[((int64_t)s * 2 + 1) * kCodeWords + w] = w1[w];
  }
  if (any_amb && ambig) atomicOr(ambig, 1u);
  // unique 8-mers per strand, masked windows skipped (unique.cc), sorted ascending
  for (int st = 0; st < 2; st++) {
    uint32_t km = 0, bad = 0;
    int cnt = 0;
    for (int y = 0; y < len; y++) {
      int x = st ? len - 1 - y : y;
      uint32_t c4 = c_map4[P.ch[x]];
      if (st) c4 = comp4(c4);
      bad = ((bad << 1) | masked_at(x)) & 0xffu;
      km = ((km << 2) | code2_of4(c4)) & 0xffffu;
      if (y >= 7 && !bad) {
        // insertion into sorted unique list
        int pos = cnt;
        bool dup = false;
        while (pos > 0 && P.km[pos - 1] >= km) {
          if (P.km[pos - 1] == km) { dup = true; break; }
          pos--;
        }
        if (!dup) {
          for (int z = cnt; z > pos; z--) P.km[z] = P.km[z - 1];
          P.km[pos] = (uint16_t)km;
          cnt++;
        }
      }
    }
    uint16_t* dst = kmers + ((int64_t)s * 2 + st) * kKmerStride;
    for (int z = 0; z < cnt; z++) dst[z] = P.km[z];
    nk[(int64_t)s * 2 + st] = (uint8_t)cnt;
  }
}

hipError_t launch_prep(const char* ascii, const int64_t* offs, const int32_t* perm, int32_t n,
                       int dust, uint32_t* codes, uint8_t* lens, uint16_t* kmers, uint8_t* nk,
                       char* masked, uint32_t* ambig, hipStream_t st) {
  hipError_t e = ensure_maps(st);
  if (e != hipSuccess) return e;
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_prep, dim3((n + kPrepThreads - 1) / kPrepThreads), dim3(kPrepThreads), 0, st,
                     ascii, offs, perm, n, dust, codes, lens, kmers, nk, masked, ambig);
  return hipGetLastError();
}

// ------------------------------------------------------------------ KI: index tile build
// One wave per tile sequence, one lane per k-mer slot (<= kMaxKmers = 65: lane and lane + 64), so a
// build issues its ~60 atomics per sequence from 60 lanes instead of one dependent chain.
__global__ __launch_bounds__(256) void k_index_count(const uint16_t* __restrict__ kmers,
                                                     const uint8_t* __restrict__ nk,
                                                     const int32_t* __restrict__ cent_seqno, int32_t first,
                                                     int32_t count, uint32_t* __restrict__ hist) {
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6), x = threadIdx.x & 63;
  if (c >= count) return;
  const int32_t s = cent_seqno[first + c];
  const int n = nk[(int64_t)s * 2];
  const uint16_t* k = kmers + (int64_t)s * 2 * kKmerStride;
  if (x < n) atomicAdd(&hist[k[x]], 1u);
  if (x + 64 < n) atomicAdd(&hist[k[x + 64]], 1u);
}

__global__ __launch_bounds__(1024) void k_index_scan(const uint32_t* __restrict__ hist,
                                                     uint32_t* __restrict__ off) {
  // exclusive scan of 65536 counters, one workgroup: 64 per thread
  __shared__ uint32_t part[1024];
  int t = threadIdx.x;
  uint32_t loc[64];
  uint32_t sum = 0;
#pragma unroll
  for (int x = 0; x < 64; x++) {
    loc[x] = sum;
    sum += hist[t * 64 + x];
  }
  part[t] = sum;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {
    uint32_t v = (t >= d) ? part[t - d] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint32_t base = part[t] - sum;
#pragma unroll
  for (int x = 0; x < 64; x++) off[t * 64 + x] = base + loc[x];
  if (t == 1023) off[65536] = part[1023];
}

__global__ __launch_bounds__(256) void k_index_fill(const uint16_t* __restrict__ kmers,
                                                    const uint8_t* __restrict__ nk,
                                                    const int32_t* __restrict__ cent_seqno, int32_t first,
                                                    int32_t count, const uint32_t* __restrict__ off,
                                                    uint32_t* __restrict__ cursor, uint16_t* __restrict__ post) {
  // posting order within a list is arbitrary: the prefilter only counts
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6), x = threadIdx.x & 63;
  if (c >= count) return;
  const int32_t s = cent_seqno[first + c];
  const int n = nk[(int64_t)s * 2];
  const uint16_t* k = kmers + (int64_t)s * 2 * kKmerStride;
  if (x < n) post[off[k[x]] + atomicAdd(&cursor[k[x]], 1u)] = (uint16_t)c;
  if (x + 64 < n) post[off[k[x + 64]] + atomicAdd(&cursor[k[x + 64]], 1u)] = (uint16_t)c;
}

hipError_t launch_index_count(const uint16_t* kmers, const uint8_t* nk, const int32_t* cent_seqno,
                              int32_t first, int32_t count, uint32_t* hist, hipStream_t st) {
  if (count <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_index_count, dim3((count + 3) / 4), dim3(256), 0, st, kmers, nk,
                     cent_seqno, first, count, hist);
  return hipGetLastError();
}
hipError_t launch_index_scan(uint32_t* hist_to_off, hipStream_t st) {
  // hist_to_off: [65536] histogram followed by [65537] offsets
  hipLaunchKernelGGL(k_index_scan, dim3(1), dim3(1024), 0, st, hist_to_off, hist_to_off + 65536);
  return hipGetLastError();
}
hipError_t launch_index_fill(const uint16_t* kmers, const uint8_t* nk, const int32_t* cent_seqno,
                             int32_t first, int32_t count, const uint32_t* off, uint32_t* cursor,
                             uint16_t* post, hipStream_t st) {
  if (count <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_index_fill, dim3((count + 3) / 4), dim3(256), 0, st, kmers, nk,
                     cent_seqno, first, count, off, cursor, post);
  return hipGetLastError();
}

// ------------------------------------------------------------------ K2: prefilter
// One 512-thread workgroup per (query, strand).  Per index tile: u8 counters (4 per u32) for up to
// 65536 centroids in 64 KiB of LDS.
//  count: the query's <= 65 posting lists are walked as one flat sequence of 16-byte chunks (8 u16
//         postings); each thread keeps 4 chunk loads in flight, then issues fire-and-forget
//         ds_add_u32 for the postings inside its list range (the memory system, not the atomics,
//         must be kept busy: one dependent 2-byte load per atomic was latency-bound);
//  scan:  the counters are read back 16 bytes per lane and a SWAR test finds every byte >= the
//         threshold min(12, #kmers) (searchcore.cc search_topscores' `count >= minmatches`);
//  top:   candidates get 30-bit keys (count desc, length asc, id asc), are bitonic-sorted and
//         merged into the running top-41 (u64 keys over all tiles; minheap.cc order).
// A threshold of 0, or more candidates than the LDS buffer holds, switches the tile to a chunked
// exact path, so the result is exact in every case.
constexpr int kPfThreads = 512;
constexpr int kPfUnroll = 4;
constexpr int kRankSel = 1024;  // candidate counts up to this are selected by rank

struct PfShared {
  uint32_t cnt[kTile / 4];        // 64 KiB packed u8 counters
  uint32_t cand[kCandCap];        // candidate local ids, then 30-bit keys
  unsigned long long top[kTopHits];
  unsigned long long merged[kTopHits];
  uint32_t best[kPeerCap + 1];    // the tile's best keys in order
  unsigned long long bestk[kTopHits];
  uint32_t kbeg[kMaxKmers + 3];   // posting range [kbeg, kend) of each query k-mer in this tile
  uint32_t kend[kMaxKmers + 3];
  uint32_t kchunk[kMaxKmers + 4]; // prefix sum of 16-byte chunks per list
  uint16_t km[kMaxKmers + 3];
  uint32_t ncand;
  uint32_t overflow;
  int32_t ntop;
  uint32_t post_local;
};

__device__ __forceinline__ uint32_t cnt_get(const uint32_t* cnt, uint32_t c) {
  return (cnt[c >> 2] >> ((c & 3) * 8)) & 0xffu;
}

// bitonic sort of n (power of two) u32 keys in LDS, ascending
__device__ void bitonic_u32(uint32_t* a, int n) {
  for (int k = 2; k <= n; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < n; i += blockDim.x) {
        int l = i ^ j;
        if (l > i) {
          uint32_t x = a[i], y = a[l];
          bool up = (i & k) == 0;
          if ((x > y) == up) {
            a[i] = y;
            a[l] = x;
          }
        }
      }
      __syncthreads();
    }
  }
}

__device__ __forceinline__ void pf_add(uint32_t* cnt, uint32_t c) {
  atomicAdd(&cnt[c >> 2], 1u << ((c & 3) * 8));  // result unused -> ds_add_u32 (no return)
}

__device__ __forceinline__ void pf_chunk(uint32_t* cnt, const uint4& v, uint32_t base, uint32_t lo,
                                         uint32_t hi) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int e = 0; e < 8; e++) {
    const uint32_t idx = base + (uint32_t)e;
    const uint32_t c = (w[e >> 1] >> ((e & 1) * 16)) & 0xffffu;
    if (idx >= lo && idx < hi) pf_add(cnt, c);
  }
}

__global__ __launch_bounds__(kPfThreads) void k_prefilter(PrefilterArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char pf_smem[];
  PfShared& S = *reinterpret_cast<PfShared*>(pf_smem);
  const int tid = threadIdx.x;
  const int qs = blockIdx.x;
  const int qlocal = qs / a.both;
  const int strand = qs % a.both;
  const int32_t q = a.q0 + qlocal;
  const int nk = a.seqs.nk[(int64_t)q * 2 + strand];
  const uint16_t* qk = a.seqs.kmers + ((int64_t)q * 2 + strand) * kKmerStride;
  const int thr = nk < a.minwordmatches ? nk : a.minwordmatches;
  for (int x = tid; x < nk; x += kPfThreads) S.km[x] = qk[x];
  if (tid == 0) {
    S.ntop = 0;
    S.post_local = 0;
  }
  __syncthreads();
  int npeer = 0;
  for (int t = 0; t < a.ntiles + 2; t++) {
    const bool peer = (t >= a.ntiles);
    TileView tv;
    if (peer) tv = a.peer[t - a.ntiles];
    else tv = a.tiles[t];
    // peers: only the window queries before q (a peer tile's base is its first seqno)
    const int limit = peer ? min(tv.n, q - tv.base) : tv.n;
    if (limit <= 0) continue;
    // zero the counters (whole uint4 groups: the scan reads 16 counters per lane)
    const int nq4 = (tv.n + 15) >> 4;
    uint4* cnt4 = reinterpret_cast<uint4*>(S.cnt);
    for (int x = tid; x < nq4; x += kPfThreads) cnt4[x] = make_uint4(0u, 0u, 0u, 0u);
    if (tid < nk) {
      const uint32_t b = tv.off[S.km[tid]], e = tv.off[S.km[tid] + 1];
      S.kbeg[tid] = b;
      S.kend[tid] = e;
    }
    if (tid == 0) {
      S.ncand = 0;
      S.overflow = 0;
    }
    __syncthreads();
    if (tid < 64) {
      // exclusive prefix of 16-byte chunk counts over the <= 65 lists (wave 0, shuffles)
      uint32_t carry = 0, touched = 0;
      for (int k0 = 0; k0 < nk; k0 += 64) {
        const int k = k0 + tid;
        uint32_t nch = 0;
        if (k < nk) {
          const uint32_t b = S.kbeg[k], e = S.kend[k];
          touched += e - b;
          nch = (e > b) ? ((e - (b & ~7u) + 7u) >> 3) : 0u;
        }
        uint32_t inc = nch;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
          const uint32_t v = __shfl_up(inc, d, 64);
          if (tid >= d) inc += v;
        }
        if (k < nk) S.kchunk[k] = carry + inc - nch;
        carry += __shfl(inc, 63, 64);
      }
#pragma unroll
      for (int d = 32; d > 0; d >>= 1) touched += __shfl_xor(touched, d, 64);
      if (tid == 0) {
        S.kchunk[nk] = carry;
        S.post_local += touched;
      }
    }
    __syncthreads();
    if (thr > 0) {
      const uint32_t total = S.kchunk[nk];
      int k = 0;
      for (uint32_t g0 = (uint32_t)tid; g0 < total; g0 += kPfThreads * kPfUnroll) {
        uint4 v[kPfUnroll];
        uint32_t base[kPfUnroll], lo[kPfUnroll], hi[kPfUnroll];
#pragma unroll
        for (int u = 0; u < kPfUnroll; u++) {
          const uint32_t g = g0 + (uint32_t)(u * kPfThreads);
          lo[u] = hi[u] = base[u] = 0;
          if (g < total) {
            while (S.kchunk[k + 1] <= g) k++;
            base[u] = (S.kbeg[k] & ~7u) + 8u * (g - S.kchunk[k]);
            lo[u] = S.kbeg[k];
            hi[u] = S.kend[k];
            v[u] = *reinterpret_cast<const uint4*>(tv.post + base[u]);
          }
        }
#pragma unroll
        for (int u = 0; u < kPfUnroll; u++)
          if (hi[u] > lo[u]) pf_chunk(S.cnt, v[u], base[u], lo[u], hi[u]);
      }
    }
    __syncthreads();
    // scan: every counter >= thr (SWAR: bytes <= 65, so byte + 128 - thr sets bit 7 iff >= thr)
    if (thr > 0) {
      const uint32_t add = (uint32_t)(128 - thr) * 0x01010101u;
      const int lim4 = (limit + 15) >> 4;
      for (int x = tid; x < lim4; x += kPfThreads) {
        const uint4 v = cnt4[x];
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; j++) {
          uint32_t m = (w[j] + add) & 0x80808080u;
          while (m) {
            const uint32_t byte = (uint32_t)__builtin_ctz(m) >> 3;
            m &= m - 1u;
            const uint32_t c = (uint32_t)x * 16u + (uint32_t)j * 4u + byte;
            if ((int)c < limit) {
              const uint32_t slot = atomicAdd(&S.ncand, 1u);
              if (slot < (uint32_t)kCandCap) S.cand[slot] = c;
              else S.overflow = 1;
            }
          }
        }
      }
    }
    __syncthreads();
    const bool scan_mode = (thr == 0) || S.overflow;
    const int nchunks = scan_mode ? (limit + kCandCap - 1) / kCandCap : 1;
    for (int ch = 0; ch < nchunks; ch++) {
      int nc;
      if (scan_mode) {
        __syncthreads();
        if (tid == 0) S.ncand = 0;
        __syncthreads();
        const int c0 = ch * kCandCap;
        const int c1 = min(limit, c0 + kCandCap);
        for (int c = c0 + tid; c < c1; c += kPfThreads)
          if ((int)cnt_get(S.cnt, (uint32_t)c) >= thr) S.cand[atomicAdd(&S.ncand, 1u)] = (uint32_t)c;
        __syncthreads();
      }
      nc = (int)min(S.ncand, (uint32_t)kCandCap);
      // keys: (127-count) << 23 | len << 16 | local id   (30 bits, unique within a tile; local-id
      // order is seqno order, so key order is (count desc, length asc, seqno asc))
      for (int x = tid; x < nc; x += kPfThreads) {
        const uint32_t c = S.cand[x];
        const uint32_t cntv = cnt_get(S.cnt, c);
        const int32_t sq = peer ? (tv.base + (int32_t)c) : a.cent_seqno[tv.base + (int32_t)c];
        S.cand[x] = ((127u - cntv) << 23) | ((uint32_t)a.seqs.lens[sq] << 16) | c;
      }
      __syncthreads();
      // best K of the tile in key order: by rank (all-pairs count, broadcast LDS reads) when the
      // candidate set is small, by a bitonic sort otherwise
      const int K = peer ? kPeerCap + 1 : kTopHits;
      int nbest = nc < K ? nc : K;
      if (nc <= kRankSel) {
        for (int x = tid; x < nc; x += kPfThreads) {
          const uint32_t kx = S.cand[x];
          int r = 0;
          for (int y = 0; y < nc; y++) r += S.cand[y] < kx;
          if (r < K) S.best[r] = kx;
        }
      } else {
        int np2 = 1;
        while (np2 < nc) np2 <<= 1;
        for (int x = nc + tid; x < np2; x += kPfThreads) S.cand[x] = 0xffffffffu;
        __syncthreads();
        bitonic_u32(S.cand, np2);
        for (int x = tid; x < nbest; x += kPfThreads) S.best[x] = S.cand[x];
      }
      __syncthreads();
      if (peer) {
        if (tid < nbest && npeer + tid < kPeerCap) {
          const uint32_t key = S.best[tid];
          a.peer_id[(int64_t)qs * kPeerCap + npeer + tid] =
              (uint16_t)(tv.base + (int32_t)(key & 0xffffu) - a.peer_base);
          a.peer_count[(int64_t)qs * kPeerCap + npeer + tid] = (uint8_t)(127u - (key >> 23));
        }
        npeer += nc;
      } else {
        // merge the tile's best into the running top-41 (u64 keys, unique seqnos): every element
        // of either sorted list finds its merged position by binary search in the other list
        const int ntop = S.ntop;
        if (tid < nbest) {
          const uint32_t key = S.best[tid];
          S.bestk[tid] = ((unsigned long long)(key >> 23) << 56) |
                         ((unsigned long long)((key >> 16) & 0x7fu) << 48) |
                         (unsigned long long)(uint32_t)a.cent_seqno[tv.base + (int32_t)(key & 0xffffu)];
        }
        __syncthreads();
        if (tid < nbest) {
          const unsigned long long kj = S.bestk[tid];
          int lo = 0, hi = ntop;
          while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (S.top[mid] < kj) lo = mid + 1;
            else hi = mid;
          }
          if (tid + lo < kTopHits) S.merged[tid + lo] = kj;
        } else if (tid >= 64 && tid - 64 < ntop) {
          const int i = tid - 64;
          const unsigned long long ki = S.top[i];
          int lo = 0, hi = nbest;
          while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (S.bestk[mid] < ki) lo = mid + 1;
            else hi = mid;
          }
          if (i + lo < kTopHits) S.merged[i + lo] = ki;
        }
        __syncthreads();
        const int nm = min(kTopHits, ntop + nbest);
        if (tid < nm) S.top[tid] = S.merged[tid];
        __syncthreads();
        if (tid == 0) S.ntop = nm;
      }
      __syncthreads();
    }
  }
  if (tid == 0) {
    const int ntop = S.ntop;
    for (int x = 0; x < ntop; x++) {
      a.top_seqno[(int64_t)qs * kTopHits + x] = (uint32_t)(S.top[x] & 0xffffffffull);
      a.top_count[(int64_t)qs * kTopHits + x] = (uint8_t)(127u - (uint32_t)(S.top[x] >> 56));
    }
    a.ntop[qs] = (uint8_t)ntop;
    a.npeer[qs] = (uint8_t)(npeer > kPeerCap ? 255 : npeer);
    if (a.postings_touched) atomicAdd(a.postings_touched, S.post_local);
  }
}

hipError_t launch_prefilter(const PrefilterArgs& a, hipStream_t st) {
  const int nqs = a.nq * a.both;
  if (nqs <= 0) return hipSuccess;
  const size_t smem = sizeof(PfShared);
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)k_prefilter,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL(k_prefilter, dim3(nqs), dim3(kPfThreads), smem, st, a);
  return hipGetLastError();
}

// ------------------------------------------------------------------ K3: alignment (stats)
__device__ __forceinline__ int sx16(uint32_t v) { return (int)(int16_t)(v & 0xffffu); }
__device__ __forceinline__ uint32_t pack_hf(int h, int f) {
  return ((uint32_t)f << 16) | ((uint32_t)h & 0xffffu);
}

constexpr int kNegInf = -16000;  // below any reachable score (|score| <= 72*40 + gaps)

// Query rows are unrolled: QL is a compile-time constant (the driver cuts greedy blocks at length
// changes, so every pair of a launch has the same query length) and the per-row state lives in
// VGPRs with compile-time indices.  Target columns run as a runtime loop (lanes may have different
// target lengths); the target's last column takes the target-right gap penalties (one select per
// column, shared by all rows).
//
// Forward-carried traceback (no direction matrix).  vsearch's acceptance needs, along the path
// backtrack16 picks, the matches m and internal_len = columns - leading gap run - trailing gap run
// (align_trim).  For every real DP cell the leading CIGAR run is exactly the boundary run (row -1
// or column -1) the path starts with, so columns - leading run = the number of moves INTO real
// cells, a.  Each DP state carries the summary a | m << 8 of the path the traceback would follow
// from it (boundary states carry 0), selected with backtrack16's strict priorities
// (diagonal > up/D > left/I; a gap extends only if strictly better than reopening).
// The trailing gap run is backtrack16's first run from the end cell (last row, last column):
//  * an I run walks left along the last row; with Lext(j) = run length when arriving at column j in
//    an I run: Lh(j) = left(j) ? 1 + Lext(j-1) : 0, Lext(j) = extleft(j) ? 1 + Lext(j-1) : Lh(j);
//  * a D run walks up the last column: the F state's summary carries the length of its trailing D
//    run in bits 16-23 (opening from H inherits H's run, so consecutive D runs merge exactly as
//    CIGAR runs do); H inherits it only when it takes F.
// Per row: HE[i] = H(i, j-1) | E(i, j) << 16 and SS[i] = S_H(i, j-1) | S_E(i, j) << 16, 16 bits each.
template <int QL, bool AMB>
__device__ __forceinline__ void align_column(uint32_t (&HE)[QL], uint32_t (&SS)[QL],
                                             const uint32_t (&qw)[(QL + 7) / 8], uint32_t tcode,
                                             int j, const Scoring& sc, int QRt, int Rt, int& Lext,
                                             int& trail) {
  const int QRqi = sc.go[2] + sc.ge[2], Rqi = sc.ge[2];
  const int QRqr = sc.go[4] + sc.ge[4], Rqr = sc.ge[4];
  const bool tamb = AMB && ((tcode & (tcode - 1u)) != 0u || tcode == 0u);
  // row -1 of this column: H(-1, j-1) (diagonal of row 0) and F(0, j); boundary summaries are 0
  int Hd = (j == 0) ? 0 : -(sc.go[0] + j * sc.ge[0]);
  uint32_t SHd = 0;
  int F = sc.boundary_open ? -(sc.go[0] + (j + 1) * sc.ge[0]) - QRt : kNegInf;
  uint32_t SF = 0x10001u;  // one real D move, trailing D run 1
#pragma unroll
  for (int i = 0; i < QL; i++) {
    const uint32_t qcode = (qw[i >> 3] >> ((i & 7) * 4)) & 15u;
    int sub;
    uint32_t e;
    if (AMB) {
      // IUPAC: any ambiguous symbol scores 0; a match is a non-empty code intersection
      const bool amb = tamb || (qcode & (qcode - 1u)) != 0u || qcode == 0u;
      sub = amb ? 0 : (qcode == tcode ? sc.match : sc.mismatch);
      e = (qcode & tcode) ? (1u << 8) : 0u;
    } else {
      const bool eq = qcode == tcode;
      sub = eq ? sc.match : sc.mismatch;
      e = eq ? (1u << 8) : 0u;
    }
    const uint32_t he = HE[i];
    const uint32_t ss = SS[i];
    const int Hl = sx16(he);
    const int E = (int)he >> 16;
    const uint32_t SE = ss >> 16;
    int h = Hd + sub;
    uint32_t sh = SHd + 1u + e;
    const bool fb = F > h;  // up: D chosen
    h = fb ? F : h;
    sh = fb ? SF : sh;
    const bool eb = E > h;  // left: I chosen
    h = eb ? E : h;
    sh = eb ? SE : sh;
    const int fo = h - QRt, fe = F - Rt;
    const bool fx = fe > fo;  // extup
    SF = (fx ? SF : sh) + 0x10001u;
    const int qrq = (i == QL - 1) ? QRqr : QRqi;
    const int rq = (i == QL - 1) ? Rqr : Rqi;
    const int eo = h - qrq, ee = E - rq;
    const bool ex = ee > eo;  // extleft
    const uint32_t sen = (ex ? SE : sh) + 1u;
    if (i == QL - 1) {
      // last row: I-run counters; the value left by the last column is the end cell's
      const int lh = eb ? 1 + Lext : 0;
      Lext = ex ? 1 + Lext : lh;
      trail = eb ? lh : (int)(sh >> 16);
    }
    F = fx ? fe : fo;
    Hd = Hl;
    SHd = ss & 0xffffu;
    // materialise the next row's diagonal now: otherwise SDWA folding reads the old packed words
    // in row i+1, both generations stay live and every column ends in a 2*QL-register copy
    asm volatile("" : "+v"(Hd), "+v"(SHd));
    HE[i] = pack_hf(h, ex ? ee : eo);
    SS[i] = (sh & 0xffffu) | (sen << 16);
  }
}

template <int QL, bool AMB>
__global__ __launch_bounds__(64) void k_align(DevSeqs s, const uint32_t* __restrict__ pq,
                                              const uint32_t* __restrict__ pt, int32_t npairs,
                                              const uint32_t* __restrict__ dev_npairs,
                                              const uint32_t* __restrict__ outidx, Scoring sc,
                                              uint32_t* __restrict__ out) {
  constexpr int CW = (QL + 7) / 8;
  const int k = blockIdx.x * 64 + threadIdx.x;
  if (k >= npairs) return;
  if (dev_npairs && k >= (int)*dev_npairs) return;
  const uint32_t qv = pq[k];
  const int32_t q = (int32_t)(qv >> 1);
  const int qstr = (int)(qv & 1u);
  const int32_t t = (int32_t)pt[k];
  const int tl = s.lens[t];
  uint32_t qw[CW];
#pragma unroll
  for (int w = 0; w < CW; w++) qw[w] = s.codes[((int64_t)q * 2 + qstr) * kCodeWords + w];
  const uint32_t* tcp = s.codes + (int64_t)t * 2 * kCodeWords;
  const int QRti = sc.go[3] + sc.ge[3], Rti = sc.ge[3];
  const int QRtr = sc.go[5] + sc.ge[5], Rtr = sc.ge[5];
  uint32_t HE[QL], SS[QL];
  {
    // boundary column -1: H(i,-1) = -(GO_TL + (i+1) GE_TL), E(i,0) opened from it; built
    // incrementally in VGPRs (an opaque zero keeps the compiler from materialising 2*QL scalars)
    int vz;
    asm volatile("v_mov_b32 %0, 0" : "=v"(vz));
    int hleft = vz - sc.go[1];
    const int QRqi = sc.go[2] + sc.ge[2], QRqr = sc.go[4] + sc.ge[4];
#pragma unroll
    for (int i = 0; i < QL; i++) {
      hleft -= sc.ge[1];
      const int qrq = (i == QL - 1) ? QRqr : QRqi;
      HE[i] = pack_hf(hleft, sc.boundary_open ? hleft - qrq : kNegInf);
      SS[i] = 1u << 16;  // S_H(i,-1) = 0 (boundary), S_E(i,0) = one real move
    }
  }
  int Lext = 0, trail = 0;
  uint32_t tword = 0;
  for (int j = 0; j < tl; j++) {
    if ((j & 7) == 0) tword = tcp[j >> 3];
    const uint32_t tcode = tword & 15u;
    tword >>= 4;
    // keep the per-row query codes from being hoisted out of the column loop (that would pin
    // QL extra VGPRs); re-extracting them is one v_bfe per cell
#pragma unroll
    for (int w = 0; w < CW; w++) asm volatile("" : "+v"(qw[w]));
    const bool lc = (j == tl - 1);
    align_column<QL, AMB>(HE, SS, qw, tcode, j, sc, lc ? QRtr : QRti, lc ? Rtr : Rti, Lext, trail);
  }
  const int H = sx16(HE[QL - 1]);
  const uint32_t S = SS[QL - 1] & 0xffffu;
  const uint32_t m = S >> 8, acols = S & 0xffu;
  const uint32_t internal = acols - (uint32_t)trail;
  out[outidx ? outidx[k] : (uint32_t)k] = m | (internal << 8) | (((uint32_t)H & 0xffffu) << 16);
}

// ------------------------------------------------------------------ K3P: packed 16-bit alignment
// The same recurrences, summaries and strict priorities as k_align, two DP cells per 32-bit VALU
// op (VOP3P v_pk_* on int16 halves).  A column is split into a top half (rows [0, TOP)) and a
// bottom half (rows [TOP, QL)) that runs one column behind: register k holds row k of column j in
// its low half and row TOP+k of column j-1 in its high half.  Within a step the rows are
// processed in order, so the bottom half's upper neighbour (row TOP-1 of column j-1) is the top
// half's carry-out of the previous step; one step costs one pass over TOP packed rows.
// Branch-free selection: for |values| well inside int16, (a - b) >> 15 (arithmetic, per half) is
// the mask of "b > a", which drives v_bfi for the summaries and v_pk_max for the scores.
// Substitution: per 16-row group a match bit-mask of the column's target base, selected per step
// from per-base masks built once per pair (non-ambiguous sequences only: one-hot codes).
typedef short v2s __attribute__((ext_vector_type(2)));

__device__ __forceinline__ v2s as_v2(uint32_t x) { return __builtin_bit_cast(v2s, x); }
__device__ __forceinline__ uint32_t as_u(v2s x) { return __builtin_bit_cast(uint32_t, x); }
__device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t a, uint32_t b) { return (m & a) | (~m & b); }
__device__ __forceinline__ uint32_t pk2(int lo, int hi) { return ((uint32_t)hi << 16) | ((uint32_t)lo & 0xffffu); }
// mask of (b > a) per half
// (opaque to the compiler, which otherwise rewrites it into per-half compares and selects)
__device__ __forceinline__ uint32_t gt_mask(v2s b, v2s a) {
  uint32_t d;
  // op_sel_hi:[0,1]: the inline constant's low half serves both halves (its high half is 0)
  asm("v_pk_sub_i16 %0, %1, %2\n\tv_pk_ashrrev_i16 %0, 15, %0 op_sel_hi:[0,1]" : "=&v"(d) : "v"(a), "v"(b));
  return d;
}

template <int QL>
__global__ __launch_bounds__(64) void k_align_pk(DevSeqs s, const uint32_t* __restrict__ pq,
                                                 const uint32_t* __restrict__ pt, int32_t npairs,
                                                 const uint32_t* __restrict__ dev_npairs,
                                                 const uint32_t* __restrict__ outidx, Scoring sc,
                                                 uint32_t* __restrict__ out) {
  constexpr int TOP = (QL + 1) / 2, BOT = QL - TOP;  // BOT == TOP or TOP - 1
  constexpr int NG = (TOP + 15) / 16;
  constexpr int KL = BOT - 1;                        // register holding row QL-1 (high half)
  const int k = blockIdx.x * 64 + threadIdx.x;
  if (k >= npairs) return;
  if (dev_npairs && k >= (int)*dev_npairs) return;
  const uint32_t qv = pq[k];
  const int32_t q = (int32_t)(qv >> 1);
  const int qstr = (int)(qv & 1u);
  const int32_t t = (int32_t)pt[k];
  const int tl = s.lens[t];
  // per-base row masks: MT[g] / MB[g] hold, for base b at bits [16b, 16b+16), the rows of group g
  // (top half / bottom half) whose query base is b
  uint64_t MT[NG], MB[NG];
#pragma unroll
  for (int g = 0; g < NG; g++) MT[g] = MB[g] = 0;
  {
    const uint32_t* qc = s.codes + ((int64_t)q * 2 + qstr) * kCodeWords;
    uint32_t w = 0;
#pragma unroll
    for (int i = 0; i < QL; i++) {
      if ((i & 7) == 0) w = qc[i >> 3];
      const uint32_t b = (uint32_t)__builtin_ctz((w & 15u) | 16u) & 3u;
      w >>= 4;
      if (i < TOP) MT[i >> 4] |= 1ull << (16 * b + (i & 15));
      else MB[(i - TOP) >> 4] |= 1ull << (16 * b + ((i - TOP) & 15));
    }
  }
  const uint32_t* tcp = s.codes + (int64_t)t * 2 * kCodeWords;
  const int QRti = sc.go[3] + sc.ge[3], Rti = sc.ge[3];
  const int QRtr = sc.go[5] + sc.ge[5], Rtr = sc.ge[5];
  const int QRqi = sc.go[2] + sc.ge[2], Rqi = sc.ge[2];
  const int QRqr = sc.go[4] + sc.ge[4], Rqr = sc.ge[4];
  const v2s MM = as_v2(pk2(sc.mismatch, sc.mismatch));
  const v2s DELTA = as_v2(pk2(sc.match - sc.mismatch, sc.match - sc.mismatch));
  v2s H[TOP], E[TOP];
  uint32_t SH[TOP], SE[TOP];  // summaries; SH stored +1 (every consumer adds the move)
  auto init_rows = [&](uint32_t keep_mask) {
    // boundary column -1: H(i,-1) = -(GO_TL + (i+1) GE_TL), E(i,0) opened from it, S_H = 0,
    // S_E = one real move; keep_mask selects the halves to (re)initialise
    int vz;
    asm volatile("v_mov_b32 %0, 0" : "=v"(vz));
#pragma unroll
    for (int kk = 0; kk < TOP; kk++) {
      const int i0 = kk, i1 = TOP + kk;
      const int h0 = vz - sc.go[1] - (i0 + 1) * sc.ge[1];
      const int h1 = vz - sc.go[1] - (i1 + 1) * sc.ge[1];
      const int q1 = (i1 == QL - 1) ? QRqr : QRqi;
      const int e0 = sc.boundary_open ? h0 - QRqi : kNegInf;
      const int e1 = sc.boundary_open ? h1 - q1 : kNegInf;
      H[kk] = as_v2(bfi(keep_mask, pk2(h0, h1), as_u(H[kk])));
      E[kk] = as_v2(bfi(keep_mask, pk2(e0, e1), as_u(E[kk])));
      SH[kk] = bfi(keep_mask, 0x00010001u, SH[kk]);
      SE[kk] = bfi(keep_mask, 0x00010001u, SE[kk]);
    }
  };
#pragma unroll
  for (int kk = 0; kk < TOP; kk++) {
    H[kk] = as_v2(0u);
    E[kk] = as_v2(0u);
    SH[kk] = SE[kk] = 0;
  }
  init_rows(0xffffffffu);
  // carries of the top half's last row, consumed by the bottom half in the next step
  uint32_t cHd = 0, cSHd = 0, cF = 0, cSF = 0, cDF = 0;
  int Lext = 0, trail = 0;
  uint32_t tword = 0, tprev = 1;
  for (int j = 0; j <= tl; j++) {
    if ((j & 7) == 0) tword = tcp[j >> 3];
    const uint32_t tcode = tword & 15u;
    tword >>= 4;
    const uint32_t bl = (uint32_t)__builtin_ctz(tcode | 16u) & 3u, bh = (uint32_t)__builtin_ctz(tprev | 16u) & 3u;
    tprev = tcode;
    uint32_t M[NG];
#pragma unroll
    for (int g = 0; g < NG; g++)
      M[g] = ((uint32_t)(MT[g] >> (16 * bl)) & 0xffffu) | ((uint32_t)(MB[g] >> (16 * bh)) << 16);
    const bool lc0 = (j == tl - 1), lc1 = (j == tl);
    const uint32_t QRt = pk2(lc0 ? QRtr : QRti, lc1 ? QRtr : QRti);
    const uint32_t Rt = pk2(lc0 ? Rtr : Rti, lc1 ? Rtr : Rti);
    // row -1 (top half, column j) | carry (bottom half, column j-1)
    const int hd0 = (j == 0) ? 0 : -(sc.go[0] + j * sc.ge[0]);
    const int f0 = sc.boundary_open ? -(sc.go[0] + (j + 1) * sc.ge[0]) - (lc0 ? QRtr : QRti) : kNegInf;
    v2s Hd = as_v2(pk2(hd0, (int)cHd));
    uint32_t SHd = pk2(1, (int)cSHd);
    v2s F = as_v2(pk2(f0, (int)cF));
    uint32_t SF = pk2(1, (int)cSF);
    uint32_t DF = pk2(-1, (int)cDF);  // row the current D run opened from (-1: boundary)
#pragma unroll
    for (int kk = 0; kk < TOP; kk++) {
      const uint32_t e = (M[kk >> 4] >> (kk & 15)) & 0x00010001u;
      v2s h = Hd + MM + as_v2(e) * DELTA;
      uint32_t sh = SHd + (e << 8);
      const uint32_t mF = gt_mask(F, h);
      h = __builtin_elementwise_max(h, F);
      sh = bfi(mF, SF, sh);
      const v2s Ec = E[kk];
      const uint32_t mE = gt_mask(Ec, h);
      h = __builtin_elementwise_max(h, Ec);
      sh = bfi(mE, SE[kk], sh);
      const uint32_t sh1 = sh + 0x00010001u;
      int dr_last = 0;
      bool eb_last = false;
      if (kk == KL) {
        // last row (high half): D run of the chosen F = rows since it opened (before DF moves on)
        eb_last = (mE >> 31) != 0;
        dr_last = (mF >> 31) != 0 ? (QL - 1) - (int)(short)(DF >> 16) : 0;
      }
      const v2s fo = h - as_v2(QRt), fe = F - as_v2(Rt);
      const uint32_t mfx = gt_mask(fe, fo);
      F = __builtin_elementwise_max(fo, fe);
      // a new D run opened from H continues H's own D run when H took F
      DF = bfi(mfx | (mF & ~mE), DF, pk2(kk, TOP + kk));
      SF = bfi(mfx, SF + 0x00010001u, sh1);
      const uint32_t qrq = pk2(QRqi, (TOP + kk == QL - 1) ? QRqr : QRqi);
      const uint32_t rq = pk2(Rqi, (TOP + kk == QL - 1) ? Rqr : Rqi);
      const v2s eo = h - as_v2(qrq), ee = Ec - as_v2(rq);
      const uint32_t mex = gt_mask(ee, eo);
      if (kk == KL) {
        // trailing I-run counters along the last row; the value left by the last column is the
        // end cell's (vsearch align_trim's trailing run)
        const bool ex = (mex >> 31) != 0;
        const int lh = eb_last ? 1 + Lext : 0;
        trail = eb_last ? lh : dr_last;
        Lext = ex ? 1 + Lext : lh;
      }
      E[kk] = __builtin_elementwise_max(eo, ee);
      SE[kk] = bfi(mex, SE[kk] + 0x00010001u, sh1);
      Hd = H[kk];
      SHd = SH[kk];
      H[kk] = h;
      SH[kk] = sh1;
    }
    // carry the top half's outputs into the bottom half of the next step
    cHd = as_u(Hd) & 0xffffu;
    cSHd = SHd & 0xffffu;
    cF = as_u(F) & 0xffffu;
    cSF = SF & 0xffffu;
    cDF = DF & 0xffffu;
    if (j == 0) {
      // the bottom half processed column -1 in this step: restore the boundary column
      init_rows(0xffff0000u);
      Lext = 0;
      trail = 0;
    }
  }
  const int Hend = (int)(short)(as_u(H[KL]) >> 16);
  const uint32_t S = ((SH[KL] >> 16) - 1u) & 0xffffu;
  const uint32_t m = S >> 8, acols = S & 0xffu;
  const uint32_t internal = acols - (uint32_t)trail;
  out[outidx ? outidx[k] : (uint32_t)k] = m | (internal << 8) | (((uint32_t)Hend & 0xffffu) << 16);
}

typedef void (*AlignFn)(DevSeqs, const uint32_t*, const uint32_t*, int32_t, const uint32_t*,
                        const uint32_t*, Scoring, uint32_t*);

template <int L>
struct AlignTable {
  static void fill(AlignFn* t) {
    t[3 * L] = k_align_pk<L>;
    t[3 * L + 1] = k_align<L, false>;
    t[3 * L + 2] = k_align<L, true>;
    AlignTable<L - 1>::fill(t);
  }
};
template <>
struct AlignTable<kMinTplLen - 1> {
  static void fill(AlignFn*) {}
};

hipError_t launch_align(const DevSeqs& s, int32_t qlen, bool ambig, const uint32_t* pq,
                        const uint32_t* pt, int32_t npairs, const uint32_t* dev_npairs,
                        const uint32_t* outidx, const Scoring& sc, uint32_t* out, hipStream_t st) {
  static AlignFn table[3 * (kMaxLen + 1)] = {};
  static bool init = false;
  static int variant0 = 0;
  if (!init) {
    AlignTable<kMaxLen>::fill(table);
    // UMICLUST_ALIGN=scalar selects the one-cell-per-op kernel (cross-checks / benchmarks)
    const char* v = getenv("UMICLUST_ALIGN");
    variant0 = (v && v[0] == 's') ? 1 : 0;
    init = true;
  }
  if (npairs <= 0) return hipSuccess;
  if (qlen < kMinTplLen || qlen > kMaxLen) return hipErrorInvalidValue;
  hipLaunchKernelGGL(table[3 * qlen + (ambig ? 2 : variant0)], dim3((npairs + 63) / 64), dim3(64), 0, st, s,
                     pq, pt, npairs, dev_npairs, outidx, sc, out);
  return hipGetLastError();
}

// ------------------------------------------------------------------ K3W: device-side walk
// vsearch search_onequery pops candidates best-first in batches of MAXDELAYED = 8 and stops
// after the batch in which it has an accept, after maxaccepts+maxrejects-1 = 32 candidates, or
// when the list is exhausted.  The walk runs on the device over the top lists (in-block peers
// are resolved later by the host): round r evaluates batch r of every unfinished query-strand and
// emits the pairs of batch r+1.  Acceptance and the id order come from host-built tables, so the
// IEEE-double test `100.0*matches/internal >= 100.0*id` is exactly vsearch's.
__global__ void k_walk(int32_t round, int32_t q0, int32_t nqs, int32_t both,
                       const uint32_t* __restrict__ top_seqno, const uint8_t* __restrict__ top_count,
                       const uint8_t* __restrict__ ntop, const uint8_t* __restrict__ lens,
                       const uint32_t* __restrict__ res, const uint8_t* __restrict__ acc_tab,
                       const uint16_t* __restrict__ rank_tab, WalkState* __restrict__ ws,
                       uint32_t* __restrict__ pq, uint32_t* __restrict__ pt,
                       uint32_t* __restrict__ outidx, uint32_t* __restrict__ npairs) {
  const int qs = blockIdx.x * blockDim.x + threadIdx.x;
  if (qs >= nqs) return;
  const int32_t q = q0 + qs / both;
  const uint32_t strand = (uint32_t)(qs % both);
  const int nt = ntop[qs];
  WalkState w;
  if (round < 0) {
    w.w = 0;
    w.done = (nt == 0) ? 1 : 0;
    w.acc = 0;
    w.best_rank = 0;
    w.best_t = 0xffffffffu;
    w.cells = 0;
    w.lastkey = 0;
  } else {
    w = ws[qs];
    if (w.done) return;
    const int b0 = round * kBatch, b1 = min(nt, b0 + kBatch);
    const int ql = lens[q];
    for (int x = b0; x < b1; x++) {
      const uint32_t r = res[(int64_t)qs * kWalk + x];
      const uint32_t m = r & 0xffu, L = (r >> 8) & 0xffu;
      const uint32_t t = top_seqno[(int64_t)qs * kTopHits + x];
      w.cells += (uint32_t)(ql * lens[t]);
      if (acc_tab[L * kTabM + m]) {
        const uint16_t rk = rank_tab[L * kTabM + m];
        if (!w.acc || rk > w.best_rank || (rk == w.best_rank && t < w.best_t)) {
          w.best_rank = rk;
          w.best_t = t;
        }
        w.acc = 1;
      }
    }
    w.w = (uint8_t)b1;
    const uint32_t tl = lens[top_seqno[(int64_t)qs * kTopHits + b1 - 1]];
    w.lastkey = ((unsigned long long)(127u - top_count[(int64_t)qs * kTopHits + b1 - 1]) << 56) |
                ((unsigned long long)tl << 48) | top_seqno[(int64_t)qs * kTopHits + b1 - 1];
    if (w.acc || b1 >= nt || b1 >= kWalk) w.done = 1;
  }
  ws[qs] = w;
  if (!w.done) {
    const int b0 = w.w, b1 = min(nt, b0 + kBatch);
    const uint32_t base = atomicAdd(npairs, (uint32_t)(b1 - b0));
    for (int x = b0; x < b1; x++) {
      const uint32_t k = base + (uint32_t)(x - b0);
      pq[k] = ((uint32_t)q << 1) | strand;
      pt[k] = top_seqno[(int64_t)qs * kTopHits + x];
      outidx[k] = (uint32_t)qs * kWalk + (uint32_t)x;
    }
  }
}

hipError_t launch_walk(int32_t round, int32_t q0, int32_t nqs, int32_t both,
                       const uint32_t* top_seqno, const uint8_t* top_count, const uint8_t* ntop,
                       const uint8_t* lens, const uint32_t* res, const uint8_t* acc_tab,
                       const uint16_t* rank_tab, WalkState* ws, uint32_t* pq, uint32_t* pt,
                       uint32_t* outidx, uint32_t* npairs, hipStream_t st) {
  if (nqs <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_walk, dim3((nqs + 255) / 256), dim3(256), 0, st, round, q0, nqs, both,
                     top_seqno, top_count, ntop, lens, res, acc_tab, rank_tab, ws, pq, pt, outidx,
                     npairs);
  return hipGetLastError();
}

// every peer pair (query vs an earlier query of the peer window [w0, q) that passed the k-mer
// threshold) is aligned speculatively in the same pass, so the host can run the exact merged walk
// without another round trip whichever peers turn out to be centroids
__global__ void k_peer_pairs(int32_t q0, int32_t w0, int32_t nqs, int32_t both, const uint16_t* __restrict__ peer_id,
                             const uint8_t* __restrict__ npeer, uint32_t* __restrict__ pq,
                             uint32_t* __restrict__ pt, uint32_t* __restrict__ outidx,
                             uint32_t* __restrict__ npairs) {
  // one thread per (query, strand): the slot allocation is one (wave-combined) atomic per wave
  // instead of one per row of kPeerCap lanes (same-address atomics saturate near 90 per us)
  const int qs = blockIdx.x * blockDim.x + threadIdx.x;
  if (qs >= nqs) return;
  const int np = npeer[qs];
  if (np == 255 || np == 0) return;
  const uint32_t base = atomicAdd(npairs, (uint32_t)np);
  const uint32_t qv = ((uint32_t)(q0 + qs / both) << 1) | (uint32_t)(qs % both);
  for (int x = 0; x < np; x++) {
    pq[base + x] = qv;
    pt[base + x] = (uint32_t)(w0 + peer_id[(int64_t)qs * kPeerCap + x]);
    outidx[base + x] = (uint32_t)(qs * kPeerCap + x);
  }
}

hipError_t launch_peer_pairs(int32_t q0, int32_t w0, int32_t nqs, int32_t both, const uint16_t* peer_id,
                             const uint8_t* npeer, uint32_t* pq, uint32_t* pt, uint32_t* outidx,
                             uint32_t* npairs, hipStream_t st) {
  if (nqs <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_peer_pairs, dim3((nqs + 255) / 256), dim3(256), 0, st, q0, w0, nqs, both, peer_id, npeer,
                     pq, pt, outidx, npairs);
  return hipGetLastError();
}

// ------------------------------------------------------------------ K3T: traceback
// Same DP (rows unrolled) without summaries; the direction nibble of every cell (bit0 up = D
// chosen, bit1 left = I chosen, bit2 D-extension, bit3 I-extension) goes to HBM as one column of
// CW words per step, laid out [column][word][pair] so a wave's stores are coalesced; then each lane
// runs backtrack16 over its own matrix.
template <int QL>
__global__ __launch_bounds__(64) void k_traceback(DevSeqs s, const uint32_t* __restrict__ pq,
                                                  const uint32_t* __restrict__ pt, int32_t npairs,
                                                  Scoring sc, uint32_t* __restrict__ dirbuf,
                                                  uint8_t* __restrict__ ops,
                                                  uint16_t* __restrict__ nops,
                                                  uint32_t* __restrict__ out) {
  constexpr int CW = (QL + 7) / 8;
  const int k = blockIdx.x * 64 + threadIdx.x;
  if (k >= npairs) return;
  const uint32_t qv = pq[k];
  const int32_t q = (int32_t)(qv >> 1);
  const int qstr = (int)(qv & 1u);
  const int32_t t = (int32_t)pt[k];
  const int tl = s.lens[t];
  uint32_t qw[CW];
#pragma unroll
  for (int w = 0; w < CW; w++) qw[w] = s.codes[((int64_t)q * 2 + qstr) * kCodeWords + w];
  const uint32_t* tcp = s.codes + (int64_t)t * 2 * kCodeWords;
  const int QRti = sc.go[3] + sc.ge[3], Rti = sc.ge[3];
  const int QRtr = sc.go[5] + sc.ge[5], Rtr = sc.ge[5];
  const int QRqi = sc.go[2] + sc.ge[2], Rqi = sc.ge[2];
  const int QRqr = sc.go[4] + sc.ge[4], Rqr = sc.ge[4];
  uint32_t HE[QL];
#pragma unroll
  for (int i = 0; i < QL; i++) {
    const int hleft = -(sc.go[1] + (i + 1) * sc.ge[1]);
    const int qrq = (i == QL - 1) ? QRqr : QRqi;
    HE[i] = pack_hf(hleft, sc.boundary_open ? hleft - qrq : kNegInf);
  }
  uint32_t tword = 0;
  for (int j = 0; j < tl; j++) {
    if ((j & 7) == 0) tword = tcp[j >> 3];
    const uint32_t tcode = tword & 15u;
    tword >>= 4;
    const bool tamb = (tcode & (tcode - 1u)) != 0u || tcode == 0u;
    // keep the per-row query codes from being hoisted out of the column loop (that would pin
    // QL extra VGPRs); re-extracting them is one v_bfe per cell
#pragma unroll
    for (int w = 0; w < CW; w++) asm volatile("" : "+v"(qw[w]));
    const bool lc = (j == tl - 1);
    const int QRt = lc ? QRtr : QRti;
    const int Rt = lc ? Rtr : Rti;
    int Hd = (j == 0) ? 0 : -(sc.go[0] + j * sc.ge[0]);
    int F = sc.boundary_open ? -(sc.go[0] + (j + 1) * sc.ge[0]) - QRt : kNegInf;
    uint32_t dw[CW];
#pragma unroll
    for (int w = 0; w < CW; w++) dw[w] = 0;
#pragma unroll
    for (int i = 0; i < QL; i++) {
      const uint32_t qcode = (qw[i >> 3] >> ((i & 7) * 4)) & 15u;
      const bool amb = tamb || (qcode & (qcode - 1u)) != 0u || qcode == 0u;
      const int sub = amb ? 0 : (qcode == tcode ? sc.match : sc.mismatch);
      const uint32_t he = HE[i];
      const int Hl = sx16(he);
      const int E = (int)he >> 16;
      int h = Hd + sub;
      uint32_t d = 0;
      if (F > h) { h = F; d |= 1u; }
      if (E > h) { h = E; d |= 2u; }
      const int fo = h - QRt, fe = F - Rt;
      if (fe > fo) { F = fe; d |= 4u; } else F = fo;
      const int qrq = (i == QL - 1) ? QRqr : QRqi;
      const int rq = (i == QL - 1) ? Rqr : Rqi;
      const int eo = h - qrq, ee = E - rq;
      int En = eo;
      if (ee > eo) { En = ee; d |= 8u; }
      dw[i >> 3] |= d << ((i & 7) * 4);
      Hd = Hl;
      HE[i] = pack_hf(h, En);
    }
#pragma unroll
    for (int w = 0; w < CW; w++) dirbuf[((int64_t)j * CW + w) * npairs + k] = dw[w];
  }
  const int H = sx16(HE[QL - 1]);
  // backtrack16
  uint8_t* o = ops + (int64_t)k * kOpsStride;
  int n = 0;
  int i = QL - 1, j = tl - 1;
  int aligned = 0, matches = 0;
  uint32_t op = 0;  // 0 none, 'M','D','I'
  while (i >= 0 && j >= 0) {
    aligned++;
    const uint32_t d = (dirbuf[((int64_t)j * CW + (i >> 3)) * npairs + k] >> ((i & 7) * 4)) & 15u;
    if (op == 'I' && (d & 8u)) {
      j--;
    } else if (op == 'D' && (d & 4u)) {
      i--;
    } else if (d & 2u) {
      j--;
      op = 'I';
    } else if (d & 1u) {
      i--;
      op = 'D';
    } else {
      const uint32_t qcode = (s.codes[((int64_t)q * 2 + qstr) * kCodeWords + (i >> 3)] >> ((i & 7) * 4)) & 15u;
      const uint32_t tcode = (tcp[j >> 3] >> ((j & 7) * 4)) & 15u;
      if (qcode & tcode) matches++;
      i--;
      j--;
      op = 'M';
    }
    o[kOpsStride - 1 - n] = (uint8_t)op;
    n++;
  }
  while (i >= 0) { aligned++; i--; o[kOpsStride - 1 - n] = 'D'; n++; }
  while (j >= 0) { aligned++; j--; o[kOpsStride - 1 - n] = 'I'; n++; }
  nops[k] = (uint16_t)n;
  // align_trim on the op string (alignment order = o[kOpsStride-n .. kOpsStride-1])
  const uint8_t* a0 = o + kOpsStride - n;
  int tlft = 0, trgt = 0;
  if (a0[0] != 'M') { while (tlft < n && a0[tlft] == a0[0]) tlft++; }
  if (a0[n - 1] != 'M') { while (trgt < n && a0[n - 1 - trgt] == a0[n - 1]) trgt++; }
  if (tlft >= aligned) trgt = 0;
  const uint32_t internal = (uint32_t)(aligned - tlft - trgt);
  out[k] = (uint32_t)matches | (internal << 8) | (((uint32_t)H & 0xffffu) << 16);
}

typedef void (*TraceFn)(DevSeqs, const uint32_t*, const uint32_t*, int32_t, Scoring, uint32_t*,
                        uint8_t*, uint16_t*, uint32_t*);
template <int L>
struct TraceTable {
  static void fill(TraceFn* t) {
    t[L] = k_traceback<L>;
    TraceTable<L - 1>::fill(t);
  }
};
template <>
struct TraceTable<kMinTplLen - 1> {
  static void fill(TraceFn*) {}
};

hipError_t launch_traceback(const DevSeqs& s, int32_t qlen, const uint32_t* pq, const uint32_t* pt,
                            int32_t npairs, const Scoring& sc, uint32_t* dirbuf, uint8_t* ops,
                            uint16_t* nops, uint32_t* out, hipStream_t st) {
  static TraceFn table[kMaxLen + 1] = {};
  static bool init = false;
  if (!init) {
    TraceTable<kMaxLen>::fill(table);
    init = true;
  }
  if (npairs <= 0) return hipSuccess;
  if (qlen < kMinTplLen || qlen > kMaxLen) return hipErrorInvalidValue;
  hipLaunchKernelGGL(table[qlen], dim3((npairs + 63) / 64), dim3(64), 0, st, s, pq, pt, npairs, sc,
                     dirbuf, ops, nops, out);
  return hipGetLastError();
}

// ------------------------------------------------------------------ K4: consensus
// One workgroup per cluster.  maxi[p] = longest member insertion before centroid position p
// (LDS atomicMax), the profile of residues per MSA column by LDS atomics; the gap count of a
// column is (members - residues) because every member contributes exactly one symbol to every
// column (msa.cc pads each insertion slot to maxi).  Columns inside the left/right centroid
// overhang are censored; a column emits the first strict maximum of A,C,G,T (N if none) iff its
// count >= the gap count.
constexpr int kConsThreads = 256;
struct ConsShared {
  int32_t maxi[kMaxLen + 1];
  int32_t slot[kMaxLen + 2];
  uint32_t prof[kMsaCols][5];
  int32_t emit[kMsaCols];
  int32_t alnlen;
};

__device__ __forceinline__ int sym_of4(uint32_t c4) {
  return c4 == 1 ? 0 : (c4 == 2 ? 1 : (c4 == 4 ? 2 : (c4 == 8 ? 3 : 4)));
}

__global__ __launch_bounds__(kConsThreads) void k_consensus(
    DevSeqs s, const int32_t* __restrict__ cstart, int32_t nclusters,
    const int32_t* __restrict__ member_seqno, const int32_t* __restrict__ member_opsidx,
    const uint8_t* __restrict__ member_strand, const uint8_t* __restrict__ ops,
    const uint16_t* __restrict__ nops, char* __restrict__ cons, uint16_t* __restrict__ conslen,
    int32_t* __restrict__ overflow) {
  extern __shared__ __attribute__((aligned(16))) unsigned char cs_smem[];
  ConsShared& S = *reinterpret_cast<ConsShared*>(cs_smem);
  const int c = blockIdx.x;
  const int tid = threadIdx.x;
  const int m0 = cstart[c], m1 = cstart[c + 1];
  const int m = m1 - m0;
  const int32_t cent = member_seqno[m0];
  const int clen = s.lens[cent];
  for (int x = tid; x <= clen; x += kConsThreads) S.maxi[x] = 0;
  __syncthreads();
  for (int mi = m0 + 1 + tid; mi < m1; mi += kConsThreads) {
    const int oi = member_opsidx[mi];
    const int n = nops[oi];
    const uint8_t* a0 = ops + (int64_t)oi * kOpsStride + kOpsStride - n;
    int pos = 0, run = 0;
    for (int x = 0; x < n; x++) {
      const uint8_t o = a0[x];
      if (o == 'D') {
        run++;
      } else {
        if (run) { atomicMax(&S.maxi[pos], run); run = 0; }
        pos++;
      }
    }
    if (run) atomicMax(&S.maxi[pos], run);
  }
  __syncthreads();
  if (tid == 0) {
    int acc = 0;
    for (int p = 0; p <= clen; p++) {
      S.slot[p] = acc;  // first column of insertion slot p; centroid residue p at acc + maxi[p]
      acc += S.maxi[p] + 1;
    }
    S.alnlen = acc - 1;
  }
  __syncthreads();
  const int alnlen = S.alnlen;
  if (alnlen > kMsaCols) {
    if (tid == 0) {
      atomicAdd(overflow, 1);
      conslen[c] = 0;
    }
    return;
  }
  for (int x = tid; x < alnlen; x += kConsThreads) {
    S.prof[x][0] = S.prof[x][1] = S.prof[x][2] = S.prof[x][3] = S.prof[x][4] = 0;
  }
  __syncthreads();
  // centroid residues
  for (int p = tid; p < clen; p += kConsThreads) {
    const uint32_t c4 = (s.codes[(int64_t)cent * 2 * kCodeWords + (p >> 3)] >> ((p & 7) * 4)) & 15u;
    atomicAdd(&S.prof[S.slot[p] + S.maxi[p]][sym_of4(c4)], 1u);
  }
  for (int mi = m0 + 1 + tid; mi < m1; mi += kConsThreads) {
    const int32_t sq = member_seqno[mi];
    const int st = member_strand[mi];
    const uint32_t* code = s.codes + ((int64_t)sq * 2 + st) * kCodeWords;
    const int oi = member_opsidx[mi];
    const int n = nops[oi];
    const uint8_t* a0 = ops + (int64_t)oi * kOpsStride + kOpsStride - n;
    int pos = 0, tpos = 0, run = 0;
    for (int x = 0; x < n; x++) {
      const uint8_t o = a0[x];
      if (o == 'D') {
        const uint32_t c4 = (code[tpos >> 3] >> ((tpos & 7) * 4)) & 15u;
        atomicAdd(&S.prof[S.slot[pos] + run][sym_of4(c4)], 1u);
        run++;
        tpos++;
      } else {
        run = 0;
        if (o == 'M') {
          const uint32_t c4 = (code[tpos >> 3] >> ((tpos & 7) * 4)) & 15u;
          atomicAdd(&S.prof[S.slot[pos] + S.maxi[pos]][sym_of4(c4)], 1u);
          tpos++;
        }
        pos++;
      }
    }
  }
  __syncthreads();
  const int left = S.maxi[0], right = S.maxi[clen];
  for (int x = tid; x < alnlen; x += kConsThreads) {
    int e = -1;
    if (x >= left && x < alnlen - right) {
      const uint32_t* pr = S.prof[x];
      int best = 0;
      uint32_t bc = 0;
      for (int y = 0; y < 4; y++)
        if (pr[y] > bc) { bc = pr[y]; best = y; }
      if (bc == 0 && pr[4] > 0) { bc = pr[4]; best = 4; }
      const uint32_t res = pr[0] + pr[1] + pr[2] + pr[3] + pr[4];
      const uint32_t gaps = (uint32_t)m - res;
      if (bc >= gaps) e = best;
    }
    S.emit[x] = e;
  }
  __syncthreads();
  if (tid == 0) {
    const char sym[5] = {'A', 'C', 'G', 'T', 'N'};
    int n = 0;
    char* dst = cons + (int64_t)c * kConsCap;
    for (int x = 0; x < alnlen; x++) {
      if (S.emit[x] >= 0) {
        if (n < kConsCap) dst[n] = sym[S.emit[x]];
        n++;
      }
    }
    if (n > kConsCap) {
      atomicAdd(overflow, 1);
      n = kConsCap;
    }
    conslen[c] = (uint16_t)n;
  }
}

hipError_t launch_consensus(const DevSeqs& s, const int32_t* cstart, int32_t nclusters,
                            const int32_t* member_seqno, const int32_t* member_opsidx,
                            const uint8_t* member_strand, const uint8_t* ops,
                            const uint16_t* nops, char* cons, uint16_t* conslen,
                            int32_t* overflow, hipStream_t st) {
  if (nclusters <= 0) return hipSuccess;
  const size_t smem = sizeof(ConsShared);
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)k_consensus,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL(k_consensus, dim3(nclusters), dim3(kConsThreads), smem, st, s, cstart,
                     nclusters, member_seqno, member_opsidx, member_strand, ops, nops, cons,
                     conslen, overflow);
  return hipGetLastError();
}

}  // namespace uc
