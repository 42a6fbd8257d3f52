// kernels.hip -- MI355X (gfx950) kernels of the UMI clustering hot path.
//
// The reference delegates this arithmetic to vsearch (`--cluster_fast`, invoked at
// /root/reference/ont_tcr_consensus/vsearch_umi_cluster.py:21-54 and :71-97).  Kernels:
//   K1 k_prep_wave   DUST soft-mask (vsearch mask.cc) + unique 8-mers both strands (unique.cc)
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

#include <atomic>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <mutex>

#include "align_kernels.h"
#include "umiclust_internal.h"

namespace uc {

// ------------------------------------------------------------------ per-device launch attributes
// hipFuncSetAttribute acts on the current device; one process may hold contexts on several GPUs
// (vsearch_umi_cluster.context(device)), so the "already set" flags are kept per device.
enum { k_attr_prefilter = 0, k_attr_consensus = 1, k_attr_count = 2 };
constexpr int kAttrDevices = 64;
// contexts on one device may run in different host threads: the flags are atomics (setting an
// attribute twice is harmless)
static std::atomic<bool> g_attr_set[kAttrDevices][k_attr_count];
static bool attr_set_on_device(int which) {
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= kAttrDevices) return false;  // set it every time
  return g_attr_set[d][which];
}
static void mark_attr_set(int which) {
  int d = 0;
  if (hipGetDevice(&d) == hipSuccess && d >= 0 && d < kAttrDevices) g_attr_set[d][which] = true;
}

// ------------------------------------------------------------------ character maps
// 4-bit IUPAC code (vsearch chrmap_4bit): A1 C2 G4 T/U8, ambiguity codes OR-ed, N15.
__constant__ uint8_t c_map4[256];

static uint8_t h_map4[256];
static std::once_flag h_maps_once;

static void host_maps_init() {
  const char* iupac = "ACGTURYSWKMBDHVN";
  const uint8_t v4[] = {1, 2, 4, 8, 8, 5, 10, 6, 9, 12, 3, 14, 13, 11, 7, 15};
  for (int i = 0; i < 256; i++) h_map4[i] = 0;
  for (int i = 0; iupac[i]; i++) {
    h_map4[(uint8_t)iupac[i]] = v4[i];
    h_map4[(uint8_t)(iupac[i] | 0x20)] = v4[i];
  }
}

static hipError_t ensure_maps(hipStream_t st) {
  std::call_once(h_maps_once, host_maps_init);
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
// K1 (k_prep_wave): one wave per sorted sequence, lane x
// holding residue positions x and x + 64.  DUST (mask.cc dust() / wo()): per 64-nt window (every 32 nt) lane i runs
// wo()'s inner loop for start i over its own triplet counts (a lane-private LDS row); wo()'s result is the
// lexicographically first (i, j) with the largest floor(10 sum / j) -- its strict `v > bestv` update never replaces
// an equal value -- so the window's best is the lanes' (v desc, i asc) maximum with the winner's own first j.
// Codes: 14 lanes pack 8 nibbles each.  Unique 8-mers (unique.cc): each lane builds the k-mers ending at its two
// positions (masked windows and short prefixes become distinct sentinels above every code), a bitonic sort of the
// 128 keys across the wave, then neighbour comparison and a ballot compaction -- ascending.
constexpr int kDustRow = 17;  // dwords per lane-private count row (64 u8 counters + 1: rotates the banks per lane)

__global__ __launch_bounds__(64) void k_prep_wave(const char* __restrict__ ascii, const int64_t* __restrict__ offs,
                                                  const int32_t* __restrict__ perm, int32_t n, int dust,
                                                  uint32_t* __restrict__ codes, uint8_t* __restrict__ lens,
                                                  uint16_t* __restrict__ kmers, uint8_t* __restrict__ nk,
                                                  char* __restrict__ masked, uint32_t* __restrict__ ambig,
                                                  uint8_t* __restrict__ mchg) {
  __shared__ uint8_t s_c2[2][kMaxLen + 8];   // 2-bit bases of the + strand and of its reverse complement
  __shared__ uint8_t s_c4[kMaxLen + 8];      // 4-bit codes of the output characters
  __shared__ uint8_t s_w[64];                // the DUST window's triplet words
  __shared__ uint32_t s_cnt[64 * kDustRow];  // lane-private triplet counts
  const int lane = (int)threadIdx.x;
  const int s = (int)blockIdx.x;
  if (s >= n) return;
  const int r = perm ? perm[s] : s;
  const int64_t b = offs[r];
  const int len = (int)(offs[r + 1] - b);
  const bool in0 = lane < len, in1 = lane + 64 < len;
  const uint8_t ch0 = in0 ? (uint8_t)ascii[b + lane] : (uint8_t)0, ch1 = in1 ? (uint8_t)ascii[b + 64 + lane] : (uint8_t)0;
  const uint32_t a0 = c_map4[ch0], a1 = c_map4[ch1];  // 0 past the sequence
  if (in0) {
    s_c2[0][lane] = (uint8_t)code2_of4(a0);
    s_c2[1][len - 1 - lane] = (uint8_t)code2_of4(comp4(a0));
  }
  if (in1) {
    s_c2[0][lane + 64] = (uint8_t)code2_of4(a1);
    s_c2[1][len - 65 - lane] = (uint8_t)code2_of4(comp4(a1));
  }
  __syncthreads();
  bool m0 = false, m1 = false;  // DUST-masked at positions lane, lane + 64
  if (dust) {
    for (int i0 = 0; i0 < len; i0 += 32) {
      const int l = len - i0 < 64 ? len - i0 : 64;
      const int l1 = l - 3 + 1 - 5;  // wo(): smallest region 8
      if (l1 < 0) continue;         // wo() returns 0: nothing masked
      if (lane < l) {
        uint32_t w = s_c2[0][i0 + lane];
        if (lane >= 1) w |= (uint32_t)s_c2[0][i0 + lane - 1] << 2;
        if (lane >= 2) w |= (uint32_t)s_c2[0][i0 + lane - 2] << 4;
        s_w[lane] = (uint8_t)(w & 63u);
      }
      __syncthreads();
      int bv = 0, bj = 0;
      if (lane < l1) {
        uint32_t* row = s_cnt + lane * kDustRow;
#pragma unroll
        for (int x = 0; x < 16; x++) row[x] = 0u;
        uint8_t* cnt = reinterpret_cast<uint8_t*>(row);
        int sum = 0;
        for (int j = 2; j < l - lane; j++) {
          const int x = s_w[lane + j];
          const int c = cnt[x];
          if (c) {
            sum += c;
            // v = 10*sum/j (integer); v > bv  <=>  10*sum >= (bv+1)*j
            if (10 * sum >= (bv + 1) * j) {
              bv = (10 * sum) / j;
              bj = j;
            }
          }
          cnt[x] = (uint8_t)(c + 1);
        }
      }
      uint32_t key = lane < l1 ? ((uint32_t)bv << 8) | (uint32_t)(63 - lane) : 0u;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) key = max(key, (uint32_t)__shfl_xor((int)key, d, 64));
      const int bestv = (int)(key >> 8), besti = 63 - (int)(key & 255u);
      const int bestj = __shfl(bj, besti, 64);
      if (bestv > 20) {
        const int lo = i0 + besti, hi = i0 + besti + bestj;
        m0 = m0 || (lane >= lo && lane <= hi);
        m1 = m1 || (lane + 64 >= lo && lane + 64 <= hi);
      }
      __syncthreads();  // s_w is rewritten by the next window
    }
  }
  // output characters: dust() upper-cases the sequence and lower-cases the masked intervals
  auto fin = [&](uint8_t c, bool m) -> uint8_t {
    const uint8_t up = (c >= 'a' && c <= 'z') ? (uint8_t)(c - 32) : c;
    return dust ? (m ? (uint8_t)(up | 0x20) : up) : c;
  };
  const uint8_t f0 = fin(ch0, m0), f1 = fin(ch1, m1);
  if (masked) {
    if (in0) masked[(int64_t)s * kMaxLen + lane] = (char)f0;
    if (in1) masked[(int64_t)s * kMaxLen + 64 + lane] = (char)f1;
    // sequences whose output characters differ from their input (DUST-masked or upper-cased): the file writer
    // prints the input bytes unless some sequence changed (ambig[1] counts them)
    const unsigned long long chg = __ballot((in0 && f0 != ch0) || (in1 && f1 != ch1));
    if (chg && lane == 0 && ambig) atomicAdd(ambig + 1, 1u);
    if (lane == 0 && mchg) mchg[s] = chg ? 1 : 0;
  }
  const uint32_t c40 = c_map4[f0], c41 = c_map4[f1];
  auto amb = [](uint32_t c4) { return c4 != 1u && c4 != 2u && c4 != 4u && c4 != 8u; };
  const unsigned long long anyamb = __ballot((in0 && amb(c40)) || (in1 && amb(c41)));
  if (lane == 0) {
    lens[s] = (uint8_t)len;
    if (anyamb && ambig) atomicOr(ambig, 1u);
  }
  if (in0) s_c4[lane] = (uint8_t)c40;
  if (in1) s_c4[lane + 64] = (uint8_t)c41;
  const unsigned long long mlo = __ballot(m0), mhi = __ballot(m1);
  __syncthreads();
  if (lane < kCodeWords) {
    uint32_t w0 = 0, w1 = 0;
#pragma unroll
    for (int t = 0; t < 8; t++) {
      const int p = lane * 8 + t;
      if (p < len) {
        w0 |= (uint32_t)s_c4[p] << (4 * t);
        w1 |= comp4(s_c4[len - 1 - p]) << (4 * t);
      }
    }
    codes[((int64_t)s * 2 + 0) * kCodeWords + lane] = w0;
    codes[((int64_t)s * 2 + 1) * kCodeWords + lane] = w1;
  }
  // any masked original position in [p, p + 8)
  auto win8 = [&](int p) -> bool {
    unsigned long long v;
    if (p >= 64) v = mhi >> (p - 64);
    else v = (mlo >> p) | (p > 0 ? (mhi << (64 - p)) : 0ull);
    return (v & 0xffull) != 0ull;
  };
  const unsigned long long lt = (1ull << lane) - 1ull;
  for (int st = 0; st < 2; st++) {
    uint32_t k[2];
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const int y = lane + 64 * h;  // the k-mer ending at strand position y
      bool ok = y < len && y >= 7;
      if (ok) ok = !win8(st ? len - 1 - y : y - 7);
      uint32_t km = 0;
      if (ok)
#pragma unroll
        for (int t = 0; t < 8; t++) km = (km << 2) | s_c2[st][y - 7 + t];
      k[h] = ok ? km : (0x10000u | (uint32_t)y);
    }
    // bitonic sort of the 128 keys (element e = lane + 64 h), ascending
#pragma unroll
    for (int size = 2; size <= 128; size <<= 1)
#pragma unroll
      for (int d = size >> 1; d > 0; d >>= 1) {
        if (d == 64) {
          const uint32_t lo = min(k[0], k[1]), hi = max(k[0], k[1]);
          k[0] = lo;
          k[1] = hi;
        } else {
#pragma unroll
          for (int h = 0; h < 2; h++) {
            const int e = lane + 64 * h;
            const uint32_t o = (uint32_t)__shfl_xor((int)k[h], d, 64);
            const bool asc = (e & size) == 0, lower = (e & d) == 0;
            k[h] = (lower == asc) ? min(k[h], o) : max(k[h], o);
          }
        }
      }
    // neighbours (every lane takes part in every shuffle: a shuffle from a lane outside EXEC reads nothing useful)
    const uint32_t p0 = (uint32_t)__shfl_up((int)k[0], 1, 64);
    const uint32_t k063 = (uint32_t)__shfl((int)k[0], 63, 64);
    const uint32_t k1up = (uint32_t)__shfl_up((int)k[1], 1, 64);
    const uint32_t p1 = lane == 0 ? k063 : k1up;
    const bool u0 = k[0] < 0x10000u && (lane == 0 || k[0] != p0);
    const bool u1 = k[1] < 0x10000u && k[1] != p1;
    const unsigned long long b0 = __ballot(u0), b1 = __ballot(u1);
    const int n0 = __builtin_popcountll(b0);
    uint16_t* dst = kmers + ((int64_t)s * 2 + st) * kKmerStride;
    if (u0) dst[__builtin_popcountll(b0 & lt)] = (uint16_t)k[0];
    if (u1) dst[n0 + __builtin_popcountll(b1 & lt)] = (uint16_t)k[1];
    if (lane == 0) nk[(int64_t)s * 2 + st] = (uint8_t)(n0 + __builtin_popcountll(b1));
  }
}

__global__ __launch_bounds__(256) void k_iota(int32_t* __restrict__ out, int32_t n) {
  const int32_t i = (int32_t)(blockIdx.x * 256 + threadIdx.x);
  if (i < n) out[i] = i;
}

hipError_t launch_iota(int32_t* out, int32_t n, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_iota, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, out, n);
  return hipGetLastError();
}

hipError_t launch_prep(const char* ascii, const int64_t* offs, const int32_t* perm, int32_t n,
                       int dust, uint32_t* codes, uint8_t* lens, uint16_t* kmers, uint8_t* nk,
                       char* masked, uint32_t* ambig, hipStream_t st, uint8_t* mchg) {
  hipError_t e = ensure_maps(st);
  if (e != hipSuccess) return e;
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_prep_wave, dim3((unsigned)n), dim3(64), 0, st, ascii, offs, perm, n, dust, codes, lens, kmers,
                     nk, masked, ambig, mchg);
  return hipGetLastError();
}

// ------------------------------------------------------------------ KI: index tile build
// CSR over bins (part << 16 | k-mer) of the tile's + strand unique 8-mers (vsearch dbindex.cc
// analogue).  The sequence with ordinal x (centroid ordinal; peer tiles: position in the block) goes
// to part x % kParts and its posting is directly its prefilter counter index (layout in
// umiclust_internal.h).  Lists are padded to multiples of 8 postings; padding postings point at 64
// spare counters.  One wave per tile sequence, one lane per k-mer slot (<= kMaxKmers = 65: lane and
// lane + 64), so a build issues its ~60 atomics per sequence from 60 lanes.
__global__ __launch_bounds__(256) void k_index_count(const uint16_t* __restrict__ kmers,
                                                     const uint8_t* __restrict__ nk,
                                                     const int32_t* __restrict__ map, int32_t first,
                                                     int32_t count, int32_t xoff, uint32_t* __restrict__ hist) {
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6), x = threadIdx.x & 63;
  if (c >= count) return;
  const int32_t s = map[first + c];
  const int n = nk[(int64_t)s * 2];
  const uint16_t* k = kmers + (int64_t)s * 2 * kKmerStride;
  const uint32_t pb = (uint32_t)((xoff + c) & (kParts - 1)) << 16;
  if (x < n) atomicAdd(&hist[pb | k[x]], 1u);
  if (x + 64 < n) atomicAdd(&hist[pb | k[x + 64]], 1u);
}

__device__ __forceinline__ uint32_t pad8(uint32_t v) { return (v + 7u) & ~7u; }

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}

// exclusive scan of the padded list sizes of kBins bins in two launches: per-block sums, then each
// block adds the sum of the blocks before it (a strided read of <= kScanBlocks partials) to its own
// scan.  The apply pass also writes the fill cursors (= list starts) and the padding postings, and
// re-zeroes the histogram for the tile's next build.
__global__ __launch_bounds__(256) void k_scan_reduce(const uint32_t* __restrict__ hist,
                                                     uint32_t* __restrict__ partial) {
  __shared__ uint32_t ws[4];
  const uint4 v = reinterpret_cast<const uint4*>(hist + (size_t)blockIdx.x * kScanPer)[threadIdx.x];
  const uint32_t s = wave_sum(pad8(v.x) + pad8(v.y) + pad8(v.z) + pad8(v.w));
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

__global__ __launch_bounds__(256) void k_scan_apply(uint32_t* __restrict__ hist,
                                                    const uint32_t* __restrict__ partial,
                                                    uint32_t* __restrict__ off, uint32_t* __restrict__ cursor,
                                                    uint16_t* __restrict__ post) {
  __shared__ uint32_t ws[4], wsum[4];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, b = blockIdx.x;
  uint32_t p = 0;
  for (int i = t; i < b; i += 256) p += partial[i];
  p = wave_sum(p);
  if (lane == 0) ws[wave] = p;
  uint4* h4 = reinterpret_cast<uint4*>(hist + (size_t)b * kScanPer);
  const uint4 v = h4[t];
  const uint32_t nn[4] = {v.x, v.y, v.z, v.w};
  const uint32_t pp[4] = {pad8(v.x), pad8(v.y), pad8(v.z), pad8(v.w)};
  const uint32_t s = pp[0] + pp[1] + pp[2] + pp[3];
  uint32_t inc = s;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t u = __shfl_up(inc, d, 64);
    if (lane >= d) inc += u;
  }
  if (lane == 63) wsum[wave] = inc;
  __syncthreads();
  uint32_t base = ws[0] + ws[1] + ws[2] + ws[3];
  for (int w = 0; w < wave; w++) base += wsum[w];
  const uint32_t e = base + inc - s;
  const uint32_t oo[4] = {e, e + pp[0], e + pp[0] + pp[1], e + pp[0] + pp[1] + pp[2]};
  const uint4 o = make_uint4(oo[0], oo[1], oo[2], oo[3]);
  reinterpret_cast<uint4*>(off + (size_t)b * kScanPer)[t] = o;
  reinterpret_cast<uint4*>(cursor + (size_t)b * kScanPer)[t] = o;
  // padding postings, spread over the 64 spare counters
#pragma unroll
  for (int j = 0; j < 4; j++)
    for (uint32_t u = oo[j] + nn[j]; u < oo[j] + pp[j]; u++)
      post[u] = (uint16_t)(kDummy + ((u ^ (u >> 6)) & 63u));
  h4[t] = make_uint4(0u, 0u, 0u, 0u);
  if (b == kScanBlocks - 1 && t == 255) off[kBins] = e + s;
}

__global__ __launch_bounds__(256) void k_index_fill(const uint16_t* __restrict__ kmers,
                                                    const uint8_t* __restrict__ nk,
                                                    const int32_t* __restrict__ map, int32_t first,
                                                    int32_t count, int32_t xoff, int32_t vbase, int32_t seg_mod,
                                                    uint32_t* __restrict__ cursor, uint16_t* __restrict__ post) {
  // posting order within a list is arbitrary: the prefilter only counts
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6), x = threadIdx.x & 63;
  if (c >= count) return;
  const int32_t s = map[first + c];
  const int n = nk[(int64_t)s * 2];
  const uint16_t* k = kmers + (int64_t)s * 2 * kKmerStride;
  const uint32_t xx = (uint32_t)(xoff + c);
  const uint32_t pb = (xx & (kParts - 1)) << 16;
  const uint16_t val = (uint16_t)(vbase + ((xx % (uint32_t)seg_mod) >> kPartShift));
  if (x < n) post[atomicAdd(&cursor[pb | k[x]], 1u)] = val;
  if (x + 64 < n) post[atomicAdd(&cursor[pb | k[x + 64]], 1u)] = val;
}

// Bank-aware posting order (round 6).  The counting loop (pf_count_stream) gives lane l the l-th 16-byte chunk of a
// 64-chunk window and issues the chunks' postings slot by slot: the e-th ds_add_u32 of the wave adds posting e of
// every lane's chunk.  ds_add_u32 is banked like ds_write_b32 (two 32-lane groups, bank = dword mod 32: a posting c
// hits bank (c >> 2) & 31), and each extra lane on a bank costs an LDS cycle; with postings in arbitrary order the
// busiest of 32 banks takes ~3.5 lanes.  Order within a list is free (the kernels only count), so after the fill
// every list is permuted so that chunk i, slot e holds a posting of bank (i + 4 e) mod 32 where the list's bank
// supply allows: then the lanes of one instruction that read consecutive chunks of one list hit consecutive banks.
// The permutation is the sorted matching of the postings (by bank) to the positions (by target bank), which
// minimises the bank displacement.  Simulated on random lists (scratch model, round 6): the busiest bank per
// 32-lane group falls from 3.5 to 2.1 inside long lists (most postings of a config-2 query) and to 3.3 for lists
// of ~11 chunks.  One 64-thread workgroup per list segment of up to kArrCap postings (longer lists: arranged per
// segment, targets by absolute chunk index, so consecutive segments continue the pattern).
constexpr int kArrCap = 4096;
__global__ __launch_bounds__(64) void k_list_arrange(const uint32_t* __restrict__ off, uint16_t* __restrict__ post,
                                                     int32_t nbins) {
  __shared__ uint16_t sa[kArrCap], ss[kArrCap];
  __shared__ uint32_t hb[32], ht[32];
  const int lane = (int)threadIdx.x;
  // a workgroup takes 64 consecutive bins at a time, one per lane, and arranges the lists of more than one chunk
  for (int32_t b0 = (int32_t)blockIdx.x * 64; b0 < nbins; b0 += (int32_t)gridDim.x * 64) {
   const int32_t mybin = b0 + lane;
   const uint32_t mlen = mybin < nbins ? off[mybin + 1] - off[mybin] : 0u;
   unsigned long long todo = __ballot(mlen > 8u);  // one chunk: its slots meet other lists' lanes only
   while (todo) {
    const int bl = __builtin_ctzll(todo);
    todo &= todo - 1ull;
    const int32_t bin = b0 + bl;
    const uint32_t o0 = off[bin], o1 = off[bin + 1];
    for (uint32_t seg = o0; seg < o1; seg += kArrCap) {
      const int m = (int)min<uint32_t>(kArrCap, o1 - seg);
      if (lane < 32) {
        hb[lane] = 0u;
        ht[lane] = 0u;
      }
      __syncthreads();
      for (int u = lane; u < m; u += 64) {
        const uint32_t p = post[seg + u];
        sa[u] = (uint16_t)p;
        atomicAdd(&hb[(p >> 2) & 31u], 1u);
        atomicAdd(&ht[(((seg + u) >> 3) + 4u * (u & 7)) & 31u], 1u);
      }
      __syncthreads();
      if (lane < 32) {  // exclusive scans -> cursors
        uint32_t b = hb[lane], t = ht[lane], xb = b, xt = t;
#pragma unroll
        for (int d = 1; d < 32; d <<= 1) {
          const uint32_t ub = (uint32_t)__shfl_up((int)xb, d, 64), ut = (uint32_t)__shfl_up((int)xt, d, 64);
          if (lane >= d) {
            xb += ub;
            xt += ut;
          }
        }
        hb[lane] = xb - b;
        ht[lane] = xt - t;
      }
      __syncthreads();
      for (int u = lane; u < m; u += 64) {
        const uint32_t p = sa[u];
        ss[atomicAdd(&hb[(p >> 2) & 31u], 1u)] = (uint16_t)p;
      }
      __syncthreads();
      for (int u = lane; u < m; u += 64) post[seg + u] = ss[atomicAdd(&ht[(((seg + u) >> 3) + 4u * (u & 7)) & 31u], 1u)];
      __syncthreads();
    }
   }
  }
}
hipError_t launch_index_arrange(const uint32_t* off, uint16_t* post, hipStream_t st) {
  hipLaunchKernelGGL(k_list_arrange, dim3(kBins / 64), dim3(64), 0, st, off, post, (int32_t)kBins);
  return hipGetLastError();
}

// An index append's host-side arrays (new centroids' seqnos and lengths, the seq -> ordinal range they fill, the
// bins they open) go to the device in one dispatch that reads the pinned host buffers over the bus, instead of up to
// four hipMemcpyAsync blit copies, each a kernel dispatch of its own queued on the append's stream.
__global__ __launch_bounds__(256) void k_append_stage(const int32_t* __restrict__ hc, const uint8_t* __restrict__ hl,
                                                      int32_t n, int32_t* __restrict__ dc, uint8_t* __restrict__ dl,
                                                      const int32_t* __restrict__ hs, int32_t* __restrict__ ds,
                                                      int32_t ns, const int32_t* __restrict__ hb,
                                                      int32_t* __restrict__ db, int32_t nb) {
  const int32_t m = max(n, max(ns, nb));
  for (int32_t i = (int32_t)(blockIdx.x * 256 + threadIdx.x); i < m; i += (int32_t)(gridDim.x * 256)) {
    if (i < n) {
      dc[i] = hc[i];
      dl[i] = hl[i];
    }
    if (i < ns) ds[i] = hs[i];
    if (i < nb) db[i] = hb[i];
  }
}
hipError_t launch_append_stage(const int32_t* hc, const uint8_t* hl, int32_t n, int32_t* dc, uint8_t* dl,
                               const int32_t* hs, int32_t* ds, int32_t ns, const int32_t* hb, int32_t* db, int32_t nb,
                               hipStream_t st) {
  const int32_t m = std::max(n, std::max(ns, nb));
  if (m <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_append_stage, dim3((unsigned)std::min(64, (m + 255) / 256)), dim3(256), 0, st, hc, hl, n, dc,
                     dl, hs, ds, ns, hb, db, nb);
  return hipGetLastError();
}

hipError_t launch_index_count(const uint16_t* kmers, const uint8_t* nk, const int32_t* map, int32_t first,
                              int32_t count, int32_t xoff, uint32_t* hist, hipStream_t st) {
  if (count <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_index_count, dim3((count + 3) / 4), dim3(256), 0, st, kmers, nk, map, first, count, xoff,
                     hist);
  return hipGetLastError();
}
hipError_t launch_index_scan(uint32_t* hist, uint32_t* partial, uint32_t* off, uint32_t* cursor, uint16_t* post,
                             hipStream_t st) {
  hipLaunchKernelGGL(k_scan_reduce, dim3(kScanBlocks), dim3(256), 0, st, hist, partial);
  hipLaunchKernelGGL(k_scan_apply, dim3(kScanBlocks), dim3(256), 0, st, hist, partial, off, cursor, post);
  return hipGetLastError();
}
hipError_t launch_index_fill(const uint16_t* kmers, const uint8_t* nk, const int32_t* map, int32_t first,
                             int32_t count, int32_t xoff, int32_t vbase, int32_t seg_mod, uint32_t* cursor,
                             uint16_t* post, hipStream_t st) {
  if (count <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_index_fill, dim3((count + 3) / 4), dim3(256), 0, st, kmers, nk, map, first, count, xoff,
                     vbase, seg_mod, cursor, post);
  return hipGetLastError();
}

// ------------------------------------------------------------------ K2: prefilter
// vsearch searchcore.cc search_topscores: for a (query, strand), count the query's unique 8-mers
// shared with every centroid (u8 counters), keep counters >= min(minwordmatches, #kmers) and take
// the top 41 by (count desc, length asc, seqno asc) (minheap.cc order).
//
// One 256-thread workgroup per (query-strand, part): blockIdx.x = qs * kParts + part, so the
// hardware's round-robin dispatch puts every part-p workgroup on one XCD, whose L2 then serves only
// part p's postings and offsets (~1/8 of the index).  Per counter segment (normally one):
//  lists: the (tile, k-mer) posting lists of the query (centroid tiles of the segment, then the two
//         peer tiles of the in-block window) are laid end to end as one stream of 16-byte chunks
//         (lists are padded to whole chunks by the index build, so no bounds are needed);
//  count: each wave streams a contiguous range of 64-chunk windows, lane l taking chunk 64w + l;
//         the list of every lane's chunk comes from one LDS read of the next 64 list starts, an OR
//         of one-hot start bits across the wave and a popcount.  A posting is its counter index,
//         so each of the chunk's 8 postings is one fire-and-forget ds_add_u32 on packed u8 counters;
//  scan:  counters are read back 16 per lane, a SWAR test finds every byte >= the threshold;
//  top:   candidates get 30-bit keys (count desc, length asc, sub-id asc = seqno asc within a
//         part), are selected by rank (few) or bitonic sort and merged into the part's running
//         top-41 (u64 keys); peers keep every candidate (<= kPeerCap), sorted by key.
// A threshold of 0, or more candidates than the LDS buffer holds, switches a segment to a chunked
// exact path.  The second kernel merges the kParts sorted part lists of each query-strand into the
// exact top-41 (the top-41 of a union is the top-41 of the parts' top-41s) and concatenates the
// peer lists.
constexpr int kPfThreads = 256;
constexpr int kPfWaves = kPfThreads / 64;
constexpr int kPfCand = 1024;   // LDS candidate buffer (centroids)
constexpr int kRankSel = 512;   // candidate counts up to this are selected by rank
constexpr int kPfTiles = 12;    // tiles per counter segment: 7 sealed + base + delta + kPeerTiles peer
static_assert(7 + 2 + kPeerTiles <= kPfTiles, "list table too small for the peer window");
constexpr int kPfLists = kMaxKmers * kPfTiles;
// the list-table scan packs (chunks << kListBits | lists) into 32 bits; a list holds <= kTile / kParts
// postings (<= 1024 chunks + padding), so the chunk total stays below 2^(32 - kListBits)
constexpr int kListBits = kPfLists < 1024 ? 10 : 11;
constexpr uint32_t kListMask = (1u << kListBits) - 1u;
static_assert(kPfLists < (1 << kListBits) && (uint64_t)kPfLists * (kTile / kParts / 8 + 1) < (1ull << (32 - kListBits)),
              "list-table scan overflows");
// the list table and the count loop for a workgroup of W waves (k_pf_full: 4; k_pf_count: 4, or 1 for small indexes)
template <int W>
struct PfW {
  static constexpr int kThreads = 64 * W;
  static constexpr int kTilesPerWave = (kPfTiles + W - 1) / W;
  static constexpr int kSlots = 2 * kTilesPerWave;
};

constexpr int kCge = (kMaxLen + 4) & ~3;  // cnt_ge entries in LDS, a whole number of 16-byte vectors
struct PfShared {
  union {
    struct {                        // list table (count phase)
      uint32_t lstart[kPfLists + 66];  // first chunk of each non-empty list, then the chunk total
      uint32_t lbias[kPfLists];        // posting index of chunk g of list L: lbias[L] + 8 g
      uint4 wtab[kPfWinBase];          // per 64-chunk window: x the list holding chunk 64 w, y / z bit b (b > 0):
                                       // a list starts at chunk 64 w + b (b < 32 / b >= 32); one b128 read
    };
    uint32_t cand[kPfCand];         // candidate sub-ids, then 30-bit keys (scan / select phases)
  };
  uint32_t pcand[kPeerCap + 1];     // peer keys
  unsigned long long top[kTopHits];
  unsigned long long merged[kTopHits];
  unsigned long long bestk[kTopHits];
  uint32_t wsum[kPfWaves];
  alignas(16) int32_t cge[kCge];    // a.cnt_ge, zero-padded
  uint32_t best[kPeerCap + 1];
  uint32_t ncand;
  uint32_t npc;
  uint32_t overflow;
  uint32_t post_local;
  int32_t ntop;
};
// the u8 counters follow in dynamic LDS (16-byte aligned offset)
constexpr int kPfSharedBytes = (int)((sizeof(PfShared) + 15) & ~(size_t)15);

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

// wave-uniform pointer (both halves through readfirstlane), so a descriptor built from it is scalar
template <typename T>
__device__ __forceinline__ const T* uniform_ptr(const T* p) {
  const uint64_t v = (uint64_t)p;
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
  return (const T*)(((uint64_t)hi << 32) | lo);
}

// postings are read with buffer loads (counted on vmcnt only): flat loads also count on lgkmcnt, so
// every wait for them would drain the fire-and-forget LDS atomics too
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t arena_rsrc(const uint16_t* uniform_base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(uniform_base), (short)0, 0x7fffffff,
                                           0x00020000);
}
__device__ __forceinline__ uint4 ld_chunk(__amdgpu_buffer_rsrc_t r, uint32_t idx) {
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(idx * 2u), 0, 0);
  return make_uint4(v.x, v.y, v.z, v.w);
}

// two consecutive list offsets of a tile (wave-uniform base): a buffer load, so nothing waits on
// lgkmcnt for it and the loads of all slots are in flight together
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u32x2 ld_off2(const uint32_t* uniform_off, uint32_t idx) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(uniform_off), (short)0, 0x7fffffff, 0x00020000);
  return __builtin_amdgcn_raw_buffer_load_b64(r, (int)(idx * 4u), 0, 0);
}

// a tile view through scalar loads (the address is wave-uniform and the views are read-only)
__device__ __forceinline__ TileView load_view(const TileView* p) {
  const __attribute__((address_space(4))) u32x4* q = (const __attribute__((address_space(4))) u32x4*)p;
  struct Raw {
    u32x4 a, b;
  } r{q[0], q[1]};
  return __builtin_bit_cast(TileView, r);
}

// centroid tile view i of a pass: from the kernel arguments, or the device array past kArgTiles tiles
__device__ __forceinline__ TileView cent_view(const PrefilterArgs& a, int i) {
  return a.ntiles <= kArgTiles ? a.tv[i] : load_view(a.tiles + i);
}

// packs: the bytes of a counter word from byte nb on (nb <= 0: all four, nb >= 4: none)
__device__ __forceinline__ uint32_t keep_from(int nb) {
  return nb <= 0 ? 0xffffffffu : nb >= 4 ? 0u : ~((1u << (8 * nb)) - 1u);
}
// packs: the query's bin bounds (PrefilterArgs::qbin): seq0 = its first seqno, ord0 = its first centroid ordinal
__device__ __forceinline__ void pack_bounds(const PrefilterArgs& a, int32_t q, int32_t& seq0, int32_t& ord0) {
  seq0 = 0;
  ord0 = 0;
  if (a.qbin) {
    const int32_t qb = __builtin_amdgcn_readfirstlane(a.qbin[q]);
    seq0 = __builtin_amdgcn_readfirstlane(a.bin_seq0[qb]);
    ord0 = __builtin_amdgcn_readfirstlane(a.bin_ord0[qb]);
  }
}
// first counter sub-id of a part whose ordinal (seg0 + (c << kPartShift) + part) is >= ord0
__device__ __forceinline__ int32_t pack_cmin(int32_t ord0, int32_t seg0, int part, int32_t nsub) {
  const int64_t d = (int64_t)ord0 - seg0 - part;
  return d <= 0 ? 0 : (int32_t)min<int64_t>((int64_t)nsub, (d + kParts - 1) >> kPartShift);
}
// first peer byte index (4 x + b) of a peer tile whose seqno (base + ((4 x + b) << kPartShift) + part) is >= seq0
__device__ __forceinline__ int32_t pack_pmin(int32_t seq0, int32_t base, int part) {
  const int64_t d = (int64_t)seq0 - base - part;
  return d <= 0 ? 0 : (int32_t)min<int64_t>(1 << 24, (d + kParts - 1) >> kPartShift);
}

// The u8 counters live at LDS byte kBase (k_pf_count: 0, k_pf_full: kPfSharedBytes).  Neither kernel has
// static LDS, so the dynamic LDS starts at address 0 and the base folds into the ds_add offset field.
typedef __attribute__((address_space(3))) uint32_t lds_u32;
template <uint32_t kBase>
__device__ __forceinline__ void lds_add(uint32_t byte_addr, uint32_t v) {
  // result unused -> ds_add_u32 (no return)
  __hip_atomic_fetch_add((lds_u32*)(uintptr_t)(kBase + byte_addr), v, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_WORKGROUP);
}
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
// the 8 postings of a chunk: one counter increment each (`one` = 0 adds nothing: lanes past the stream).
// Posting c is the counter byte: dword c & ~3, byte c & 3, i.e. add one << 8 (c & 3).  Per posting pair
// (a u32 of the chunk): one packed shift puts (c & 3) << 3 into the low 5 bits of both halves (the
// shifter reads only those), the high half's shift selects word 1 by SDWA: 5 VALU per pair.
template <uint32_t kBase>
__device__ __forceinline__ void pf_chunk(const uint4& v, uint32_t one) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int e = 0; e < 4; e++) {
    const uint32_t x = w[e];
    const uint32_t t = __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, x) << (u16x2){3, 3});
    uint32_t vhi;
    asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD"
        : "=v"(vhi)
        : "v"(t), "v"(one));
    lds_add<kBase>(x & 0xfffcu, one << (t & 31u));
    lds_add<kBase>((x >> 16) & 0xfffcu, vhi);
  }
}

// Inclusive wave scans on the VALU through DPP (no LDS traffic, unlike ds_bpermute shuffles, whose
// lgkmcnt waits would also drain the counting loop's LDS atomics): Hillis-Steele over rows of 16
// lanes (row_shr 1, 2, 4, 8; lanes shifted in from outside the row read 0), then lane 15 of rows 0/2
// into rows 1/3 (row_bcast:15) and lane 31 into rows 2/3 (row_bcast:31).  All 64 lanes must be active.
template <typename Op>
__device__ __forceinline__ uint32_t wave_scan_dpp(uint32_t v, Op op) {
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true));
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true));
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true));
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true));
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false));
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false));
  return v;
}
// two independent OR scans interleaved (fills the DPP read-after-write wait states)
__device__ __forceinline__ void wave_or2_dpp(uint32_t& a, uint32_t& b) {
#define UC_DPP2(ctrl, rmask, bc)                                                    \
  {                                                                                 \
    const uint32_t ta = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)a, ctrl, rmask, 0xf, bc); \
    const uint32_t tb = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)b, ctrl, rmask, 0xf, bc); \
    a |= ta;                                                                        \
    b |= tb;                                                                        \
  }
  UC_DPP2(0x111, 0xf, true)
  UC_DPP2(0x112, 0xf, true)
  UC_DPP2(0x114, 0xf, true)
  UC_DPP2(0x118, 0xf, true)
  UC_DPP2(0x142, 0xa, false)
  UC_DPP2(0x143, 0xc, false)
#undef UC_DPP2
}
struct OpAdd {
  __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a + b; }
};
struct OpOr {
  __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a | b; }
};
__device__ __forceinline__ uint32_t lane63(uint32_t v) { return (uint32_t)__builtin_amdgcn_readlane((int)v, 63); }

// wave-aggregated allocation of n slots per lane from an LDS counter (all 64 lanes active): one
// atomic per wave; returns the lane's first slot
__device__ __forceinline__ uint32_t wave_alloc(uint32_t n, uint32_t* counter) {
  const uint32_t inc = wave_scan_dpp(n, OpAdd());
  const uint32_t tot = lane63(inc);
  uint32_t b = 0;
  if (tot) {
    if ((threadIdx.x & 63) == 0) b = atomicAdd(counter, tot);
    b = (uint32_t)__builtin_amdgcn_readfirstlane((int)b);
  }
  return b + inc - n;
}

// exclusive scan over the workgroup (every thread must call it); one DPP scan per wave, one barrier: the caller
// must pass another barrier before wsum is written again (pf_list_table ends with one)
template <int W = kPfWaves>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* wsum, uint32_t& total) {
  const int wave = threadIdx.x >> 6;
  const uint32_t inc = wave_scan_dpp(v, OpAdd());
  if (W == 1) {  // one wave: no barrier, no LDS
    total = lane63(inc);
    return inc - v;
  }
  if ((threadIdx.x & 63) == 63) wsum[wave] = inc;
  __syncthreads();
  uint32_t base = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < W; w++) {
    const uint32_t x = wsum[w];
    base += (w < wave) ? x : 0u;
    tot += x;
  }
  total = tot;
  return base + inc - v;
}

// The list table of one counting pass.  Wave w takes tiles w, w + kPfWaves, ... (the tile view is
// wave-uniform: scalar loads, issued before anything waits) and lane l the query's k-mers l and l + 64;
// every slot's offsets are loaded unconditionally (an absent tile reads the own peer tile's offsets, a
// k-mer slot past nk reads list 0) and masked afterwards.  A packed block scan lays the non-empty lists
// end to end as one stream of T 16-byte chunks: lstart[L] = first chunk of list L (then T), lbias[L] =
// posting index of chunk g of list L minus 8 g; per 64-chunk window w < kPfWinBase, wtab[w].x = the list
// holding chunk 64 w and wtab[w].y / .z bit b = a list starts at chunk 64 w + b (b > 0).  Ends with a barrier.
// a part candidate for the merge: count << 24 | ordinal (ordinals stay below kMaxSegs * kSegCentroids < 2^23)
static_assert(kMaxSegs * kSegCentroids < (1 << 24), "ordinal field");
__device__ __forceinline__ uint32_t cand_entry(unsigned long long key64) {
  return ((127u - (uint32_t)(key64 >> 56)) << 24) | (uint32_t)(key64 & 0xffffffu);
}
struct PfTable {
  uint32_t* lstart;
  uint32_t* lbias;
  uint4* wtab;  // per window {base list, start bits 0-31, start bits 32-63, 0}
  uint32_t* wsum;
};
// the list offsets of a wave's tiles, issued as loads (pf_list_table waits for them): k_pf_count issues them before
// zeroing its counters, so the zeroing's LDS stores overlap their memory latency
template <int W = kPfWaves>
struct PfOffsets {
  TileView tvs[PfW<W>::kTilesPerWave];
  u32x2 o0[PfW<W>::kTilesPerWave], o1[PfW<W>::kTilesPerWave];
};
template <int W = kPfWaves>
__device__ __forceinline__ void pf_list_offsets(const PrefilterArgs& a, int t0, int nct, int ntl, int part, int thr,
                                                uint32_t km0, uint32_t km1, int wv, PfOffsets<W>& r) {
  constexpr int kTPW = PfW<W>::kTilesPerWave;
#pragma unroll
  for (int it = 0; it < kTPW; it++) {
    const int ti = wv + it * W;
    if (ti < nct) r.tvs[it] = cent_view(a, t0 + ti);
    else if (ti < ntl) r.tvs[it] = a.peer[ti - nct];
    else r.tvs[it].n = 0;
  }
#pragma unroll
  for (int it = 0; it < kTPW; it++) {
    const bool live = thr > 0 && r.tvs[it].n > 0;
    const uint32_t* op = uniform_ptr((live ? r.tvs[it].off : a.peer[kPeerTiles - 1].off) + ((uint32_t)part << 16));
    r.o0[it] = ld_off2(op, km0);
    r.o1[it] = ld_off2(op, km1);
  }
}
template <int W = kPfWaves>
__device__ __forceinline__ void pf_list_table(const PrefilterArgs& a, const PfTable& tb, const PfOffsets<W>& r,
                                              uint64_t pbase, int thr, int nk, int lane, int tid, uint32_t& T,
                                              uint32_t& nlc, bool prof = false, unsigned long long* clk0 = nullptr,
                                              unsigned long long* clk1 = nullptr) {
  constexpr int kTPW = PfW<W>::kTilesPerWave, kSl = PfW<W>::kSlots;
  const TileView* tvs = r.tvs;
  const u32x2* o0 = r.o0;
  const u32x2* o1 = r.o1;
  uint32_t nch[kSl], bse[kSl], sum_ch = 0, sum_ne = 0;
#pragma unroll
  for (int it = 0; it < kTPW; it++) {
    const bool live = thr > 0 && tvs[it].n > 0;
    const uint32_t tbase = (uint32_t)(tvs[it].post_base - pbase);
    const uint32_t c0 = (live && lane < nk) ? (o0[it].y - o0[it].x) >> 3 : 0u;
    const uint32_t c1 = (live && lane + 64 < nk) ? (o1[it].y - o1[it].x) >> 3 : 0u;
    nch[2 * it] = c0;
    bse[2 * it] = tbase + o0[it].x;
    nch[2 * it + 1] = c1;
    bse[2 * it + 1] = tbase + o1[it].x;
  }
#pragma unroll
  for (int j = 0; j < kSl; j++) {
    sum_ch += nch[j];
    sum_ne += nch[j] ? 1u : 0u;
  }
  if (prof) *clk0 = __builtin_readcyclecounter();  // phase probe: the list offsets have arrived
  // window start masks (set below, after block_excl_scan's barriers; one wave: its LDS operations stay in order)
  for (int i = tid; i < kPfWinBase; i += PfW<W>::kThreads) tb.wtab[i] = make_uint4(0u, 0u, 0u, 0u);
  // packed scan: chunks << kListBits | lists (see kListBits)
  uint32_t tot;
  const uint32_t ex = block_excl_scan<W>((sum_ch << kListBits) | sum_ne, tb.wsum, tot);
  if (prof) *clk1 = __builtin_readcyclecounter();
  T = tot >> kListBits;
  nlc = tot & kListMask;
  uint32_t li = ex & kListMask, ci = ex >> kListBits;
#pragma unroll
  for (int j = 0; j < kSl; j++)
    if (nch[j]) {
      tb.lstart[li] = ci;
      tb.lbias[li] = bse[j] - 8u * ci;
      if ((ci & 63u) != 0u && (ci >> 6) < (uint32_t)kPfWinBase)
        atomicOr(reinterpret_cast<uint32_t*>(tb.wtab + (ci >> 6)) + ((ci & 32u) ? 2 : 1), 1u << (ci & 31u));
      // windows whose first chunk lies in this list
      for (uint32_t w = (ci + 63u) >> 6; (w << 6) < ci + nch[j] && w < (uint32_t)kPfWinBase; w++)
        tb.wtab[w].x = li;
      li++;
      ci += nch[j];
    }
  for (int i = tid; i < 66; i += PfW<W>::kThreads) tb.lstart[nlc + i] = T;
  __syncthreads();
}

// Count the stream of T chunks into the u8 counters at LDS byte kBase (every wave; no barrier).
// Arena index of a lane's chunk of window w (~0u past the stream's end): the window's base list m (the one
// holding chunk 64 w) and the lists starting inside it come from the table (windows past kPfWinBase: a
// binary search over lstart and a DPP OR-scan of the starts), and the lane's list is m + the starts at or
// before it.  Wave v counts windows v, v + 4, v + 8, ... in batches of two, one batch of loads in flight
// ahead of the batch being counted; two register sets are used alternately (a copy between them would wait
// for the loads in flight).  A lane past the end of the stream reads chunk 0 and adds 0; a window past the
// end is skipped (wave-uniform branch).
template <uint32_t kBase, int W = kPfWaves>
__device__ __forceinline__ void pf_count_stream(__amdgpu_buffer_rsrc_t arena, uint32_t T, uint32_t nlc,
                                                const uint32_t* lstart, const uint32_t* lbias,
                                                const uint4* wtab, int lane, int wv) {
  const uint32_t nwin = (T + 63u) >> 6;
  const unsigned long long below = (2ull << lane) - 1ull;  // lanes <= this one
  const uint32_t below_lo = lane < 32 ? (2u << lane) - 1u : 0xffffffffu;
  const uint32_t below_hi = lane < 32 ? 0u : (2u << (lane - 32)) - 1u;
  auto window = [&](uint32_t w) -> uint32_t {
    if (w >= nwin) return 0xffffffffu;
    const uint32_t g0 = w << 6, g = g0 + (uint32_t)lane;
    if (w < (uint32_t)kPfWinBase) {
      const uint4 t = wtab[w];  // one uniform b128 read (was three)
      const uint32_t L0 = t.x + (uint32_t)__builtin_popcount(t.y & below_lo) + (uint32_t)__builtin_popcount(t.z & below_hi);
      return g < T ? lbias[L0] + 8u * g : 0xffffffffu;
    }
    int lo = 0, hi = (int)nlc - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (lstart[mid] <= g0) lo = mid;
      else hi = mid - 1;
    }
    const uint32_t m = (uint32_t)lo;
    const uint32_t bit = lstart[m + 1 + lane] - g0;
    uint32_t lo32 = bit < 32u ? 1u << bit : 0u, hi32 = bit - 32u < 32u ? 1u << (bit - 32u) : 0u;
    wave_or2_dpp(lo32, hi32);
    const unsigned long long sm = ((unsigned long long)lane63(hi32) << 32) | lane63(lo32);
    const uint32_t L0 = m + (uint32_t)__builtin_popcountll(sm & below);
    return g < T ? lbias[L0] + 8u * g : 0xffffffffu;
  };
  // a lane past the end of the stream adds 0 to the postings of chunk `lane` (any valid chunk): with every such lane
  // on chunk 0, as before round 6, a partial last window's idle lanes all hit the same 8 counter dwords, and
  // same-address atomics serialise (up to 32 lanes of a group on one address)
  auto ldv = [&](uint32_t i) { return ld_chunk(arena, i == 0xffffffffu ? (uint32_t)lane << 3 : i); };
  auto one = [](uint32_t i) { return i != 0xffffffffu ? 1u : 0u; };
  constexpr uint32_t S1 = W;
  uint32_t w = (uint32_t)wv;  // wave-uniform (SGPR): the window bounds are scalar branches
  uint32_t a0 = window(w), a1 = window(w + S1);
  uint4 v0 = ldv(a0), v1 = ldv(a1);
  for (; w < nwin; w += 4 * S1) {
    const uint32_t b0 = window(w + 2 * S1), b1 = window(w + 3 * S1);
    const uint4 u0 = ldv(b0), u1 = ldv(b1);
    pf_chunk<kBase>(v0, one(a0));
    if (w + S1 < nwin) pf_chunk<kBase>(v1, one(a1));
    a0 = window(w + 4 * S1);
    a1 = window(w + 5 * S1);
    v0 = ldv(a0);
    v1 = ldv(a1);
    if (w + 2 * S1 < nwin) pf_chunk<kBase>(u0, one(b0));
    if (w + 3 * S1 < nwin) pf_chunk<kBase>(u1, one(b1));
  }
}

// The full counting kernel: every counter segment (bins beyond kSegCentroids centroids) and the exact
// selection of a part's top-41 for any candidate count (it also re-runs the units the lean kernel could
// not finish: more than kPartCand candidates, or a threshold of 0).  One (query-strand, part) unit.
__device__ __forceinline__ void pf_full_unit(const PrefilterArgs& a, uint32_t unit, unsigned char* pf_smem) {
  PfShared& S = *reinterpret_cast<PfShared*>(pf_smem);
  uint32_t* cnt = reinterpret_cast<uint32_t*>(pf_smem + kPfSharedBytes);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // optional phase timing (a.prof != nullptr): thread 0's shader-clock deltas between barriers
  const bool prof = a.prof != nullptr && tid == 0 && unit % 61u == 0;  // sampled units
  unsigned long long tprev = prof ? __builtin_readcyclecounter() : 0ull, tacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define PF_MARK(i)                                              \
  if (prof) {                                                   \
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); \
    const unsigned long long t_ = __builtin_readcyclecounter(); \
    tacc[i] += t_ - tprev;                                      \
    tprev = t_;                                                 \
  }
  const int part = (int)(unit & (kParts - 1));
  const int qs = (int)(unit >> kPartShift);
  const int qlocal = qs / a.both;
  const int strand = qs % a.both;
  const int32_t q = a.q0 + qlocal;
  // every wave keeps the query's k-mers in registers: lane l holds k-mers l and l + 64 (the k-mer
  // slots are loaded unconditionally, together with their count, and masked afterwards)
  const int nk = a.seqs.nk[(int64_t)q * 2 + strand];
  const uint16_t* qk = a.seqs.kmers + ((int64_t)q * 2 + strand) * kKmerStride;
  const uint32_t raw0 = qk[lane], raw1 = qk[64 + (lane < kKmerStride - 64 ? lane : 0)];
  const int thr = nk < a.minwordmatches ? nk : a.minwordmatches;
  const uint32_t km0 = lane < nk ? raw0 : 0u, km1 = lane + 64 < nk ? raw1 : 0u;
  PF_MARK(5)
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  if (tid == 0) {
    S.ntop = 0;
    S.post_local = 0;
  }
  if (tid < kCge) S.cge[tid] = tid <= kMaxLen ? a.cnt_ge[tid] : 0;
  const int64_t pq_ = (int64_t)qs * kParts + part;
  int32_t seq0, ord0;
  pack_bounds(a, q, seq0, ord0);
  const int npass = a.nseg > 0 ? a.nseg : 1;
  uint4* cnt4 = reinterpret_cast<uint4*>(cnt);
  for (int sg = 0; sg < npass; sg++) {
    const bool last = sg == npass - 1;
    const int t0 = a.nseg > 0 ? a.seg_tile[sg] : 0;
    const int nct = a.nseg > 0 ? a.seg_tile[sg + 1] - t0 : 0;  // centroid tiles of this segment
    const int ntl = nct + (last ? kPeerTiles : 0);              // + the peer tiles in the last pass
    const int seg0 = sg * kSegCentroids;
    const int segn = min(a.ncent - seg0, kSegCentroids);
    const int nsubC = segn > part ? (segn - part + kParts - 1) >> kPartShift : 0;
    const int ncnt = kCentBase + ((nsubC + 15) & ~15);         // counter bytes in use
    // the pass's postings are addressed from its lowest arena slot (32-bit buffer offsets)
    const uint64_t pbase = a.seg_base[sg];
    const __amdgpu_buffer_rsrc_t arena = arena_rsrc(uniform_ptr(a.arena + pbase));
    for (int x = tid; x < (ncnt >> 4); x += kPfThreads) cnt4[x] = make_uint4(0u, 0u, 0u, 0u);
    if (tid == 0) {
      S.ncand = 0;
      S.npc = 0;
      S.overflow = 0;
    }
    uint32_t T, nlc;
    PfOffsets offs;
    pf_list_offsets(a, t0, nct, ntl, part, thr, km0, km1, wv, offs);
    pf_list_table(a, PfTable{S.lstart, S.lbias, S.wtab, S.wsum}, offs, pbase, thr, nk, lane, tid, T, nlc);
    PF_MARK(0)
    if (T > 0) pf_count_stream<kPfSharedBytes>(arena, T, nlc, S.lstart, S.lbias, S.wtab, lane, wv);
    __syncthreads();
    PF_MARK(1)
    if (wave == 0) {
      // postings touched (stats): every chunk posting minus the padding ones, counted by the spare
      // counters (<= 7 pads per list spread over 64 counters: no u8 overflow in practice)
      const uint8_t* cb = reinterpret_cast<const uint8_t*>(cnt);
      const uint32_t pads = lane63(wave_scan_dpp((uint32_t)cb[kDummy + lane], OpAdd()));
      if (lane == 0) S.post_local += 8u * T - pads;
    }
    // scan: centroid counters >= thr (SWAR: bytes <= 65, so byte + 128 - thr sets bit 7 iff >= thr);
    // each wave sweeps 64 counter vectors per step and takes LDS slots with one atomic per step
    const uint32_t add = (uint32_t)(128 - thr) * 0x01010101u;
    const int32_t cmin = pack_cmin(ord0, seg0, part, nsubC);  // packs: earlier bins' centroids are never candidates
    if (thr > 0) {
      const int lim4 = (nsubC + 15) >> 4;  // counters past nsubC are zero (< thr)
      const uint4* c4 = cnt4 + kCentBase / 16;
      for (int x0 = (cmin >> 4) + wv * 64; x0 < lim4; x0 += kPfThreads) {
        const int x = x0 + lane;
        uint4 v = x < lim4 ? c4[x] : make_uint4(0u, 0u, 0u, 0u);
        const int cb = cmin - x * 16;
        if (cb > 0) v = make_uint4(v.x & keep_from(cb), v.y & keep_from(cb - 4), v.z & keep_from(cb - 8), v.w & keep_from(cb - 12));
        // most sweeps hold no candidate: one OR over the four words decides (no carries cross bytes)
        if (__ballot((((v.x + add) | (v.y + add) | (v.z + add) | (v.w + add)) & 0x80808080u) != 0u) == 0ull)
          continue;
        uint32_t mk[4] = {(v.x + add) & 0x80808080u, (v.y + add) & 0x80808080u, (v.z + add) & 0x80808080u,
                          (v.w + add) & 0x80808080u};
        const uint32_t n = (uint32_t)(__builtin_popcount(mk[0]) + __builtin_popcount(mk[1]) +
                                      __builtin_popcount(mk[2]) + __builtin_popcount(mk[3]));
        uint32_t slot = wave_alloc(n, &S.ncand);
#pragma unroll
        for (int j = 0; j < 4; j++) {
          while (mk[j]) {
            const uint32_t byte = (uint32_t)__builtin_ctz(mk[j]) >> 3;
            mk[j] &= mk[j] - 1u;
            if (slot < (uint32_t)kPfCand) S.cand[slot] = (uint32_t)x * 16u + (uint32_t)j * 4u + byte;
            else S.overflow = 1;
            slot++;
          }
        }
      }
    }
    if (last) {
      // peers: the window queries before q, every count >= thr (all of them when thr == 0)
#pragma unroll
      for (int v = 0; v < kPeerTiles; v++) {
        const TileView pv = a.peer[v];
        if (pv.n <= 0) continue;
        const int lim = min(pv.n, q - pv.base);
        const int nsubP = lim > part ? (lim - part + kParts - 1) >> kPartShift : 0;
        const int nwords = (nsubP + 3) >> 2;
        const uint32_t* pw = cnt + pv.seg * (kPeerRegion / 4);
        const int32_t pmin = pack_pmin(seq0, pv.base, part);  // packs: earlier bins' queries are never peers
        for (int x0 = (pmin >> 2) + wv * 64; x0 < nwords; x0 += kPfThreads) {
          const int x = x0 + lane;
          const uint32_t w = x < nwords ? pw[x] & keep_from(pmin - 4 * x) : 0u;
          const int valid = x < nwords ? min(4, nsubP - 4 * x) : 0;  // bytes of peers before q
          uint32_t mk = (w + add) & 0x80808080u & (valid >= 4 ? 0xffffffffu : (1u << (8 * valid)) - 1u);
          if (__ballot(mk != 0u) == 0ull) continue;
          uint32_t slot = wave_alloc((uint32_t)__builtin_popcount(mk), &S.npc);
          while (mk) {
            const uint32_t byte = (uint32_t)__builtin_ctz(mk) >> 3;
            mk &= mk - 1u;
            const uint32_t cv = (w >> (8 * byte)) & 0xffu;
            const int32_t sq = pv.base + ((4 * x + (int)byte) << kPartShift) + part;
            // the peer's own length (an O4 round tile spans several lengths; k_pf_merge keys peers the same way)
            const uint32_t key = ((127u - cv) << 23) | ((uint32_t)a.seqs.lens[sq] << 16) | (uint32_t)(sq - a.peer_base);
            if (slot <= (uint32_t)kPeerCap) S.pcand[slot] = key;
            slot++;
          }
        }
      }
    }
    __syncthreads();
    PF_MARK(2)
    const bool scan_mode = (thr == 0) || S.overflow;
    const int nchunks = scan_mode ? (nsubC + kPfCand - 1) / kPfCand : 1;
    for (int ch = 0; ch < nchunks; ch++) {
      if (scan_mode) {
        __syncthreads();
        if (tid == 0) S.ncand = 0;
        __syncthreads();
        const int c0 = ch * kPfCand;
        const int c1 = min(nsubC, c0 + kPfCand);
        for (int c = max(c0, cmin) + tid; c < c1; c += kPfThreads)
          if ((int)cnt_get(cnt, (uint32_t)(kCentBase + c)) >= thr) S.cand[atomicAdd(&S.ncand, 1u)] = (uint32_t)c;
        __syncthreads();
      }
      const int nc = (int)min(S.ncand, (uint32_t)kPfCand);
      // keys: (127-count) << 23 | len << 16 | sub-id   (30 bits, unique within the part of a segment;
      // sub-id order is ordinal = seqno order, so key order is (count desc, length asc, seqno asc))
      for (int x = tid; x < nc; x += kPfThreads) {
        const uint32_t c = S.cand[x];
        const uint32_t cntv = cnt_get(cnt, kCentBase + c);
        const int32_t ord = seg0 + (int32_t)(c << kPartShift) + part;
        // the centroid's length from the ordinal table (a packs' lengths are not monotone in the ordinal across bins,
        // so the cnt_ge count of round 2 no longer applies; one L2 read per candidate on this rare path)
        const uint32_t len = (uint32_t)a.cent_len[ord];
        S.cand[x] = ((127u - cntv) << 23) | (len << 16) | c;
      }
      __syncthreads();
      // best 41 of the segment part in key order: by rank (all-pairs count, broadcast LDS reads)
      // when the candidate set is small, by a bitonic sort otherwise.  With one pass (one counter
      // segment, no chunked scan) they are the part's final list and go straight to HBM.
      const bool direct = npass == 1 && !scan_mode;
      // u64 key: (127-count) << 56 | len << 48 | ordinal (the ordinal stands in for the seqno: same
      // order; k_pf_merge maps it)
      auto key64 = [&](uint32_t key) {
        const int32_t ord = seg0 + (int32_t)((key & 0xffffu) << kPartShift) + part;
        return ((unsigned long long)(key >> 23) << 56) | ((unsigned long long)((key >> 16) & 0x7fu) << 48) |
               (unsigned long long)(uint32_t)ord;
      };
      const int nbest = nc < kTopHits ? nc : kTopHits;
      if (nc <= kRankSel) {
        for (int x = tid; x < nc; x += kPfThreads) {
          const uint32_t kx = S.cand[x];
          int r = 0;
          for (int y = 0; y < nc; y++) r += S.cand[y] < kx;
          if (r < kTopHits) {
            if (direct) a.pcand[pq_ * kPartCand + r] = cand_entry(key64(kx));
            else S.best[r] = kx;
          }
        }
      } else {
        int np2 = 1;
        while (np2 < nc) np2 <<= 1;
        for (int x = nc + tid; x < np2; x += kPfThreads) S.cand[x] = 0xffffffffu;
        __syncthreads();
        bitonic_u32(S.cand, np2);
        for (int x = tid; x < nbest; x += kPfThreads) {
          if (direct) a.pcand[pq_ * kPartCand + x] = cand_entry(key64(S.cand[x]));
          else S.best[x] = S.cand[x];
        }
      }
      if (direct) {
        if (tid == 0) S.ntop = -1 - nbest;  // written already
        break;
      }
      __syncthreads();
      // merge into the running top-41 (u64 keys, unique seqnos): every element of either sorted
      // list finds its merged position by binary search in the other list
      const int ntop = S.ntop;
      if (tid < nbest) S.bestk[tid] = key64(S.best[tid]);
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
      __syncthreads();
    }
    PF_MARK(3)
  }
  // peers in key order (<= kPeerCap, else the query-strand overflows)
  const int np = (int)S.npc;
  if (np <= kPeerCap) {
    for (int x = tid; x < np; x += kPfThreads) {
      const uint32_t kx = S.pcand[x];
      int r = 0;
      for (int y = 0; y < np; y++) r += S.pcand[y] < kx;
      a.ppeer_id[pq_ * kPeerCap + r] = (uint16_t)((kx & 0xffffu) + (uint32_t)a.peer_id_add);
      a.ppeer_count[pq_ * kPeerCap + r] = (uint8_t)(127u - (kx >> 23));
    }
  }
  __syncthreads();
  const int ntop = S.ntop;  // < 0: -1 - (entries written directly)
  if (tid < ntop) a.pcand[pq_ * kPartCand + tid] = cand_entry(S.top[tid]);
  if (tid == 0) {
    a.pncand[pq_] = (uint8_t)(ntop < 0 ? -1 - ntop : ntop);
    a.pnpeer[pq_] = (uint8_t)(np > kPeerCap ? 255 : np);
    a.ppost[pq_] = S.post_local;  // summed by the merge: a per-workgroup atomic on one address serialises
  }
  PF_MARK(4)
  if (prof) {
#pragma unroll
    for (int i = 0; i < 8; i++) atomicAdd(&a.prof[i], tacc[i]);
    atomicAdd(&a.prof[8], 1ull);
  }
#undef PF_MARK
}

__global__ __launch_bounds__(kPfThreads, 5) void k_pf_full(PrefilterArgs a, int unit_mode) {
  extern __shared__ __attribute__((aligned(16))) unsigned char pf_smem[];
  if (!unit_mode) {
    pf_full_unit(a, blockIdx.x, pf_smem);
    return;
  }
  // the overflowed units of the lean kernel (usually none)
  const uint32_t nu = *a.nunits;
  for (uint32_t u = blockIdx.x; u < nu; u += gridDim.x) {
    pf_full_unit(a, a.units[u], pf_smem);
    __syncthreads();
  }
}

// The lean counting kernel (one counter segment): list table, count, then every centroid counter >= the
// threshold becomes a part candidate (count << 24 | ordinal, unsorted, at most kPartCand) and every earlier
// window query over it a peer (unsorted); lengths, keys and the top-41 are the merge's.  Only what counting
// needs lives in LDS -- the u8 counters from address 0, then the list table sized by a.nlist_cap -- and
// the kernel keeps few registers, so up to 8 workgroups share a CU.
struct PfCountHdr {
  uint32_t wsum[kPfWaves];
  uint32_t ncand, npc, pad0, pad1;
};
__host__ __device__ constexpr uint32_t pf_count_table_bytes(int nlist_cap) {
  return (uint32_t)(sizeof(PfCountHdr) + kPfWinBase * 16 + (2 * nlist_cap + 66) * 4);
}
// W waves per workgroup: 4 (8 workgroups per CU), or 1 when the index is small (up to 32 one-wave workgroups per CU;
// launch_prefilter): then the table, count and scan phases need no workgroup barrier, and 4x more units are in flight
// to hide the latency chain (k-mers -> list offsets -> table) that dominates a unit with few postings.
template <int CM, int W>
__global__ __launch_bounds__(64 * W, 8) void k_pf_count(PrefilterArgs a, uint32_t tab_off) {
  constexpr int kThr = PfW<W>::kThreads;
  extern __shared__ __attribute__((aligned(16))) unsigned char pf_smem[];
  PfCountHdr& H = *reinterpret_cast<PfCountHdr*>(pf_smem + tab_off);
  uint4* wtab = reinterpret_cast<uint4*>(pf_smem + tab_off + sizeof(PfCountHdr));
  uint32_t* lstart = reinterpret_cast<uint32_t*>(wtab + kPfWinBase);
  uint32_t* lbias = lstart + a.nlist_cap + 66;
  uint32_t* cnt = reinterpret_cast<uint32_t*>(pf_smem);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int part = (int)(blockIdx.x & (kParts - 1));
  const int qs = (int)(blockIdx.x >> kPartShift);
  const int strand = qs % a.both;
  const int32_t q = a.q0 + qs / a.both;
  const int nk = a.seqs.nk[(int64_t)q * 2 + strand];
  const uint16_t* qk = a.seqs.kmers + ((int64_t)q * 2 + strand) * kKmerStride;
  const uint32_t raw0 = qk[lane], raw1 = qk[64 + (lane < kKmerStride - 64 ? lane : 0)];
  const int thr = nk < a.minwordmatches ? nk : a.minwordmatches;
  const uint32_t km0 = lane < nk ? raw0 : 0u, km1 = lane + 64 < nk ? raw1 : 0u;
  const int64_t pq_ = (int64_t)qs * kParts + part;
  int32_t seq0, ord0;
  pack_bounds(a, q, seq0, ord0);
  const int nct = a.nseg > 0 ? a.seg_tile[1] - a.seg_tile[0] : 0;
  const int nsubC = a.ncent > part ? (a.ncent - part + kParts - 1) >> kPartShift : 0;
  const int ncnt = kCentBase + ((nsubC + 15) & ~15);
  const uint64_t pbase = a.seg_base[0];
  const __amdgpu_buffer_rsrc_t arena = arena_rsrc(uniform_ptr(a.arena + pbase));
  // optional phase timing (UMICLUST_PFPROF: a.prof != nullptr): thread 0's shader-clock deltas between the
  // phase barriers of sampled workgroups, into a.prof[9 + i] (k_pf_full uses [0, 9))
  const bool prof = a.prof != nullptr && tid == 0 && (blockIdx.x % 61u) == 0u;
  unsigned long long tprev = prof ? __builtin_readcyclecounter() : 0ull, tacc[5] = {0, 0, 0, 0, 0};
  // ... and the workgroup's life in shader cycles and in the 100 MHz real-time clock: their ratio is the clock the
  // kernel ran at inside the pipeline (PMC runs serialise dispatches and see only the solo clock)
  const unsigned long long rt0 = prof ? __builtin_amdgcn_s_memrealtime() : 0ull, cy0 = tprev;
  // table sub-phases: offsets arrived, block scan done (scalars, not an address-taken array: that one lived in
  // scratch, and its zeroing store from every lane of every workgroup was 537 MB of HBM writes per launch)
  unsigned long long clk0 = 0, clk1 = 0, tsub[2] = {0, 0};
#define PFC_MARK(i)                                             \
  if (prof) {                                                   \
    const unsigned long long tn = __builtin_readcyclecounter(); \
    tacc[i] += tn - tprev;                                      \
    tprev = tn;                                                 \
  }
  uint4* cnt4 = reinterpret_cast<uint4*>(cnt);
  PfOffsets<W> offs;
  pf_list_offsets<W>(a, 0, nct, nct + kPeerTiles, part, thr, km0, km1, wv, offs);  // in flight during the zeroing
  for (int x = tid; x < (ncnt >> 4); x += kThr) cnt4[x] = make_uint4(0u, 0u, 0u, 0u);
  if (tid == 0) {
    H.ncand = 0;
    H.npc = 0;
  }
  uint32_t T, nlc;
  PFC_MARK(0)
  pf_list_table<W>(a, PfTable{lstart, lbias, wtab, H.wsum}, offs, pbase, thr, nk, lane, tid, T, nlc, prof, &clk0, &clk1);
  if (prof) {
    tsub[0] += clk0 - tprev;
    tsub[1] += clk1 - clk0;
  }
  PFC_MARK(1)
  if (T > 0 && CM != 2)  // CM 2: the timing probe without the count loop (UMICLUST_PFPROBE)
    pf_count_stream<0, W>(arena, T, nlc, lstart, lbias, wtab, lane, wv);
  __syncthreads();
  PFC_MARK(2)
  if (wv == 0) {
    // postings touched (stats): every chunk posting minus the padding ones (the spare counters)
    const uint8_t* cb = reinterpret_cast<const uint8_t*>(cnt);
    const uint32_t pads = lane63(wave_scan_dpp((uint32_t)cb[kDummy + lane], OpAdd()));
    if (lane == 0) a.ppost[pq_] = 8u * T - pads;
  }
  // centroid counters >= thr (SWAR: bytes <= 112, so byte + 128 - thr sets bit 7 iff >= thr); a sweep
  // of 64 counter vectors with no candidate costs one OR and a ballot.
  const uint32_t add = (uint32_t)(128 - thr) * 0x01010101u;
  if (thr > 0) {
    const int lim4 = (nsubC + 15) >> 4;  // counters past nsubC are zero (< thr)
    const uint4* c4 = cnt4 + kCentBase / 16;
    const int32_t cmin = pack_cmin(ord0, 0, part, nsubC);  // packs: earlier bins' centroids are never candidates
    for (int x0 = (cmin >> 4) + wv * 64; x0 < lim4; x0 += kThr) {
      const int x = x0 + lane;
      uint4 v = x < lim4 ? c4[x] : make_uint4(0u, 0u, 0u, 0u);
      const int cb = cmin - x * 16;
      if (cb > 0) v = make_uint4(v.x & keep_from(cb), v.y & keep_from(cb - 4), v.z & keep_from(cb - 8), v.w & keep_from(cb - 12));
      if (__ballot((((v.x + add) | (v.y + add) | (v.z + add) | (v.w + add)) & 0x80808080u) != 0u) == 0ull) continue;
      const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
      uint32_t mk[4] = {(v.x + add) & 0x80808080u, (v.y + add) & 0x80808080u, (v.z + add) & 0x80808080u,
                        (v.w + add) & 0x80808080u};
      const uint32_t n = (uint32_t)(__builtin_popcount(mk[0]) + __builtin_popcount(mk[1]) +
                                    __builtin_popcount(mk[2]) + __builtin_popcount(mk[3]));
      uint32_t slot = wave_alloc(n, &H.ncand);
#pragma unroll
      for (int j = 0; j < 4; j++) {
        while (mk[j]) {
          const uint32_t byte = (uint32_t)__builtin_ctz(mk[j]) >> 3;
          mk[j] &= mk[j] - 1u;
          const uint32_t c = (uint32_t)x * 16u + (uint32_t)j * 4u + byte;
          const uint32_t cv = (wd[j] >> (8 * byte)) & 0xffu;
          if (slot < (uint32_t)kPartCand) a.pcand[pq_ * kPartCand + slot] = (cv << 24) | ((c << kPartShift) + part);
          slot++;
        }
      }
    }
  }
  PFC_MARK(3)
  // peers: the window queries before q, every count >= thr (all of them when thr == 0)
#pragma unroll
  for (int v = 0; v < kPeerTiles; v++) {
    const TileView pv = a.peer[v];
    if (pv.n <= 0 || v == a.flag_tile) continue;
    const int lim = min(pv.n, q - pv.base);
    const int nsubP = lim > part ? (lim - part + kParts - 1) >> kPartShift : 0;
    const int nwords = (nsubP + 3) >> 2;
    const uint32_t* pw = cnt + pv.seg * (kPeerRegion / 4);
    const int32_t pmin = pack_pmin(seq0, pv.base, part);  // packs: earlier bins' queries are never peers
    for (int x0 = (pmin >> 2) + wv * 64; x0 < nwords; x0 += kThr) {
      const int x = x0 + lane;
      const uint32_t w = x < nwords ? pw[x] & keep_from(pmin - 4 * x) : 0u;
      const int valid = x < nwords ? min(4, nsubP - 4 * x) : 0;  // bytes of peers before q
      uint32_t mk = (w + add) & 0x80808080u & (valid >= 4 ? 0xffffffffu : (1u << (8 * valid)) - 1u);
      if (__ballot(mk != 0u) == 0ull) continue;
      uint32_t slot = wave_alloc((uint32_t)__builtin_popcount(mk), &H.npc);
      while (mk) {
        const uint32_t byte = (uint32_t)__builtin_ctz(mk) >> 3;
        mk &= mk - 1u;
        if (slot < (uint32_t)kPeerCap) {
          const int32_t sq = pv.base + ((4 * x + (int)byte) << kPartShift) + part;
          a.ppeer_id[pq_ * kPeerCap + slot] = (uint16_t)(sq - a.cand_base);
          a.ppeer_count[pq_ * kPeerCap + slot] = (uint8_t)((w >> (8 * byte)) & 0xffu);
        }
        slot++;
      }
    }
  }
  // the flagged tile (a split pass's unresolved oldest block): its hits are candidates for the merge
  if (a.flag_tile >= 0) {
    const TileView pv = a.peer[a.flag_tile];
    const int nsubP = pv.n > part ? (pv.n - part + kParts - 1) >> kPartShift : 0;
    const int nwords = (nsubP + 3) >> 2;
    const uint32_t* pw = cnt + pv.seg * (kPeerRegion / 4);
    const int32_t pmin = pack_pmin(seq0, pv.base, part);
    for (int x0 = (pmin >> 2) + wv * 64; x0 < nwords; x0 += kThr) {
      const int x = x0 + lane;
      const uint32_t w = x < nwords ? pw[x] & keep_from(pmin - 4 * x) : 0u;
      const int valid = x < nwords ? min(4, nsubP - 4 * x) : 0;
      uint32_t mk = (w + add) & 0x80808080u & (valid >= 4 ? 0xffffffffu : (1u << (8 * valid)) - 1u);
      if (__ballot(mk != 0u) == 0ull) continue;
      uint32_t slot = wave_alloc((uint32_t)__builtin_popcount(mk), &H.ncand);
      while (mk) {
        const uint32_t byte = (uint32_t)__builtin_ctz(mk) >> 3;
        mk &= mk - 1u;
        const int32_t sq = pv.base + ((4 * x + (int)byte) << kPartShift) + part;
        if (slot < (uint32_t)kPartCand)
          a.pcand[pq_ * kPartCand + slot] = (((w >> (8 * byte)) & 0xffu) << 24) | 0x800000u | (uint32_t)(sq - a.cand_base);
        slot++;
      }
    }
  }
  __syncthreads();
  if (tid == 0) {
    const uint32_t nc = H.ncand, np = H.npc;
    const bool ovf = thr == 0 || nc > (uint32_t)kPartCand;
    a.pncand[pq_] = (uint8_t)(ovf ? 255u : nc);
    a.pnpeer[pq_] = (uint8_t)(np > (uint32_t)kPeerCap ? 255u : np);
    if (ovf) a.units[atomicAdd(a.nunits, 1u)] = (uint32_t)pq_;
  }
  PFC_MARK(4)
  if (prof) {
    for (int i = 0; i < 5; i++) atomicAdd(&a.prof[9 + i], tacc[i]);
    atomicAdd(&a.prof[14], 1ull);
    atomicAdd(&a.prof[15], (unsigned long long)T);
    atomicAdd(&a.prof[16], tsub[0]);
    atomicAdd(&a.prof[17], tsub[1]);
    atomicAdd(&a.prof[18], __builtin_readcyclecounter() - cy0);
    atomicAdd(&a.prof[19], __builtin_amdgcn_s_memrealtime() - rt0);
  }
#undef PFC_MARK
}

// One wave per query-strand.  Candidates: the parts' lists (distinct ordinals) get their u64 keys
// (127-count) << 56 | length << 48 | ordinal -- vsearch's order: count desc, length asc, seqno asc (ordinal
// order is seqno order) -- and every key its rank in the union by counting smaller keys; ranks < 41 are
// the exact top-41 (a part's list holds every candidate over the threshold, or the full kernel's exact
// part top-41: top-41 of a union = top-41 of the parts' top-41s).  Peers: sorted within each part by
// (count desc, length asc, window id asc) and concatenated in part order.
constexpr int kMergeWaves = 4;
__global__ __launch_bounds__(64 * kMergeWaves) void k_pf_merge(PrefilterArgs a, int32_t nqs) {
  __shared__ unsigned long long keys[kMergeWaves][kParts * kPartCand];
  __shared__ uint32_t pkeys[kMergeWaves][kPeerCap];
  __shared__ uint32_t wpost[kMergeWaves];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int qs = (int)blockIdx.x * kMergeWaves + wave;
  const bool live = qs < nqs;
  unsigned long long* K = keys[wave];
  const int64_t p0 = (int64_t)qs * kParts;
  // postings touched (stats): the parts' counts, one atomic per workgroup into one of kPostSpread lines
  {
    uint32_t pp = (live && lane < kParts) ? a.ppost[p0 + lane] : 0u;
#pragma unroll
    for (int d = 1; d < kParts; d <<= 1) pp += __shfl_xor(pp, d, 64);
    if (lane == 0) wpost[wave] = pp;
    __syncthreads();
    if (threadIdx.x == 0 && a.postings_touched) {
      uint32_t t = 0;
#pragma unroll
      for (int w = 0; w < kMergeWaves; w++) t += wpost[w];
      if (t) atomicAdd(a.postings_touched + 16 + 32 * (blockIdx.x % kPostSpread), t);
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) *a.nunits = 0;  // the full kernel has read it (stream order)
  if (!live) return;
  // list sizes and offsets (lanes 0..kParts-1)
  const int n_l = lane < kParts ? min((int)a.pncand[p0 + lane], kPartCand) : 0;
  int inc = n_l;
#pragma unroll
  for (int d = 1; d < kParts; d <<= 1) {
    const int u = __shfl_up(inc, d, 64);
    if (lane >= d) inc += u;
  }
  const int o_l = inc - n_l;
  const int total = __shfl(inc, kParts - 1, 64);
#pragma unroll
  for (int l = 0; l < kParts; l++) {
    const int n = __shfl(n_l, l, 64), o = __shfl(o_l, l, 64);
    for (int x = lane; x < n; x += 64) {
      const uint32_t e = a.pcand[(p0 + l) * kPartCand + x];
      unsigned long long key = ~0ull;  // a flagged hit that turned out a member: no candidate
      if (e & 0x800000u) {
        const int32_t sq = a.cand_base + (int32_t)(e & 0x7fffffu);
        const int32_t ord = a.seq2ord[sq];
        if (ord >= 0)
          key = ((unsigned long long)(127u - (e >> 24)) << 56) | ((unsigned long long)a.seqs.lens[sq] << 48) |
                (uint32_t)ord;
      } else {
        const uint32_t ord = e & 0xffffffu;
        const uint32_t len = a.seqs.lens[a.cent_seqno[ord]];
        key = ((unsigned long long)(127u - (e >> 24)) << 56) | ((unsigned long long)len << 48) | ord;
      }
      K[o + x] = key;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // compact the valid keys in place (chunk i reads [64 i, 64 i + 64) and writes below its own start, after its
  // reads: LDS operations of a wave complete in order)
  int nvalid = 0;
  for (int e0 = 0; e0 < total; e0 += 64) {
    const int e = e0 + lane;
    const unsigned long long key = e < total ? K[e] : ~0ull;
    const unsigned long long vb = __ballot(key != ~0ull);
    if (key != ~0ull) K[nvalid + (int)__builtin_popcountll(vb & ((1ull << lane) - 1ull))] = key;
    nvalid += (int)__builtin_popcountll(vb);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  for (int e = lane; e < nvalid; e += 64) {
    const unsigned long long key = K[e];
    int rank = 0;
    for (int y = 0; y < nvalid; y++) rank += K[y] < key;
    if (rank < kTopHits) {
      a.top_seqno[(int64_t)qs * kTopHits + rank] = (uint32_t)a.cent_seqno[(uint32_t)(key & 0xffffffu)];
      a.top_count[(int64_t)qs * kTopHits + rank] = (uint8_t)(127u - (uint32_t)(key >> 56));
    }
  }
  // peers
  const int np_l = lane < kParts ? (int)a.pnpeer[p0 + lane] : 0;
  const bool over = __any(np_l == 255);
  int pinc = np_l;
#pragma unroll
  for (int d = 1; d < kParts; d <<= 1) {
    const int u = __shfl_up(pinc, d, 64);
    if (lane >= d) pinc += u;
  }
  const int ptotal = __shfl(pinc, kParts - 1, 64);
  const int po_l = pinc - np_l;
  const bool povf = over || ptotal > kPeerCap;
  if (lane == 0) {
    a.ntop[qs] = (uint8_t)min(nvalid, kTopHits);
    a.npeer[qs] = (uint8_t)(povf ? 255 : ptotal);
  }
  if (povf) return;
  uint32_t* P = pkeys[wave];
  for (int l = 0; l < kParts; l++) {
    const int n = __shfl(np_l, l, 64), o = __shfl(po_l, l, 64);
    if (n == 0) continue;
    uint32_t key[kPeerCap / 64];
#pragma unroll
    for (int hh = 0; hh < kPeerCap / 64; hh++) {
      const int x = lane + 64 * hh;
      key[hh] = 0xffffffffu;
      if (x < n) {
        const uint32_t id = a.ppeer_id[(p0 + l) * kPeerCap + x] - (uint32_t)a.peer_shift;  // peer_base-relative
        const uint32_t cv = a.ppeer_count[(p0 + l) * kPeerCap + x];
        key[hh] = ((127u - cv) << 23) | ((uint32_t)a.seqs.lens[a.peer_base + (int32_t)id] << 16) | id;
        P[x] = key[hh];
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int hh = 0; hh < kPeerCap / 64; hh++) {
      if (lane + 64 * hh < n) {
        int r = 0;
        for (int y = 0; y < n; y++) r += P[y] < key[hh];
        a.peer_id[(int64_t)qs * kPeerCap + o + r] = (uint16_t)(key[hh] & 0xffffu);
        a.peer_count[(int64_t)qs * kPeerCap + o + r] = (uint8_t)(127u - (key[hh] >> 23));
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// ------------------------------------------------------------------ packs: per-bin k-mer scrambling
__global__ __launch_bounds__(256) void k_kmer_xor(uint16_t* __restrict__ kmers, const uint8_t* __restrict__ nk,
                                                  int64_t n2, const int32_t* __restrict__ bin,
                                                  const uint16_t* __restrict__ xmask) {
  const int64_t ss = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);  // sequence * 2 + strand
  const int x = threadIdx.x & 63;
  if (ss >= n2) return;
  const int m = nk[ss];
  const uint16_t xm = xmask[bin[ss >> 1]];
  uint16_t* k = kmers + ss * kKmerStride;
  if (x < m) k[x] ^= xm;
  if (x + 64 < m) k[x + 64] ^= xm;
}
hipError_t launch_kmer_xor(uint16_t* kmers, const uint8_t* nk, int32_t n, const int32_t* bin, const uint16_t* xmask,
                           hipStream_t st) {
  const int64_t n2 = (int64_t)n * 2;
  if (n2 <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_kmer_xor, dim3((unsigned)((n2 + 3) / 4)), dim3(256), 0, st, kmers, nk, n2, bin, xmask);
  return hipGetLastError();
}

hipError_t launch_prefilter(const PrefilterArgs& a, hipStream_t st, int mode) {
  const int nqs = a.nq * a.both;
  if (nqs <= 0) return hipSuccess;
  const int full_most = kPfSharedBytes + kCentBase + kSegCentroids / kParts + 16;
  const int count_most = kCentBase + kSegCentroids / kParts + 16 + (int)pf_count_table_bytes(kPfLists) + 16;
  if (!attr_set_on_device(k_attr_prefilter)) {
    hipError_t e = hipFuncSetAttribute((const void*)k_pf_full, hipFuncAttributeMaxDynamicSharedMemorySize, full_most);
    if (e == hipSuccess)
      e = hipFuncSetAttribute((const void*)k_pf_count<0, kPfWaves>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              count_most);
    if (e == hipSuccess)
      e = hipFuncSetAttribute((const void*)k_pf_count<0, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, count_most);
    if (e == hipSuccess)
      e = hipFuncSetAttribute((const void*)k_pf_count<2, kPfWaves>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              count_most);
    if (e != hipSuccess) return e;
    mark_attr_set(k_attr_prefilter);
  }
  // LDS of the full kernel: the fixed part + counters for the peer regions, the spares and one
  // segment's centroids
  const int segn = a.ncent < kSegCentroids ? a.ncent : kSegCentroids;
  const size_t sub = (size_t)(((segn + kParts - 1) >> kPartShift) + 15) & ~(size_t)15;
  const size_t smem_full = (size_t)kPfSharedBytes + kCentBase + sub;
  if (mode == 1 || mode == 3 || (mode == 0 && a.nseg <= 1)) {
    // lean counting (one counter segment)
    if (a.nseg > 1 || a.nlist_cap < 1 || a.nlist_cap > kPfLists) return hipErrorInvalidValue;
    const uint32_t tab_off = (uint32_t)(kCentBase + sub);
    size_t lds = tab_off + pf_count_table_bytes(a.nlist_cap) + 16;  // (+16: the table copy's last vector)
    if (mode == 3)  // the timing probe: every phase but the count loop, into scratch outputs (UMICLUST_PFPROBE)
      hipLaunchKernelGGL((k_pf_count<2, kPfWaves>), dim3(nqs * kParts), dim3(kPfThreads), lds, st, a, tab_off);
    else if ((int64_t)lds <= (int64_t)a.pf1_lds)  // small index: one-wave units
      hipLaunchKernelGGL((k_pf_count<0, 1>), dim3(nqs * kParts), dim3(64), lds, st, a, tab_off);
    else
      hipLaunchKernelGGL((k_pf_count<0, kPfWaves>), dim3(nqs * kParts), dim3(kPfThreads), lds, st, a, tab_off);
    if (mode == 1 || mode == 3) return hipGetLastError();
  }
  if (mode == 2 || a.nseg <= 1) {
    // the full kernel over the units the lean kernel could not finish (exits at once when there are none); its
    // workgroups loop over the units (256: one per CU; 1024 / 2048 measured within noise, round 4 full_wg/)
    hipLaunchKernelGGL(k_pf_full, dim3(256), dim3(kPfThreads), smem_full, st, a, 1);
  } else {
    hipLaunchKernelGGL(k_pf_full, dim3(nqs * kParts), dim3(kPfThreads), smem_full, st, a, 0);
  }
  hipLaunchKernelGGL(k_pf_merge, dim3((nqs + kMergeWaves - 1) / kMergeWaves), dim3(64 * kMergeWaves), 0, st, a, nqs);
  return hipGetLastError();
}

static AlignFn g_align[kAlignSlots * (kMaxLen + 1)];
static std::once_flag g_align_once;
static void init_align_tables() {
  std::call_once(g_align_once, [] {
    fill_align_part0(g_align);
    fill_align_part1(g_align);
    fill_align_part2(g_align);
    fill_align_part3(g_align);
    fill_align_part4(g_align);
    fill_align_part5(g_align);
  });
}

hipError_t launch_align(const DevSeqs& s, int32_t qlen, bool ambig, const uint32_t* pq,
                        const uint32_t* pt, int32_t npairs, const uint32_t* dev_npairs,
                        const uint32_t* outidx, const Scoring& sc, uint32_t* out, hipStream_t st,
                        int32_t band_max) {
  init_align_tables();
  if (npairs <= 0) return hipSuccess;
  if (qlen < kMinTplLen || qlen > kMaxLen) return hipErrorInvalidValue;
  const bool band = !ambig && npairs <= band_max;
  const int64_t lanes = (int64_t)npairs * (band ? band_lanes(qlen) : 1);
  const int v = ambig ? 1 : band ? 2 : 0;
  int64_t grid = (lanes + 63) / 64;
  // banded launches are latency-bound (about one wave per SIMD) and sit on the pass chain the host waits for, while
  // the next pass's counting waves share their SIMDs: UMICLUST_BAND_WPRIO=1 raises their issue priority
  static const int band_prio = [] {
    const char* e = getenv("UMICLUST_BAND_WPRIO");
    return e ? atoi(e) : 0;
  }();
  Scoring scl = sc;
  if (band && band_prio > 0) scl.wave_prio = 1;
  hipLaunchKernelGGL(g_align[kAlignSlots * qlen + v], dim3((unsigned)grid),
                     dim3(64), 0, st, s, pq, pt, npairs, dev_npairs, outidx, scl, out);
  return hipGetLastError();
}

// ------------------------------------------------------------------ K3W: device-side walk
// vsearch search_onequery pops candidates best-first in batches of MAXDELAYED = 8 and stops
// after the batch in which it has an accept, after maxaccepts+maxrejects-1 = 32 candidates, or
// when the list is exhausted.  The walk runs on the device over the top lists (in-block peers
// are resolved later by the host): round r evaluates batch r of every unfinished query-strand and
// emits the pairs of batch r+1.  Acceptance and the id order come from host-built tables, so the
// IEEE-double test `100.0*matches/internal >= 100.0*id` is exactly vsearch's.
// Pairs are appended to per-query-length segments (SegTab: a block may hold several lengths, and the aligner is
// compiled per query length): segment i = query length sg.lmax - i, its pairs from sg.base[i], its counter cnt[i].
// Slots are allocated per wave (queries are length-sorted, so a wave's lanes hold one or two segments): one atomic
// per segment present in the wave.  All 64 lanes must be active.
__device__ __forceinline__ uint32_t seg_alloc(uint32_t n, uint32_t si, uint32_t* cnt) {
  uint32_t start = 0;
  unsigned long long pending = __ballot(n > 0u);
  while (pending) {
    const int lead = __builtin_ctzll(pending);
    const uint32_t L = (uint32_t)__builtin_amdgcn_readlane((int)si, lead);
    const bool mine = n > 0u && si == L;
    const unsigned long long grp = __ballot(mine);
    const uint32_t v = mine ? n : 0u;
    const uint32_t incl = wave_scan_dpp(v, OpAdd());
    const uint32_t tot = lane63(incl);
    uint32_t b = 0;
    if ((int)(threadIdx.x & 63) == lead) b = atomicAdd(cnt + L, tot);
    b = (uint32_t)__builtin_amdgcn_readlane((int)b, lead);
    if (mine) start = b + incl - v;
    pending &= ~grp;
  }
  return start;
}

__global__ __launch_bounds__(256) void k_walk(int32_t round, int32_t q0, int32_t nqs, int32_t both, int32_t spec_thr,
                                              const uint32_t* __restrict__ top_seqno, const uint8_t* __restrict__ top_count,
                                              const uint8_t* __restrict__ ntop, const uint8_t* __restrict__ lens,
                                              const uint32_t* __restrict__ res, const uint8_t* __restrict__ acc_tab,
                                              const uint16_t* __restrict__ rank_tab, WalkState* __restrict__ ws,
                                              uint32_t* __restrict__ pq, uint32_t* __restrict__ pt,
                                              uint32_t* __restrict__ outidx, SegTab sg, uint32_t* __restrict__ seg_cnt,
                                              unsigned long long* __restrict__ cells) {
  const int qs = blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = qs < nqs;  // every lane stays to the slot allocation
  const int32_t q = q0 + (live ? qs : 0) / both;
  const uint32_t strand = (uint32_t)((live ? qs : 0) % both);
  const int nt = live ? ntop[qs] : 0;
  const int ql = lens[q];
  WalkState w{};
  bool act = live;
  int emit_to = 0;  // emit candidates [w.e, emit_to)
  if (round < 0) {
    w.w = 0;
    w.done = (nt == 0) ? 1 : 0;
    w.acc = 0;
    w.best_rank = 0;
    w.best_t = 0xffffffffu;
    w.cells = 0;
    w.lastkey = 0;
    w.e = 0;
    const bool spec = nt > 0 && (int)top_count[(int64_t)(live ? qs : 0) * kTopHits] < spec_thr;
    emit_to = min(nt, spec ? kWalk : kBatch);
  } else if (live) {
    w = ws[qs];
    act = !w.done;
    if (act) {
      // every batch whose results exist, in order
      while (!w.done && w.w < w.e) {
        const int b0 = w.w, b1 = min(nt, b0 + kBatch);
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
      // the rest of an unfinished walk is emitted at once (one more align launch instead of up to three
      // dependent ones); walks are still evaluated batch by batch
      emit_to = w.done ? (int)w.e : min(nt, kWalk);
    }
  }
  const uint32_t n = (act && emit_to > (int)w.e) ? (uint32_t)(emit_to - (int)w.e) : 0u;
  const uint32_t si = (uint32_t)(sg.lmax - ql);
  const uint32_t k0 = seg_alloc(n, si, seg_cnt);
  if (n) {
    const int b0 = w.e, b1 = emit_to;
    const uint32_t base = sg.base[si] + k0;
    uint32_t tl = 0;
    for (int x = b0; x < b1; x++) {
      const uint32_t k = base + (uint32_t)(x - b0);
      const uint32_t t = top_seqno[(int64_t)qs * kTopHits + x];
      pq[k] = ((uint32_t)q << 1) | strand;
      pt[k] = t;
      outidx[k] = (uint32_t)qs * kWalk + (uint32_t)x;
      tl += lens[t];
    }
    atomicAdd(cells, (unsigned long long)ql * tl);  // cells the device computes for these pairs
    w.e = (uint8_t)b1;
  }
  if (act) ws[qs] = w;
}

hipError_t launch_walk(int32_t round, int32_t q0, int32_t nqs, int32_t both, int32_t spec_thr,
                       const uint32_t* top_seqno, const uint8_t* top_count, const uint8_t* ntop,
                       const uint8_t* lens, const uint32_t* res, const uint8_t* acc_tab,
                       const uint16_t* rank_tab, WalkState* ws, uint32_t* pq, uint32_t* pt,
                       uint32_t* outidx, const SegTab& sg, uint32_t* seg_cnt, unsigned long long* cells,
                       hipStream_t st) {
  if (nqs <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_walk, dim3((nqs + 255) / 256), dim3(256), 0, st, round, q0, nqs, both, spec_thr,
                     top_seqno, top_count, ntop, lens, res, acc_tab, rank_tab, ws, pq, pt, outidx,
                     sg, seg_cnt, cells);
  return hipGetLastError();
}

__device__ __forceinline__ unsigned long long cand_key_dev(uint32_t count, uint32_t len, uint32_t seqno) {
  return ((unsigned long long)(127u - count) << 56) | ((unsigned long long)len << 48) | seqno;
}
// the device walk's last batch is still open: a candidate inserted anywhere could join it
__device__ __forceinline__ bool walk_open(const WalkState& w) {
  return (w.w % kBatch) != 0 || w.w == 0 || (!w.acc && w.w < kWalk);
}
// a peer (an earlier query of the peer window [w0, q) passing the k-mer threshold) can change the
// query-strand's walk only if it is a centroid AND it ranks before the walk's last candidate, or
// the last batch is open; exactly those peers are aligned here, speculatively, in the same pass
__device__ __forceinline__ bool peer_relevant(const WalkState& w, uint32_t count, uint32_t len, uint32_t seqno) {
  return walk_open(w) || cand_key_dev(count, len, seqno) < w.lastkey;
}

// A peer whose own device walk has already accepted a hit is (almost surely) going to be a member, and members never
// enter a query's merged walk: its alignment would never be read.  Certain when w plus the peer's own in-window peer
// count is <= kWalk (no merge can push that hit out of its walk); taken as a member whenever it accepted since round 5
// (the rare peer that then turns out a centroid only costs a round-B alignment -- the host aligns every needed peer the
// pass did not -- so the result never changes; configs 3 / 4: 6 % / 11 % fewer peer pairs, round-B pairs 10.7 k ->
// 11.8 k per config-4 step, `profiles/r05/cert_relax_ab/`).  The peer's walk state is this pass's (an in-block peer,
// after round 0's evaluation) or the previous block's pass's (final).
__device__ __forceinline__ bool member_expected(uint32_t ps, int32_t q0, int32_t nqb, int32_t both,
                                               const WalkState* __restrict__ ws, const uint8_t* __restrict__ npeer,
                                               const WalkState* __restrict__ ws_prev,
                                               const uint8_t* __restrict__ npeer_prev, int32_t q0_prev,
                                               int32_t nq_prev) {
  (void)npeer;
  (void)npeer_prev;
  const WalkState* W;
  int32_t base;
  if ((int32_t)ps >= q0 && (int32_t)ps < q0 + nqb) {
    W = ws;
    base = q0;
  } else if (ws_prev && (int32_t)ps >= q0_prev && (int32_t)ps < q0_prev + nq_prev) {
    W = ws_prev;
    base = q0_prev;
  } else {
    return false;
  }
  for (int s = 0; s < both; s++)
    if (W[(int64_t)((int32_t)ps - base) * both + s].acc) return true;
  return false;
}

// The relevant peers not expected to be members, of every query-strand as bit masks (aligned[qs * kPH + h], peers 64 h ..
// 64 h + 63), one wave per query-strand, a lane per peer: the per-peer tests are dependent loads (the peer's id, then
// its length and walk states), which a thread per query-strand ran in series over up to kPeerCap peers (~170 us per
// launch on config 3's dense windows).  k_peer_pairs then allocates and emits the pairs from the masks.
__global__ __launch_bounds__(256) void k_peer_rel(int32_t q0, int32_t w0, int32_t nqs, int32_t both,
                                                  const uint8_t* __restrict__ lens, const WalkState* __restrict__ ws,
                                                  const uint16_t* __restrict__ peer_id,
                                                  const uint8_t* __restrict__ peer_count,
                                                  const uint8_t* __restrict__ npeer,
                                                  unsigned long long* __restrict__ aligned, int32_t emit,
                                                  const WalkState* __restrict__ ws_prev,
                                                  const uint8_t* __restrict__ npeer_prev, int32_t q0_prev,
                                                  int32_t nq_prev) {
  constexpr int kPH = kPeerCap / 64;
  const int lane = threadIdx.x & 63;
  const int qs = (int)blockIdx.x * 4 + (int)(threadIdx.x >> 6);  // wave-uniform
  if (qs >= nqs) return;
  const int np = npeer[qs];
  const bool any = np != 255 && np != 0 && emit;
  const WalkState w = ws[qs];
  const int32_t nqb = nqs / both;
#pragma unroll
  for (int hh = 0; hh < kPH; hh++) {
    const int x = lane + 64 * hh;
    bool r = false;
    if (any && x < np) {
      const uint32_t ps = (uint32_t)(w0 + peer_id[(int64_t)qs * kPeerCap + x]);
      r = peer_relevant(w, peer_count[(int64_t)qs * kPeerCap + x], lens[ps], ps) &&
          !member_expected(ps, q0, nqb, both, ws, npeer, ws_prev, npeer_prev, q0_prev, nq_prev);
    }
    const unsigned long long m = __ballot(r);
    if (lane == 0) aligned[(int64_t)qs * kPH + hh] = m;
  }
}

__global__ __launch_bounds__(256) void k_peer_pairs(int32_t q0, int32_t w0, int32_t nqs, int32_t both,
                                                    const uint8_t* __restrict__ lens, const WalkState* __restrict__ ws,
                                                    const uint16_t* __restrict__ peer_id,
                                                    const uint8_t* __restrict__ peer_count, const uint8_t* __restrict__ npeer,
                                                    uint32_t* __restrict__ pq, uint32_t* __restrict__ pt,
                                                    uint32_t* __restrict__ outidx, SegTab sg, uint32_t* __restrict__ seg_cnt,
                                                    unsigned long long* __restrict__ cells, uint32_t* __restrict__ nstat,
                                                    uint32_t out0, unsigned long long* __restrict__ aligned, int32_t emit,
                                                    const WalkState* __restrict__ ws_prev,
                                                    const uint8_t* __restrict__ npeer_prev, int32_t q0_prev,
                                                    int32_t nq_prev) {
  // one thread per (query, strand); the slots come from a wave-aggregated allocation per query length (seg_alloc)
  const int qs = blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = qs < nqs;  // every lane stays to the slot allocation
  constexpr int kPH = kPeerCap / 64;  // 64-bit masks per query-strand: peers 0..63, 64..127, ...
  // the relevant, not certainly-member peers, from k_peer_rel (zero masks when nothing is emitted)
  unsigned long long rel[kPH] = {};
  if (live)
    for (int hh = 0; hh < kPH; hh++) rel[hh] = aligned[(int64_t)qs * kPH + hh];
  const int32_t q = q0 + (live ? qs : 0) / both;
  const int ql = lens[q];
  uint32_t n = 0;
  for (int hh = 0; hh < kPH; hh++) n += (uint32_t)__builtin_popcountll(rel[hh]);
  const uint32_t si = (uint32_t)(sg.lmax - ql);
  const uint32_t k0 = seg_alloc(n, si, seg_cnt);
  if (!n) return;
  atomicAdd(nstat, n);
  uint32_t k = sg.base[si] + k0;
  const uint32_t qv = ((uint32_t)q << 1) | (uint32_t)(qs % both);
  uint32_t tl = 0;
  for (int hh = 0; hh < kPH; hh++)
    for (unsigned long long m = rel[hh]; m; m &= m - 1ull) {
      const int x = 64 * hh + __builtin_ctzll(m);
      const uint32_t t = (uint32_t)(w0 + peer_id[(int64_t)qs * kPeerCap + x]);
      pq[k] = qv;
      pt[k] = t;
      outidx[k] = out0 + (uint32_t)(qs * kPeerCap + x);
      tl += lens[t];
      k++;
    }
  atomicAdd(cells, (unsigned long long)ql * tl);
}

hipError_t launch_peer_pairs(int32_t q0, int32_t w0, int32_t nqs, int32_t both, const uint8_t* lens,
                             const WalkState* ws, const uint16_t* peer_id, const uint8_t* peer_count,
                             const uint8_t* npeer, uint32_t* pq, uint32_t* pt, uint32_t* outidx, const SegTab& sg,
                             uint32_t* seg_cnt, unsigned long long* cells, uint32_t* nstat, uint32_t out0,
                             unsigned long long* aligned, int32_t emit, const WalkState* ws_prev,
                             const uint8_t* npeer_prev, int32_t q0_prev, int32_t nq_prev, hipStream_t st) {
  if (nqs <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_peer_rel, dim3((nqs + 3) / 4), dim3(256), 0, st, q0, w0, nqs, both, lens, ws, peer_id,
                     peer_count, npeer, aligned, emit, ws_prev, npeer_prev, q0_prev, nq_prev);
  hipLaunchKernelGGL(k_peer_pairs, dim3((nqs + 255) / 256), dim3(256), 0, st, q0, w0, nqs, both, lens, ws, peer_id,
                     peer_count, npeer, pq, pt, outidx, sg, seg_cnt, cells, nstat, out0, aligned, emit, ws_prev,
                     npeer_prev, q0_prev, nq_prev);
  return hipGetLastError();
}

// What the host needs of a pass, written to device buffers the host receives by DMA: per
// query-strand the device walk's outcome (HostQs), and -- only for query-strands with a relevant
// peer, whose outcome depends on which peers turn out to be centroids -- a record with the walk's
// candidate list (seqno, k-mer count, result of the walked ones) and every peer (window id, count,
// relevant flag, result of the aligned ones).  One wave per kPackQ consecutive query-strands, lanes writing
// consecutive words.  Record layout (u32 words): nt | np << 8, seqno[nt], res[nt], counts[(nt+3)/4] (u8 x4),
// peer[np] (id | count << 16 | relevant << 24 | aligned << 25), peer_res[np] (valid if aligned).  Record
// space is taken with one device-scope atomic per workgroup of kPackWaves x kPackQ query-strands: a returning
// atomic on one word saturates at ~88 per us on MI355X (MI355X_MICROARCH.md, "dequeue"), so one per 4
// query-strands held a 16k-query-strand pack at ~46 us of atomics alone (115-131 us per launch measured).
constexpr int kPackWaves = 4, kPackQ = 4;
__global__ __launch_bounds__(64 * kPackWaves) void k_pack(int32_t nqs, int32_t w0, const uint8_t* __restrict__ lens,
                                              const WalkState* __restrict__ ws, const uint8_t* __restrict__ ntop,
                                              const uint32_t* __restrict__ top_seqno,
                                              const uint8_t* __restrict__ top_count, const uint32_t* __restrict__ res,
                                              const uint8_t* __restrict__ npeer, const uint16_t* __restrict__ peer_id,
                                              const uint8_t* __restrict__ peer_count,
                                              const uint32_t* __restrict__ peer_res,
                                              const unsigned long long* __restrict__ aligned,
                                              uint32_t* __restrict__ reccount,
                                              HostQs* __restrict__ hq, uint32_t* __restrict__ rec,
                                              uint32_t* __restrict__ counters, uint32_t* __restrict__ hcounters,
                                              uint32_t* __restrict__ hreccount) {
  __shared__ uint32_t wsize[kPackWaves * kPackQ];
  __shared__ uint32_t last_wg;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int qs0 = ((int)blockIdx.x * kPackWaves + wave) * kPackQ;
  if (blockIdx.x == 0 && threadIdx.x < 64) {
    // counters[0] = the postings partial sums (k_pf_merge spreads its atomics over kPostSpread lines)
    uint32_t v = threadIdx.x < kPostSpread ? counters[16 + 32 * threadIdx.x] : 0u;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) v += __shfl_xor(v, d, 64);
    if (threadIdx.x < 16) hcounters[threadIdx.x] = threadIdx.x == 0 ? v : counters[threadIdx.x];
  }
  constexpr int kH = kPeerCap / 64;  // peers lane, lane + 64, ...
  static_assert(kPackQ * kH <= 32, "relevant / aligned bits per lane");
  // phase 1: every query-strand's peer words and record size (the lane's relevant / aligned peers as bits
  // i * kH + hh)
  uint32_t pw[kPackQ][kH], relb = 0u, alb = 0u;
#pragma unroll
  for (int i = 0; i < kPackQ; i++) {
    const int qs = qs0 + i;
    const bool live = qs < nqs;
    const WalkState w = ws[live ? qs : 0];
    const int np = live ? npeer[qs] : 0;
    bool anyrel = false;
#pragma unroll
    for (int hh = 0; hh < kH; hh++) {
      const int x = lane + 64 * hh;
      pw[i][hh] = 0;
      if (live && np != 255 && x < np) {
        const uint32_t id = peer_id[(int64_t)qs * kPeerCap + x];
        const uint32_t cnt = peer_count[(int64_t)qs * kPeerCap + x];
        const uint32_t ps = (uint32_t)w0 + id;
        const bool rel = peer_relevant(w, cnt, lens[ps], ps);
        const bool al = (aligned[(int64_t)qs * kH + hh] >> lane) & 1ull;
        pw[i][hh] = id | (cnt << 16) | (rel ? 1u << 24 : 0u) | (al ? 1u << 25 : 0u);
        relb |= rel ? 1u << (i * kH + hh) : 0u;
        alb |= al ? 1u << (i * kH + hh) : 0u;
        anyrel |= rel;
      }
    }
    const bool has_rec = __any(anyrel);
    const int nt = live ? min((int)ntop[qs], kWalk) : 0;
    if (lane == 0) wsize[wave * kPackQ + i] = has_rec ? (uint32_t)(1 + 2 * nt + ((nt + 3) >> 2) + 2 * np) : 0u;
  }
  // record space: the workgroup's sizes scanned in LDS, one atomic
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t tot = 0;
    for (int i = 0; i < kPackWaves * kPackQ; i++) {
      const uint32_t x = wsize[i];
      wsize[i] = x ? tot : 0xffffffffu;
      tot += x;
    }
    const uint32_t b0 = tot ? atomicAdd(reccount, tot) : 0u;
    for (int i = 0; i < kPackWaves * kPackQ; i++)
      if (wsize[i] != 0xffffffffu) wsize[i] += b0;
    // the workgroup taking the last ticket (reccount[1]) sees every allocation: it writes the record total to
    // pinned host memory and re-zeroes both counters for the buffer set's next pass, so the chain the host waits on
    // holds no memset and no 4-byte copy (each a blit dispatch)
    __threadfence();
    last_wg = 0u;
    if (atomicAdd(reccount + 1, 1u) == gridDim.x - 1) {
      *hreccount = atomicAdd(reccount, 0u);
      atomicExch(reccount, 0u);
      atomicExch(reccount + 1, 0u);
      last_wg = 1u;
    }
  }
  __syncthreads();
  // the last workgroup also re-zeroes the pass counters (every kernel of the pass that adds to them ran before this
  // one on the align stream, and workgroup 0 copied them out before taking its ticket): the main stream's next pass
  // on this buffer set needs no memset, a blit dispatch that waited for a CU slot behind the alignment waves
  // (4-125 us per pass, round 6)
  if (last_wg) {
    __threadfence();
    for (int i = (int)threadIdx.x; i < kCountersLen; i += 64 * kPackWaves) counters[i] = 0u;
  }
  // phase 2: records and outcomes
#pragma unroll
  for (int i = 0; i < kPackQ; i++) {
    const int qs = qs0 + i;
    if (qs >= nqs) break;  // wave-uniform
    const WalkState w = ws[qs];
    const int np = npeer[qs];
    const int nt = min((int)ntop[qs], kWalk);
    const int ncw = (nt + 3) >> 2;
    const uint32_t base = wsize[wave * kPackQ + i];
    if (base != 0xffffffffu) {
      uint32_t* r = rec + base;
      if (lane == 0) r[0] = (uint32_t)nt | ((uint32_t)np << 8);
      if (lane < nt) {
        r[1 + lane] = top_seqno[(int64_t)qs * kTopHits + lane];
        r[1 + nt + lane] = lane < w.e ? res[(int64_t)qs * kWalk + lane] : 0u;
      }
      if (lane < ncw) {
        uint32_t cw = 0;
#pragma unroll
        for (int e = 0; e < 4; e++)
          if (4 * lane + e < nt) cw |= (uint32_t)top_count[(int64_t)qs * kTopHits + 4 * lane + e] << (8 * e);
        r[1 + 2 * nt + lane] = cw;
      }
#pragma unroll
      for (int hh = 0; hh < kH; hh++) {
        const int x = lane + 64 * hh;
        if (x < np) {
          const bool al = (alb >> (i * kH + hh)) & 1u;
          r[1 + 2 * nt + ncw + x] = pw[i][hh];
          r[1 + 2 * nt + ncw + np + x] = al ? peer_res[(int64_t)qs * kPeerCap + x] : 0u;
        }
      }
    }
    // the first kInlineRel relevant peers' ids, gathered from their lanes (wave-uniform masks, peer order)
    unsigned long long rm[kH];
    uint32_t nrel = 0;
#pragma unroll
    for (int hh = 0; hh < kH; hh++) {
      rm[hh] = __ballot((relb >> (i * kH + hh)) & 1u);
      nrel += (uint32_t)__builtin_popcountll(rm[hh]);
    }
    uint16_t ids[kInlineRel];
    int hcur = 0;
#pragma unroll
    for (int j = 0; j < kInlineRel; j++) {
      uint32_t id = 0;
      while (hcur < kH && !rm[hcur]) hcur++;
      if (hcur < kH) {
        const int l = __builtin_ctzll(rm[hcur]);
        rm[hcur] &= rm[hcur] - 1ull;
        uint32_t v = pw[i][0];
#pragma unroll
        for (int hh = 1; hh < kH; hh++) v = hh == hcur ? pw[i][hh] : v;
        id = (uint32_t)__builtin_amdgcn_readlane((int)(v & 0xffffu), l);
      }
      ids[j] = (uint16_t)id;
    }
    if (lane == 0) {
      HostQs h;
      h.best_t = w.best_t;
      h.cells = w.cells;
      h.rec = base;
      h.best_rank = w.best_rank;
      h.w = w.w;
      h.flags = (uint8_t)((w.acc ? 1u : 0u) | (np == 255 ? 2u : 0u));
      h.nrel = (uint16_t)nrel;
      h.e = w.e;
      h.npeer = (uint8_t)np;
#pragma unroll
      for (int j = 0; j < kInlineRel; j++) h.rel[j] = ids[j];
      hq[qs] = h;
    }
  }
}

hipError_t launch_pack(int32_t nqs, int32_t w0, const uint8_t* lens, const WalkState* ws, const uint8_t* ntop,
                       const uint32_t* top_seqno, const uint8_t* top_count, const uint32_t* res,
                       const uint8_t* npeer, const uint16_t* peer_id, const uint8_t* peer_count,
                       const uint32_t* peer_res, const unsigned long long* aligned, uint32_t* reccount, HostQs* hq,
                       uint32_t* rec, uint32_t* counters, uint32_t* hcounters, uint32_t* hreccount,
                       hipStream_t st) {
  if (nqs <= 0) {
    *hreccount = 0;  // no launch: nothing of this pass is in flight on the buffer set
    return hipSuccess;
  }
  constexpr int per = kPackWaves * kPackQ;
  hipLaunchKernelGGL(k_pack, dim3((nqs + per - 1) / per), dim3(64 * kPackWaves), 0, st, nqs, w0, lens,
                     ws, ntop, top_seqno, top_count,
                     res, npeer, peer_id, peer_count, peer_res, aligned, reccount, hq, rec, counters, hcounters,
                     hreccount);
  return hipGetLastError();
}

// ------------------------------------------------------------------ K3T: traceback (one wave per alignment)
// The same DP as k_align / backtrack16 for the one chosen hit of every member (the CIGAR feeding the
// consensus).  A wave computes one alignment: lane l holds query row 64 s + l of stripe s and sweeps the
// anti-diagonals, lane l computing column j = step - l; the vertical state (H(i-1, j), F(i, j)) and the
// target code move one lane down per step by DPP wave_shr:1, the horizontal state (H(i, j-1), E(i, j))
// stays in the lane, and the diagonal H(i-1, j-1) is what the lane received one step earlier.  Stripe
// s > 0 takes row 64 s - 1 from LDS (written by lane 63 of stripe s - 1).  Every cell's direction nibble
// (bit 0 up = D chosen, bit 1 left = I chosen, bit 2 D-extension, bit 3 I-extension) goes to LDS, 8 steps
// per word, and lane 0 runs backtrack16 over it.  Any query length up to kMaxLen in one launch; latency
// ~(ql + tl) steps instead of ql * tl serial cells.
// A wave's LDS is sized by the longest sequence of the launch (maxl): dir[stripes][words][64] (cell
// (64 s + l, t - l): word t / 8 of lane l, nibble t % 8), botH[maxl] (H(64 s - 1, j) for the next stripe),
// botF[maxl] (F(64 s, j)), hend, tcode[maxl + 64] -- 9.4 KB for 68-nt UMIs instead of 12.4 KB at kMaxLen
// (16 waves per CU instead of 12).
constexpr int kTwWaves = 4;
// maxq: the launch's longest query (its stripes: a launch of queries <= 64 nt needs half the direction store, so
// more waves fit a CU); maxl: its longest sequence.
struct TwLayout {
  int words, dir_u32, wave_bytes;
  __host__ __device__ TwLayout(int maxq, int maxl) {
    words = (maxl + 63 + 7) / 8;
    dir_u32 = ((maxq + 63) / 64) * words * 64;
    // tcode: maxl + 64 + 8 (whole 8-step groups); qraw, traw: maxl each (the backtrack's match test)
    wave_bytes = (dir_u32 * 4 + 2 * maxl * 4 + 4 + maxl + 72 + 2 * maxl + 15) & ~15;
  }
};
static_assert(kMaxLen <= 128, "the backtrack's register prefetch covers two stripes");

__device__ __forceinline__ uint32_t wave_shr1(uint32_t v, uint32_t lane0) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)lane0, (int)v, 0x138, 0xf, 0xf, false);  // wave_shr:1
}

__global__ __launch_bounds__(64 * kTwWaves) void k_trace_wave(DevSeqs s, const uint32_t* __restrict__ pq,
                                                              const uint32_t* __restrict__ pt, int32_t npairs,
                                                              Scoring sc, uint8_t* __restrict__ ops,
                                                              uint16_t* __restrict__ nops, uint32_t* __restrict__ out,
                                                              int32_t maxq, int32_t maxl) {
  extern __shared__ __attribute__((aligned(16))) uint8_t tw_smem[];
  // wave-uniform by construction (readfirstlane), so the pair's lengths, the sweep bounds and the backtrack are
  // scalar
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), lane = threadIdx.x & 63;
  const int k = (int)blockIdx.x * kTwWaves + wave;
  if (k >= npairs) return;  // wave-uniform
  const TwLayout lay(maxq, maxl);
  struct {
    uint32_t* dir;
    int32_t *botH, *botF, *hendp;
    uint8_t *tcode, *qraw, *traw;
  } S;
  S.dir = (uint32_t*)(tw_smem + (size_t)wave * lay.wave_bytes);
  S.botH = (int32_t*)(S.dir + lay.dir_u32);
  S.botF = S.botH + maxl;
  S.hendp = S.botF + maxl;
  S.tcode = (uint8_t*)(S.hendp + 1);
  S.qraw = S.tcode + maxl + 72;
  S.traw = S.qraw + maxl;
  const int TW = lay.words;
  const uint32_t qv = pq[k];
  const int32_t q = (int32_t)(qv >> 1);
  const int qstr = (int)(qv & 1u);
  const int32_t t = (int32_t)pt[k];
  const int tl = s.lens[t], ql = s.lens[q];
  const uint32_t* tcp = s.codes + (int64_t)t * 2 * kCodeWords;
  const uint32_t* qcp = s.codes + ((int64_t)q * 2 + qstr) * kCodeWords;
  // the target codes staged one-hot (0 = ambiguous or past the end), so the substitution score is two tests
  for (int j = lane; j < tl + 72; j += 64) {
    const uint32_t c = j < tl ? (tcp[j >> 3] >> ((j & 7) * 4)) & 15u : 0u;
    S.tcode[j] = (uint8_t)((c & (c - 1u)) == 0u ? c : 0u);
    if (j < tl) S.traw[j] = (uint8_t)c;
  }
  // both sequences' code words in VGPRs (lane w holds word w): the backtrack reads them by v_readlane
  // instead of a global / LDS load per diagonal step
  const uint32_t qword = lane < kCodeWords ? qcp[lane] : 0u, tword = lane < kCodeWords ? tcp[lane] : 0u;
  for (int i = lane; i < ql; i += 64) S.qraw[i] = (uint8_t)((qcp[i >> 3] >> ((i & 7) * 4)) & 15u);
  // identical sequences of one-hot codes (a member equal to its centroid: about (1 - error)^L of them): the all-M
  // path is the only optimum -- any other path trades matches for gaps or mismatches -- so its ops, matches and
  // internal length are known without the DP (codes past the length are 0 in both)
  if (ql == tl) {
    bool same = qword == tword;
    if (same && lane < kCodeWords)
#pragma unroll
      for (int e = 0; e < 8; e++) {
        const uint32_t c = (qword >> (4 * e)) & 15u;
        same = same && (lane * 8 + e >= ql || (c != 0u && (c & (c - 1u)) == 0u));
      }
    if (__all(same)) {
      uint8_t* o = ops + (int64_t)k * kOpsStride + (kOpsStride - ql);
      for (int x = lane; x < ql; x += 64) o[x] = (uint8_t)'M';
      if (lane == 0) {
        nops[k] = (uint16_t)ql;
        out[k] = (uint32_t)ql | ((uint32_t)ql << 8) | (((uint32_t)(ql * sc.match)) & 0xffffu) << 16;
      }
      return;
    }
  }
  const int QRti = sc.go[3] + sc.ge[3], Rti = sc.ge[3];
  const int QRtr = sc.go[5] + sc.ge[5], Rtr = sc.ge[5];
  const int QRqi = sc.go[2] + sc.ge[2], Rqi = sc.ge[2];
  const int QRqr = sc.go[4] + sc.ge[4], Rqr = sc.ge[4];
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  const int nstripe = (ql + 63) >> 6;
  int hend = 0;
  // The sweep in groups of 8 steps (one direction word per group, no per-step store test), the diagonal's
  // column -1 and H(ql - 1, tl - 1) without per-step tests: a lane's H starts as H(i, -1), which the lane below
  // reads as its diagonal at column 0, and H(ql - 1, tl - 1) is the last H lane (ql - 1) % 64 of the last stripe
  // kept.  Steps past the stripe's end (to the group's end) touch no live cell.
  // one sweep per stripe, specialised on the top boundary (stripe 0: computed; later stripes: the previous
  // stripe's bottom row from LDS) and on whether a stripe follows (lane 63 then stores its row)
  auto sweep = [&](int st, auto top_c, auto bot_c) {
    constexpr bool kTop = decltype(top_c)::value, kBot = decltype(bot_c)::value;
    const int i = st * 64 + lane;
    const int rows = min(64, ql - st * 64);
    const uint32_t qcode = i < ql ? (qcp[i >> 3] >> ((i & 7) * 4)) & 15u : 0u;
    const bool qamb = (qcode & (qcode - 1u)) != 0u || qcode == 0u;
    const uint32_t qm = qamb ? 0u : qcode;
    const int Mq = qamb ? 0 : sc.match, Xq = qamb ? 0 : sc.mismatch;
    const int qrq = (i == ql - 1) ? QRqr : QRqi, rq = (i == ql - 1) ? Rqr : Rqi;
    const uint32_t tle = i < ql ? (uint32_t)tl : 0u;  // live columns of this lane
    int hout = -(sc.go[1] + (i + 1) * sc.ge[1]);      // H(i, -1)
    int E = sc.boundary_open ? hout - qrq : kNegInf;
    int Hd = i == 0 ? 0 : -(sc.go[1] + i * sc.ge[1]);  // H(i - 1, -1)
    int fout = 0;
    uint32_t tc = 0;
    const int nsteps = tl + rows - 1;
    for (int t8 = 0; t8 < nsteps; t8 += 8) {
      uint32_t dword = 0;
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const int tt = t8 + u;
        int hb, fb;
        if constexpr (kTop) {
          hb = -(sc.go[0] + (tt + 1) * sc.ge[0]);
          fb = sc.boundary_open ? hb - ((tt == tl - 1) ? QRtr : QRti) : kNegInf;
        } else {
          hb = tt < tl ? S.botH[tt] : 0;
          fb = tt < tl ? S.botF[tt] : 0;
        }
        const uint32_t recv = wave_shr1(pack_hf(hout, fout), pack_hf(hb, fb));
        tc = wave_shr1(tc, (uint32_t)S.tcode[tt]);
        const int Hup = sx16(recv), Fin = (int)recv >> 16;
        const int j = tt - lane;
        const bool live = (uint32_t)j < tle;
        const bool lc = j == tl - 1;
        const int QRt = lc ? QRtr : QRti, Rt = lc ? Rtr : Rti;
        const int sub = (qm & tc) ? Mq : (tc ? Xq : 0);
        const int diag = Hd + sub;
        const int m1 = max(diag, Fin);
        const int h = max(m1, E);
        const int fo = h - QRt, fe = Fin - Rt;
        const int eo = h - qrq, ee = E - rq;
        const uint32_t d = (Fin > diag ? 1u : 0u) | (E > m1 ? 2u : 0u) | (fe > fo ? 4u : 0u) | (ee > eo ? 8u : 0u);
        E = live ? max(eo, ee) : E;
        hout = live ? h : hout;
        fout = live ? max(fo, fe) : fout;
        if constexpr (kBot) {
          if (live && lane == 63) {
            S.botH[j] = hout;
            S.botF[j] = fout;
          }
        }
        Hd = Hup;
        dword |= d << (4 * u);
      }
      S.dir[(st * TW + (t8 >> 3)) * 64 + lane] = dword;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    return hout;
  };
  using T1 = std::integral_constant<bool, true>;
  using T0 = std::integral_constant<bool, false>;
  int hlast;
  if (nstripe == 1) {
    hlast = sweep(0, T1{}, T0{});
  } else {
    sweep(0, T1{}, T1{});
    for (int st = 1; st + 1 < nstripe; st++) sweep(st, T0{}, T1{});
    hlast = sweep(nstripe - 1, T0{}, T0{});
  }
  hend = __builtin_amdgcn_readlane(hlast, (ql - 1) & 63);
  uint8_t* o = ops + (int64_t)k * kOpsStride;
  // backtrack16 from (ql-1, tl-1) by runs, the wave deciding up to 64 steps at once: from a cell reached by a
  // diagonal step (or the start) the path continues diagonally while the cells say neither up nor left -- lane x
  // reads cell (i - x, j - x), a ballot gives the run; after an I (D) step it continues left (up) while the cells'
  // extension bits say so -- lane x reads (i, j - x) ((i - x, j)).  A run's ops are stored by its lanes; the
  // counters, states and align_trim's runs (the first run generated is the alignment's last, the last one its
  // first) are scalar.  Same decisions as the per-cell loop below, cell for cell.
  auto nib = [&](int ii, int jj) -> uint32_t {
    const int l = ii & 63, tt = jj + l;
    return (S.dir[((ii >> 6) * TW + (tt >> 3)) * 64 + l] >> ((tt & 7) * 4)) & 15u;
  };
  int n = 0, i = ql - 1, j = tl - 1, matches = 0;
  uint32_t first_op = 0, run_op = 0;
  int first_run = 0, run_len = 0;
  bool first_open = true;
  auto emit_run = [&](uint32_t c, int r) {  // r >= 1 ops c (wave-uniform)
    if (lane < r) o[kOpsStride - 1 - (n + lane)] = (uint8_t)c;
    if (n == 0) first_op = c;
    if (first_open) {
      if (c == first_op) first_run += r;
      else first_open = false;
    }
    run_len = c == run_op ? run_len + r : r;
    run_op = c;
    n += r;
  };
  enum { kFresh = 0, kInI = 1, kInD = 2 };
  int state = kFresh;
  while (i >= 0 && j >= 0) {
    if (state == kFresh) {
      const int ii = i - lane, jj = j - lane;
      const bool valid = ii >= 0 && jj >= 0;
      const uint32_t d = valid ? nib(ii, jj) : 3u;
      const unsigned long long stop = __ballot((d & 3u) != 0u);  // invalid cells stop the run too
      const int r = stop ? __builtin_ctzll(stop) : 64;
      if (r > 0) {
        const bool m = lane < r && (S.qraw[valid ? ii : 0] & S.traw[valid ? jj : 0]) != 0;
        matches += __builtin_popcountll(__ballot(m));
        emit_run('M', r);
        i -= r;
        j -= r;
      } else {
        const uint32_t d0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)d);
        if (d0 & 2u) {
          emit_run('I', 1);
          j--;
          state = kInI;
        } else {
          emit_run('D', 1);
          i--;
          state = kInD;
        }
      }
    } else if (state == kInI) {
      const int jj = j - lane;
      const uint32_t d = jj >= 0 ? nib(i, jj) : 0u;
      const unsigned long long stop = __ballot((d & 8u) == 0u);
      const int r = stop ? __builtin_ctzll(stop) : 64;
      if (r > 0) {
        emit_run('I', r);
        j -= r;
      }
      if (r < 64) state = kFresh;
    } else {
      const int ii = i - lane;
      const uint32_t d = ii >= 0 ? nib(ii, j) : 0u;
      const unsigned long long stop = __ballot((d & 4u) == 0u);
      const int r = stop ? __builtin_ctzll(stop) : 64;
      if (r > 0) {
        emit_run('D', r);
        i -= r;
      }
      if (r < 64) state = kFresh;
    }
  }
  for (; i >= 0; i -= 64) emit_run('D', min(i + 1, 64));
  for (; j >= 0; j -= 64) emit_run('I', min(j + 1, 64));
  if (lane != 0) return;
  nops[k] = (uint16_t)n;
  const int tlft = run_op != 'M' ? run_len : 0;
  const int trgt = (first_op != 'M' && tlft < n) ? first_run : 0;
  const uint32_t internal = (uint32_t)(n - tlft - trgt);
  out[k] = (uint32_t)matches | (internal << 8) | (((uint32_t)hend & 0xffffu) << 16);
}

hipError_t launch_traceback(const DevSeqs& s, const uint32_t* pq, const uint32_t* pt, int32_t npairs,
                            const Scoring& sc, uint8_t* ops, uint16_t* nops, uint32_t* out, hipStream_t st,
                            int32_t maxl, int32_t maxq) {
  if (npairs <= 0) return hipSuccess;
  if (maxl < 1 || maxl > kMaxLen) return hipErrorInvalidValue;
  if (maxq <= 0 || maxq > maxl) maxq = maxl;
  const TwLayout lay(maxq, maxl);
  hipLaunchKernelGGL(k_trace_wave, dim3((npairs + kTwWaves - 1) / kTwWaves), dim3(64 * kTwWaves),
                     (size_t)lay.wave_bytes * kTwWaves, st, s, pq, pt, npairs, sc, ops, nops, out, maxq, maxl);
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
  if (!attr_set_on_device(k_attr_consensus)) {
    hipError_t e = hipFuncSetAttribute((const void*)k_consensus,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return e;
    mark_attr_set(k_attr_consensus);
  }
  hipLaunchKernelGGL(k_consensus, dim3(nclusters), dim3(kConsThreads), smem, st, s, cstart,
                     nclusters, member_seqno, member_opsidx, member_strand, ops, nops, cons,
                     conslen, overflow);
  return hipGetLastError();
}

}  // namespace uc
