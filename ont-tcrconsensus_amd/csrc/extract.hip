// extract.hip -- UMI extraction on the GPU.
//
// Replaces the per-read edlib calls of /root/reference/ont_tcr_consensus/extract_umis.py:19-107
// (`edlib.align(pattern, window, task="path", mode="HW", k=max_pattern_dist, additionalEqualities=IUPAC)`,
// python-edlib >= 1.3.9, pyproject.toml:34) on the 5' and 3' adapter windows of every read (:110-126,
// :189-245).  One thread per (read, window), Myers' bit-parallel edit distance with the pattern (<= 64
// symbols) in one 64-bit word:
//   HW pass: free target start (top row 0, no carry-in), bottom-row score tracked along the window; the
//     edit distance is the minimum (reported if <= k) and locations[0]'s end is the first column with it;
//   start pass (edlib obtainLocations for mode HW): SHW of the reversed pattern against the reversed window
//     prefix [0, end] (top row j: carry-in +1); the LAST reversed column with the edit distance gives
//     start = end - column.
// Equality is a 256-entry match mask per pattern (identical bytes or an IUPAC pair of the reference's
// additionalEqualities, either order), built on the host.  Integer VALU work, a few hundred bytes per read.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "umiclust_internal.h"

namespace uc {

__device__ __forceinline__ void myers_step(uint64_t Eq, uint64_t mask, uint64_t hb, uint64_t hin, uint64_t& Pv,
                                           uint64_t& Mv, int& score) {
  const uint64_t Xv = Eq | Mv;
  const uint64_t Xh = (((Eq & Pv) + Pv) ^ Pv) | Eq;
  uint64_t Ph = Mv | ~(Xh | Pv);
  uint64_t Mh = Pv & Xh;
  score += (Ph & hb) ? 1 : ((Mh & hb) ? -1 : 0);
  Ph = (Ph << 1) | hin;
  Mh <<= 1;
  Pv = (Mh | ~(Xv | Ph)) & mask;
  Mv = Ph & Xv & mask;
}

// out[(i * 2 + w) * 3 + {0, 1, 2}] = edit distance (-1: none <= k), start, end within window w of read i
__global__ void k_extract(const char* __restrict__ seqs, const int64_t* __restrict__ offs, int64_t n, int32_t a5,
                          int32_t a3, int32_t k, const ExtractPatterns* __restrict__ P, int32_t* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 2 * n) return;
  const int64_t i = t >> 1;
  const int w = (int)(t & 1);
  const int64_t b = offs[i], len = offs[i + 1] - b;
  // Python slicing: seq[:a5] and seq[-a3:] (a3 == 0 is the whole read)
  int64_t w0, wl;
  if (w == 0) {
    w0 = b;
    wl = a5 < len ? a5 : len;
  } else {
    wl = (a3 == 0 || a3 > len) ? len : a3;
    w0 = b + len - wl;
  }
  const int m = P->m[w];
  const uint64_t* peq = P->peq[w];
  const uint64_t* peqr = P->peqr[w];
  const uint64_t mask = m == 64 ? ~0ull : ((1ull << m) - 1ull), hb = 1ull << (m - 1);
  uint64_t Pv = mask, Mv = 0;
  int score = m, best = 1 << 30, end = -1;
  for (int64_t j = 0; j < wl; j++) {
    myers_step(peq[(uint8_t)seqs[w0 + j]], mask, hb, 0ull, Pv, Mv, score);
    if (score < best) {
      best = score;
      end = (int)j;
    }
  }
  int32_t* o = out + t * 3;
  if (end < 0 || best > k) {
    o[0] = -1;
    o[1] = -1;
    o[2] = -1;
    return;
  }
  Pv = mask;
  Mv = 0;
  score = m;
  int last = -1;
  for (int p = 0; p <= end; p++) {
    myers_step(peqr[(uint8_t)seqs[w0 + end - p]], mask, hb, 1ull, Pv, Mv, score);
    if (score == best) last = p;
  }
  o[0] = best;
  o[1] = end - last;
  o[2] = end;
}

// Compact-window form: the host gathered every read's two windows into win[i * S, i * S + S) (5' window at
// offset 0, 3' window at a5; S = a5 + a3 rounded to 4), their lengths in wlen[2 i + w].  A workgroup of
// 256 threads takes 128 reads: their S-byte slots are copied into LDS with coalesced 16-byte loads, then each
// thread runs the same two Myers passes on its window from LDS (the byte-per-lane gathers of k_extract touch
// one cache line per lane per step).
constexpr int kExReads = 128;
__global__ __launch_bounds__(256) void k_extract_win(const char* __restrict__ win, const uint8_t* __restrict__ wlen,
                                                     int64_t n, int32_t S, int32_t a5, int32_t k,
                                                     const ExtractPatterns* __restrict__ P, int32_t* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) char ex_smem[];
  const int64_t i0 = (int64_t)blockIdx.x * kExReads;
  const int nr = (int)(n - i0 < kExReads ? n - i0 : kExReads);
  {
    const uint4* src = reinterpret_cast<const uint4*>(win + i0 * S);
    uint4* dst = reinterpret_cast<uint4*>(ex_smem);
    const int nv = (nr * S + 15) >> 4;
    for (int x = threadIdx.x; x < nv; x += blockDim.x) dst[x] = src[x];
  }
  __syncthreads();
  const int r = threadIdx.x >> 1, w = threadIdx.x & 1;
  if (r >= nr) return;
  const int64_t t = (i0 + r) * 2 + w;
  const char* wp = ex_smem + r * S + (w ? a5 : 0);
  const int wl = wlen[t];
  const int m = P->m[w];
  const uint64_t* peq = P->peq[w];
  const uint64_t* peqr = P->peqr[w];
  const uint64_t mask = m == 64 ? ~0ull : ((1ull << m) - 1ull), hb = 1ull << (m - 1);
  uint64_t Pv = mask, Mv = 0;
  int score = m, best = 1 << 30, end = -1;
  for (int j = 0; j < wl; j++) {
    myers_step(peq[(uint8_t)wp[j]], mask, hb, 0ull, Pv, Mv, score);
    if (score < best) {
      best = score;
      end = j;
    }
  }
  int32_t* o = out + t * 3;
  if (end < 0 || best > k) {
    o[0] = -1;
    o[1] = -1;
    o[2] = -1;
    return;
  }
  Pv = mask;
  Mv = 0;
  score = m;
  int last = -1;
  for (int q = 0; q <= end; q++) {
    myers_step(peqr[(uint8_t)wp[end - q]], mask, hb, 1ull, Pv, Mv, score);
    if (score == best) last = q;
  }
  o[0] = best;
  o[1] = end - last;
  o[2] = end;
}

hipError_t launch_extract_win(const char* win, const uint8_t* wlen, int64_t n, int32_t S, int32_t a5, int32_t k,
                              const ExtractPatterns* P, int32_t* out, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const size_t smem = (size_t)kExReads * S + 16;
  hipLaunchKernelGGL(k_extract_win, dim3((unsigned)((n + kExReads - 1) / kExReads)), dim3(2 * kExReads), smem, st, win,
                     wlen, n, S, a5, k, P, out);
  return hipGetLastError();
}

hipError_t launch_extract(const char* seqs, const int64_t* offs, int64_t n, int32_t a5, int32_t a3, int32_t k,
                          const ExtractPatterns* P, int32_t* out, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_extract, dim3((unsigned)((2 * n + 255) / 256)), dim3(256), 0, st, seqs, offs, n, a5, a3, k,
                     P, out);
  return hipGetLastError();
}

}  // namespace uc
