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

hipError_t launch_extract(const char* seqs, const int64_t* offs, int64_t n, int32_t a5, int32_t a3, int32_t k,
                          const ExtractPatterns* P, int32_t* out, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_extract, dim3((unsigned)((2 * n + 255) / 256)), dim3(256), 0, st, seqs, offs, n, a5, a3, k,
                     P, out);
  return hipGetLastError();
}

}  // namespace uc
