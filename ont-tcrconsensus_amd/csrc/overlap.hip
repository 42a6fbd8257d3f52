// overlap.hip -- region-vs-region UMI overlap counts on the GPU.
//
// Replaces the O(R^2 n m) Python string scan of /root/reference/ont_tcr_consensus/extract_umis.py:
//   count_single_umi_overlaps (:270-290): for one region-1 UMI, the number of region-2 consensus UMIs
//       that are string-equal to it (the edlib comparison is commented out upstream, so equality it is);
//   count_overlapping_umis_between_2_regions (:293-342): the sum of those counts over region 1 (the TSV
//       value) and whether any count exceeds 1 (the warning);
//   count_overlapping_umis_between_all_regions (:345-369): every unordered region pair.
// As a hash join: every sequence of every region is hashed (64-bit, seeded), inserted into one
// open-addressing table (the slot = the distinct sequence; its representative = the lowest index), checked
// byte-for-byte against the representative (a 64-bit hash collision between different sequences is
// detected and the host re-runs with the next seed, so the result is always exact), bucketed by slot (CSR),
// and each multi-member slot adds c_a(s) * c_b(s) to total[a][b] and max c_b(s) to maxc[a][b] for every
// region pair a < b that holds s.  HBM/atomic-bound integer work, no MFMA.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "../../include/umiclust.h"
#include "umiclust_internal.h"

namespace uc {

constexpr uint64_t kOvEmpty = ~0ull;
constexpr int kOvThreads = 256;
constexpr int kOvScan = 1024;  // counts per scan block (4 per thread)

__device__ __forceinline__ uint64_t ov_mix(uint64_t h) {
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdull;
  h ^= h >> 33;
  h *= 0xc4ceb9fe1a85ec53ull;
  h ^= h >> 33;
  return h;
}

// per sequence: hash of its bytes (seeded, length mixed in), never kOvEmpty; its region
__global__ void k_ov_hash(const char* __restrict__ seqs, const int64_t* __restrict__ offs, int64_t n,
                          const int64_t* __restrict__ rstart, int32_t nreg, uint64_t seed, uint64_t hmask,
                          uint64_t* __restrict__ hash, int32_t* __restrict__ region) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t a = offs[i], b = offs[i + 1];
  uint64_t h = seed ^ ((uint64_t)(b - a) * 0x9e3779b97f4a7c15ull);
  for (int64_t x = a; x < b; x++) h = (h ^ (uint8_t)seqs[x]) * 0x100000001b3ull;
  h = ov_mix(h) & hmask;  // hmask < ~0 only in the collision test (UMICLUST_OVERLAP_TEST_COLLIDE)
  hash[i] = h == kOvEmpty ? h - 1 : h;
  int lo = 0, hi = nreg - 1;  // last region with rstart <= i
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (rstart[mid] <= i) lo = mid;
    else hi = mid - 1;
  }
  region[i] = lo;
}

__device__ __forceinline__ int64_t ov_find(const uint64_t* __restrict__ keys, uint64_t mask, uint64_t h) {
  uint64_t s = h & mask;
  while (true) {
    const uint64_t k = keys[s];
    if (k == h) return (int64_t)s;
    if (k == kOvEmpty) return -1;
    s = (s + 1) & mask;
  }
}

// claim a slot per distinct hash (linear probing); the representative is the lowest index
__global__ void k_ov_insert(const uint64_t* __restrict__ hash, int64_t n, uint64_t mask,
                            unsigned long long* __restrict__ keys, unsigned long long* __restrict__ rep) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t h = hash[i];
  uint64_t s = h & mask;
  while (true) {
    const unsigned long long prev = atomicCAS(&keys[s], (unsigned long long)kOvEmpty, (unsigned long long)h);
    if (prev == kOvEmpty || prev == h) break;
    s = (s + 1) & mask;
  }
  atomicMin(&rep[s], (unsigned long long)i);
}

// every sequence: its slot, equality with the slot's representative (else: a collision), slot sizes
__global__ void k_ov_verify(const char* __restrict__ seqs, const int64_t* __restrict__ offs, int64_t n,
                            const uint64_t* __restrict__ hash, uint64_t mask, const uint64_t* __restrict__ keys,
                            const unsigned long long* __restrict__ rep, int64_t* __restrict__ slot,
                            uint32_t* __restrict__ cnt, uint32_t* __restrict__ collision) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t s = ov_find(keys, mask, hash[i]);
  slot[i] = s;
  const int64_t r = (int64_t)rep[s];
  const int64_t a = offs[i], b = offs[i + 1], ra = offs[r], rb = offs[r + 1];
  bool eq = (b - a) == (rb - ra);
  for (int64_t x = 0; eq && x < b - a; x++) eq = seqs[a + x] == seqs[ra + x];
  if (!eq) atomicOr(collision, 1u);
  atomicAdd(&cnt[s], 1u);
}

// exclusive scan of cnt[0, m) into start[0, m] (three launches: block sums, their scan, apply)
__global__ void k_ov_scan_sum(const uint32_t* __restrict__ cnt, int64_t m, uint32_t* __restrict__ bsum) {
  __shared__ uint32_t red[kOvThreads / 64];
  const int64_t base = (int64_t)blockIdx.x * kOvScan;
  uint32_t v = 0;
  for (int j = 0; j < kOvScan / kOvThreads; j++) {
    const int64_t x = base + threadIdx.x + (int64_t)j * kOvThreads;
    v += x < m ? cnt[x] : 0u;
  }
  for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int w = 0; w < kOvThreads / 64; w++) t += red[w];
    bsum[blockIdx.x] = t;
  }
}

__global__ void k_ov_scan_top(uint32_t* __restrict__ bsum, int64_t nb) {
  // one block: exclusive scan of the block sums in chunks of 256
  __shared__ uint32_t buf[kOvThreads];
  __shared__ uint32_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int64_t c0 = 0; c0 < nb; c0 += kOvThreads) {
    const int64_t x = c0 + threadIdx.x;
    const uint32_t v = x < nb ? bsum[x] : 0u;
    buf[threadIdx.x] = v;
    __syncthreads();
    for (int d = 1; d < kOvThreads; d <<= 1) {
      const uint32_t u = threadIdx.x >= (unsigned)d ? buf[threadIdx.x - d] : 0u;
      __syncthreads();
      buf[threadIdx.x] += u;
      __syncthreads();
    }
    if (x < nb) bsum[x] = carry + buf[threadIdx.x] - v;
    __syncthreads();
    if (threadIdx.x == kOvThreads - 1) carry += buf[kOvThreads - 1];
    __syncthreads();
  }
}

__global__ void k_ov_scan_apply(const uint32_t* __restrict__ cnt, int64_t m, const uint32_t* __restrict__ bsum,
                                uint32_t* __restrict__ start, uint32_t* __restrict__ cursor) {
  __shared__ uint32_t buf[kOvScan];
  const int64_t base = (int64_t)blockIdx.x * kOvScan;
  for (int j = threadIdx.x; j < kOvScan; j += kOvThreads) buf[j] = base + j < m ? cnt[base + j] : 0u;
  __syncthreads();
  if (threadIdx.x == 0) {  // serial scan of 1024 counts in LDS (small next to the table passes)
    uint32_t acc = bsum[blockIdx.x];
    for (int j = 0; j < kOvScan; j++) {
      const uint32_t v = buf[j];
      buf[j] = acc;
      acc += v;
    }
  }
  __syncthreads();
  for (int j = threadIdx.x; j < kOvScan; j += kOvThreads)
    if (base + j < m) {
      start[base + j] = buf[j];
      cursor[base + j] = buf[j];
    }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) {
    int64_t last = m - 1 - base;
    start[m] = buf[last] + cnt[m - 1];
  }
}

__global__ void k_ov_fill(const int64_t* __restrict__ slot, int64_t n, uint32_t* __restrict__ cursor,
                          uint32_t* __restrict__ members) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  members[atomicAdd(&cursor[slot[i]], 1u)] = (uint32_t)i;
}

// one thread per slot: members in index (= region) order, run lengths per region, then every region pair.
// Buckets of more than kOvSmallBucket members (one UMI present many times: an artifact shared by many regions)
// are handed to k_ov_pairs_big, so no thread runs a quadratic sort or pair loop over a large bucket.
__global__ void k_ov_pairs(const uint32_t* __restrict__ start, int64_t m, uint32_t* __restrict__ members,
                           const int32_t* __restrict__ region, int32_t nreg,
                           unsigned long long* __restrict__ total, uint32_t* __restrict__ maxc,
                           uint32_t* __restrict__ big, uint32_t* __restrict__ nbig) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= m) return;
  const uint32_t a = start[s], b = start[s + 1];
  if (b - a < 2) return;
  if (b - a > (uint32_t)kOvSmallBucket) {
    big[atomicAdd(nbig, 1u)] = (uint32_t)s;
    return;
  }
  uint32_t* mb = members + a;
  const uint32_t nb = b - a;
  // insertion sort (buckets are small: one distinct consensus UMI)
  for (uint32_t x = 1; x < nb; x++) {
    const uint32_t v = mb[x];
    uint32_t y = x;
    while (y > 0 && mb[y - 1] > v) {
      mb[y] = mb[y - 1];
      y--;
    }
    mb[y] = v;
  }
  if (region[mb[0]] == region[mb[nb - 1]]) return;  // one region only
  // region runs: (region, count) in order; pairs a < b of runs
  for (uint32_t i0 = 0; i0 < nb;) {
    const int ra = region[mb[i0]];
    uint32_t i1 = i0;
    while (i1 < nb && region[mb[i1]] == ra) i1++;
    const uint32_t ca = i1 - i0;
    for (uint32_t j0 = i1; j0 < nb;) {
      const int rb = region[mb[j0]];
      uint32_t j1 = j0;
      while (j1 < nb && region[mb[j1]] == rb) j1++;
      const uint32_t cb = j1 - j0;
      const int64_t cell = (int64_t)ra * nreg + rb;
      atomicAdd(&total[cell], (unsigned long long)ca * cb);
      atomicMax(&maxc[cell], cb);
      j0 = j1;
    }
    i0 = i1;
  }
}

// large buckets: one workgroup per bucket (persistent grid over the list k_ov_pairs built).  A region histogram
// in LDS replaces the sort (regions are index ranges, so the nonzero entries in region order are the runs), a
// block scan compacts it, and the pairs of runs are spread over the threads row by row.
constexpr int kOvMaxRegions = UMICLUST_OVERLAP_MAX_REGIONS;
__global__ __launch_bounds__(kOvThreads) void k_ov_pairs_big(const uint32_t* __restrict__ start,
                                                           const uint32_t* __restrict__ members,
                                                           const int32_t* __restrict__ region, int32_t nreg,
                                                           const uint32_t* __restrict__ big,
                                                           const uint32_t* __restrict__ nbig,
                                                           unsigned long long* __restrict__ total,
                                                           uint32_t* __restrict__ maxc) {
  __shared__ uint32_t hist[kOvMaxRegions];
  __shared__ uint16_t rr[kOvMaxRegions];
  __shared__ uint32_t rc[kOvMaxRegions];
  __shared__ uint32_t part[kOvThreads];
  __shared__ uint32_t nz_s;
  const int tid = threadIdx.x;
  const uint32_t nbuckets = *nbig;
  for (uint32_t q = blockIdx.x; q < nbuckets; q += gridDim.x) {
    const uint32_t s = big[q];
    const uint32_t a = start[s], nb = start[s + 1] - a;
    for (int r = tid; r < nreg; r += kOvThreads) hist[r] = 0;
    if (tid == 0) nz_s = 0;
    __syncthreads();
    for (uint32_t i = tid; i < nb; i += kOvThreads) atomicAdd(&hist[region[members[a + i]]], 1u);
    __syncthreads();
    // compaction in region order: chunks of kOvThreads regions, an exclusive scan of the nonzero flags
    for (int r0 = 0; r0 < nreg; r0 += kOvThreads) {
      const int r = r0 + tid;
      const uint32_t f = (r < nreg && hist[r] != 0u) ? 1u : 0u;
      part[tid] = f;
      __syncthreads();
      for (int d = 1; d < kOvThreads; d <<= 1) {
        const uint32_t v = tid >= d ? part[tid - d] : 0u;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
      }
      const uint32_t base = nz_s;
      if (f) {
        rr[base + part[tid] - 1u] = (uint16_t)r;
        rc[base + part[tid] - 1u] = hist[r];
      }
      __syncthreads();
      if (tid == kOvThreads - 1) nz_s = base + part[tid];
      __syncthreads();
    }
    const uint32_t nz = nz_s;
    for (uint32_t i = 0; i + 1 < nz; i++) {
      const uint32_t ra = rr[i], ca = rc[i];
      for (uint32_t j = i + 1 + tid; j < nz; j += kOvThreads) {
        const int64_t cell = (int64_t)ra * nreg + rr[j];
        atomicAdd(&total[cell], (unsigned long long)ca * rc[j]);
        atomicMax(&maxc[cell], rc[j]);
      }
    }
    __syncthreads();
  }
}

// two-set form: cnt2[slot] = members from set 2 (region 1); counts[i] for set 1 (region 0)
__global__ void k_ov_count2(const int64_t* __restrict__ slot, const int32_t* __restrict__ region, int64_t n,
                            uint32_t* __restrict__ cnt2) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || region[i] != 1) return;
  atomicAdd(&cnt2[slot[i]], 1u);
}
__global__ void k_ov_gather2(const int64_t* __restrict__ slot, int64_t n1, const uint32_t* __restrict__ cnt2,
                             int64_t* __restrict__ counts) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n1) return;
  counts[i] = cnt2[slot[i]];
}

// table pass with one seed; returns the collision flag through *collided (synchronous)
hipError_t launch_overlap_table(const char* seqs, const int64_t* offs, int64_t n, const int64_t* rstart, int32_t nreg,
                                uint64_t seed, uint64_t hmask, uint64_t mask, const OvBuffers& B, bool csr,
                                uint32_t* collided, hipStream_t st) {
  const int64_t m = (int64_t)mask + 1;
  const dim3 gn((unsigned)((n + kOvThreads - 1) / kOvThreads)), blk(kOvThreads);
  hipError_t e;
  if ((e = hipMemsetAsync(B.keys, 0xff, (size_t)m * 8, st)) != hipSuccess) return e;
  if ((e = hipMemsetAsync(B.rep, 0xff, (size_t)m * 8, st)) != hipSuccess) return e;
  if ((e = hipMemsetAsync(B.cnt, 0, (size_t)m * 4, st)) != hipSuccess) return e;
  if ((e = hipMemsetAsync(B.collision, 0, 4, st)) != hipSuccess) return e;
  if (n > 0) {
    hipLaunchKernelGGL(k_ov_hash, gn, blk, 0, st, seqs, offs, n, rstart, nreg, seed, hmask, B.hash, B.region);
    hipLaunchKernelGGL(k_ov_insert, gn, blk, 0, st, B.hash, n, mask, B.keys, B.rep);
    hipLaunchKernelGGL(k_ov_verify, gn, blk, 0, st, seqs, offs, n, B.hash, mask, (const uint64_t*)B.keys, B.rep,
                       B.slot, B.cnt, B.collision);
    if (csr) {
      const int64_t nb = (m + kOvScan - 1) / kOvScan;
      hipLaunchKernelGGL(k_ov_scan_sum, dim3((unsigned)nb), blk, 0, st, B.cnt, m, B.bsum);
      hipLaunchKernelGGL(k_ov_scan_top, dim3(1), blk, 0, st, B.bsum, nb);
      hipLaunchKernelGGL(k_ov_scan_apply, dim3((unsigned)nb), blk, 0, st, B.cnt, m, B.bsum, B.start, B.cursor);
      hipLaunchKernelGGL(k_ov_fill, gn, blk, 0, st, B.slot, n, B.cursor, B.members);
    }
  }
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if ((e = hipMemcpyAsync(collided, B.collision, 4, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
  return hipStreamSynchronize(st);
}

hipError_t launch_overlap_pairs(const OvBuffers& B, uint64_t mask, int32_t nreg, unsigned long long* total,
                                uint32_t* maxc, hipStream_t st) {
  const int64_t m = (int64_t)mask + 1;
  if (nreg > kOvMaxRegions) return hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(B.nbig, 0, 4, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_ov_pairs, dim3((unsigned)((m + kOvThreads - 1) / kOvThreads)), dim3(kOvThreads), 0, st,
                     B.start, m, B.members, B.region, nreg, total, maxc, B.big, B.nbig);
  hipLaunchKernelGGL(k_ov_pairs_big, dim3(512), dim3(kOvThreads), 0, st, B.start, B.members, B.region, nreg, B.big,
                     B.nbig, total, maxc);
  return hipGetLastError();
}

hipError_t launch_overlap_two(const OvBuffers& B, uint64_t mask, int64_t n, int64_t n1, int64_t* counts,
                              hipStream_t st) {
  const int64_t m = (int64_t)mask + 1;
  hipError_t e = hipMemsetAsync(B.cnt, 0, (size_t)m * 4, st);
  if (e != hipSuccess) return e;
  if (n > 0)
    hipLaunchKernelGGL(k_ov_count2, dim3((unsigned)((n + kOvThreads - 1) / kOvThreads)), dim3(kOvThreads), 0, st,
                       B.slot, B.region, n, B.cnt);
  if (n1 > 0)
    hipLaunchKernelGGL(k_ov_gather2, dim3((unsigned)((n1 + kOvThreads - 1) / kOvThreads)), dim3(kOvThreads), 0, st,
                       B.slot, n1, B.cnt, counts);
  return hipGetLastError();
}

}  // namespace uc
