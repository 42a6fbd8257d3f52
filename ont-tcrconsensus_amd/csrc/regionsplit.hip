// regionsplit.hip -- region binning of aligned reads on the GPU.
//
// Replaces the per-record loop of filter_and_split_reads_by_region_cluster
// (/root/reference/ont_tcr_consensus/region_split.py:219-333), which sets the shard sizes of the clustering
// hot path: every BAM record is classified (unmapped / secondary or supplementary / too short an overlap /
// too long / kept) and every kept read is written to region_cluster<k>.fasta as
// `>{query_name};strand={+|-}` + its forward sequence (pysam get_forward_sequence: reverse-complemented for
// reverse-strand records).  The host inflates the BGZF blocks on all its threads and finds the record
// offsets; on the device one thread per record decodes the fixed fields and the CIGAR (reference_length =
// M/D/N/=/X lengths) and classifies it, and one wave per kept record writes its FASTA bytes -- the 4-bit
// sequence decoded (and reverse-complemented) lane-parallel -- at its slot in a cluster-grouped output
// buffer, which the host appends to the cluster files.  Byte work: HBM/PCIe-bound, no MFMA.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "umiclust_internal.h"

namespace uc {

__device__ __forceinline__ uint32_t ld_u32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
__device__ __forceinline__ uint32_t ld_u16(const uint8_t* p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8); }

// per record: class (kBamUnmapped ... kBamNoCluster), cluster, output bytes
__global__ void k_bam_classify(const uint8_t* __restrict__ raw, const int64_t* __restrict__ roff, int64_t n,
                               int32_t nref, const int64_t* __restrict__ ref_len, const int32_t* __restrict__ ref_cluster,
                               double minov, int32_t s5, int32_t s3, int8_t* __restrict__ cls,
                               int32_t* __restrict__ cluster, int64_t* __restrict__ outlen) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const uint8_t* p = raw + roff[r] + 4;  // past block_size
  const int32_t ref = (int32_t)ld_u32(p);
  const uint32_t lrn = p[8], ncig = ld_u16(p + 12), flag = ld_u16(p + 14);
  const int32_t lseq = (int32_t)ld_u32(p + 16);
  int8_t c;
  int32_t k = -1;
  int64_t len = 0;
  if (flag & 0x4u) {
    c = kBamUnmapped;
  } else if (flag & 0x900u) {
    c = kBamSecondary;
  } else if (ref < 0 || ref >= nref || ref_len[ref] < 0) {
    c = kBamNoRegion;  // region_length_dict[entry.reference_name] raises
  } else {
    const uint8_t* cg = p + 32 + lrn;
    int64_t rl = 0;
    for (uint32_t x = 0; x < ncig; x++) {
      const uint32_t v = ld_u32(cg + 4 * x), op = v & 15u;
      if (op == 0 || op == 2 || op == 3 || op == 7 || op == 8) rl += v >> 4;
    }
    // pysam's reference_length = bam_endpos - pos, and htslib's bam_endpos counts a zero reference span (no CIGAR,
    // or only I/S/H/P ops) as 1: such a record is 1 base long and drops as short (:261-263)
    if (rl == 0) rl = 1;
    const double L = (double)ref_len[ref];
    if ((double)rl < L * minov) {
      c = kBamShort;
    } else if ((double)lseq > L * (2.0 - minov) + (double)(s5 + s3)) {
      c = kBamLong;
    } else if (ref_cluster[ref] < 0) {
      c = kBamNoCluster;  // region_cluster_dict[entry.reference_name] raises
    } else {
      c = kBamKept;
      k = ref_cluster[ref];
      len = 1 + (int64_t)(lrn - 1) + 9 + 1 + (lseq > 0 ? lseq : 4) + 1;  // ">name;strand=s\nSEQ\n" ("None")
    }
  }
  cls[r] = c;
  cluster[r] = k;
  outlen[r] = len;
}

// one wave per kept record: ">{name};strand={s}\n{forward sequence}\n" at pos[r]
__global__ void k_bam_emit(const uint8_t* __restrict__ raw, const int64_t* __restrict__ roff, int64_t n,
                           const int8_t* __restrict__ cls, const int64_t* __restrict__ pos, char* __restrict__ out) {
  const int64_t r = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= n || cls[r] != kBamKept) return;
  const uint8_t* p = raw + roff[r] + 4;
  const uint32_t lrn = p[8], ncig = ld_u16(p + 12), flag = ld_u16(p + 14);
  const int32_t lseq = (int32_t)ld_u32(p + 16);
  const uint8_t* name = p + 32;
  const uint8_t* sq = name + lrn + 4 * ncig;
  char* o = out + pos[r];
  const int nl = (int)lrn - 1;
  for (int x = lane; x < nl; x += 64) o[1 + x] = (char)name[x];
  if (lane == 0) {
    o[0] = '>';
    const char* tag = ";strand=";
    for (int x = 0; x < 8; x++) o[1 + nl + x] = tag[x];
    o[1 + nl + 8] = (flag & 0x10u) ? '-' : '+';
    o[1 + nl + 9] = '\n';
  }
  char* s = o + 1 + nl + 10;
  const char kSym[16] = {'=', 'A', 'C', 'M', 'G', 'R', 'S', 'V', 'T', 'W', 'Y', 'H', 'K', 'D', 'B', 'N'};
  if (lseq <= 0) {
    if (lane < 4) s[lane] = "None"[lane];
    if (lane == 0) s[4] = '\n';
    return;
  }
  const bool rev = (flag & 0x10u) != 0;
  for (int x = lane; x < lseq; x += 64) {
    // forward sequence: position x of the read = stored position (rev ? lseq - 1 - x : x), complemented if rev
    const int y = rev ? lseq - 1 - x : x;
    const uint32_t code = (sq[y >> 1] >> (((y & 1) ^ 1) * 4)) & 15u;
    char ch = kSym[code];
    if (rev) ch = ch == 'A' ? 'T' : ch == 'C' ? 'G' : ch == 'G' ? 'C' : ch == 'T' ? 'A' : ch;
    s[x] = ch;
  }
  if (lane == 0) s[lseq] = '\n';
}

hipError_t launch_bam_classify(const uint8_t* raw, const int64_t* roff, int64_t n, int32_t nref, const int64_t* ref_len,
                               const int32_t* ref_cluster, double minov, int32_t s5, int32_t s3, int8_t* cls,
                               int32_t* cluster, int64_t* outlen, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_bam_classify, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, raw, roff, n, nref, ref_len,
                     ref_cluster, minov, s5, s3, cls, cluster, outlen);
  return hipGetLastError();
}

hipError_t launch_bam_emit(const uint8_t* raw, const int64_t* roff, int64_t n, const int8_t* cls, const int64_t* pos,
                           char* out, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_bam_emit, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st, raw, roff, n, cls, pos, out);
  return hipGetLastError();
}

}  // namespace uc
