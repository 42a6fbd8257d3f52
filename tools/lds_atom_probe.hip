// lds_atom_probe.hip -- measures the cost of one ds_add_u32 wave-instruction per CU for address patterns
// (measurement only, not product code): which lanes conflict on MI355X LDS atomics?  The counting kernel's cost is
// set by these.  Pattern of lane l's dword at slot e (8 slots, one instruction each):
//   0 seq       l + 64 e                          distinct dwords, banks l mod 32 / mod 64
//   1 dupgrp    (l & 31) + 64 e                   lanes l and l + 32 on the same dword
//   2 xgrp64    (l & 31) + 64 (l >> 5) + 128 e    lanes l and l + 32 on the same bank mod 64, distinct dwords
//   3 stride2   2 l + 128 e                       2-way per 32-bank group; lanes l, l+32 same bank mod 64
//   4 random    hash(l, e) mod 4096
//   5 arranged  (l + 4 e) mod 32 + 32 rnd(l, e)   distinct banks mod 32 in each 32-lane group, random rows
//   6 same32    32 l + e                          one bank per 32-lane group (32-way)
//   7 arr64     (l + 4 e) mod 64 + 64 rnd(l, e)   distinct banks mod 64 over the wave
// Prints one JSON line per pattern: ns and cycles (at the given clock) per wave-instruction per CU.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

constexpr int kIters = 2048;
constexpr int kDw = 4096;  // 16 KB of counters

__device__ __forceinline__ uint32_t hsh(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

template <int P>
__global__ __launch_bounds__(256) void k_probe(uint32_t* out, uint32_t seed) {
  __shared__ uint32_t buf[kDw];
  for (int i = threadIdx.x; i < kDw; i += 256) buf[i] = 0;
  __syncthreads();
  const uint32_t l = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t a[8];
#pragma unroll
  for (int e = 0; e < 8; e++) {
    const uint32_t r = hsh(seed * 977u + w * 131u + l * 8u + (uint32_t)e + blockIdx.x * 7919u);
    uint32_t d;
    if (P == 0) d = l + 64u * e;
    else if (P == 1) d = (l & 31u) + 64u * e;
    else if (P == 2) d = (l & 31u) + 64u * (l >> 5) + 128u * e;
    else if (P == 3) d = 2u * l + 128u * e;
    else if (P == 4) d = r % kDw;
    else if (P == 5) d = ((l + 4u * e) & 31u) + 32u * (r % (kDw / 32));
    else if (P == 6) d = 32u * l + e;
    else d = ((l + 4u * e) & 63u) + 64u * (r % (kDw / 64));
    a[e] = (d % kDw) * 4u;
  }
  for (int i = 0; i < kIters; i++) {
    asm volatile(
        "ds_add_u32 %0, %8\n ds_add_u32 %1, %8\n ds_add_u32 %2, %8\n ds_add_u32 %3, %8\n"
        "ds_add_u32 %4, %8\n ds_add_u32 %5, %8\n ds_add_u32 %6, %8\n ds_add_u32 %7, %8\n s_waitcnt lgkmcnt(0)\n"
        :
        : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7]), "v"(1u));
  }
  __syncthreads();
  out[blockIdx.x * 256 + threadIdx.x] = buf[threadIdx.x];
}

template <int P>
void run(int cus, uint32_t* out, double ghz) {
  const int grid = cus * 8;
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL(k_probe<P>, dim3(grid), dim3(256), 0, 0, out, 1u);  // warm-up
  CHECK(hipEventRecord(a, 0));
  hipLaunchKernelGGL(k_probe<P>, dim3(grid), dim3(256), 0, 0, out, 2u);
  CHECK(hipEventRecord(b, 0));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  const double instrs_per_cu = (double)grid * 4 * kIters * 8 / cus;
  const double ns = ms * 1e6 / instrs_per_cu;
  printf("{\"pattern\": %d, \"ms\": %.4f, \"ns_per_instr_per_cu\": %.4f, \"cycles_per_instr_per_cu\": %.3f}\n", P, ms, ns,
         ns * ghz);
  fflush(stdout);
}

int main(int argc, char** argv) {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const double ghz = argc > 1 ? atof(argv[1]) : 2.4;
  uint32_t* out;
  CHECK(hipMalloc(&out, (size_t)cus * 8 * 256 * 4));
  run<0>(cus, out, ghz);
  run<1>(cus, out, ghz);
  run<2>(cus, out, ghz);
  run<3>(cus, out, ghz);
  run<4>(cus, out, ghz);
  run<5>(cus, out, ghz);
  run<6>(cus, out, ghz);
  run<7>(cus, out, ghz);
  CHECK(hipFree(out));
  return 0;
}
