// pmc_calib.hip -- calibration kernels for the rocprofv3 SQ counters used in bench.py's roofline block
// (measurement only; not product code).  Each kernel saturates one unit with a known instruction stream:
//   k_valu      independent v_add_u32 chains, 8 waves per SIMD: VALU issue-bound
//   k_lds_read  conflict-free ds_read_b32 (2 LDS-array cycles each, MI355X_MICROARCH.md §LDS), 8 waves per
//               SIMD, no dependent use inside the loop: LDS-array-bound
//   k_lds_atom  ds_add_u32 to 64 distinct dwords in distinct banks (conflict-free), then to 64 lanes on one
//               bank of a 32-lane group (32-way conflicts): SQ_LDS_BANK_CONFLICT's unit
// Run under `rocprofv3 --pmc <counters> -- ./pmc_calib`; the per-dispatch counters divided by the known
// instruction counts printed here give the factors of profiles/r03/pmc_calib.json (tools/pmc_calib.py).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                 \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                    \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

constexpr int kIters = 4096;

__global__ __launch_bounds__(256) void k_valu(uint32_t* out, uint32_t seed) {
  uint32_t a = seed + threadIdx.x, b = a ^ 0x9e37u, c = a * 3u, d = a + 7u;
  for (int i = 0; i < kIters; i++) {
    // 16 independent-ish adds per iteration (4 chains)
    asm volatile(
        "v_add_u32 %0, %0, %4\n v_add_u32 %1, %1, %4\n v_add_u32 %2, %2, %4\n v_add_u32 %3, %3, %4\n"
        "v_add_u32 %0, %0, %4\n v_add_u32 %1, %1, %4\n v_add_u32 %2, %2, %4\n v_add_u32 %3, %3, %4\n"
        "v_add_u32 %0, %0, %4\n v_add_u32 %1, %1, %4\n v_add_u32 %2, %2, %4\n v_add_u32 %3, %3, %4\n"
        "v_add_u32 %0, %0, %4\n v_add_u32 %1, %1, %4\n v_add_u32 %2, %2, %4\n v_add_u32 %3, %3, %4\n"
        : "+v"(a), "+v"(b), "+v"(c), "+v"(d)
        : "v"(seed));
  }
  out[blockIdx.x * 256 + threadIdx.x] = a ^ b ^ c ^ d;
}

__global__ __launch_bounds__(256) void k_lds_read(uint32_t* out, uint32_t seed) {
  __shared__ uint32_t buf[256 * 4];
  for (int i = threadIdx.x; i < 256 * 4; i += 256) buf[i] = i ^ seed;
  __syncthreads();
  const uint32_t addr = (uint32_t)(threadIdx.x * 4);  // lane l -> dword l: conflict-free
  uint32_t acc = 0, v0, v1, v2, v3;
  for (int i = 0; i < kIters; i++) {
    asm volatile(
        "ds_read_b32 %0, %4\n ds_read_b32 %1, %4 offset:1024\n ds_read_b32 %2, %4 offset:2048\n"
        "ds_read_b32 %3, %4 offset:3072\n s_waitcnt lgkmcnt(0)\n"
        : "=v"(v0), "=v"(v1), "=v"(v2), "=v"(v3)
        : "v"(addr));
    acc += v0 ^ v1 ^ v2 ^ v3;
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int STRIDE>
__global__ __launch_bounds__(256) void k_lds_atom(uint32_t* out, uint32_t seed) {
  __shared__ uint32_t buf[64 * 33 * 4];
  for (int i = threadIdx.x; i < 64 * 33 * 4; i += 256) buf[i] = 0;
  __syncthreads();
  // STRIDE 1: lane l -> dword l (distinct banks); STRIDE 32: lane l -> dword 32 l (one bank per 32-lane group)
  const uint32_t addr = (uint32_t)(((threadIdx.x & 63) * STRIDE + (threadIdx.x >> 6) * 64 * 33) * 4);
  for (int i = 0; i < kIters; i++) {
    asm volatile(
        "ds_add_u32 %0, %1\n ds_add_u32 %0, %1\n ds_add_u32 %0, %1\n ds_add_u32 %0, %1\n s_waitcnt lgkmcnt(0)\n"
        :
        : "v"(addr), "v"(seed));
  }
  __syncthreads();
  out[blockIdx.x * 256 + threadIdx.x] = buf[threadIdx.x];
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const int grid = cus * 8;  // 8 workgroups of 4 waves per CU: 8 waves per SIMD
  uint32_t* out;
  CHECK(hipMalloc(&out, (size_t)grid * 256 * 4));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const long long waves = (long long)grid * 4;
  struct K {
    const char* name;
    void (*fn)(uint32_t*, uint32_t);
    long long insts_per_wave;
  } ks[] = {{"k_valu", k_valu, 16LL * kIters},
            {"k_lds_read", k_lds_read, 4LL * kIters},
            {"k_lds_atom<1>", k_lds_atom<1>, 4LL * kIters},
            {"k_lds_atom<32>", k_lds_atom<32>, 4LL * kIters}};
  printf("{\"cus\": %d, \"clock_khz\": %d, \"grid\": %d, \"waves\": %lld, \"kernels\": {", cus, prop.clockRate, grid,
         waves);
  for (int k = 0; k < 4; k++) {
    hipLaunchKernelGGL(ks[k].fn, dim3(grid), dim3(256), 0, 0, out, 1u);  // warm
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(ks[k].fn, dim3(grid), dim3(256), 0, 0, out, 2u);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    printf("%s\"%s\": {\"ms\": %.4f, \"insts_per_wave\": %lld, \"insts\": %lld}", k ? ", " : "", ks[k].name, ms,
           ks[k].insts_per_wave, ks[k].insts_per_wave * waves);
  }
  printf("}}\n");
  CHECK(hipFree(out));
  return 0;
}
