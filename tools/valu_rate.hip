// VALU issue-rate probe for the aligner's instruction mix (gfx950): cycles per wave-instruction per SIMD of
// each op the k_align_pk column loop issues, with W waves per SIMD, 8 independent chains per wave (rate) or one
// dependent chain (latency).  Build: hipcc -O3 --offload-arch=gfx950 -o tools/valu_rate tools/valu_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define OP2(name, ins) \
  struct name { static __device__ __forceinline__ void run(uint32_t& a, uint32_t b) { asm volatile(ins " %0, %0, %1" : "+v"(a) : "v"(b)); } };
#define OP3(name, ins) \
  struct name { static __device__ __forceinline__ void run(uint32_t& a, uint32_t b) { asm volatile(ins " %0, %0, %1, %1" : "+v"(a) : "v"(b)); } };
OP2(AddU32, "v_add_u32")
OP2(PkSub, "v_pk_sub_i16")
OP2(PkMax, "v_pk_max_i16")
OP2(PkAshr, "v_pk_ashrrev_i16")
OP3(PkMad, "v_pk_mad_u16")
OP3(Add3, "v_add3_u32")
OP3(AndOr, "v_and_or_b32")
struct Bitop3 {
  static __device__ __forceinline__ void run(uint32_t& a, uint32_t b) {
    asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0xca" : "+v"(a) : "v"(b));
  }
};

template <typename Op, int CH>
__global__ __launch_bounds__(64) void k_rate(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a[CH];
#pragma unroll
  for (int c = 0; c < CH; c++) a[c] = seed + threadIdx.x * 7u + c;
  const uint32_t b = seed ^ threadIdx.x;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int r = 0; r < 8; r++)
#pragma unroll
      for (int c = 0; c < CH; c++) Op::run(a[c], b);
  }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < CH; c++) s ^= a[c];
  if (s == 0x12345678u) out[blockIdx.x] = s;
}

template <typename Op, int CH>
void probe(const char* name, int wps, int iters, uint32_t* d) {
  const int cus = 256, simds = cus * 4;
  const int grid = simds * wps;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL((k_rate<Op, CH>), dim3(grid), dim3(64), 0, 0, d, 16, 1u);  // warm
  hipEventRecord(e0, 0);
  hipLaunchKernelGGL((k_rate<Op, CH>), dim3(grid), dim3(64), 0, 0, d, iters, 1u);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  const double instr_per_simd = (double)wps * iters * 8 * CH;  // wave-instructions per SIMD
  const double ghz = 2.4;
  printf("{\"op\": \"%s\", \"chains\": %d, \"waves_per_simd\": %d, \"ms\": %.4f, \"cycles_per_instr_at_2.4GHz\": %.3f}\n",
         name, CH, wps, ms, ms * 1e-3 * ghz * 1e9 / instr_per_simd);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
}

template <typename Op>
void all(const char* name, uint32_t* d) {
  for (int w : {1, 2, 3, 4}) probe<Op, 8>(name, w, 4096, d);
  probe<Op, 1>(name, 1, 4096, d);
  probe<Op, 1>(name, 3, 4096, d);
}

int main() {
  uint32_t* d = nullptr;
  if (hipMalloc(&d, 1 << 20) != hipSuccess) return 1;
  all<AddU32>("v_add_u32", d);
  all<PkSub>("v_pk_sub_i16", d);
  all<PkMax>("v_pk_max_i16", d);
  all<PkAshr>("v_pk_ashrrev_i16", d);
  all<PkMad>("v_pk_mad_u16", d);
  all<Add3>("v_add3_u32", d);
  all<AndOr>("v_and_or_b32", d);
  all<Bitop3>("v_bitop3_b32", d);
  hipFree(d);
  return 0;
}
