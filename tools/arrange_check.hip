// arrange_check.hip -- checks kernels.hip k_list_arrange (bank-aware posting order) on synthetic lists, linked
// against the built libumiclust.so (measurement / test tool, not product code): every list stays a permutation of
// its postings, and for 32 consecutive chunks of one list the postings of one slot should fall on distinct LDS banks
// (bank = (posting >> 2) & 31, as the counting kernel's ds_add_u32 sees them).  Prints one JSON line.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../ont-tcrconsensus_amd/csrc/umiclust_internal.h"

static double window_load(const std::vector<uint16_t>& post, const std::vector<uint32_t>& off) {
  double tot = 0;
  long cnt = 0;
  for (size_t b = 0; b + 1 < off.size(); b++) {
    const uint32_t o0 = off[b], o1 = off[b + 1], nch = (o1 - o0) / 8;
    for (uint32_t c0 = 0; c0 + 32 <= nch; c0 += 32)
      for (int e = 0; e < 8; e++) {
        int h[32] = {0}, mx = 0;
        for (int l = 0; l < 32; l++) mx = std::max(mx, ++h[(post[o0 + 8 * (c0 + l) + e] >> 2) & 31]);
        tot += mx;
        cnt++;
      }
  }
  return cnt ? tot / cnt : 0.0;
}

int main() {
  std::mt19937 rng(7);
  std::vector<uint32_t> off(uc::kBins + 1, 0);
  std::uniform_int_distribution<int> pick(0, 99);
  for (int b = 0; b < uc::kBins; b++) {
    const int r = pick(rng);
    uint32_t n = 0;
    if (b % 64 == 0) n = 8u * (uint32_t)(1 + pick(rng));            // 1..100 chunks
    else if (r < 3) n = 8u * (uint32_t)(1 + (pick(rng) % 4));       // short lists
    off[b + 1] = off[b] + n;
  }
  const uint32_t N = off[uc::kBins];
  std::vector<uint16_t> post(N);
  std::uniform_int_distribution<int> cv(uc::kCentBase, uc::kCentBase + 14700);
  for (auto& p : post) p = (uint16_t)cv(rng);
  uint32_t* d_off;
  uint16_t* d_post;
  if (hipMalloc(&d_off, off.size() * 4) != hipSuccess || hipMalloc(&d_post, (size_t)N * 2 + 16) != hipSuccess) return 1;
  (void)hipMemcpy(d_off, off.data(), off.size() * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(d_post, post.data(), (size_t)N * 2, hipMemcpyHostToDevice);
  hipEvent_t a, z;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&z);
  (void)hipEventRecord(a, 0);
  if (uc::launch_index_arrange(d_off, d_post, 0) != hipSuccess) return 2;
  (void)hipEventRecord(z, 0);
  (void)hipEventSynchronize(z);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, z);
  std::vector<uint16_t> got(N);
  (void)hipMemcpy(got.data(), d_post, (size_t)N * 2, hipMemcpyDeviceToHost);
  bool perm = true;
  for (int b = 0; b < uc::kBins && perm; b++) {
    std::vector<uint16_t> x(post.begin() + off[b], post.begin() + off[b + 1]), y(got.begin() + off[b], got.begin() + off[b + 1]);
    std::sort(x.begin(), x.end());
    std::sort(y.begin(), y.end());
    perm = x == y;
  }
  printf("{\"postings\": %u, \"permutation\": %s, \"ms\": %.3f, \"busiest_bank_before\": %.3f, \"busiest_bank_after\": %.3f}\n",
         N, perm ? "true" : "false", ms, window_load(post, off), window_load(got, off));
  return perm ? 0 : 3;
}
