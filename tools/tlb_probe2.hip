// tlb_probe2.hip — TLB reach on this part, as seen in TCC_UC_REQ (page-table
// walks): a random gather of 2^20 1-KiB records spread over one buffer of
// 1, 4 or 16 GiB, or over 64 separate 16-MiB allocations; each case launched
// four times (the first launch after the order upload is the cold one).
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/tlb_probe2 tools/tlb_probe2.hip
// Test infrastructure only.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <random>
#include <vector>

__global__ __launch_bounds__(256) void k_gather(const uint4* const* __restrict__ bases, uint32_t shift,
                                                const uint64_t* __restrict__ ord, uint32_t n,
                                                uint4* __restrict__ out) {
  const uint32_t i = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
  if (i >= n) return;
  const uint64_t r = ord[i];
  const uint4* b = bases[r >> shift];
  const uint4 v = b[(r & ((1ull << shift) - 1)) * 64 + lane];
  out[(uint64_t)i * 64 + lane] = v;
}

int main() {
  const uint32_t n = 1u << 20;
  uint4 *out;
  uint64_t* ord;
  const uint4** bases;
  if (hipMalloc(&out, (uint64_t)n * 1024) != hipSuccess || hipMalloc(&ord, n * 8) != hipSuccess ||
      hipMalloc(&bases, 64 * 8) != hipSuccess)
    return 1;
  std::mt19937_64 g(11);
  // cases: (number of allocations, records per allocation as a power of two)
  const int cases[][2] = {{1, 20}, {1, 22}, {1, 24}, {64, 14}};
  for (auto& c : cases) {
    const int na = c[0], sh = c[1];
    std::vector<const uint4*> hb(64, nullptr);
    for (int a = 0; a < na; ++a) {
      uint4* p;
      if (hipMalloc(&p, (1ull << sh) * 1024) != hipSuccess) return 3;
      (void)hipMemset(p, 5, (1ull << sh) * 1024);
      hb[a] = p;
    }
    std::vector<uint64_t> o(n);
    const uint64_t tot = (uint64_t)na << sh;
    for (uint32_t i = 0; i < n; ++i) o[i] = g() % tot;
    (void)hipMemcpy(ord, o.data(), n * 8, hipMemcpyHostToDevice);
    (void)hipMemcpy(bases, hb.data(), 64 * 8, hipMemcpyHostToDevice);
    for (int r = 0; r < 4; ++r) hipLaunchKernelGGL(k_gather, dim3(n / 4), dim3(256), 0, 0, bases, (uint32_t)sh, ord, n, out);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    for (int a = 0; a < na; ++a) (void)hipFree((void*)hb[a]);
  }
  printf("tlb_probe2 ok\n");
  return 0;
}
