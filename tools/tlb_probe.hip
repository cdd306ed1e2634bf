// tlb_probe.hip — do uncached L2 reads (TCC_UC_REQ) follow the ORDER of a
// gather (page-table walks on TLB misses) rather than the set of lines read?
// One wave per 1 KiB record, the record index taken from an order array:
//   order 0: sequential, 1: random permutation, 2: bit-reversed index,
//   3: sequential inside 64-record chunks whose order is random
// over buffers of 64 MiB and 1 GiB.  Every order reads every record once.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/tlb_probe tools/tlb_probe.hip
// Test infrastructure only.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>

__global__ __launch_bounds__(256) void k_gather(const uint4* __restrict__ buf, const uint32_t* __restrict__ ord,
                                                uint32_t n, uint4* __restrict__ out) {
  const uint32_t i = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
  if (i >= n) return;
  const uint32_t r = ord[i];
  const uint4 v = buf[(uint64_t)r * 64 + lane];
  out[(uint64_t)i * 64 + lane] = v;
}

int main() {
  const uint32_t sizes[] = {1u << 16, 1u << 20};  // records of 1 KiB: 64 MiB, 1 GiB
  uint4 *buf, *out;
  uint32_t* ord;
  if (hipMalloc(&buf, (1ull << 20) * 1024) != hipSuccess || hipMalloc(&out, (1ull << 20) * 1024) != hipSuccess ||
      hipMalloc(&ord, (1u << 20) * 4) != hipSuccess)
    return 1;
  (void)hipMemset(buf, 3, (1ull << 20) * 1024);
  std::mt19937 g(7);
  for (uint32_t n : sizes) {
    for (int o = 0; o < 4; ++o) {
      std::vector<uint32_t> v(n);
      for (uint32_t i = 0; i < n; ++i) v[i] = i;
      if (o == 1) std::shuffle(v.begin(), v.end(), g);
      if (o == 2) {
        int b = 0;
        while ((1u << b) < n) ++b;
        for (uint32_t i = 0; i < n; ++i) {
          uint32_t x = i, y = 0;
          for (int k = 0; k < b; ++k) y |= ((x >> k) & 1u) << (b - 1 - k);
          v[i] = y;
        }
      }
      if (o == 3) {
        std::vector<uint32_t> c(n / 64);
        for (uint32_t i = 0; i < n / 64; ++i) c[i] = i;
        std::shuffle(c.begin(), c.end(), g);
        for (uint32_t i = 0; i < n; ++i) v[i] = c[i / 64] * 64 + i % 64;
      }
      (void)hipMemcpy(ord, v.data(), n * 4, hipMemcpyHostToDevice);
      for (int r = 0; r < 4; ++r) hipLaunchKernelGGL(k_gather, dim3(n / 4), dim3(256), 0, 0, buf, ord, n, out);
      (void)hipDeviceSynchronize();
    }
  }
  printf("tlb_probe ok\n");
  return 0;
}
