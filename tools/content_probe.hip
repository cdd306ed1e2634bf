// content_probe.hip — do the read-request counts of a streaming pass depend on
// the CONTENT of the rows?  An in-place pass over 2^20 rows of 1 KiB (the
// k_rpass2 shape: one workgroup of 4 waves per 1024-row partition, 16 rows per
// chunk, NT loads and stores, v ^= key with key = 0 from the host) over
// tables filled (0) all zero, (1) all random, (2) 20% random rows, 80% zero,
// (3) all 0x01.  Counted by rocprofv3: TCP_TCC_READ_REQ, TCC_BUBBLE.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/content_probe tools/content_probe.hip
// Test infrastructure only.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <random>
#include <vector>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_stream(uint4* table, uint32_t key) {
  constexpr int U = 16, ROWS = 1024;
  const uint32_t w = blockIdx.x, wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  uint4* part = table + (uint64_t)w * ROWS * 64;
  for (uint32_t j = wave * U; j < ROWS; j += 4 * U) {
    v4u v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(&part[(uint64_t)(j + u) * 64 + lane]));
#pragma unroll
    for (int u = 0; u < U; ++u) {
      v[u].x ^= key;
      __builtin_nontemporal_store(v[u], reinterpret_cast<v4u*>(&part[(uint64_t)(j + u) * 64 + lane]));
    }
  }
}

int main() {
  const uint64_t rows = 1ull << 20, bytes = rows * 1024;
  uint4* table;
  if (hipMalloc(&table, bytes) != hipSuccess) return 1;
  std::vector<uint32_t> h(bytes / 4);
  std::mt19937 g(3);
  for (int fill = 0; fill < 4; ++fill) {
    for (uint64_t r = 0; r < rows; ++r) {
      const bool rnd = fill == 1 || (fill == 2 && (g() % 5) == 0);
      for (int k = 0; k < 256; ++k) h[r * 256 + k] = fill == 3 ? 0x01010101u : rnd ? g() : 0u;
    }
    (void)hipMemcpy(table, h.data(), bytes, hipMemcpyHostToDevice);
    for (int rep = 0; rep < 4; ++rep) hipLaunchKernelGGL(k_stream, dim3(rows / 1024), dim3(256), 0, 0, table, 0u);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
  }
  printf("content_probe ok\n");
  return 0;
}
