// fetch_probe.hip — does rocprofv3 FETCH_SIZE depend on the ORDER in which a
// kernel gathers whole 1 KiB rows (same rows, same bytes)?  Each kernel reads
// 65536 rows of 1 KiB (one wave per row, 16 B per lane) from a 256 MiB buffer
// and writes one word per row:
//   k_seq      row p                        (sequential)
//   k_perm     row perm(p), a fixed random permutation of [0, 65536)
//   k_scatter  row perm(p) * 4              (random rows over the whole buffer)
//   k_mixed    first half sequential, second half permuted
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/fetch_probe tools/fetch_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

__global__ __launch_bounds__(256) void k_rows(const uint4* __restrict__ src, const uint32_t* __restrict__ idx,
                                              uint32_t* __restrict__ out, uint32_t n) {
  const uint32_t w = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
  if (w >= n) return;
  const uint4 v = src[(uint64_t)idx[w] * 64 + lane];
  uint32_t x = v.x ^ v.y ^ v.z ^ v.w;
  for (int o = 32; o > 0; o >>= 1) x ^= __shfl_xor(x, o);
  if (lane == 0) out[w] = x;
}

// 16 rows per wave, all loads in flight together (as the phase-C walks)
__global__ __launch_bounds__(256) void k_rows16(const uint4* __restrict__ src, const uint32_t* __restrict__ idx,
                                                uint32_t* __restrict__ out, uint32_t n) {
  const uint32_t w = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
  if (w * 16 >= n) return;
  uint4 v[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) v[j] = src[(uint64_t)idx[w * 16 + j] * 64 + lane];
  uint32_t x = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) x ^= v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
  for (int o = 32; o > 0; o >>= 1) x ^= __shfl_xor(x, o);
  if (lane == 0) out[w] = x;
}

#define CK(x)                                                   \
  do {                                                          \
    hipError_t e_ = (x);                                        \
    if (e_ != hipSuccess) {                                     \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));   \
      return 1;                                                 \
    }                                                           \
  } while (0)

int main() {
  const uint32_t n = 65536, rows = 262144;  // 256 MiB of rows
  uint4 *src, *flush;
  uint32_t *idx, *out;
  CK(hipMalloc(&src, (size_t)rows * 1024));
  CK(hipMalloc(&flush, (size_t)rows * 1024));
  CK(hipMemset(src, 1, (size_t)rows * 1024));
  CK(hipMalloc(&idx, 4 * (size_t)n * 4));
  CK(hipMalloc(&out, (size_t)n * 4));
  std::vector<uint32_t> seq(n), perm(n), scat(n), mixed(n);
  std::iota(seq.begin(), seq.end(), 0u);
  perm = seq;
  std::mt19937 rng(7);
  std::shuffle(perm.begin(), perm.end(), rng);
  for (uint32_t i = 0; i < n; ++i) scat[i] = perm[i] * 4u;
  for (uint32_t i = 0; i < n; ++i) mixed[i] = i < n / 2 ? i : perm[i];
  const std::vector<uint32_t>* v[4] = {&seq, &perm, &scat, &mixed};
  for (int k = 0; k < 4; ++k) CK(hipMemcpy(idx + (size_t)k * n, v[k]->data(), n * 4, hipMemcpyHostToDevice));
  // 4 rounds of the four orders; a 256 MiB memset of another buffer between launches clears L2
  for (int r = 0; r < 4; ++r)
    for (int k = 0; k < 4; ++k) {
      CK(hipMemset(flush, r + k, (size_t)rows * 1024));
      hipLaunchKernelGGL(k_rows, dim3(n / 4), dim3(256), 0, 0, src, idx + (size_t)k * n, out, n);
      CK(hipGetLastError());
      CK(hipMemset(flush, r + k + 1, (size_t)rows * 1024));
      hipLaunchKernelGGL(k_rows16, dim3(n / 64), dim3(256), 0, 0, src, idx + (size_t)k * n, out, n);
      CK(hipGetLastError());
    }
  CK(hipDeviceSynchronize());
  printf("fetch_probe done: 16 launches (order seq, perm, scatter, mixed) x 4\n");
  return 0;
}
