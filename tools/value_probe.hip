// value_probe.hip — do rocprofv3 FETCH_SIZE / WRITE_SIZE depend on the VALUES
// a kernel moves (same addresses, same instructions)?  The obliviousness test
// (tests/test_oblivious.py) saw small systematic differences in kernels whose
// address stream is fixed (the bitonic merge steps) under mixes whose sort
// keys are regular (all-miss-read: keys already in order).
//
// k_cx: bitonic-style compare-exchange over 2^20 16-B keys (pairs i, i ^ 512),
// every key read and both written back unconditionally, as k_bitonic_global.
// Buffers are filled with: random words, an increasing sequence (already
// sorted), a constant, zero.  Each fill runs 4 times; FETCH/WRITE per launch.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/value_probe tools/value_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <algorithm>
#include <random>
#include <vector>

struct alignas(16) K {
  uint64_t hi, lo;
};

__global__ __launch_bounds__(256) void k_cx(K* keys, uint32_t n, uint32_t j) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  const uint32_t i = ((t & ~(j - 1)) << 1) | (t & (j - 1));  // lower element of a pair
  if (i + j >= n) return;
  const K a = keys[i], b = keys[i + j];
  const bool sw = a.hi > b.hi || (a.hi == b.hi && a.lo > b.lo);
  keys[i] = sw ? b : a;
  keys[i + j] = sw ? a : b;
}

#define CK(x)                                                 \
  do {                                                        \
    hipError_t e_ = (x);                                      \
    if (e_ != hipSuccess) {                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); \
      return 1;                                               \
    }                                                         \
  } while (0)

int main() {
  const uint32_t n = 1u << 20;
  K* d;
  uint8_t* flush;
  CK(hipMalloc(&d, (size_t)n * sizeof(K)));
  CK(hipMalloc(&flush, (size_t)512 << 20));
  std::vector<K> h(n);
  std::mt19937_64 rng(3);
  // random (half the pairs swap), random_sorted (random values, no swap),
  // regular_sorted (no swap), regular_reversed (every pair swaps), zero
  const char* names[5] = {"random", "random_sorted", "regular_sorted", "regular_reversed", "zero"};
  for (int r = 0; r < 4; ++r)
    for (int f = 0; f < 5; ++f) {
      for (uint32_t i = 0; i < n; ++i) {
        if (f == 0 || f == 1) h[i] = K{rng(), rng()};
        if (f == 2) h[i] = K{~0ull, (~0ull << 21) | ((uint64_t)i << 1)};
        if (f == 3) h[i] = K{~0ull, (~0ull << 21) | ((uint64_t)(n - 1 - i) << 1)};
        if (f == 4) h[i] = K{0, 0};
      }
      if (f == 1)
        std::sort(h.begin(), h.end(), [](const K& x, const K& y) { return x.hi < y.hi || (x.hi == y.hi && x.lo < y.lo); });
      CK(hipMemcpy(d, h.data(), (size_t)n * sizeof(K), hipMemcpyHostToDevice));
      CK(hipMemset(flush, r, (size_t)512 << 20));
      hipLaunchKernelGGL(k_cx, dim3(n / 2 / 256), dim3(256), 0, 0, d, n, 512u);
      CK(hipGetLastError());
      CK(hipDeviceSynchronize());
      printf("round %d fill %s\n", r, names[f]);
    }
  return 0;
}
