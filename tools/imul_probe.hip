// imul_probe.hip — issue rate of the integer multiplies a 2^255-19 field
// multiply can be built from, on gfx950 (not part of the product):
//   hipcc -O3 --offload-arch=gfx950 -o tools/imul_probe tools/imul_probe.hip
//   tools/imul_probe
// Each thread runs 8 independent chains of 4096 multiply steps; the grid puts
// W waves on every SIMD.  Reported: wave-instructions per cycle per SIMD.
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kSteps = 4096;

template <int K>
__global__ __launch_bounds__(256) void k_op(uint32_t* out, uint32_t seed) {
  uint32_t a[8];
  uint64_t c[8];
  for (int i = 0; i < 8; ++i) {
    a[i] = seed * (threadIdx.x + 3 * i + 1);
    c[i] = a[i];
  }
  const uint32_t b = seed | 1u;
  for (int s = 0; s < kSteps; ++s) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (K == 0) {  // v_mad_u64_u32
        c[i] = (uint64_t)a[i] * b + c[i];
        a[i] = (uint32_t)(c[i] >> 32);
      } else if (K == 1) {  // v_mul_lo_u32 + v_mul_hi_u32
        const uint32_t lo = a[i] * b, hi = __umulhi(a[i], b);
        a[i] = lo ^ hi;
      } else if (K == 2) {  // v_mul_u32_u24 + v_mul_hi_u32_u24
        const uint32_t x = a[i] & 0xFFFFFFu, y = b & 0xFFFFFFu;
        const uint32_t lo = x * y, hi = (uint32_t)(((uint64_t)x * y) >> 32);
        a[i] = lo ^ hi;
      } else if (K == 3) {  // fp64 fma
        double x = (double)a[i];
        x = __builtin_fma(x, 1.0000001, 3.0);
        a[i] = (uint32_t)(x);
      } else {  // v_add3_u32 baseline
        a[i] = a[i] + b + (a[i] >> 3);
      }
    }
  }
  uint32_t r = 0;
  for (int i = 0; i < 8; ++i) r ^= a[i] ^ (uint32_t)c[i];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

template <int K>
void run(const char* name, int waves_per_simd, uint32_t* d) {
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  const int blocks = p.multiProcessorCount * waves_per_simd;  // 4 waves per block = 1 per SIMD
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(k_op<K>, dim3(blocks), dim3(256), 0, 0, d, 7u);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(k_op<K>, dim3(blocks), dim3(256), 0, 0, d, 9u);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double cycles = ms * 1e-3 * p.clockRate * 1e3;
  const double insts = (double)kSteps * 8 * waves_per_simd;  // per SIMD, one "step" per chain
  printf("%-28s waves/SIMD=%d  %.3f ms  %.3f steps/cycle/SIMD (clock %.0f MHz)\n", name,
         waves_per_simd, ms, insts / cycles, p.clockRate / 1e3);
}

int main() {
  uint32_t* d;
  (void)hipMalloc(&d, 256u * 4096 * 16 * 4);
  for (int w : {1, 2, 4}) {
    run<0>("mad_u64_u32", w, d);
    run<1>("mul_lo + mul_hi u32", w, d);
    run<2>("mul_u24 + mulhi_u24", w, d);
    run<3>("fma_f64 (+cvt)", w, d);
    run<4>("add3 baseline", w, d);
  }
  (void)hipFree(d);
  return 0;
}
