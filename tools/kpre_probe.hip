// kpre_probe.hip — uncached kernarg reads (TCC_UC_REQ) with arguments passed
// by value (a 256-B struct read by every wave) against a device-memory struct
// behind one preloaded pointer (-mllvm -amdgpu-kernarg-preload-count=2).
// Build: hipcc -O3 --offload-arch=gfx950 -mllvm -amdgpu-kernarg-preload-count=2 -o tools/kpre_probe tools/kpre_probe.hip
// Test infrastructure only.
#include <hip/hip_runtime.h>

#include <cstdio>

struct Big {
  uint32_t w[64];
};

__global__ __launch_bounds__(256) void k_byval(Big a, uint32_t* out) {
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 64; ++i) x += a.w[i] * (threadIdx.x + i);
  if (x == 0x12345u) out[blockIdx.x] = x;
}

__global__ __launch_bounds__(256) void k_byptr(const Big* __restrict__ pa, uint32_t* out) {
  const Big& a = *pa;
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 64; ++i) x += a.w[i] * (threadIdx.x + i);
  if (x == 0x12345u) out[blockIdx.x] = x;
}

int main() {
  Big h{};
  for (int i = 0; i < 64; ++i) h.w[i] = i * 7 + 1;
  Big* d;
  uint32_t* out;
  if (hipMalloc(&d, sizeof(Big)) != hipSuccess || hipMalloc(&out, 1 << 20) != hipSuccess) return 1;
  (void)hipMemcpy(d, &h, sizeof(Big), hipMemcpyHostToDevice);
  for (int r = 0; r < 10; ++r) {
    hipLaunchKernelGGL(k_byval, dim3(4096), dim3(256), 0, 0, h, out);
    hipLaunchKernelGGL(k_byptr, dim3(4096), dim3(256), 0, 0, d, out);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("kpre_probe ok\n");
  return 0;
}
