// uc_time_probe.hip — is the uncached L2 traffic (TCC_UC_REQ) seen inside the
// engine's kernels their own?  A kernel that touches no memory but one store
// spins for T microseconds; rocprofv3 counts TCC_UC_REQ / TCC_EA0_RDREQ_64B in
// its window.  Counts that grow with T are traffic of other agents during the
// kernel (DESIGN.md §3 "Counters").  Test infrastructure only.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/uc_time_probe tools/uc_time_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ __launch_bounds__(64) void k_spin(uint64_t ticks, uint32_t* out) {
  const uint64_t t0 = wall_clock64();  // 100 MHz constant clock
  uint32_t n = 0;
  while (wall_clock64() - t0 < ticks) {
    __builtin_amdgcn_s_sleep(8);
    ++n;
  }
  if (threadIdx.x == 0 && n == 0xFFFFFFFFu) out[blockIdx.x] = n;
}

int main() {
  uint32_t* out;
  if (hipMalloc(&out, 1 << 16) != hipSuccess) return 1;
  const uint64_t us[] = {10, 30, 100, 300, 1000, 3000};
  for (int r = 0; r < 5; ++r)
    for (uint64_t u : us) hipLaunchKernelGGL(k_spin, dim3(256), dim3(64), 0, 0, u * 100, out);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("uc_time_probe ok\n");
  return 0;
}
