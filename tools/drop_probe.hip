// drop_probe.hip — do sc1 stores (buffer_store ... sc1) leave the line out
// of L2?  Kernel w_* writes 16 MiB of rows with one policy, kernel r reads
// them back at once; the reader's TCC_HIT tells how many lines stayed.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/drop_probe tools/drop_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef unsigned int u4v __attribute__((ext_vector_type(4)));

__global__ void w_plain(uint4* p) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  p[i] = make_uint4((uint32_t)i, 1, 2, 3);
}
__global__ void w_nt(uint4* p) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  u4v v = {(uint32_t)i, 1, 2, 3};
  __builtin_nontemporal_store(v, reinterpret_cast<u4v*>(p + i));
}
__global__ void w_sc1(uint4* p) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  u4v v = {(uint32_t)i, 1, 2, 3};
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(p, (short)0, -1, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(v, r, (uint32_t)(i * 16), 0, 16);
}
__global__ void r_all(const uint4* p, uint32_t* out) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint4 v = p[i];
  if ((v.x ^ v.y) == 0xdeadbeef) out[0] = 1;
}

int main() {
  const size_t n = (16u << 20) / 16;  // 16 MiB of uint4
  uint4* p;
  uint32_t* out;
  if (hipMalloc(&p, n * 16) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) return 1;
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(w_plain, dim3(n / 256), dim3(256), 0, 0, p);
    hipLaunchKernelGGL(r_all, dim3(n / 256), dim3(256), 0, 0, p, out);
    hipLaunchKernelGGL(w_nt, dim3(n / 256), dim3(256), 0, 0, p);
    hipLaunchKernelGGL(r_all, dim3(n / 256), dim3(256), 0, 0, p, out);
    hipLaunchKernelGGL(w_sc1, dim3(n / 256), dim3(256), 0, 0, p);
    hipLaunchKernelGGL(r_all, dim3(n / 256), dim3(256), 0, 0, p, out);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  printf("drop_probe done\n");
  return 0;
}
