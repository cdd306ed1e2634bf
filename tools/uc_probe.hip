// uc_probe.hip — L2 residency rules that the obliviousness contract rests on
// (DESIGN.md §3 rule 3).  Which accesses leave a line in an XCD's L2, and does
// it survive a non-temporal stream of the whole table?
//
// Each case: flush (write a 512 MiB buffer), PRODUCER kernel on a 16 MiB
// region (16384 rows of 1 KiB, one wave per row, 16 B per lane), optionally a
// 2 GiB non-temporal read stream, then the CONSUMER: plain loads of the region
// with the producer's exact workgroup -> row mapping (same XCD per row).
// rocprofv3 FETCH_SIZE / TCC_HIT of the consumer tell whether the lines were
// still in L2.  Producers: plain load, nt load, sc1 store, plain store, nt
// store, and "none" (flush only).
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/uc_probe tools/uc_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

__device__ inline void st_sc1(const void* base, uint32_t i, uint4 x) {
  const v4u v = {x.x, x.y, x.z, x.w};
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, -1, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(v, r, i * 16u, 0, 16 /* sc1 */);
}

// MODE 0 plain load, 1 nt load, 2 sc1 store, 3 plain store, 4 nt store, 5 nothing
template <int MODE>
__global__ __launch_bounds__(256) void k_prod(uint4* buf, uint32_t* out) {
  const uint32_t row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
  uint4* p = buf + (uint64_t)row * 64 + lane;
  uint32_t x = 0;
  if (MODE == 0) {
    const uint4 v = *p;
    x = v.x ^ v.y ^ v.z ^ v.w;
  } else if (MODE == 1) {
    const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
    x = v.x ^ v.y ^ v.z ^ v.w;
  } else if (MODE == 2) {
    st_sc1(buf, row * 64 + lane, make_uint4(row, lane, 1, 2));
  } else if (MODE == 3) {
    *p = make_uint4(row, lane, 3, 4);
  } else if (MODE == 4) {
    const v4u v = {row, lane, 5, 6};
    __builtin_nontemporal_store(v, reinterpret_cast<v4u*>(p));
  }
  if (x == 0x12345678u) out[row] = x;
}

__global__ __launch_bounds__(256) void k_cons(const uint4* buf, uint32_t* out) {
  const uint32_t row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
  const uint4 v = buf[(uint64_t)row * 64 + lane];
  uint32_t x = v.x ^ v.y ^ v.z ^ v.w;
  for (int o = 32; o > 0; o >>= 1) x ^= __shfl_xor(x, o);
  if (lane == 0) out[row] = x;
}

// grid-stride non-temporal read of a big buffer
__global__ __launch_bounds__(256) void k_stream(const uint4* big, uint64_t n16, uint32_t* out) {
  uint32_t x = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) {
    const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(big + i));
    x ^= v.x;
  }
  if (x == 0x12345678u) out[0] = x;
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
  const uint32_t rows = 16384;  // 16 MiB region
  const size_t big_bytes = (size_t)2 << 30;
  uint4 *region, *flush, *big;
  uint32_t* out;
  CK(hipMalloc(&region, (size_t)rows * 1024));
  CK(hipMalloc(&flush, (size_t)512 << 20));
  CK(hipMalloc(&big, big_bytes));
  CK(hipMalloc(&out, (size_t)rows * 4));
  CK(hipMemset(region, 1, (size_t)rows * 1024));
  CK(hipMemset(big, 2, big_bytes));
  const char* names[6] = {"plain_load", "nt_load", "sc1_store", "plain_store", "nt_store", "none"};
  // dispatch order per case: k_prod, [k_stream], k_cons
  for (int r = 0; r < 2; ++r)
    for (int st = 0; st < 2; ++st)
      for (int m = 0; m < 6; ++m) {
        CK(hipMemset(flush, r + m, (size_t)512 << 20));
        dim3 g(rows / 4), b(256);
        switch (m) {
          case 0: hipLaunchKernelGGL(k_prod<0>, g, b, 0, 0, region, out); break;
          case 1: hipLaunchKernelGGL(k_prod<1>, g, b, 0, 0, region, out); break;
          case 2: hipLaunchKernelGGL(k_prod<2>, g, b, 0, 0, region, out); break;
          case 3: hipLaunchKernelGGL(k_prod<3>, g, b, 0, 0, region, out); break;
          case 4: hipLaunchKernelGGL(k_prod<4>, g, b, 0, 0, region, out); break;
          default: hipLaunchKernelGGL(k_prod<5>, g, b, 0, 0, region, out); break;
        }
        if (st) hipLaunchKernelGGL(k_stream, dim3(4096), dim3(256), 0, 0, big, big_bytes / 16, out);
        hipLaunchKernelGGL(k_cons, g, b, 0, 0, region, out);
        hipLaunchKernelGGL(k_cons, g, b, 0, 0, region, out);  // back to back: residency across a boundary
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        printf("case round=%d stream=%d producer=%s\n", r, st, names[m]);
      }
  return 0;
}
