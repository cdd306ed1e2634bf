// ladder_probe.hip — does the schnorrkel ladder (gvs_sr25519.h
// double_scalar_mul + ristretto_encode) run faster at 2 waves per SIMD than
// at 1?  Not part of the product:
//   hipcc -O3 --offload-arch=gfx950 -o tools/ladder_probe tools/ladder_probe.hip
// The same kernel is launched over 64K threads with 0 B of dynamic LDS (its
// VGPR count allows 2 waves per SIMD) and with 40 KiB per 64-thread block
// (4 blocks, so 1 wave per SIMD, per CU).
#include "../grapevine_amd/csrc/gvs_sr25519.h"

#include <cstdio>
#include <vector>

using namespace gvs::sr;

__global__ void __launch_bounds__(64) k_ladder(const uint32_t* in, uint32_t* out) {
  extern __shared__ uint32_t pad[];
  const uint32_t t = blockIdx.x * 64 + threadIdx.x;
  Fe s, k;
  Pt A;
  for (int i = 0; i < 8; ++i) {
    s.v[i] = in[t * 48 + i] & 0x0FFFFFFFu;
    k.v[i] = in[t * 48 + 8 + i] & 0x0FFFFFFFu;
    A.X.v[i] = in[t * 48 + 16 + i];
    A.Y.v[i] = in[t * 48 + 24 + i];
    A.Z.v[i] = in[t * 48 + 32 + i];
    A.T.v[i] = in[t * 48 + 40 + i];
  }
  const Fe e = ristretto_encode(double_scalar_mul(s, k, A));
  for (int i = 0; i < 8; ++i) out[t * 8 + i] = e.v[i];
  if (t == 0xFFFFFFFFu) pad[0] = 0;  // keeps the dynamic LDS declared
}

#define CK(x)                                                      \
  do {                                                             \
    hipError_t err_ = (x);                                         \
    if (err_ != hipSuccess) {                                      \
      std::printf("%s: %s\n", #x, hipGetErrorString(err_));        \
      return 1;                                                    \
    }                                                              \
  } while (0)

int main() {
  const uint32_t n = 65536;
  std::vector<uint32_t> h(n * 48);
  uint32_t x = 12345;
  for (auto& v : h) v = (x = x * 1664525u + 1013904223u);
  uint32_t *din, *dout;
  CK(hipMalloc(&din, h.size() * 4));
  CK(hipMalloc(&dout, n * 32));
  CK(hipMemcpy(din, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int rep = 0; rep < 2; ++rep)
    for (uint32_t lds : {0u, 40960u}) {
      hipLaunchKernelGGL(k_ladder, dim3(n / 64), dim3(64), lds, 0, din, dout);
      CK(hipEventRecord(a));
      for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k_ladder, dim3(n / 64), dim3(64), lds, 0, din, dout);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      std::printf("dyn LDS %6u B per block: %.3f ms per 64K ladders+encodes\n", lds, ms / 3);
    }
  return 0;
}
