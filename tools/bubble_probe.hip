// bubble_probe.hip — what makes a 128-B memory read count twice in FETCH_SIZE
// (TCC_BUBBLE: FETCH_SIZE = (BUBBLE*128 + (RDREQ - BUBBLE - RDREQ_32B)*64 +
// RDREQ_32B*32) / 1024 on gfx950)?  One workgroup of 4 waves per 256-row
// partition streams its rows (1 KiB each, NT loads, U rows per chunk) and
// reads 16 extra 1-KiB "slot" lines of its own, either
//   MODE 0: all after the stream (the k_rpass2 tail loop shape),
//   MODE 1: one inside every 4th chunk of wave 0 (in-stream),
//   MODE 2: plain (not NT) slot loads after the stream,
//   MODE 3: no slot lines (stream only),
//   MODE 4: slot lines before the stream (prologue).
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/bubble_probe tools/bubble_probe.hip
// Test infrastructure only.
#include <hip/hip_runtime.h>

#include <cstdio>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
__device__ inline uint4 ldnt(const uint4* p) {
  const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ inline void stnt(uint4* p, uint4 x) {
  v4u v = {x.x, x.y, x.z, x.w};
  __builtin_nontemporal_store(v, reinterpret_cast<v4u*>(p));
}

template <int MODE>
__global__ __launch_bounds__(256) void k_pass(uint4* table, const uint4* slots, uint32_t* out) {
  constexpr int U = 16, ROWS = 256, NS = 16;
  const uint32_t w = blockIdx.x, wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  uint4* part = table + (uint64_t)w * ROWS * 64;
  const uint4* sl = slots + (uint64_t)w * NS * 64;
  uint32_t acc = 0;
  if (MODE == 4)
    for (uint32_t k = wave; k < NS; k += 4) {
      const uint4 x = ldnt(&sl[k * 64 + lane]);
      acc ^= x.x ^ x.w;
    }
  uint32_t ns = 0;
  for (uint32_t j = wave * U; j < ROWS; j += 4 * U) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ldnt(&part[(uint64_t)(j + u) * 64 + lane]);
    if (MODE == 1 && ns < NS) {  // 16 chunks per workgroup carry a slot each
      const uint4 x = ldnt(&sl[ns * 64 + lane]);
      v[0].x ^= x.x & 0u;
      acc ^= x.y;
      ++ns;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) stnt(&part[(uint64_t)(j + u) * 64 + lane], v[u]);
  }
  if (MODE == 1)
    for (uint32_t k = ns + wave * 0; k < 0; ++k) acc ^= k;
  if (MODE == 0 || MODE == 2)
    for (uint32_t k = wave; k < NS; k += 4) {
      const uint4 x = MODE == 0 ? ldnt(&sl[k * 64 + lane]) : sl[k * 64 + lane];
      acc ^= x.x ^ x.w;
    }
  if (acc == 0x9e3779b9u) out[w] = acc;
}

int main() {
  const uint32_t W = 4096;  // 4096 partitions x 256 rows = 1 GiB table, 64 MiB of slots
  uint4 *table, *slots;
  uint32_t* out;
  if (hipMalloc(&table, (uint64_t)W * 256 * 1024) != hipSuccess ||
      hipMalloc(&slots, (uint64_t)W * 16 * 1024) != hipSuccess || hipMalloc(&out, W * 4) != hipSuccess)
    return 1;
  (void)hipMemset(table, 1, (uint64_t)W * 256 * 1024);
  (void)hipMemset(slots, 2, (uint64_t)W * 16 * 1024);
  for (int r = 0; r < 4; ++r) {
    hipLaunchKernelGGL(k_pass<0>, dim3(W), dim3(256), 0, 0, table, slots, out);
    hipLaunchKernelGGL(k_pass<1>, dim3(W), dim3(256), 0, 0, table, slots, out);
    hipLaunchKernelGGL(k_pass<2>, dim3(W), dim3(256), 0, 0, table, slots, out);
    hipLaunchKernelGGL(k_pass<3>, dim3(W), dim3(256), 0, 0, table, slots, out);
    hipLaunchKernelGGL(k_pass<4>, dim3(W), dim3(256), 0, 0, table, slots, out);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("bubble_probe ok\n");
  return 0;
}
