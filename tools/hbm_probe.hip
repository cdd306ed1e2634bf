// hbm_probe.hip — ceiling of in-place read+write streaming on MI355X for the
// message-table pass's access shape (1 KiB rows, 16 B per lane, every row read
// and written back once).  Not part of the product; run on the GPU box:
//   hipcc -O3 --offload-arch=gfx950 -o tools/hbm_probe tools/hbm_probe.hip
//   tools/hbm_probe [GiB]      (the pass shapes on one buffer)
//   tools/hbm_probe sweep      (read-only and copy rates against buffer size)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <algorithm>
#include <cstdlib>
#include <string>
#include <vector>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ inline v4u ld(const v4u* p) {
  if (NT) return __builtin_nontemporal_load(p);
  return *p;
}
template <bool NT>
__device__ inline void st(v4u* p, v4u v) {
  if (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// grid-stride in place: each thread 16 B per iteration
template <bool NT>
__global__ __launch_bounds__(256) void k_gs(v4u* a, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    v4u v = ld<NT>(a + i);
    v.x ^= 1u;
    st<NT>(a + i, v);
  }
}

// rpass shape: one workgroup per partition of `rows` rows; each wave streams
// chunks of U rows (loads, then stores), 64 rows per wave per 256-row tile
template <int U, bool NT, int MINW>
__global__ __launch_bounds__(256, MINW) void k_part(v4u* a, uint32_t rows) {
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  v4u* part = a + (size_t)blockIdx.x * rows * 64;
  for (uint32_t t = 0; t < rows / 256; ++t) {
    const uint32_t rb = t * 256 + wave * 64;
    for (uint32_t j = 0; j < 64; j += U) {
      v4u v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = ld<NT>(&part[(size_t)(rb + j + u) * 64 + lane]);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        v[u].x ^= 1u;
        st<NT>(&part[(size_t)(rb + j + u) * 64 + lane], v[u]);
      }
    }
    __syncthreads();
  }
}

// same, software-pipelined: next chunk's loads issued before this chunk's stores
template <int U, bool NT, int MINW>
__global__ __launch_bounds__(256, MINW) void k_pipe(v4u* a, uint32_t rows) {
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  v4u* part = a + (size_t)blockIdx.x * rows * 64;
  const uint32_t per_wave = rows / 4;  // contiguous rows per wave
  v4u* w = part + (size_t)wave * per_wave * 64;
  v4u cur[U], nxt[U];
#pragma unroll
  for (int u = 0; u < U; ++u) cur[u] = ld<NT>(&w[(size_t)u * 64 + lane]);
  for (uint32_t j = 0; j < per_wave; j += U) {
    if (j + U < per_wave) {
#pragma unroll
      for (int u = 0; u < U; ++u) nxt[u] = ld<NT>(&w[(size_t)(j + U + u) * 64 + lane]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      cur[u].x ^= 1u;
      st<NT>(&w[(size_t)(j + u) * 64 + lane], cur[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) cur[u] = nxt[u];
  }
}

// k_pipe with a per-workgroup start: workgroup b begins its waves' streams at
// chunk (b * STAG) mod chunks and wraps, so that at any moment the grid's
// accesses are not all at one offset of equal, power-of-two-strided partitions
template <int U, int STAG, int MINW>
__global__ __launch_bounds__(256, MINW) void k_pipe_stag(v4u* a, uint32_t rows) {
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  v4u* part = a + (size_t)blockIdx.x * rows * 64;
  const uint32_t per_wave = rows / 4, chunks = per_wave / U;
  v4u* w = part + (size_t)wave * per_wave * 64;
  const uint32_t c0 = (blockIdx.x * STAG) % chunks;
  v4u cur[U], nxt[U];
#pragma unroll
  for (int u = 0; u < U; ++u) cur[u] = ld<true>(&w[(size_t)(c0 * U + u) * 64 + lane]);
  for (uint32_t i = 0; i < chunks; ++i) {
    const uint32_t c = (c0 + i) % chunks, cn = (c + 1) % chunks;
    if (i + 1 < chunks) {
#pragma unroll
      for (int u = 0; u < U; ++u) nxt[u] = ld<true>(&w[(size_t)(cn * U + u) * 64 + lane]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      cur[u].x ^= 1u;
      st<true>(&w[(size_t)(c * U + u) * 64 + lane], cur[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) cur[u] = nxt[u];
  }
}

// k_part with block-interleaved partitions: partition w's local row k lives
// at physical row ((k / G) * W + w) * G + k % G, so that the workgroups in
// flight together sweep a compact window of the table (grid-stride-like DRAM
// locality) while each still owns a fixed set of rows
template <int U, int G, int MINW>
__global__ __launch_bounds__(256, MINW) void k_ipart(v4u* a, uint32_t rows) {
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t W = gridDim.x, w = blockIdx.x;
  for (uint32_t t = 0; t < rows / 256; ++t) {
    const uint32_t rb = t * 256 + wave * 64;
    for (uint32_t j = 0; j < 64; j += U) {
      v4u v[U];
      uint64_t pr[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint64_t k = rb + j + u;
        pr[u] = ((k / G) * W + w) * G + k % G;
        v[u] = ld<true>(&a[pr[u] * 64 + lane]);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        v[u].x ^= 1u;
        st<true>(&a[pr[u] * 64 + lane], v[u]);
      }
    }
    __syncthreads();
  }
}

// grid-stride with U independent 16-B accesses in flight per thread: thread t
// of block b handles elements (b * U + u) * 256 + t, then jumps the grid
template <int U, bool NT, bool COPY>
__global__ __launch_bounds__(256) void k_wide(const v4u* s, v4u* d, size_t n) {
  const size_t step = (size_t)gridDim.x * U * 256;
  for (size_t base = (size_t)blockIdx.x * U * 256 + threadIdx.x; base < n; base += step) {
    v4u v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = base + u * 256 < n ? ld<NT>(s + base + u * 256) : v4u{0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!COPY) v[u].x ^= 1u;
      if (base + u * 256 < n) st<NT>(d + base + u * 256, v[u]);
    }
  }
}

// read only: U independent 16-B loads per thread per step, XOR-folded into one
// word per thread (stored once, so the loads are not dead)
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_read(const v4u* s, uint32_t* out, size_t n) {
  const size_t step = (size_t)gridDim.x * U * 256;
  uint32_t acc = 0;
  for (size_t base = (size_t)blockIdx.x * U * 256 + threadIdx.x; base < n; base += step) {
    v4u v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = base + u * 256 < n ? ld<NT>(s + base + u * 256) : v4u{0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

// out-of-place copy, grid-stride
template <bool NT>
__global__ __launch_bounds__(256) void k_copy(const v4u* s, v4u* d, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    st<NT>(d + i, ld<NT>(s + i));
}

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e = (x);                                                \
    if (e != hipSuccess) {                                             \
      std::printf("%s: %s\n", #x, hipGetErrorString(e));               \
      std::exit(1);                                                    \
    }                                                                  \
  } while (0)

template <typename F>
static void timeit(const char* name, double bytes, F launch) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  launch();
  CK(hipDeviceSynchronize());
  std::vector<float> ts;
  for (int r = 0; r < 7; ++r) {
    CK(hipEventRecord(a));
    launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    ts.push_back(ms);
  }
  std::sort(ts.begin(), ts.end());
  std::printf("%-34s %8.3f ms  %7.0f GB/s (min %.3f)\n", name, ts[3], bytes / ts[3] / 1e6,
              ts[0]);
  std::fflush(stdout);
}

// `hbm_probe sweep`: read-only and copy rates against the buffer size, to
// place the 16-GiB figures beside the guide's (float4 copy, smaller buffers)
static int sweep() {
  const size_t maxb = 16ull << 30;
  v4u* a;
  uint32_t* o;
  CK(hipMalloc(&a, maxb));
  CK(hipMalloc(&o, 8192 * 256 * 4));
  CK(hipMemset(a, 1, maxb));
  for (double gib : {0.125, 0.5, 1.0, 4.0, 16.0}) {
    const size_t bytes = (size_t)(gib * (1ull << 30)), n = bytes / 16, h = n / 2;
    char nm[64];
    for (int g : {2048, 8192}) {
      std::snprintf(nm, sizeof nm, "%.3g GiB read U8 nt grid=%d", gib, g);
      timeit(nm, (double)bytes, [&] { hipLaunchKernelGGL((k_read<8, true>), dim3(g), dim3(256), 0, 0, a, o, n); });
      std::snprintf(nm, sizeof nm, "%.3g GiB read U8 plain grid=%d", gib, g);
      timeit(nm, (double)bytes, [&] { hipLaunchKernelGGL((k_read<8, false>), dim3(g), dim3(256), 0, 0, a, o, n); });
    }
    std::snprintf(nm, sizeof nm, "%.3g GiB copy float4 plain grid=4096", gib);
    timeit(nm, 2.0 * h * 16, [&] { hipLaunchKernelGGL(k_copy<false>, dim3(4096), dim3(256), 0, 0, a, a + h, h); });
    std::snprintf(nm, sizeof nm, "%.3g GiB copy U8 nt grid=8192", gib);
    timeit(nm, 2.0 * h * 16, [&] { hipLaunchKernelGGL((k_wide<8, true, true>), dim3(8192), dim3(256), 0, 0, a, a + h, h); });
    std::snprintf(nm, sizeof nm, "%.3g GiB inplace U8 nt grid=8192", gib);
    timeit(nm, 2.0 * bytes, [&] { hipLaunchKernelGGL((k_wide<8, true, false>), dim3(8192), dim3(256), 0, 0, a, a, n); });
  }
  CK(hipFree(a));
  CK(hipFree(o));
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 1 && std::string(argv[1]) == "sweep") return sweep();
  const double gib = argc > 1 ? std::atof(argv[1]) : 16.0;
  const size_t bytes = (size_t)(gib * (1ull << 30));
  const size_t n = bytes / 16;
  v4u* a;
  CK(hipMalloc(&a, bytes));
  CK(hipMemset(a, 1, bytes));
  const double rw = 2.0 * bytes;
  const uint32_t rows_total = (uint32_t)(bytes / 1024);
  for (int g : {1024, 2048, 4096, 8192}) {
    char nm[64];
    std::snprintf(nm, sizeof nm, "gs nt grid=%d", g);
    timeit(nm, rw, [&] { hipLaunchKernelGGL(k_gs<true>, dim3(g), dim3(256), 0, 0, a, n); });
  }
  timeit("gs plain grid=4096", rw, [&] { hipLaunchKernelGGL(k_gs<false>, dim3(4096), dim3(256), 0, 0, a, n); });
  for (uint32_t rows : {1024u, 4096u}) {
    const uint32_t nb = rows_total / rows;
    char nm[64];
    std::snprintf(nm, sizeof nm, "part U16 nt rows=%u", rows);
    timeit(nm, rw, [&] { hipLaunchKernelGGL((k_part<16, true, 2>), dim3(nb), dim3(256), 0, 0, a, rows); });
    std::snprintf(nm, sizeof nm, "part U8 nt w4 rows=%u", rows);
    timeit(nm, rw, [&] { hipLaunchKernelGGL((k_part<8, true, 4>), dim3(nb), dim3(256), 0, 0, a, rows); });
    std::snprintf(nm, sizeof nm, "part U16 plain rows=%u", rows);
    timeit(nm, rw, [&] { hipLaunchKernelGGL((k_part<16, false, 2>), dim3(nb), dim3(256), 0, 0, a, rows); });
    std::snprintf(nm, sizeof nm, "pipe U8 nt rows=%u", rows);
    timeit(nm, rw, [&] { hipLaunchKernelGGL((k_pipe<8, true, 2>), dim3(nb), dim3(256), 0, 0, a, rows); });
    std::snprintf(nm, sizeof nm, "pipe U4 nt w4 rows=%u", rows);
    timeit(nm, rw, [&] { hipLaunchKernelGGL((k_pipe<4, true, 4>), dim3(nb), dim3(256), 0, 0, a, rows); });
    std::snprintf(nm, sizeof nm, "pipe U16 nt w1 rows=%u", rows);
    timeit(nm, rw, [&] { hipLaunchKernelGGL((k_pipe<16, true, 1>), dim3(nb), dim3(256), 0, 0, a, rows); });
    std::snprintf(nm, sizeof nm, "ipart U16 G16 nt rows=%u", rows);
    timeit(nm, rw, [&] { hipLaunchKernelGGL((k_ipart<16, 16, 2>), dim3(nb), dim3(256), 0, 0, a, rows); });
    std::snprintf(nm, sizeof nm, "ipart U16 G64 nt rows=%u", rows);
    timeit(nm, rw, [&] { hipLaunchKernelGGL((k_ipart<16, 64, 2>), dim3(nb), dim3(256), 0, 0, a, rows); });
    std::snprintf(nm, sizeof nm, "ipart U16 G256 nt rows=%u", rows);
    timeit(nm, rw, [&] { hipLaunchKernelGGL((k_ipart<16, 256, 2>), dim3(nb), dim3(256), 0, 0, a, rows); });
    std::snprintf(nm, sizeof nm, "ipart U16 G1 nt rows=%u", rows);
    timeit(nm, rw, [&] { hipLaunchKernelGGL((k_ipart<16, 1, 2>), dim3(nb), dim3(256), 0, 0, a, rows); });
    std::snprintf(nm, sizeof nm, "pipe U8 nt stag1 rows=%u", rows);
    timeit(nm, rw, [&] { hipLaunchKernelGGL((k_pipe_stag<8, 1, 2>), dim3(nb), dim3(256), 0, 0, a, rows); });
    std::snprintf(nm, sizeof nm, "pipe U8 nt stag7 rows=%u", rows);
    timeit(nm, rw, [&] { hipLaunchKernelGGL((k_pipe_stag<8, 7, 2>), dim3(nb), dim3(256), 0, 0, a, rows); });
    std::snprintf(nm, sizeof nm, "pipe U8 nt stag0 rows=%u", rows);
    timeit(nm, rw, [&] { hipLaunchKernelGGL((k_pipe_stag<8, 0, 2>), dim3(nb), dim3(256), 0, 0, a, rows); });
  }
  // copy between two halves
  const size_t h = n / 2;
  for (int g : {2048, 4096, 8192}) {
    char nm[64];
    std::snprintf(nm, sizeof nm, "wide copy U4 nt grid=%d", g);
    timeit(nm, 2.0 * h * 16, [&] { hipLaunchKernelGGL((k_wide<4, true, true>), dim3(g), dim3(256), 0, 0, a, a + h, h); });
    std::snprintf(nm, sizeof nm, "wide copy U8 plain grid=%d", g);
    timeit(nm, 2.0 * h * 16, [&] { hipLaunchKernelGGL((k_wide<8, false, true>), dim3(g), dim3(256), 0, 0, a, a + h, h); });
    std::snprintf(nm, sizeof nm, "wide copy U8 nt grid=%d", g);
    timeit(nm, 2.0 * h * 16, [&] { hipLaunchKernelGGL((k_wide<8, true, true>), dim3(g), dim3(256), 0, 0, a, a + h, h); });
    std::snprintf(nm, sizeof nm, "wide inplace U8 nt grid=%d", g);
    timeit(nm, rw, [&] { hipLaunchKernelGGL((k_wide<8, true, false>), dim3(g), dim3(256), 0, 0, a, a, n); });
    std::snprintf(nm, sizeof nm, "wide inplace U8 plain grid=%d", g);
    timeit(nm, rw, [&] { hipLaunchKernelGGL((k_wide<8, false, false>), dim3(g), dim3(256), 0, 0, a, a, n); });
  }
  timeit("copy nt half->half grid=4096", 2.0 * h * 16, [&] {
    hipLaunchKernelGGL(k_copy<true>, dim3(4096), dim3(256), 0, 0, a, a + h, h);
  });
  timeit("copy plain half->half grid=4096", 2.0 * h * 16, [&] {
    hipLaunchKernelGGL(k_copy<false>, dim3(4096), dim3(256), 0, 0, a, a + h, h);
  });
  CK(hipFree(a));
  return 0;
}
