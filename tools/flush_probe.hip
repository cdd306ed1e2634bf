// flush_probe.hip — what makes a kernel re-walk the page tables (TCC_UC_REQ
// bursts) between two identical launches?  One kernel reads a 1 GiB buffer
// (512 x 2 MiB pages), ITERS times, the host idle ~100 ms between launches:
//   MODE 0  idle only (sleep)
//   MODE 1  + malloc / memset / free of 70 MB host memory (a numpy batch array)
//   MODE 2  + hipHostMalloc / hipHostFree of 1 MiB (positive control: unmaps
//           GPU-visible memory)
//   MODE 3  + a pageable hipMemcpy of 70 MB host -> device (the old host path)
//   MODE 4  idle only, but 70 small launches per iteration (a batch's worth of
//           dispatch records for the profiler)
//   MODE 5  as 4, after 2000 small launches before the first iteration
//   MODE 6  as 4, + a 68 MB pinned host -> device and device -> host copy
//   MODE 7  as 4, + hipPointerGetAttributes of a pageable 68 MB array
//   MODE 8  as 4, + 8 host threads copying 68 MB pageable -> pinned
//   MODE 9  as 4, + the host -> device copy of mode 6 only
//   MODE 10 as 4, + the device -> host copy of mode 6 only
//   MODE 11 as 4, + both copies by a kernel reading / writing the pinned
//           buffer directly (no runtime copy)
//   MODE 12 as 11, the pinned buffer given its own memory policy (mbind
//           MPOL_LOCAL): automatic NUMA balancing then leaves its pages alone
//   MODE 13 as 11, after set_mempolicy(MPOL_LOCAL) for the process's thread
//   MODE 14 as 11, the pinned buffer madvise(MADV_NOHUGEPAGE): khugepaged
//           leaves it alone
//   MODE 15 as 11, the pinned buffer 2-MiB pages: mmap'd, madvise(MADV_HUGEPAGE),
//           touched, then hipHostRegister'd (34K 4-KiB host pages are 34K GPU
//           translations competing with the device buffer's 512)
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/flush_probe tools/flush_probe.hip
// Run:   rocprofv3 --pmc TCC_UC_REQ_sum TCC_EA0_RDREQ_sum -- tools/flush_probe MODE
// Test infrastructure only.
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

__global__ __launch_bounds__(256) void k_tiny(uint32_t* out, uint32_t it) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && it == 0xffffffffu) out[1] = it;
}

__global__ __launch_bounds__(256) void k_xcopy(const uint4* src, uint4* dst, uint64_t n16) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256)
    dst[i] = src[i];
}

__global__ __launch_bounds__(256) void k_read(const uint4* buf, uint64_t n16, uint32_t* out) {
  uint32_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) {
    const uint4 v = buf[i];
    acc ^= v.x ^ v.w;
  }
  if (acc == 0x9e3779b9u) out[0] = acc;  // practically never: keeps the loads
}

int main(int argc, char** argv) {
  const int mode = argc > 1 ? atoi(argv[1]) : 0;
  const int iters = argc > 2 ? atoi(argv[2]) : 60;
  const uint64_t bytes = 1ull << 30;
  uint4* buf;
  uint32_t* out;
  void* dstage;
  if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess ||
      hipMalloc(&dstage, 70u << 20) != hipSuccess)
    return 1;
  (void)hipMemset(buf, 1, bytes);
  void* pin = nullptr;
  char* pageable = (char*)malloc(68u << 20);
  memset(pageable, 3, 68u << 20);
  if (mode == 13) printf("set_mempolicy: %ld\n", syscall(SYS_set_mempolicy, 4 /* MPOL_LOCAL */, nullptr, 0));
  if (mode == 15) {
    const size_t sz = 68ul << 20, al = 2ul << 20;
    char* raw = (char*)mmap(nullptr, sz + al, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (raw == MAP_FAILED) return 7;
    pin = (void*)(((uintptr_t)raw + al - 1) & ~(uintptr_t)(al - 1));
    printf("madvise huge: %d\n", madvise(pin, sz, MADV_HUGEPAGE));
    memset(pin, 5, sz);
    if (hipHostRegister(pin, sz, hipHostRegisterDefault) != hipSuccess) return 8;
    FILE* f = fopen("/proc/self/smaps_rollup", "r");
    char line[256];
    while (f && fgets(line, sizeof line, f))
      if (strstr(line, "AnonHugePages")) printf("%s", line);
    if (f) fclose(f);
  } else if (mode >= 6 && hipHostMalloc(&pin, 68u << 20, hipHostMallocDefault) != hipSuccess) return 5;
  if (mode == 14) printf("madvise: %d\n", madvise(pin, 68ul << 20, MADV_NOHUGEPAGE));
  if (mode == 12) printf("mbind: %ld\n", syscall(SYS_mbind, pin, 68ul << 20, 4 /* MPOL_LOCAL */, nullptr, 0, 0));
  (void)hipDeviceSynchronize();
  if (mode == 5) {
    for (int j = 0; j < 2000; ++j) hipLaunchKernelGGL(k_tiny, dim3(64), dim3(256), 0, 0, out, (uint32_t)j);
    (void)hipDeviceSynchronize();
  }
  for (int it = 0; it < iters; ++it) {
    if (mode >= 4)
      for (int j = 0; j < 70; ++j) hipLaunchKernelGGL(k_tiny, dim3(64), dim3(256), 0, 0, out, (uint32_t)j);
    hipLaunchKernelGGL(k_read, dim3(4096), dim3(256), 0, 0, buf, bytes / 16, out);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    if (mode == 1) {
      char* p = (char*)malloc(70u << 20);
      memset(p, it, 70u << 20);
      free(p);
    } else if (mode == 2) {
      void* p;
      if (hipHostMalloc(&p, 1u << 20, hipHostMallocDefault) != hipSuccess) return 3;
      memset(p, it, 1u << 20);
      (void)hipHostFree(p);
    } else if (mode == 6) {
      if (hipMemcpyAsync(dstage, pin, 68u << 20, hipMemcpyHostToDevice, 0) != hipSuccess) return 6;
      if (hipMemcpyAsync(pin, dstage, 68u << 20, hipMemcpyDeviceToHost, 0) != hipSuccess) return 6;
      (void)hipDeviceSynchronize();
    } else if (mode == 9) {
      if (hipMemcpyAsync(dstage, pin, 68u << 20, hipMemcpyHostToDevice, 0) != hipSuccess) return 6;
      (void)hipDeviceSynchronize();
    } else if (mode == 10) {
      if (hipMemcpyAsync(pin, dstage, 68u << 20, hipMemcpyDeviceToHost, 0) != hipSuccess) return 6;
      (void)hipDeviceSynchronize();
    } else if (mode >= 11 && mode <= 15) {
      hipLaunchKernelGGL(k_xcopy, dim3(2048), dim3(256), 0, 0, (const uint4*)pin, (uint4*)dstage, (68ull << 20) / 16);
      hipLaunchKernelGGL(k_xcopy, dim3(2048), dim3(256), 0, 0, (const uint4*)dstage, (uint4*)pin, (68ull << 20) / 16);
      (void)hipDeviceSynchronize();
    } else if (mode == 7) {
      hipPointerAttribute_t at{};
      if (hipPointerGetAttributes(&at, pageable + it) != hipSuccess) (void)hipGetLastError();
    } else if (mode == 8) {
      std::vector<std::thread> th;
      const size_t chunk = (68u << 20) / 8;
      for (int k = 0; k < 8; ++k)
        th.emplace_back([=] { memcpy((char*)pin + k * chunk, pageable + k * chunk, chunk); });
      for (auto& t : th) t.join();
    } else if (mode == 3) {
      char* p = (char*)malloc(70u << 20);
      memset(p, it, 70u << 20);
      if (hipMemcpy(dstage, p, 70u << 20, hipMemcpyHostToDevice) != hipSuccess) return 4;
      free(p);
    }
    usleep(100000);
  }
  printf("flush_probe ok mode %d\n", mode);
  return 0;
}
