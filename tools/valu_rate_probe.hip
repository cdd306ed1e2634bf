// valu_rate_probe.hip — issue rate of the vector instructions the sealed
// passes are made of (BLAKE2b: 64-bit adds, XOR, rotates; AES: v_perm_b32
// addresses, LDS table reads, v_bitop3 / v_alignbit combines), on gfx950 (not
// part of the product):
//   hipcc -O3 --offload-arch=gfx950 -o tools/valu_rate_probe tools/valu_rate_probe.hip
//   tools/valu_rate_probe
// Each thread runs 8 independent chains of kSteps steps (inline asm, so the
// instruction is exactly the one named); the grid puts W waves on every SIMD.
// Reported: wave-instructions per cycle per SIMD (1 = one every cycle).
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kSteps = 32768;  // long enough that launch and setup (~7 us) do not matter

template <int K>
__global__ __launch_bounds__(1024) void k_op(uint32_t* out, uint32_t seed) {
  __shared__ uint32_t s_t[16384];
  for (uint32_t i = threadIdx.x; i < 16384; i += blockDim.x) s_t[i] = i * 2654435761u;
  __syncthreads();
  uint32_t a[8];
  uint64_t c[8];
  for (int i = 0; i < 8; ++i) {
    a[i] = seed * (threadIdx.x + 3 * i + 1);
    c[i] = ((uint64_t)a[i] << 32) | (a[i] ^ 0x5bd1e995u);
  }
  const uint32_t b = seed | 1u, lane4 = (threadIdx.x & 31u) * 4u;
  const uint64_t d = ((uint64_t)b << 32) | 0x9e3779b9u;
  for (int s = 0; s < kSteps; ++s) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (K == 0) {
        asm volatile("v_lshl_add_u64 %0, %1, 0, %2" : "=v"(c[i]) : "v"(c[i]), "v"(d));
      } else if (K == 1) {
        uint32_t lo = (uint32_t)c[i], hi = (uint32_t)(c[i] >> 32);
        asm volatile("v_add_co_u32 %0, vcc, %0, %2\n\tv_addc_co_u32 %1, vcc, %1, %3, vcc"
                     : "+v"(lo), "+v"(hi) : "v"((uint32_t)d), "v"((uint32_t)(d >> 32)) : "vcc");
        c[i] = ((uint64_t)hi << 32) | lo;
      } else if (K == 2) {
        asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "s"(0x0c0c0501u));
      } else if (K == 3) {
        asm volatile("v_alignbit_b32 %0, %0, %0, 8" : "+v"(a[i]));
      } else if (K == 4) {
        asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a[i]) : "v"(b), "v"(lane4));
      } else if (K == 5) {
        asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
      } else if (K == 6) {  // table read: address from the previous value, conflict-free
        const uint32_t addr = ((a[i] & 0xffu) << 8) | lane4;
        a[i] = s_t[addr >> 2] ^ b;
      } else if (K == 8) {  // the same XOR in the 8-byte VOP3 encoding
        asm volatile("v_xor_b32_e64 %0, %0, %1" : "+v"(a[i]) : "v"(b));
      } else if (K == 9) {  // v_add_u32 (VOP2)
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
      } else if (K == 7) {  // v_xor_b32 pair (64-bit XOR) + 2 v_alignbit (64-bit rotate by 24)
        uint32_t lo = (uint32_t)c[i], hi = (uint32_t)(c[i] >> 32);
        asm volatile("v_xor_b32 %0, %0, %2\n\tv_xor_b32 %1, %1, %3\n\t"
                     "v_alignbit_b32 %0, %1, %0, 24\n\tv_alignbit_b32 %1, %0, %1, 24"
                     : "+v"(lo), "+v"(hi) : "v"((uint32_t)d), "v"((uint32_t)(d >> 32)));
        c[i] = ((uint64_t)hi << 32) | lo;
      }
    }
  }
  uint32_t r = 0;
  for (int i = 0; i < 8; ++i) r ^= a[i] ^ (uint32_t)c[i] ^ (uint32_t)(c[i] >> 32);
  out[blockIdx.x * 1024 + threadIdx.x] = r;
}

template <int K>
void run(const char* name, int ipc, int waves_per_simd, uint32_t* d) {
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  // one workgroup of 4 * W waves per CU: W waves on every SIMD
  const int blocks = p.multiProcessorCount;
  const int threads = 256 * waves_per_simd;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(k_op<K>, dim3(blocks), dim3(threads), 0, 0, d, 7u);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(k_op<K>, dim3(blocks), dim3(threads), 0, 0, d, 9u);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double cycles = ms * 1e-3 * p.clockRate * 1e3;
  const double insts = (double)kSteps * 8 * ipc * waves_per_simd;  // per SIMD
  printf("%-34s waves/SIMD=%d  %.3f ms  %.3f wave-instr/cycle/SIMD\n", name, waves_per_simd, ms, insts / cycles);
}

int main() {
  uint32_t* d;
  (void)hipMalloc(&d, 1024u * 4096 * 4);
  for (int w : {1, 2, 3, 4}) {
    run<0>("v_lshl_add_u64 (64-bit add)", 1, w, d);
    run<1>("v_add_co_u32 + v_addc_co_u32", 2, w, d);
    run<2>("v_perm_b32", 1, w, d);
    run<3>("v_alignbit_b32", 1, w, d);
    run<4>("v_bitop3_b32", 1, w, d);
    run<5>("v_xor_b32", 1, w, d);
    run<6>("ds_read_b32 (+and/or/xor)", 1, w, d);
    run<7>("2 x v_xor_b32 + 2 x v_alignbit_b32", 4, w, d);
    run<8>("v_xor_b32_e64 (VOP3 encoding)", 1, w, d);
    run<9>("v_add_u32 (VOP2)", 1, w, d);
  }
  (void)hipFree(d);
  return 0;
}
