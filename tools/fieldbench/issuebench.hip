// Chip-wide VALU issue rate of the instructions the field arithmetic is made of (gfx950): many waves per SIMD, each
// running 8 independent accumulator chains of one instruction kind, so the figure is issue throughput, not latency.
// Prints wave64 instructions per second and SIMD cycles per wave64 instruction at the measured clock-free rate
// (256 CUs x 4 SIMDs x 2.4 GHz).
// build: hipcc --offload-arch=gfx950 -O3 -o issuebench issuebench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int ITERS = 512, UNROLL = 8;

template <int KIND>
__global__ __launch_bounds__(256) void k_issue(uint32_t* out, uint32_t seed) {
  uint32_t a[UNROLL], b = seed ^ threadIdx.x;
  uint64_t w[UNROLL];
#pragma unroll
  for (int i = 0; i < UNROLL; i++) { a[i] = seed * (i + 3) + threadIdx.x; w[i] = a[i]; }
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < UNROLL; i++) {
      if constexpr (KIND == 0) {  // v_add_u32
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
      } else if constexpr (KIND == 1) {  // v_mad_u64_u32 (64-bit accumulate, SGPR carry-out)
        uint64_t c;
        asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(w[i]), "=s"(c) : "v"(a[i]), "v"(b));
      } else if constexpr (KIND == 2) {  // v_mul_lo_u32
        asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
      } else if constexpr (KIND == 3) {  // v_mul_hi_u32
        asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
      } else if constexpr (KIND == 4) {  // v_add_co_u32 (VCC carry-out)
        asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(a[i]) : "v"(b) : "vcc");
      } else if constexpr (KIND == 5) {  // v_mov_b32 with a DPP row broadcast
        asm volatile("v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "=v"(a[i]) : "v"(a[(i + 1) % UNROLL]));
      } else {  // v_lshl_add_u64
        asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(w[i]) : "v"(w[(i + 1) % UNROLL]));
      }
    }
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < UNROLL; i++) s += a[i] + (uint32_t)w[i] + (uint32_t)(w[i] >> 32);
  if (s == 0x12345678u) out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int KIND>
static int run(const char* name, uint32_t* d) {
  const int blocks = 256 * 4 * 8 * 4 / 4;  // 8 waves per SIMD (256-thread workgroups = 4 waves)
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k_issue<KIND>, dim3(blocks), dim3(256), 0, 0, d, 7u);
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(e0));
  const int reps = 5;
  for (int r = 0; r < reps; r++) hipLaunchKernelGGL(k_issue<KIND>, dim3(blocks), dim3(256), 0, 0, d, 7u + r);
  CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
  float ms = 0; CHK(hipEventElapsedTime(&ms, e0, e1));
  const double waves = (double)blocks * 4 * reps, insts = waves * ITERS * UNROLL;
  const double rate = insts / (ms * 1e-3);
  printf("%-16s %8.3f ms  %7.1f G wave-instr/s  %.2f SIMD cycles per instruction at 2.4 GHz\n", name, ms, rate / 1e9,
         256.0 * 4 * 2.4e9 / rate);
  return 0;
}

int main() {
  uint32_t* d;
  CHK(hipMalloc(&d, 4u << 22));
  if (run<0>("v_add_u32", d) || run<4>("v_add_co_u32", d) || run<1>("v_mad_u64_u32", d) || run<2>("v_mul_lo_u32", d) ||
      run<3>("v_mul_hi_u32", d) || run<5>("v_mov_b32_dpp", d) || run<6>("v_lshl_add_u64", d))
    return 1;
  CHK(hipFree(d));
  return 0;
}
