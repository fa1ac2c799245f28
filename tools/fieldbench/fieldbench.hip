// BN254 Fr multiplication throughput on MI355X: the emitters' and cores' VALU work is Fr
// products; this measures fr_mul per second for the CIOS variant in csrc/fr.hpp and variants.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include "../../passport-zk-circuits_amd/csrc/fr.hpp"

using namespace pzk;

// variant B: 32x32 products via v_mul_lo_u32 / v_mul_hi_u32 and explicit carry chains
__device__ __forceinline__ fr fr_mul_b(const fr& a, const fr& b) {
  uint32_t t[10];
#pragma unroll
  for (int j = 0; j < 10; j++) t[j] = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      uint32_t lo = a.v[j] * b.v[i], hi = __umulhi(a.v[j], b.v[i]);
      uint64_t s = (uint64_t)t[j] + lo + c;
      t[j] = (uint32_t)s;
      c = hi + (uint32_t)(s >> 32);
    }
    uint64_t s8 = (uint64_t)t[8] + c; t[8] = (uint32_t)s8; t[9] = (uint32_t)(s8 >> 32);
    uint32_t m = t[0] * PINV;
    c = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      uint32_t lo = m * P_[j], hi = __umulhi(m, P_[j]);
      uint64_t s = (uint64_t)t[j] + lo + c;
      t[j] = (uint32_t)s;
      c = hi + (uint32_t)(s >> 32);
    }
    uint64_t s8b = (uint64_t)t[8] + c; t[8] = (uint32_t)s8b; t[9] += (uint32_t)(s8b >> 32);
#pragma unroll
    for (int j = 0; j < 9; j++) t[j] = t[j + 1];
    t[9] = 0;
  }
  fr r;
#pragma unroll
  for (int j = 0; j < 8; j++) r.v[j] = t[j];
  return fr_reduce_once(r);
}

// variant C: dedicated squaring (SOS: 28 cross + 8 square products, then Montgomery REDC)
__device__ __forceinline__ fr fr_sqr_c(const fr& a) {
  uint32_t t[16];
#pragma unroll
  for (int j = 0; j < 16; j++) t[j] = 0;
#pragma unroll
  for (int i = 0; i < 7; i++) {
    uint32_t c = 0;
#pragma unroll
    for (int j = i + 1; j < 8; j++) {
      uint64_t s = (uint64_t)a.v[i] * a.v[j] + t[i + j] + c;
      t[i + j] = (uint32_t)s; c = (uint32_t)(s >> 32);
    }
    t[i + 8] = c;
  }
  // double
#pragma unroll
  for (int j = 15; j > 0; j--) t[j] = (t[j] << 1) | (t[j - 1] >> 31);
  t[0] <<= 1;
  // add squares
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t s = (uint64_t)a.v[i] * a.v[i] + t[2 * i] + c;
    t[2 * i] = (uint32_t)s;
    uint64_t s2 = (s >> 32) + t[2 * i + 1];
    t[2 * i + 1] = (uint32_t)s2; c = (uint32_t)(s2 >> 32);
  }
  // REDC
  uint32_t hc = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint32_t m = t[i] * PINV, cc = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      uint64_t s = (uint64_t)m * P_[j] + t[i + j] + cc;
      t[i + j] = (uint32_t)s; cc = (uint32_t)(s >> 32);
    }
    uint64_t s = (uint64_t)t[i + 8] + cc + hc;
    t[i + 8] = (uint32_t)s; hc = (uint32_t)(s >> 32);
  }
  fr r;
#pragma unroll
  for (int j = 0; j < 8; j++) r.v[j] = t[8 + j];
  return fr_reduce_once(r);
}

__global__ void k_check(const fr* io, int n, int* bad) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  fr a = io[i];
  a.v[7] &= 0x1fffffff;  // < p
  fr x = fr_mul(a, a), y = fr_sqr_c(a);
  for (int k = 0; k < 8; k++) if (x.v[k] != y.v[k]) { atomicAdd(bad, 1); break; }
}

template <int V>
__global__ void __launch_bounds__(256) k_bench(fr* io, int iters) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  fr a0 = io[tid], a1 = fr_add(a0, a0), a2 = fr_add(a1, a0), a3 = fr_add(a2, a0), b = io[tid + 1];
  for (int i = 0; i < iters; i++) {
    if (V == 0) { a0 = fr_mul(a0, b); a1 = fr_mul(a1, b); a2 = fr_mul(a2, b); a3 = fr_mul(a3, b); }
    else if (V == 1) { a0 = fr_mul_b(a0, b); a1 = fr_mul_b(a1, b); a2 = fr_mul_b(a2, b); a3 = fr_mul_b(a3, b); }
    else if (V == 2) { a0 = fr_mul(a0, a0); a1 = fr_mul(a1, a1); a2 = fr_mul(a2, a2); a3 = fr_mul(a3, a3); }
    else { a0 = fr_sqr_c(a0); a1 = fr_sqr_c(a1); a2 = fr_sqr_c(a2); a3 = fr_sqr_c(a3); }
  }
  io[tid] = fr_add(fr_add(a0, a1), fr_add(a2, a3));
}

int main() {
  const int blocks = 256 * 32, threads = 256, iters = 200;
  fr* io;
  hipMalloc(&io, sizeof(fr) * (blocks * threads + 1));
  hipMemset(io, 0x11, sizeof(fr) * (blocks * threads + 1));
  // check both variants agree on the same data
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  {
    // random-ish data, then check sqr == mul(a, a)
    fr* h = (fr*)malloc(sizeof(fr) * 65536);
    uint64_t x = 88172645463325252ull;
    for (int i = 0; i < 65536; i++) for (int k = 0; k < 8; k++) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; h[i].v[k] = (uint32_t)x; }
    hipMemcpy(io, h, sizeof(fr) * 65536, hipMemcpyHostToDevice);
    int* bad; hipMalloc(&bad, 4); hipMemset(bad, 0, 4);
    hipLaunchKernelGGL(k_check, dim3(256), dim3(256), 0, 0, io, 65536, bad);
    int hb = -1; hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
    printf("sqr check: %d mismatches of 65536\n", hb);
  }
  for (int v = 0; v < 4; v++) {
    for (int rep = 0; rep < 3; rep++) {
      hipEventRecord(e0);
      if (v == 0) hipLaunchKernelGGL(k_bench<0>, dim3(blocks), dim3(threads), 0, 0, io, iters);
      else if (v == 1) hipLaunchKernelGGL(k_bench<1>, dim3(blocks), dim3(threads), 0, 0, io, iters);
      else if (v == 2) hipLaunchKernelGGL(k_bench<2>, dim3(blocks), dim3(threads), 0, 0, io, iters);
      else hipLaunchKernelGGL(k_bench<3>, dim3(blocks), dim3(threads), 0, 0, io, iters);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      double muls = 4.0 * iters * blocks * threads;
      if (rep == 2)
        printf("variant %d: %.2f Gmul/s  (%.1f ms)  => %.0f cycles per wave64 fr_mul per SIMD at 2.4 GHz\n", v,
               muls / ms / 1e6, ms, (ms * 1e-3 * 2.4e9 * 1024) / (muls / 64));
    }
  }
  return 0;
}
