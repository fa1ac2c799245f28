// BN254 Fr multiplication throughput on MI355X: the emitters' and cores' VALU work is Fr
// products; this measures products per second for csrc/fr.hpp (0: fr_mul, CIOS; 4: fr_mul_fast, FIPS
// with padded carries; 3: fr_sqr) and experimental variants (7: FIPS without the carry pad).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include "../../passport-zk-circuits_amd/csrc/fr.hpp"

using namespace pzk;

// reference: the operand-scanning CIOS product csrc/fr.hpp used before the FIPS form
__device__ __forceinline__ fr fr_mul_cios(const fr& a, const fr& b) {
  uint32_t t[8];
#pragma unroll
  for (int j = 0; j < 8; j++) t[j] = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t s = (uint64_t)a.v[0] * b.v[i] + t[0];
    uint32_t C = (uint32_t)(s >> 32);
    uint32_t t0 = (uint32_t)s;
    uint32_t m = t0 * PINV;
    uint64_t s2 = (uint64_t)m * P_[0] + t0;
    uint32_t C2 = (uint32_t)(s2 >> 32);
#pragma unroll
    for (int j = 1; j < 8; j++) {
      s = (uint64_t)a.v[j] * b.v[i] + t[j] + C;
      C = (uint32_t)(s >> 32);
      s2 = (uint64_t)m * P_[j] + (uint32_t)s + C2;
      C2 = (uint32_t)(s2 >> 32);
      t[j - 1] = (uint32_t)s2;
    }
    t[7] = C + C2;
  }
  fr r;
#pragma unroll
  for (int j = 0; j < 8; j++) r.v[j] = t[j];
  return fr_reduce_once(r);
}

// stress: divergent lanes, chains of products, inversions; every result checked against CIOS
__global__ void k_stress(const fr* io, int n, int rounds, int* bad) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  fr a = io[i], b = io[(i * 7 + 3) % n];
  a.v[7] &= 0x1fffffff; b.v[7] &= 0x1fffffff;
  fr x = a, y = a;
  for (int r = 0; r < rounds; r++) {
    if ((i + r) % 3 == 0) { x = fr_mul_fast(x, b); y = fr_mul_cios(y, b); }
    else if ((i + r) % 3 == 1) { x = fr_sqr_fast(x); y = fr_mul_cios(y, y); }
    else { x = fr_from_mont_fast(fr_mul_fast(x, b)); y = fr_mul_cios(fr_mul_cios(y, b), fr_u64(1)); }
  }
  fr iv = fr_inv(x), one = fr_mul_fast(iv, x), R1 = fr_mont_one();
  int e = 0;
  for (int k = 0; k < 8; k++) e |= (x.v[k] != y.v[k]) | (!fr_is_zero(x) && one.v[k] != R1.v[k]);
  if (e) atomicAdd(bad, 1);
}

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

// variant D: FIPS product scanning (Montgomery product and reduction interleaved per column) with
// a 96-bit column accumulator: each 32x32 product is one v_mad_u64_u32 into the 64-bit
// accumulator with its carry-out (vcc) added into the top word: 2 VALU per product, no moves
__device__ __forceinline__ void mac_d(uint64_t& acc, uint32_t& t2, uint32_t x, uint32_t y) {
  asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc" : "+v"(acc), "+v"(t2) : "v"(x), "v"(y) : "vcc");
}
__device__ __forceinline__ void mac_ds(uint64_t& acc, uint32_t& t2, uint32_t x, uint32_t y) {
  asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc" : "+v"(acc), "+v"(t2) : "v"(x), "s"(y) : "vcc");
}
__device__ __forceinline__ fr fr_mul_d(const fr& a, const fr& b) {
  uint32_t m[8], u[8];
  uint64_t acc = 0; uint32_t t2 = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
#pragma unroll
    for (int j = 0; j < i; j++) { mac_d(acc, t2, a.v[j], b.v[i - j]); mac_ds(acc, t2, m[j], P_[i - j]); }
    mac_d(acc, t2, a.v[i], b.v[0]);
    m[i] = (uint32_t)acc * PINV;
    mac_ds(acc, t2, m[i], P_[0]);
    acc = (acc >> 32) | ((uint64_t)t2 << 32); t2 = 0;
  }
#pragma unroll
  for (int i = 8; i < 16; i++) {
#pragma unroll
    for (int j = i - 7; j < 8; j++) { mac_d(acc, t2, a.v[j], b.v[i - j]); mac_ds(acc, t2, m[j], P_[i - j]); }
    u[i - 8] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)t2 << 32); t2 = 0;
  }
  fr r;
#pragma unroll
  for (int j = 0; j < 8; j++) r.v[j] = u[j];
  return fr_reduce_once(r);
}

// variant E: FIPS with two column accumulators (even / odd product index), halving the dependent
// mad chain for latency-bound callers; the two are summed at the column end
__device__ __forceinline__ void add96(uint64_t& acc, uint32_t& t2, uint64_t x, uint32_t x2) {
  asm("v_add_co_u32_e32 %0, vcc, %0, %2\n\tv_addc_co_u32_e32 %1, vcc, %1, %3, vcc" : "+v"(acc), "+v"(t2) : "v"(x), "v"(x2) : "vcc");
}
__device__ __forceinline__ fr fr_mul_e(const fr& a, const fr& b) {
  uint32_t m[8], u[8];
  uint64_t acc = 0; uint32_t t2 = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) {
    uint64_t c1 = 0; uint32_t h1 = 0;
    const int j0 = i < 8 ? 0 : i - 7, j1 = i < 8 ? i : 7;
#pragma unroll
    for (int j = j0; j <= j1; j++) {
      if (j < i || i >= 8) mac_ds(c1, h1, m[j], P_[i - j]);
      mac_d(acc, t2, a.v[j], b.v[i - j]);
    }
    // acc += c1 (96-bit): lo 64 with carry into t2, then h1
    uint64_t s = acc + c1; uint32_t cy = s < acc; acc = s; t2 += h1 + cy;
    if (i < 8) { m[i] = (uint32_t)acc * PINV; mac_ds(acc, t2, m[i], P_[0]); }
    else u[i - 8] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)t2 << 32); t2 = 0;
  }
  fr r;
#pragma unroll
  for (int j = 0; j < 8; j++) r.v[j] = u[j];
  return fr_reduce_once(r);
}
// variant F: FIPS squaring: per column the cross products once, doubled, plus the square term
__device__ __forceinline__ fr fr_sqr_f(const fr& a) {
  uint32_t m[8], u[8];
  uint64_t cin = 0;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    uint64_t c = 0; uint32_t h = 0;
#pragma unroll
    for (int i = (k < 8 ? 0 : k - 7); i < k - i; i++) mac_d(c, h, a.v[i], a.v[k - i]);
    h = (h << 1) | (uint32_t)(c >> 63); c <<= 1;
    if (!(k & 1)) mac_d(c, h, a.v[k >> 1], a.v[k >> 1]);
    { uint64_t s = c + cin; h += s < c; c = s; }
#pragma unroll
    for (int j = (k < 8 ? 0 : k - 7); j < (k < 8 ? k : 8); j++) mac_ds(c, h, m[j], P_[k - j]);
    if (k < 8) { m[k] = (uint32_t)c * PINV; mac_ds(c, h, m[k], P_[0]); }
    else u[k - 8] = (uint32_t)c;
    cin = (c >> 32) | ((uint64_t)h << 32);
  }
  fr r;
#pragma unroll
  for (int j = 0; j < 8; j++) r.v[j] = u[j];
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
  fr b = io[(i + 1) % n];
  b.v[7] &= 0x1fffffff;
  fr x = fr_mul(a, a), y = fr_sqr_c(a), z = fr_mul(a, b), zd = fr_mul_fast(a, b), ze = fr_mul_e(a, b), yf = fr_sqr_f(a);
  for (int k = 0; k < 8; k++)
    if (x.v[k] != y.v[k] || z.v[k] != zd.v[k] || z.v[k] != ze.v[k] || x.v[k] != yf.v[k]) { atomicAdd(bad, 1); break; }
}

// latency: one dependent chain per lane, one wave per SIMD
template <int V>
__global__ void __launch_bounds__(64) k_lat(fr* io, int iters) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  fr a = io[tid], b = io[tid + 1];
  for (int i = 0; i < iters; i++) {
    if (V == 0) a = fr_mul(a, b);
    else if (V == 4) a = fr_mul_fast(a, b);
    else if (V == 5) a = fr_mul_e(a, b);
    else if (V == 3) a = fr_sqr(a);
    else a = fr_sqr_f(a);
  }
  io[tid] = a;
}

template <int V>
__global__ void __launch_bounds__(256) k_bench(fr* io, int iters) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  fr a0 = io[tid], a1 = fr_add(a0, a0), a2 = fr_add(a1, a0), a3 = fr_add(a2, a0), b = io[tid + 1];
  for (int i = 0; i < iters; i++) {
    if (V == 0) { a0 = fr_mul(a0, b); a1 = fr_mul(a1, b); a2 = fr_mul(a2, b); a3 = fr_mul(a3, b); }
    else if (V == 1) { a0 = fr_mul_b(a0, b); a1 = fr_mul_b(a1, b); a2 = fr_mul_b(a2, b); a3 = fr_mul_b(a3, b); }
    else if (V == 5) { a0 = fr_mul_e(a0, b); a1 = fr_mul_e(a1, b); a2 = fr_mul_e(a2, b); a3 = fr_mul_e(a3, b); }
    else if (V == 6) { a0 = fr_sqr_f(a0); a1 = fr_sqr_f(a1); a2 = fr_sqr_f(a2); a3 = fr_sqr_f(a3); }
    else if (V == 4) { a0 = fr_mul_fast(a0, b); a1 = fr_mul_fast(a1, b); a2 = fr_mul_fast(a2, b); a3 = fr_mul_fast(a3, b); }
    else if (V == 7) { a0 = fr_mul_d(a0, b); a1 = fr_mul_d(a1, b); a2 = fr_mul_d(a2, b); a3 = fr_mul_d(a3, b); }
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
    printf("sqr / FIPS check: %d mismatches of 65536\n", hb);
    for (int rep = 0; rep < 20; rep++) {
      hipMemset(bad, 0, 4);
      hipLaunchKernelGGL(k_stress, dim3(256), dim3(256), 0, 0, io, 65536, 40 + rep, bad);
      hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
      if (hb || rep == 19) printf("stress rep %d: %d mismatches of 65536\n", rep, hb);
    }
  }
  for (int v = 0; v < 8; v++) {
    for (int rep = 0; rep < 3; rep++) {
      hipEventRecord(e0);
      if (v == 0) hipLaunchKernelGGL(k_bench<0>, dim3(blocks), dim3(threads), 0, 0, io, iters);
      else if (v == 1) hipLaunchKernelGGL(k_bench<1>, dim3(blocks), dim3(threads), 0, 0, io, iters);
      else if (v == 2) hipLaunchKernelGGL(k_bench<2>, dim3(blocks), dim3(threads), 0, 0, io, iters);
      else if (v == 7) hipLaunchKernelGGL(k_bench<7>, dim3(blocks), dim3(threads), 0, 0, io, iters);
      else if (v == 5) hipLaunchKernelGGL(k_bench<5>, dim3(blocks), dim3(threads), 0, 0, io, iters);
      else if (v == 6) hipLaunchKernelGGL(k_bench<6>, dim3(blocks), dim3(threads), 0, 0, io, iters);
      else if (v == 4) hipLaunchKernelGGL(k_bench<4>, dim3(blocks), dim3(threads), 0, 0, io, iters);
      else hipLaunchKernelGGL(k_bench<3>, dim3(blocks), dim3(threads), 0, 0, io, iters);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      double muls = 4.0 * iters * blocks * threads;
      if (rep == 2)
        printf("variant %d: %.2f Gmul/s  (%.1f ms)  => %.0f cycles per wave64 fr_mul per SIMD at 2.4 GHz\n", v,
               muls / ms / 1e6, ms, (ms * 1e-3 * 2.4e9 * 1024) / (muls / 64));
    }
  }
  const int lv[5] = {0, 4, 5, 3, 6};
  for (int q = 0; q < 5; q++) {
    for (int rep = 0; rep < 2; rep++) {
      hipEventRecord(e0);
      switch (lv[q]) {
        case 0: hipLaunchKernelGGL(k_lat<0>, dim3(1024), dim3(64), 0, 0, io, 2000); break;
        case 4: hipLaunchKernelGGL(k_lat<4>, dim3(1024), dim3(64), 0, 0, io, 2000); break;
        case 5: hipLaunchKernelGGL(k_lat<5>, dim3(1024), dim3(64), 0, 0, io, 2000); break;
        case 3: hipLaunchKernelGGL(k_lat<3>, dim3(1024), dim3(64), 0, 0, io, 2000); break;
        default: hipLaunchKernelGGL(k_lat<6>, dim3(1024), dim3(64), 0, 0, io, 2000); break;
      }
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      if (rep == 1) printf("latency variant %d: %.0f ns per dependent op (one wave per SIMD)\n", lv[q], ms * 1e6 / 2000);
    }
  }
  return 0;
}
