// Quad-spread Fr products (csrc/fq.hpp) on MI355X: correctness against the one-lane CIOS product (fr_mul) and the
// latency of a dependent chain at one wave per SIMD, next to fr_mul / fr_mul_fast on the same chain.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/fieldbench/quadbench.hip -o /tmp/quadbench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include "../../passport-zk-circuits_amd/csrc/fq.hpp"

using namespace pzk;

__device__ fr canon_in(fr a) { a.v[7] &= 0x1fffffffu; return a; }  // < p

// every quad: a chain of `iters` products a <- a * b (and a <- a^2 on odd steps), against fr_mul on each lane
__global__ void __launch_bounds__(64) k_check(const fr* io, int n, int iters, int* bad) {
  const int e = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 2);
  const QLane c = QLane::make();
  const fr a1 = canon_in(io[e % n]), b1 = canon_in(io[(e * 7 + 3) % n]);
  fr x = a1;
  fq xq = fq_digit(a1, c.q), bq = fq_digit(b1, c.q);
  for (int i = 0; i < iters; i++) {
    if (i & 1) { x = fr_mul(x, x); xq = (i & 2) ? fq_mul64(xq, xq, c) : (i & 4) ? fq_mulq(xq, xq, c) : fq_mul(xq, xq, c); }
    else { x = fr_mul(x, b1); xq = (i & 2) ? fq_mul(xq, bq, c) : (i & 4) ? fq_mulq(xq, bq, c) : fq_mul64(xq, bq, c); }
  }
  const fq r = fq_canon(xq, c);
  const fr g = fq_gather(r);
  int err = 0;
  for (int k = 0; k < 8; k++) err |= g.v[k] != x.v[k];
  // sums: a + b (both < p, so < 2p) canonicalised
  const fq s = fq_canon(fq_add_raw(fq_digit(a1, c.q), bq), c);
  const fr gs = fq_gather(s), rs = fr_add(a1, b1);
  for (int k = 0; k < 8; k++) err |= gs.v[k] != rs.v[k];
  // a 3-row lazy sum with a constant: K R^-1 + a1 b1' + a2 b2' + a3 b3' (rows from quads 0, 1, 2 of the row, b from
  // this quad), against fr_mul sums; every quad of a 16-lane row holds a different element
  {
    const int row0 = e & ~3;
    const fr r0 = canon_in(io[row0 % n]), r1 = canon_in(io[(row0 + 1) % n]), r2 = canon_in(io[(row0 + 2) % n]);
    const fr kk = canon_in(io[(e * 5 + 1) % n]);
    const fr d0 = canon_in(io[(e * 3 + 2) % n]), d1 = canon_in(io[(e * 11 + 5) % n]), d2 = canon_in(io[(e * 13 + 7) % n]);
    const fq aq = fq_digit((e & 3) == 0 ? r0 : (e & 3) == 1 ? r1 : (e & 3) == 2 ? r2 : r0, c.q);
    const fq bb[3] = {fq_digit(d0, c.q), fq_digit(d1, c.q), fq_digit(d2, c.q)};
    const fq dq = fq_canon(fq_dot<3>([&](int r, auto J) {
      constexpr int j = decltype(J)::value;
      return r == 0 ? rword<0, j>(aq) : r == 1 ? rword<1, j>(aq) : rword<2, j>(aq);
    }, bb, fq_digit(kk, c.q), c), c);
    fr one = fr_zero(); one.v[0] = 1;
    const fr want = fr_add(fr_add(fr_mul(kk, one), fr_mul(r0, d0)), fr_add(fr_mul(r1, d1), fr_mul(r2, d2)));
    const fr got = fq_gather(dq);
    for (int k = 0; k < 8; k++) err |= got.v[k] != want.v[k];
  }
  if (err && (threadIdx.x & 3) == 0) atomicAdd(bad, 1);
}

template <int V>
__global__ void __launch_bounds__(64) k_lat(fr* io, int iters) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  if constexpr (V < 2) {
    fr a = io[tid], b = io[tid + 1];
    for (int i = 0; i < iters; i++) a = V == 0 ? fr_mul(a, b) : fr_mul_fast(a, b);
    io[tid] = a;
  } else {
    const QLane c = QLane::make();
    const int e = tid >> 2;
    fq a = fq_digit(canon_in(io[e]), c.q), b = fq_digit(canon_in(io[e + 1]), c.q);
    for (int i = 0; i < iters; i++) {
      a = V == 4 ? fq_mul64(a, b, c) : V == 5 ? fq_mulq(a, b, c) : fq_mul(a, b, c);
      if (V == 3) a = fq_canon(a, c);
    }
    io[tid] = fq_gather(a);
  }
}

// throughput: 4 independent chains per lane (quads), 256-thread blocks
template <int V>
__global__ void __launch_bounds__(256) k_tput(fr* io, int iters) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  const QLane c = QLane::make();
  const int e = tid >> 2;
  fq a0 = fq_digit(canon_in(io[e]), c.q), b = fq_digit(canon_in(io[e + 1]), c.q), a1 = b, a2 = a0, a3 = b;
  for (int i = 0; i < iters; i++) {
    if (V == 0) { a0 = fq_mul(a0, b, c); a1 = fq_mul(a1, b, c); a2 = fq_mul(a2, b, c); a3 = fq_mul(a3, b, c); }
    else if (V == 1) { a0 = fq_mul64(a0, b, c); a1 = fq_mul64(a1, b, c); a2 = fq_mul64(a2, b, c); a3 = fq_mul64(a3, b, c); }
    else { a0 = fq_mulq(a0, b, c); a1 = fq_mulq(a1, b, c); a2 = fq_mulq(a2, b, c); a3 = fq_mulq(a3, b, c); }
  }
  io[tid] = fq_gather(fq_add_raw(fq_add_raw(a0, a1), fq_add_raw(a2, a3)));
}

// DPP semantics on gfx950: row_newbcast:5 and row_ror:4 / row_ror:12 of the lane index
__global__ void k_dpp(int* out) {
  const int l = threadIdx.x;
  out[l] = __builtin_amdgcn_update_dpp(0, l, 0x155, 0xF, 0xF, false);
  out[64 + l] = __builtin_amdgcn_update_dpp(0, l, 0x124, 0xF, 0xF, false);
  out[128 + l] = __builtin_amdgcn_update_dpp(0, l, 0x12C, 0xF, 0xF, false);
}

int main() {
  {
    int* d;
    hipMalloc(&d, 4 * 192);
    hipLaunchKernelGGL(k_dpp, dim3(1), dim3(64), 0, 0, d);
    int hd[192];
    hipMemcpy(hd, d, sizeof(hd), hipMemcpyDeviceToHost);
    const char* nm[3] = {"row_newbcast:5", "row_ror:4", "row_ror:12"};
    for (int k = 0; k < 3; k++) {
      printf("%-15s", nm[k]);
      for (int l = 0; l < 20; l++) printf(" %d", hd[64 * k + l]);
      printf("\n");
    }
  }
  const int n = 65536;
  fr* io;
  hipMalloc(&io, sizeof(fr) * (256 * 32 * 256 + 8));
  fr* h = (fr*)malloc(sizeof(fr) * n);
  uint64_t x = 88172645463325252ull;
  for (int i = 0; i < n; i++)
    for (int k = 0; k < 8; k++) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; h[i].v[k] = (uint32_t)x; }
  hipMemcpy(io, h, sizeof(fr) * n, hipMemcpyHostToDevice);
  int* bad;
  hipMalloc(&bad, 4);
  int tot = 0;
  for (int it = 1; it <= 33; it += 8) {
    hipMemset(bad, 0, 4);
    hipLaunchKernelGGL(k_check, dim3(4 * n / 64), dim3(64), 0, 0, io, n, it, bad);
    int hb = -1;
    hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
    printf("check iters %d: %d mismatches of %d\n", it, hb, n);
    tot += hb;
  }
  hipMemcpy(io, h, sizeof(fr) * n, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[6] = {"fr_mul (lane)", "fr_mul_fast (lane)", "fq_mul (quad)", "fq_mul + fq_canon (quad)",
                          "fq_mul64 (quad)", "fq_mulq (quad, E/O columns)"};
  for (int v = 0; v < 6; v++) {
    for (int rep = 0; rep < 2; rep++) {
      hipEventRecord(e0);
      const int iters = 2000;
      if (v == 0) hipLaunchKernelGGL(k_lat<0>, dim3(1024), dim3(64), 0, 0, io, iters);
      else if (v == 1) hipLaunchKernelGGL(k_lat<1>, dim3(1024), dim3(64), 0, 0, io, iters);
      else if (v == 2) hipLaunchKernelGGL(k_lat<2>, dim3(1024), dim3(64), 0, 0, io, iters);
      else if (v == 3) hipLaunchKernelGGL(k_lat<3>, dim3(1024), dim3(64), 0, 0, io, iters);
      else if (v == 4) hipLaunchKernelGGL(k_lat<4>, dim3(1024), dim3(64), 0, 0, io, iters);
      else hipLaunchKernelGGL(k_lat<5>, dim3(1024), dim3(64), 0, 0, io, iters);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (rep == 1) printf("latency %-26s %7.1f ns per dependent product (one wave per SIMD)\n", names[v], ms * 1e6 / iters);
    }
  }
  for (int rep = 0; rep < 6; rep++) {
    const int blocks = 256 * 32, iters = 100;
    hipEventRecord(e0);
    if (rep < 2) hipLaunchKernelGGL(k_tput<0>, dim3(blocks), dim3(256), 0, 0, io, iters);
    else if (rep < 4) hipLaunchKernelGGL(k_tput<1>, dim3(blocks), dim3(256), 0, 0, io, iters);
    else hipLaunchKernelGGL(k_tput<2>, dim3(blocks), dim3(256), 0, 0, io, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double prods = 4.0 * iters * blocks * 256 / 4;
    if (rep & 1) printf("throughput %s: %.2f G products/s (%.1f ms)\n", rep < 2 ? "fq_mul" : rep < 4 ? "fq_mul64" : "fq_mulq", prods / ms / 1e6, ms);
  }
  return tot ? 1 : 0;
}
