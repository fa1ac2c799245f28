// Poseidon (hasher/poseidon/poseidon.circom:10-226) on gfx950.
//
//  * core — one lane per (witness, permutation task); wave = 64 witnesses of the SAME task,
//           so t, the round constants and every control decision are wave-uniform (scalar
//           loads of constants, no divergence). Keeps only the layer states that enter each
//           S-box layer (X0..X3, Y0..Y_RP, Z1..Z3; (RP+8)*t Fr in Montgomery form) — the
//           sequential critical path does no format conversion and no per-signal stores.
//  * emit — one workgroup per (permutation, witness): rebuilds x^2, x^4, x^5, ark outputs and
//           every constant-times-state product into LDS in parallel, then writes the
//           PoseidonHash(n) block (1 + n + |PoseidonEx|) as consecutive 32-byte elements.
#pragma once
#include <type_traits>
#include "fr.hpp"
#include "layout.hpp"
#include "pos_prog.hpp"

namespace pzk {

struct PosConsts {
  const fr* base;   // Montgomery-form constants
  const fr* nbase;  // the same constants in normal form
  PosParamIndex ix;
  __device__ __forceinline__ const fr& Cn(int t, int i) const { return nbase[ix.c_off[t] + i]; }
  __device__ __forceinline__ const fr& C(int t, int i) const { return base[ix.c_off[t] + i]; }
  __device__ __forceinline__ const fr& M(int t, int i, int j) const { return base[ix.m_off[t] + i * t + j]; }
  __device__ __forceinline__ const fr& Pm(int t, int i, int j) const { return base[ix.p_off[t] + i * t + j]; }
  __device__ __forceinline__ const fr& S(int t, int i) const { return base[ix.s_off[t] + i]; }
};

__device__ __forceinline__ fr pow5(const fr& x) { fr x2 = fr_sqr(x), x4 = fr_sqr(x2); return fr_mul(x4, x); }

// value store: SoA [slot][witness], Montgomery form
struct ValueStore {
  fr* v;
  uint32_t batch;
  __device__ __forceinline__ fr& at(int slot, uint32_t w) const { return v[(size_t)slot * batch + w]; }
};

// Round-state sink of pos_core_lane. Each lane's core slice starts on a 128-byte line (the builder aligns
// task.core_off and the per-witness core to 4 Fr); element k is parked in the lane's 4-element line in LDS
// and the line leaves as one whole 128-byte write when its last element arrives. Writing the 32-byte
// elements as they come (one partial line per lane per round, 64 lanes on 64 different lines) let L2 evict
// most lines half-written under the emitters' store stream: 2.2x the algorithmic write bytes.
struct PosLineSink {
  fr* out;   // the lane's task slice (128-byte aligned)
  fr* line;  // the wave's LDS lines, element i of lane l at line[i * 64 + l]
  __device__ __forceinline__ void flush(int k0, int n) const {
#pragma unroll
    for (int i = 0; i < 4; i++)
      if (i < n) out[k0 + i] = line[i * 64];
  }
  __device__ __forceinline__ void put(int k, const fr& v) const {
    line[(k & 3) * 64] = v;
    if ((k & 3) == 3) flush(k - 3, 4);  // k is wave-uniform
  }
  __device__ __forceinline__ void finish(int k_end) const {
    if (k_end & 3) flush(k_end & ~3, k_end & 3);
  }
};

// compile-time loop: f(std::integral_constant<int, I>) for I in [B, E)
template <int B, int E, class F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    sfor<B + 1, E>(f);
  }
}

// (every index into st[] / nx[] is a constant expression from the start, so the arrays are registers: with
// `#pragma unroll` loops the state of t <= 6 stayed a 96-400 B scratch array)
template <int T>
__device__ __forceinline__ void pos_core_lane(const PosConsts& K, const PosTask& task, const ValueStore& vs, uint32_t w,
                                              const PosLineSink& out) {
  constexpr int t = T;
  const int RP = pos_nrp(t);
  fr st[t], nx[t];
  st[0] = K.C(t, 0);
  sfor<1, t>([&](auto J) { st[J] = fr_add(vs.at(task.in_slot[J - 1], w), K.C(t, J)); });
  int o = 0;
  auto full = [&](int c0, bool use_p) __attribute__((always_inline)) {  // S-box layer (Ark constants from c0), then the t x t mix
    sfor<0, t>([&](auto J) { out.put(o + J, st[J]); });
    o += t;
    sfor<0, t>([&](auto J) { st[J] = fr_add(pow5(st[J]), K.C(t, c0 + J)); });
    sfor<0, t>([&](auto I) {
      fr acc = fr_zero();
      sfor<0, t>([&](auto J) { acc = fr_add(acc, fr_mul(use_p ? K.Pm(t, J, I) : K.M(t, J, I), st[J])); });
      nx[I] = acc;
    });
    sfor<0, t>([&](auto J) { st[J] = nx[J]; });
  };
  for (int r = 0; r < 4; r++) full((r + 1) * t, r == 3);  // full rounds 0..3 (round 3 mixes with P)
  for (int r = 0; r < RP; r++) {                          // partial rounds
    sfor<0, t>([&](auto J) { out.put(o + J, st[J]); });
    o += t;
    const fr s0 = fr_add(pow5(st[0]), K.C(t, 5 * t + r));
    const int sb = (2 * t - 1) * r;
    fr acc = fr_mul(K.S(t, sb), s0);
    sfor<1, t>([&](auto I) { acc = fr_add(acc, fr_mul(K.S(t, sb + I), st[I])); });
    sfor<1, t>([&](auto I) { st[I] = fr_add(st[I], fr_mul(s0, K.S(t, sb + t + I - 1))); });
    st[0] = acc;
  }
  for (int r = 0; r < 3; r++) full(5 * t + RP + r * t, false);  // full rounds 4..6
  sfor<0, t>([&](auto J) { out.put(o + J, st[J]); });         // Z3
  out.finish(o + t);
  fr h = fr_zero();
  sfor<0, t>([&](auto J) { h = fr_add(h, fr_mul(K.M(t, J, 0), pow5(st[J]))); });
  vs.at(task.out_slot, w) = h;
}

// Cooperative permutation: G lanes per (witness, task), lane j < t holds state element j; returns
// the hash to every lane of the group
// (G = 4 for t <= 4, 8 otherwise; the lanes j >= t carry zeros). A full round is one S-box per
// lane and a t-term mix gathered with shuffles; a partial round is lane 0's S-box, one product
// per lane and a butterfly sum. Same core output as pos_core_lane (Montgomery layer states,
// X0..X3, Y0..Y_RP, Z1..Z3), written by the owning lanes. ~3.5x shorter dependency chain than
// one lane per permutation and ~70 VGPRs instead of 256, so the kernel can be placed next to
// the emitters.
template <int T, int G>
__device__ __forceinline__ fr pos_core_group(const PosConsts& K, const PosTask& task, const ValueStore& vs, uint32_t w,
                                               fr* core /* this witness's Poseidon core */, int j) {
  constexpr int t = T;
  const int RP = pos_nrp(t);
  const bool act = j < t;
  const int jj = act ? j : 0;
  fr* out = core + task.core_off;
  fr st = fr_zero();
  if (act && j > 0) st = vs.at(task.in_slot[j - 1], w);
  if (act) st = fr_add(st, K.C(t, j));
  const int lane = threadIdx.x & 63, gb = lane & ~(G - 1);
  auto mix = [&](const fr& x, bool use_p) -> fr {  // sum_k Mat[k][j] * x_k
    fr acc = fr_zero();
#pragma unroll
    for (int k = 0; k < t; k++) {
      fr xk = fr_shfl(x, gb + k, 64);
      acc = fr_add(acc, fr_mul(use_p ? K.Pm(t, k, jj) : K.M(t, k, jj), xk));
    }
    return act ? acc : fr_zero();
  };
  auto group_sum = [&](fr v) -> fr {  // butterfly: every lane of the group gets the sum
#pragma unroll
    for (int d = 1; d < G; d <<= 1) {
      fr o;
#pragma unroll
      for (int k = 0; k < 8; k++) o.v[k] = (uint32_t)__shfl_xor((int)v.v[k], d, 64);
      v = fr_add(v, o);
    }
    return v;
  };
  int o = 0;
  for (int r = 0; r < 4; r++) {  // full rounds 0..3 (round 3 mixes with P)
    if (act) out[o + j] = st;
    o += t;
    fr a = act ? fr_add(pow5(st), K.C(t, (r + 1) * t + jj)) : fr_zero();
    st = mix(a, r == 3);
  }
  for (int r = 0; r < RP; r++) {  // partial rounds
    if (act) out[o + j] = st;
    o += t;
    fr s0 = fr_zero();
    if (j == 0) s0 = fr_add(pow5(st), K.C(t, 5 * t + r));
    s0 = fr_shfl(s0, gb, 64);
    const int sb = (2 * t - 1) * r;
    fr term = act ? fr_mul(K.S(t, sb + jj), j == 0 ? s0 : st) : fr_zero();
    fr sum = group_sum(term);
    if (j == 0) st = sum;
    else if (act) st = fr_add(st, fr_mul(s0, K.S(t, sb + t + j - 1)));
  }
  for (int r = 0; r < 3; r++) {  // full rounds 4..6
    if (act) out[o + j] = st;
    o += t;
    fr a = act ? fr_add(pow5(st), K.C(t, 5 * t + RP + r * t + jj)) : fr_zero();
    st = mix(a, false);
  }
  if (act) out[o + j] = st;  // Z3
  fr h = group_sum(act ? fr_mul(K.M(t, jj, 0), pow5(st)) : fr_zero());
  if (j == 0) vs.at(task.out_slot, w) = h;
  return h;  // every lane of the group holds the hash (Montgomery)
}

// ------------------------------------------------------------------------------ emit
// Image fill (pos_prog.hpp layout, normal form), two phases:
//  A: per S-box (8t full-layer elements, RP partial rounds): x, x^2, x^4, x^5 and the Ark output
//     from the Montgomery layer state of the core; the remaining partial-round states; inputs,
//     hash, zero.
//  B: per GetSum row (7t full, 1 last, RP partial): t products constant*value, kept (products
//     1..t-1, the row's `in` signals) and turned into prefix sums. mont_mul(c * R, v) = c * v, so
//     products of Montgomery constants with normal-form values come out in normal form.
template <int T>
__device__ __forceinline__ void pos_img_fill(fr* img, const PosConsts& K, const fr* core, const ValueStore& vs,
                                             const PosTask& task, uint32_t w) {
  constexpr int t = T;
  constexpr PosImg I(T);
  constexpr int RP = I.rp;
  const int tid = threadIdx.x, nt = blockDim.x;
  // core order: X0..X3 (4t), Y0..Y_RP ((RP+1)t), Z1..Z3 (3t), all Montgomery
  constexpr int NA = 8 * t + RP, NC = RP * (t - 1) + t;
  for (int q = tid; q < NA + NC + 7; q += nt) {
    if (q < 8 * t) {
      const int f = q / t, j = q - f * t;
      const int ci = f < 4 ? f * t + j : f == 4 ? 4 * t + RP * t + j : 4 * t + (RP + 1) * t + (f - 5) * t + j;
      // mixed forms: mont_mul(aR, b) = ab, so normal-form powers come straight out of products
      // with the Montgomery-form x and x^2 (3.4 products per S-box instead of 5.3)
      const fr xm = core[ci], x2m = fr_sqr_fast(xm), x2 = fr_from_mont_fast(x2m), x4 = fr_mul_fast(x2m, x2), x5 = fr_mul_fast(x4, xm);
      img[I.in + q] = fr_from_mont_fast(xm); img[I.p2 + q] = x2;
      img[I.p4 + q] = x4; img[I.p5 + q] = x5;
      if (f < 7) {
        const int cidx = f < 4 ? (f + 1) * t + j : 5 * t + RP + (f - 4) * t + j;
        img[I.ark + q] = fr_add(x5, K.Cn(t, cidx));
      }
    } else if (q < NA) {
      const int r = q - 8 * t;
      const fr xm = core[4 * t + r * t], x2m = fr_sqr_fast(xm), x2 = fr_from_mont_fast(x2m), x4 = fr_mul_fast(x2m, x2),
               x5 = fr_mul_fast(x4, xm);
      img[I.pin + r * t] = fr_from_mont_fast(xm); img[I.pp2 + r] = x2;
      img[I.pp4 + r] = x4; img[I.pp5 + r] = x5;
      img[I.pin0 + r] = fr_add(x5, K.Cn(t, 5 * t + r));
    } else if (q < NA + NC) {
      const int c = q - NA;
      int r, i;
      if (c < RP * (t - 1)) { r = c / (t - 1); i = 1 + (c - r * (t - 1)); }
      else { r = RP; i = c - RP * (t - 1); }
      img[I.pin + r * t + i] = fr_from_mont_fast(core[4 * t + r * t + i]);
    } else {
      const int k = q - NA - NC;
      if (k < task.n) img[I.inp + k] = fr_from_mont_fast(vs.at(task.in_slot[k], w));
      else if (k == 5) img[I.hash] = fr_from_mont_fast(vs.at(task.out_slot, w));
      else if (k == 6) img[I.zero] = fr_zero();
    }
  }
  __syncthreads();
  constexpr int NF = 7 * t, NR = NF + 1 + RP;
  // products, one per thread: row r, term k (full mix f, output i: Mat_f[k][i] * ark[f][k];
  // mixLast: M[k][0] * x5[7][k]; partial r: S[(2t-1)r + k] * in_k, in_0 = the S-box's Ark output)
  for (int q = tid; q < NR * t; q += nt) {
    const int row = q / t, k = q - row * t;
    fr c, v;
    int dst;
    if (row < NF) {
      const int f = row / t, i = row - f * t;
      c = f == 3 ? K.Pm(t, k, i) : K.M(t, k, i);
      v = img[I.ark + f * t + k];
      dst = I.fs + row * t + k;
    } else if (row == NF) {
      c = K.M(t, k, 0);
      v = img[I.p5 + 7 * t + k];
      dst = I.ls + k;
    } else {
      const int r = row - NF - 1;
      c = K.S(t, (2 * t - 1) * r + k);
      v = k == 0 ? img[I.pin0 + r] : img[I.pin + r * t + k];
      dst = I.ps + r * t + k;
    }
    const fr pr = fr_mul_fast(c, v);
    img[dst] = pr;
    if (k) img[I.prod(row, k)] = pr;
  }
  __syncthreads();
  // prefix sums along each row
  for (int row = tid; row < NR; row += nt) {
    const int base = row < NF ? I.fs + row * t : row == NF ? I.ls : I.ps + (row - NF - 1) * t;
    fr acc = img[base];
#pragma unroll
    for (int k = 1; k < t; k++) { acc = fr_add(acc, img[base + k]); img[base + k] = acc; }
  }
  __syncthreads();
}

}  // namespace pzk
