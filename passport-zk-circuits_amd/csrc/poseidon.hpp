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
#include "fr.hpp"
#include "layout.hpp"

namespace pzk {

struct PosConsts {
  const fr* base;   // Montgomery-form constants
  PosParamIndex ix;
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

template <int T>
__device__ __forceinline__ void pos_core_lane(const PosConsts& K, const PosTask& task, const ValueStore& vs, uint32_t w,
                                              fr* core /* this witness's Poseidon core */) {
  constexpr int t = T;
  const int RP = pos_nrp(t);
  fr st[t], nx[t];
  fr* out = core + task.core_off;
  st[0] = fr_zero();
#pragma unroll
  for (int j = 1; j < t; j++) st[j] = vs.at(task.in_slot[j - 1], w);
#pragma unroll
  for (int j = 0; j < t; j++) st[j] = fr_add(st[j], K.C(t, j));
  int o = 0;
  // full rounds 0..3 (round 3 mixes with P)
  for (int r = 0; r < 4; r++) {
#pragma unroll
    for (int j = 0; j < t; j++) out[o + j] = st[j];
    o += t;
#pragma unroll
    for (int j = 0; j < t; j++) st[j] = fr_add(pow5(st[j]), K.C(t, (r + 1) * t + j));
#pragma unroll
    for (int i = 0; i < t; i++) {
      fr acc = fr_zero();
#pragma unroll
      for (int j = 0; j < t; j++) acc = fr_add(acc, fr_mul(r == 3 ? K.Pm(t, j, i) : K.M(t, j, i), st[j]));
      nx[i] = acc;
    }
#pragma unroll
    for (int j = 0; j < t; j++) st[j] = nx[j];
  }
  // partial rounds
  for (int r = 0; r < RP; r++) {
#pragma unroll
    for (int j = 0; j < t; j++) out[o + j] = st[j];
    o += t;
    fr s0 = fr_add(pow5(st[0]), K.C(t, 5 * t + r));
    const int sb = (2 * t - 1) * r;
    fr acc = fr_mul(K.S(t, sb), s0);
#pragma unroll
    for (int i = 1; i < t; i++) acc = fr_add(acc, fr_mul(K.S(t, sb + i), st[i]));
#pragma unroll
    for (int i = 1; i < t; i++) st[i] = fr_add(st[i], fr_mul(s0, K.S(t, sb + t + i - 1)));
    st[0] = acc;
  }
  // full rounds 4..6
  for (int r = 0; r < 3; r++) {
#pragma unroll
    for (int j = 0; j < t; j++) out[o + j] = st[j];
    o += t;
#pragma unroll
    for (int j = 0; j < t; j++) st[j] = fr_add(pow5(st[j]), K.C(t, 5 * t + RP + r * t + j));
#pragma unroll
    for (int i = 0; i < t; i++) {
      fr acc = fr_zero();
#pragma unroll
      for (int j = 0; j < t; j++) acc = fr_add(acc, fr_mul(K.M(t, j, i), st[j]));
      nx[i] = acc;
    }
#pragma unroll
    for (int j = 0; j < t; j++) st[j] = nx[j];
  }
#pragma unroll
  for (int j = 0; j < t; j++) out[o + j] = st[j];  // Z3
  fr h = fr_zero();
#pragma unroll
  for (int j = 0; j < t; j++) h = fr_add(h, fr_mul(K.M(t, j, 0), pow5(st[j])));
  vs.at(task.out_slot, w) = h;
}

// ------------------------------------------------------------------------------ emit
// LDS image of one permutation (all Montgomery form). Layers: full layers f = 0..7
// (inputs X0..X3, Z0..Z3), partial rounds r = 0..RP-1 (inputs Y_r), plus derived values.
struct PosLds {
  int t, RP;
  fr* full_in;    // [8][t]  sigma inputs of full layers
  fr* full_p2;    // [8][t]
  fr* full_p4;    // [8][t]
  fr* full_p5;    // [8][t]
  fr* full_ark;   // [7][t]  ark outputs (layers 0..6)
  fr* full_prod;  // [7][t][t] prod[f][i][j] = Mat_f[j][i] * ark[f][j]; mixLast: [7][0][j] uses M[j][0]*p5[7][j]
  fr* last_prod;  // [t]
  fr* part_in;    // [RP+1][t] Y_0..Y_RP
  fr* part_p2;    // [RP]
  fr* part_p4;    // [RP]
  fr* part_p5;    // [RP]
  fr* part_in0;   // [RP]  p5 + C
  fr* part_prod;  // [RP][t]  S[..+i] * in_i
  fr* part_out;   // [RP][t]  mixS outputs (= Y_{r+1})
  fr* inputs;     // [5] PoseidonHash inputs
  fr* hash;       // [1]
  fr* base;       // whole image: pos_lds_elems(t) elements
};

__host__ __device__ inline int pos_lds_elems(int t) {
  int RP = pos_nrp(t);
  return 8 * t * 4 + 7 * t + 7 * t * t + t + (RP + 1) * t + 4 * RP + RP * t + 6;
}

__device__ __forceinline__ void pos_lds_carve(PosLds& L, fr* base, int t) {
  int RP = pos_nrp(t);
  L.t = t; L.RP = RP;
  L.base = base;
  fr* p = base;
  L.full_in = p; p += 8 * t;
  L.full_p2 = p; p += 8 * t;
  L.full_p4 = p; p += 8 * t;
  L.full_p5 = p; p += 8 * t;
  L.full_ark = p; p += 7 * t;
  L.full_prod = p; p += 7 * t * t;
  L.last_prod = p; p += t;
  L.part_in = p; p += (RP + 1) * t;
  L.part_p2 = p; p += RP;
  L.part_p4 = p; p += RP;
  L.part_p5 = p; p += RP;
  L.part_in0 = p; p += RP;
  L.part_prod = p; p += RP * t;
  L.inputs = p; p += 5;
  L.hash = p; p += 1;
  L.part_out = L.part_in + t;  // Y_{r+1}
}

// Cooperative fill: all threads of the workgroup. core = this witness's states for the task.
__device__ __forceinline__ void pos_lds_fill(PosLds& L, const PosConsts& K, const fr* core) {
  const int t = L.t, RP = L.RP;
  const int tid = threadIdx.x, nt = blockDim.x;
  // core order: X0..X3 (4t), Y0..Y_RP ((RP+1)t), Z1..Z3 (3t)
  for (int i = tid; i < 4 * t; i += nt) L.full_in[i] = core[i];
  for (int i = tid; i < (RP + 1) * t; i += nt) L.part_in[i] = core[4 * t + i];
  for (int i = tid; i < t; i += nt) L.full_in[4 * t + i] = core[4 * t + RP * t + i];  // Z0 = Y_RP
  for (int i = tid; i < 3 * t; i += nt) L.full_in[5 * t + i] = core[4 * t + (RP + 1) * t + i];
  __syncthreads();
  for (int i = tid; i < 8 * t; i += nt) {
    fr x = L.full_in[i], x2 = fr_sqr(x), x4 = fr_sqr(x2), x5 = fr_mul(x4, x);
    L.full_p2[i] = x2; L.full_p4[i] = x4; L.full_p5[i] = x5;
    int f = i / t, j = i - f * t;
    if (f < 7) {
      int cidx = f < 4 ? (f + 1) * t + j : 5 * t + RP + (f - 4) * t + j;
      L.full_ark[i] = fr_add(x5, K.C(t, cidx));
    }
  }
  for (int r = tid; r < RP; r += nt) {
    fr x = L.part_in[r * t], x2 = fr_sqr(x), x4 = fr_sqr(x2), x5 = fr_mul(x4, x);
    L.part_p2[r] = x2; L.part_p4[r] = x4; L.part_p5[r] = x5;
    L.part_in0[r] = fr_add(x5, K.C(t, 5 * t + r));
  }
  __syncthreads();
  for (int q = tid; q < 7 * t * t; q += nt) {
    int f = q / (t * t), rem = q - f * t * t, i = rem / t, j = rem - i * t;
    fr m = f == 3 ? K.Pm(t, j, i) : K.M(t, j, i);
    L.full_prod[q] = fr_mul(m, L.full_ark[f * t + j]);
  }
  for (int j = tid; j < t; j += nt) L.last_prod[j] = fr_mul(K.M(t, j, 0), L.full_p5[7 * t + j]);
  for (int q = tid; q < RP * t; q += nt) {
    int r = q / t, i = q - r * t;
    fr in = i == 0 ? L.part_in0[r] : L.part_in[r * t + i];
    L.part_prod[q] = fr_mul(K.S(t, (2 * t - 1) * r + i), in);
  }
  __syncthreads();
  // the image is emitted in normal form: convert every element once here rather than every
  // signal at store time (GetSumOfNElements sums are linear, so they are summed in normal form)
  for (int q = tid, n = pos_lds_elems(t); q < n; q += nt) L.base[q] = fr_from_mont(L.base[q]);
  __syncthreads();
}

// GetSumOfNElements(t) block over an LDS product row: out | in[t] | sum[t-1]
__device__ __forceinline__ fr pos_getsum(const fr* prod, int t, int j) {
  if (j == 0 || j > t) {
    int upto = j == 0 ? t - 1 : j - t;  // sum[q] (j = t+1+q) = prod[0..q+1]
    fr acc = prod[0];
    for (int q = 1; q <= upto; q++) acc = fr_add(acc, prod[q]);
    return acc;
  }
  return prod[j - 1];
}

// value (normal form, after pos_lds_fill) of local signal s of the PoseidonHash(n) block
__device__ __forceinline__ fr pos_block_sig(const PosLds& L, int n, uint32_t s) {
  const int t = L.t, RP = L.RP;
  if (s == 0) return *L.hash;
  if (s <= (uint32_t)n) return L.inputs[s - 1];
  s -= 1 + n;
  // PoseidonEx own: out | in[n] | initialState
  if (s == 0) return *L.hash;
  if (s <= (uint32_t)n) return L.inputs[s - 1];
  if (s == (uint32_t)n + 1) return fr_zero();
  s -= 2 + n;
  // ark[0]: out[t] | in[t]
  if (s < (uint32_t)(2 * t)) {
    if (s < (uint32_t)t) return L.full_in[s];
    int j = s - t;
    return j == 0 ? fr_zero() : L.inputs[j - 1];
  }
  s -= 2 * t;
  const uint32_t SIG = 4 * t, ARK = 2 * t, MIX = 2 * t + 2 * t * t;
  auto sigma_sig = [&](int f, uint32_t q) -> fr {  // sigmaF[f][j]: out | in | in2 | in4
    int j = q >> 2, k = q & 3;
    int i = f * t + j;
    return k == 0 ? L.full_p5[i] : k == 1 ? L.full_in[i] : k == 2 ? L.full_p2[i] : L.full_p4[i];
  };
  auto ark_sig = [&](int f, uint32_t q) -> fr {  // ark[f+1]: out[t] | in[t]
    return q < (uint32_t)t ? L.full_ark[f * t + q] : L.full_p5[f * t + q - t];
  };
  auto mix_sig = [&](int f, uint32_t q) -> fr {  // mix: out[t] | in[t] | sum[i] blocks (2t each)
    const fr* nxt = f == 3 ? L.part_in : L.full_in + (f < 3 ? (f + 1) * t : (f + 1) * t);
    if (q < (uint32_t)t) return nxt[q];
    if (q < (uint32_t)(2 * t)) return L.full_ark[f * t + q - t];
    q -= 2 * t;
    int i = q / (2 * t), j = q - i * 2 * t;
    return pos_getsum(L.full_prod + (f * t + i) * t, t, j);
  };
  // three full rounds 0..2: sigmaF[r][*], ark[r+1], mix[r]
  const uint32_t FR = SIG + ARK + MIX;
  if (s < 3 * FR) {
    int r = s / FR; uint32_t q = s - r * FR;
    if (q < SIG) return sigma_sig(r, q);
    q -= SIG;
    if (q < ARK) return ark_sig(r, q);
    return mix_sig(r, q - ARK);
  }
  s -= 3 * FR;
  if (s < FR) {  // round 3 with P
    if (s < SIG) return sigma_sig(3, s);
    s -= SIG;
    if (s < ARK) return ark_sig(3, s);
    return mix_sig(3, s - ARK);
  }
  s -= FR;
  const uint32_t PR = 4 + 4 * t;
  if (s < RP * PR) {  // sigmaP[r] (4) | mixS[r]: out[t] | in[t] | sum (2t)
    int r = s / PR; uint32_t q = s - r * PR;
    if (q < 4) return q == 0 ? L.part_p5[r] : q == 1 ? L.part_in[r * t] : q == 2 ? L.part_p2[r] : L.part_p4[r];
    q -= 4;
    if (q < (uint32_t)t) return L.part_out[r * t + q];
    if (q < (uint32_t)(2 * t)) { int i = q - t; return i == 0 ? L.part_in0[r] : L.part_in[r * t + i]; }
    return pos_getsum(L.part_prod + r * t, t, q - 2 * t);
  }
  s -= RP * PR;
  if (s < 3 * FR) {  // full rounds 4..6 (layers 4..6)
    int r = s / FR; uint32_t q = s - r * FR;
    int f = 4 + r;
    if (q < SIG) return sigma_sig(f, q);
    q -= SIG;
    if (q < ARK) return ark_sig(f, q);
    return mix_sig(f, q - ARK);
  }
  s -= 3 * FR;
  if (s < SIG) return sigma_sig(7, s);
  s -= SIG;
  // mixLast: out | in[t] | sum (2t)
  if (s == 0) return *L.hash;
  if (s <= (uint32_t)t) return L.full_p5[7 * t + s - 1];
  return pos_getsum(L.last_prod, t, s - 1 - t);
}

}  // namespace pzk
