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

// PoseidonHash(n) of all-zero inputs is one constant block per width (the SMT levels below a proof's insertion
// level hash Switcher(0, 0), merkleTree/SMTVerifier.circom:104-106): per t, its image in pos_img_fill's layout
// (normal form) followed by the hash (Montgomery), computed once per instance (k_pos_zero_img)
__host__ __device__ constexpr uint32_t pos_zimg_off(int t) {
  uint32_t o = 0;
  for (int u = 2; u < t; u++) o += (uint32_t)PosImg(u).size + 1;
  return o;
}
constexpr uint32_t POS_ZIMG_TOTAL = pos_zimg_off(POS_MAX_T + 1);
// ... followed by the zero-input blocks themselves in the O0 signal order (the image permuted by the width's block
// program, pos_prog.hpp; built on the host at instance creation): a zero block of an O0 layout is a plain copy
__host__ __device__ constexpr uint32_t pos_zrow_off(int t) {
  uint32_t o = POS_ZIMG_TOTAL;
  for (int u = 2; u < t; u++) o += pos_hash_size_c(u - 1);
  return o;
}
constexpr uint32_t POS_ZBUF_TOTAL = pos_zrow_off(POS_MAX_T + 1);

struct PosConsts {
  const fr* base;   // Montgomery-form constants
  const fr* nbase;  // the same constants in normal form
  PosParamIndex ix;
  const fr* sbase;  // partial-round products S[i] * C[5t + r] (Montgomery) at S's indices (k_pos_sc, runtime.cpp)
  const fr* zimg;   // zero-input images and hashes (pos_zimg_off)
  const fr* qc;     // the quad SMT chain's constant table (smt_chain4.hpp, QC_SIZE entries)
  __device__ __forceinline__ const fr* Zimg(int t) const { return zimg + pos_zimg_off(t); }
  __device__ __forceinline__ const fr& Zhash(int t) const { return zimg[pos_zimg_off(t) + PosImg(t).size]; }
  __device__ __forceinline__ const fr* Zrow(int t) const { return zimg + pos_zrow_off(t); }
  __device__ __forceinline__ const fr& SC(int t, int i) const { return sbase[ix.s_off[t] + i]; }
  __device__ __forceinline__ const fr& Cn(int t, int i) const { return nbase[ix.c_off[t] + i]; }
  __device__ __forceinline__ const fr& C(int t, int i) const { return base[ix.c_off[t] + i]; }
  __device__ __forceinline__ const fr& M(int t, int i, int j) const { return base[ix.m_off[t] + i * t + j]; }
  __device__ __forceinline__ const fr& Pm(int t, int i, int j) const { return base[ix.p_off[t] + i * t + j]; }
  __device__ __forceinline__ const fr& S(int t, int i) const { return base[ix.s_off[t] + i]; }
  __device__ __forceinline__ const fr& Sn(int t, int i) const { return nbase[ix.s_off[t] + i]; }
};

__device__ __forceinline__ fr pow5(const fr& x) { fr x2 = fr_sqr(x), x4 = fr_sqr(x2); return fr_mul(x4, x); }

// value store: SoA [slot][witness], Montgomery form
struct ValueStore {
  fr* v;
  uint32_t batch;
  __device__ __forceinline__ fr& at(int slot, uint32_t w) const { return v[(size_t)slot * batch + w]; }
};

// every input of the task is 0 (Montgomery 0 = 0): the permutation is the constant zero-input one (PosConsts.Zimg)
__device__ __forceinline__ bool pos_inputs_zero(const PosTask& task, const ValueStore& vs, uint32_t w) {
  uint32_t acc = 0;
  for (int k = 0; k < task.n; k++) {
    const fr& v = vs.at(task.in_slot[k], w);
#pragma unroll
    for (int i = 0; i < 8; i++) acc |= v.v[i];
  }
  return acc == 0;
}

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

// The constants of one width T staged in LDS, with PosConsts' accessors (t fixed): k_smt_chain reads them every
// round of every level, and from LDS those reads never wait for the round-state stores in flight (a global load
// issued after a store waits for it: gfx9 vmcnt counts both).
template <int T>
struct PosConstsLds {
  static constexpr int RP = pos_rp(T), NC = RP + 8 * T, NM = T * T, NS = (2 * T - 1) * RP;
  static constexpr int SIZE = NC + 2 * NM + 2 * NS;  // C | M | P | S | S * C
  const fr* c;
  __device__ __forceinline__ const fr& C(int, int i) const { return c[i]; }
  __device__ __forceinline__ const fr& M(int, int i, int j) const { return c[NC + i * T + j]; }
  __device__ __forceinline__ const fr& Pm(int, int i, int j) const { return c[NC + NM + i * T + j]; }
  __device__ __forceinline__ const fr& S(int, int i) const { return c[NC + 2 * NM + i]; }
  __device__ __forceinline__ const fr& SC(int, int i) const { return c[NC + 2 * NM + NS + i]; }
  // every thread of the workgroup; the caller syncs before use
  __device__ static void stage(fr* lds, const PosConsts& K) {
    for (int i = threadIdx.x; i < SIZE; i += blockDim.x) {
      const fr* src = i < NC ? K.base + K.ix.c_off[T] + i
                    : i < NC + NM ? K.base + K.ix.m_off[T] + (i - NC)
                    : i < NC + 2 * NM ? K.base + K.ix.p_off[T] + (i - NC - NM)
                    : i < NC + 2 * NM + NS ? K.base + K.ix.s_off[T] + (i - NC - 2 * NM)
                                           : K.sbase + K.ix.s_off[T] + (i - NC - 2 * NM - NS);
      lds[i] = *src;
    }
  }
};

// Cooperative permutation: G lanes per (witness, task), lane j < t holds state element j; returns
// the hash to every lane of the group
// (G = 4 for t <= 4, 8 otherwise; the lanes j >= t carry zeros). A full round is one S-box per
// lane and a t-term mix gathered with shuffles; a partial round is lane 0's S-box, one product
// per lane and a butterfly sum. Same core output as pos_core_lane (Montgomery layer states,
// X0..X3, Y0..Y_RP, Z1..Z3), written by the owning lanes. ~3.5x shorter dependency chain than
// one lane per permutation and ~70 VGPRs instead of 256, so the kernel can be placed next to
// the emitters.
// Product policies of the cooperative permutation: inline (the Poseidon cores) or out of line (k_smt_chain: one
// copy of each product in the level loop, whose code then stays in the instruction cache it shares with the
// emitter kernels on the same CUs)
struct FrMulInline {
  __device__ static __forceinline__ fr mul(const fr& a, const fr& b) { return fr_mul(a, b); }
  __device__ static __forceinline__ fr sqr(const fr& a) { return fr_sqr(a); }
};
__device__ __attribute__((noinline)) static fr fr_mul_ool(fr a, fr b) { return fr_mul(a, b); }
__device__ __attribute__((noinline)) static fr fr_sqr_ool(fr a) { return fr_sqr(a); }
struct FrMulCall {
  __device__ static __forceinline__ fr mul(const fr& a, const fr& b) { return fr_mul_ool(a, b); }
  __device__ static __forceinline__ fr sqr(const fr& a) { return fr_sqr_ool(a); }
};
// FIPS products (fr.hpp fr_mul_fast: the throughput product, 1,200 vs 1,560 cycles per wave64 product)
struct FrMulFips {
  __device__ static __forceinline__ fr mul(const fr& a, const fr& b) { return fr_mul_fast(a, b); }
  __device__ static __forceinline__ fr sqr(const fr& a) { return fr_mul_fast(a, a); }
};
template <class PM>
__device__ __forceinline__ fr pow5p(const fr& x) { fr x2 = PM::sqr(x), x4 = PM::sqr(x2); return PM::mul(x4, x); }

// The cooperative permutation itself: lane j < t enters with its input (lane 0: 0), the round states go to out
// (this task's core slice), every lane of the group gets the hash (Montgomery).
template <int T, int G, class KC, class PM = FrMulInline>
__device__ __forceinline__ fr pos_perm_group(const KC& K, fr st, fr* out, int j) {
  constexpr int t = T;
  const int RP = pos_nrp(t);
  const bool act = j < t;
  const int jj = act ? j : 0;
  if (act) st = fr_add(st, K.C(t, j));
  else st = fr_zero();
  const int lane = threadIdx.x & 63, gb = lane & ~(G - 1);
  auto mix = [&](const fr& x, bool use_p) -> fr {  // sum_k Mat[k][j] * x_k
    fr acc = fr_zero();
#pragma unroll
    for (int k = 0; k < t; k++) {
      fr xk = fr_shfl(x, gb + k, 64);
      acc = fr_add(acc, PM::mul(use_p ? K.Pm(t, k, jj) : K.M(t, k, jj), xk));
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
  // One loop over the 7 full rounds with the partial rounds in front of full round 4, none unrolled: each round
  // body exists once in the code (two full-round copies made k_smt_chain's level loop ~9,000 instructions, more
  // than the instruction cache holds beside the emitters' code).
  int o = 0;
#pragma unroll 1
  for (int f = 0; f < 7; f++) {
    if (f == 4) {
#pragma unroll 1
      for (int r = 0; r < RP; r++) {  // partial rounds
        if (act) out[o + j] = st;
        o += t;
        const int sb = (2 * t - 1) * r;
        if constexpr (G > T) {
          // 3 product times per round, with the group's spare lane t: s0 = x^5 + C with x = st_0, and
          //   lane 0:   st_0' = S[0] s0 + sum_k S[k] st_k      (S[0] s0 = x^3 (S[0] x^2) + S[0] C)
          //   lane k:   st_k' = st_k + S'[k] s0                (S'[k] s0 = x^3 (S'[k] x^2) + S'[k] C)
          // A: lane 0 x^2, lanes k their terms S[k] st_k | B: lane 0 x^3, lanes k S'[k] x^2, lane t S[0] x^2 |
          // C: every lane x^3 times its B product. The S * C constants come precomputed (K.SC).
          const fr a = PM::mul(j == 0 ? st : K.S(t, sb + jj), st);
          const fr x2 = fr_shfl(a, gb, 64);
          const fr b = PM::mul(j == 0 ? st : act ? K.S(t, sb + t + jj - 1) : K.S(t, sb), x2);
          const fr x3 = fr_shfl(b, gb, 64), s0x2 = fr_shfl(b, gb + t, 64);
          const fr c = PM::mul(x3, j == 0 ? s0x2 : b);
          const fr sum = group_sum(j == 0 ? fr_add(c, K.SC(t, sb)) : act ? a : fr_zero());
          if (j == 0) st = sum;
          else if (act) st = fr_add(st, fr_add(c, K.SC(t, sb + t + jj - 1)));
        } else {
          // 4 product times (no spare lane: t = 4 on 4 lanes): one product on every lane: lane 0 squares its state
          // (the S-box's first step), lanes 1..t-1 take their sparse-matrix terms S[k] * st_k
          const fr p = PM::mul(j == 0 ? st : K.S(t, sb + jj), st);
          fr s0 = fr_zero();
          if (j == 0) s0 = fr_add(PM::mul(PM::sqr(p), st), K.C(t, 5 * t + r));
          s0 = fr_shfl(s0, gb, 64);
          // one product on every lane: lane 0's term S[0] * s0, the others' updates s0 * S'[k]
          const fr q = PM::mul(j == 0 ? K.S(t, sb) : K.S(t, sb + t + jj - 1), s0);
          const fr sum = group_sum(j == 0 ? q : act ? p : fr_zero());
          if (j == 0) st = sum;
          else if (act) st = fr_add(st, q);
        }
      }
    }
    if (act) out[o + j] = st;  // full round f (round 3 mixes with P)
    o += t;
    const int c0 = f < 4 ? (f + 1) * t : 5 * t + RP + (f - 4) * t;
    fr a = act ? fr_add(pow5p<PM>(st), K.C(t, c0 + jj)) : fr_zero();
    st = mix(a, f == 3);
  }
  if (act) out[o + j] = st;  // Z3
  return group_sum(act ? PM::mul(K.M(t, jj, 0), pow5p<PM>(st)) : fr_zero());  // every lane of the group: the hash
}

// The product of the narrow-level Poseidon cores and the BabyJubJub core (round 6): FIPS, the throughput product —
// the lines those cores sit on are VALU-bound; -DPZK_CORE_CIOS builds the latency product (A/B).
#ifdef PZK_CORE_CIOS
using CoreMul = FrMulInline;
#else
using CoreMul = FrMulFips;
#endif

template <int T, int G>
__device__ __forceinline__ fr pos_core_group(const PosConsts& K, const PosTask& task, const ValueStore& vs, uint32_t w,
                                               fr* core /* this witness's Poseidon core */, int j) {
  fr in = fr_zero();
  if (j > 0 && j < T) in = vs.at(task.in_slot[j - 1], w);
  const fr h = pos_perm_group<T, G, PosConsts, CoreMul>(K, in, core + task.core_off, j);
  if (j == 0) vs.at(task.out_slot, w) = h;
  return h;  // every lane of the group holds the hash (Montgomery)
}

// ------------------------------------------------------------------------------ emit
// Image fill (pos_prog.hpp layout, normal form). Mixed forms give normal-form results straight from the FIPS product:
// mont_mul(aR, b) = ab, so a Montgomery core value times a normal-form constant (or the reverse) is a normal-form
// product. The work: NS = 8t + RP S-box chains (x^2 = sqr(xR) -> x^2 = from_mont(x^2 R) -> x^4 = (x^2 R) x^2 ->
// x^5 = x^4 (xR), + the Ark constant), NA = RP (t-1) partial-round products S * Y_r[k] (k >= 1, from the core, no
// dependency), the format conversions (S-box inputs, the other partial-round states, hash inputs / output), and the
// GetSum products that need an S-box output (full mixes, mixLast, the partial rounds' k = 0 term).
// Scheduled so that every wave runs ONE operation per step on all its lanes: thread q < NS keeps S-box q's chain
// in registers across steps 1-4, and the lanes of a step beyond NS take independent products (steps 1, 3, 4) or
// conversions (step 2), with operands and destinations selected per lane around a single product call. (The
// previous fill gave each lane one S-box chain OR one conversion in a branchy loop: waves holding both ran both, and
// the 81 S-box chains of t = 3 occupied two waves for 4 product times while the others idled: 14.5 product-times
// of wave work per block against 10.5 here.)
// Image parts a block's stored signals may need beyond the S-box powers x^2, x^4, x^5 and the Ark outputs, which are
// always filled: a mapped block (a .sym layout) fills only those its kept signals read (pos_img_need)
template <int T>
__device__ __forceinline__ uint32_t pos_img_need(uint32_t d) { return pos_img_need_t(T, d); }

// core: the permutation's round states in Montgomery form, canonical (k_pos_core, k_pos_core1) or below 2.2p
// (k_smt_chain4): every core value read here goes through fr_mul_fast or fr_from_mont_fast, whose results are
// canonical for such inputs.
template <int T>
__device__ __forceinline__ void pos_img_fill(fr* img, const PosConsts& K, const fr* core, const ValueStore& vs,
                                             const PosTask& task, uint32_t w, uint32_t need = PI_ALL) {
  constexpr int t = T;
  constexpr PosImg I(T);
  constexpr int RP = I.rp;
  // core order: X0..X3 (4t), Y0..Y_RP ((RP+1)t), Z1..Z3 (3t), all Montgomery
  constexpr int NS = 8 * t + RP, NA = RP * (t - 1), NC = RP * (t - 1) + t, NF = NS + NC + 7;
  constexpr int PAD = (NS + 63) / 64 * 64 - NS;  // lanes left in the S-box waves of a product step
  constexpr int A1 = NA < PAD ? NA : PAD, A3 = NA - A1 < PAD ? NA - A1 : PAD, A4 = NA - A1 - A3;
  static_assert(NS <= 256, "one S-box chain per thread of a 256-thread workgroup");
  const int tid = threadIdx.x, nt = blockDim.x;
  // S-box q: core index, image slots of x, x^2, x^4, x^5 and of the Ark output (-1: none), its Ark constant index
  auto sbox = [&](int q, int& ci, int& din, int& d2, int& d4, int& d5, int& dark, int& cidx) {
    if (q < 8 * t) {
      const int f = q / t, j = q - f * t;
      ci = f < 4 ? f * t + j : f == 4 ? 4 * t + RP * t + j : 4 * t + (RP + 1) * t + (f - 5) * t + j;
      din = I.in + q; d2 = I.p2 + q; d4 = I.p4 + q; d5 = I.p5 + q;
      dark = f < 7 ? I.ark + q : -1;
      cidx = f < 4 ? (f + 1) * t + j : 5 * t + RP + (f - 4) * t + j;
    } else {
      const int r = q - 8 * t;
      ci = 4 * t + r * t;
      din = I.pin + r * t; d2 = I.pp2 + r; d4 = I.pp4 + r; d5 = I.pp5 + r;
      dark = I.pin0 + r;
      cidx = 5 * t + r;
    }
  };
  // independent product a: S[(2t-1) r + k] * Y_r[k] (k >= 1) -> the row's prefix-sum slot and its product slot
  auto aprod = [&](int a, fr& x, fr& y, int& d1, int& d2) {
    const int r = a / (t - 1), k = 1 + (a - r * (t - 1));
    x = K.Sn(t, (2 * t - 1) * r + k);
    y = core[4 * t + r * t + k];
    d1 = I.ps + r * t + k;
    d2 = I.prod(7 * t + 1 + r, k);
  };
  const bool chain = tid < NS;
  int ci = 0, din = 0, d2 = 0, d4 = 0, d5 = 0, dark = -1, cidx = 0;
  if (chain) sbox(tid, ci, din, d2, d4, d5, dark, cidx);
  fr xm = chain ? core[ci] : fr_zero(), x2m = xm, x2 = xm, x4 = xm;
  const bool mix = need & PI_MIX;
  // step 1 (product): x^2 R = sqr(x R) | independent products [0, A1)
  for (int q = tid; q < NS + (mix ? A1 : 0); q += nt) {
    fr x = xm, y = xm;
    int e1 = -1, e2 = -1;
    if (q >= NS) aprod(q - NS, x, y, e1, e2);
    const fr r = fr_mul_fast(x, y);
    if (q < NS) x2m = r;
    else { img[e1] = r; img[e2] = r; }
  }
  // step 2 (conversion): x^2 | S-box inputs, partial-round states, hash inputs / output, zero (the parts asked for).
  // With the GetSum rows built, an S-box input other than layers 0 and 4 is the previous mix's output — its row's
  // last prefix sum — and is copied from there at the end (a copy instead of a conversion: 77 of t = 3's 81)
  const bool nx = need & PI_X, nst = need & PI_ST, nmisc = need & PI_MISC;
  const int NXC = nx ? (mix ? 2 * t : NS) : 0;
  for (int q = tid; q < NS + NXC + (nst ? NC : 0) + (nmisc ? NF - NS - NC : 0); q += nt) {
    fr x = x2m;
    int e = q < NS ? d2 : -1;
    if (q >= NS) {
      int f = q - NS;
      if (f < NXC) {  // S-box input x (mix: layers 0 and 4 only)
        int c_, i_, a_, b_, g_, h_, k_;
        sbox(mix ? (f < t ? f : 3 * t + f) : f, c_, i_, a_, b_, g_, h_, k_);
        x = core[c_]; e = i_;
        f = -1;
      } else {
        f -= NXC;
        if (!nst) f += NC;
      }
      if (f < 0) {
      } else if (f < NC) {
        const int c = f;
        int r, i;
        if (c < RP * (t - 1)) { r = c / (t - 1); i = 1 + (c - r * (t - 1)); }
        else { r = RP; i = c - RP * (t - 1); }
        x = core[4 * t + r * t + i]; e = I.pin + r * t + i;
      } else {
        const int k = f - NC;
        x = fr_zero();
        if (k < task.n) { x = vs.at(task.in_slot[k], w); e = I.inp + k; }
        else if (k == 5) { x = vs.at(task.out_slot, w); e = I.hash; }
        else if (k == 6) e = I.zero;  // from_mont(0) = 0
      }
    }
    const fr r = fr_from_mont_fast(x);
    if (q < NS) x2 = r;
    if (e >= 0) img[e] = r;
  }
  // step 3 (product): x^4 = (x^2 R) x^2 | independent products [A1, A1 + A3)
  for (int q = tid; q < NS + (mix ? A3 : 0); q += nt) {
    fr x = x2m, y = x2;
    int e1 = d4, e2 = -1;
    if (q >= NS) aprod(A1 + q - NS, x, y, e1, e2);
    const fr r = fr_mul_fast(x, y);
    if (q < NS) x4 = r;
    img[e1] = r;
    if (e2 >= 0) img[e2] = r;
  }
  // step 4 (product): x^5 = x^4 (x R), Ark output | independent products [A1 + A3, NA)
  for (int q = tid; q < NS + (mix ? A4 : 0); q += nt) {
    fr x = x4, y = xm;
    int e1 = d5, e2 = -1;
    if (q >= NS) aprod(A1 + A3 + q - NS, x, y, e1, e2);
    const fr r = fr_mul_fast(x, y);
    img[e1] = r;
    if (e2 >= 0) img[e2] = r;
    if (q < NS && dark >= 0) img[dark] = fr_add(r, K.Cn(t, cidx));
  }
  __syncthreads();
  if (!mix) return;
  // step 5 (product): the GetSum terms of an S-box output (full mix f, output i: Mat_f[k][i] * ark[f][k]; mixLast:
  // M[k][0] * x5[7][k]; partial r, k = 0: S[(2t-1) r] * (S-box output + Ark))
  constexpr int NFR = 7 * t;
  for (int q = tid; q < NFR * t + t + RP; q += nt) {
    fr c, v;
    int e1, e2 = -1;
    if (q < NFR * t) {
      const int row = q / t, k = q - row * t, f = row / t, i = row - f * t;
      c = f == 3 ? K.Pm(t, k, i) : K.M(t, k, i);
      v = img[I.ark + f * t + k];
      e1 = I.fs + row * t + k;
      if (k) e2 = I.prod(row, k);
    } else if (q < NFR * t + t) {
      const int k = q - NFR * t;
      c = K.M(t, k, 0);
      v = img[I.p5 + 7 * t + k];
      e1 = I.ls + k;
      if (k) e2 = I.prod(NFR, k);
    } else {
      const int r = q - NFR * t - t;
      c = K.S(t, (2 * t - 1) * r);
      v = img[I.pin0 + r];
      e1 = I.ps + r * t;
    }
    const fr pr = fr_mul_fast(c, v);
    img[e1] = pr;
    if (e2 >= 0) img[e2] = pr;
  }
  __syncthreads();
  // prefix sums along each row (7t full, mixLast, RP partial)
  constexpr int NR = NFR + 1 + RP;
  for (int row = tid; row < NR; row += nt) {
    const int base = row < NFR ? I.fs + row * t : row == NFR ? I.ls : I.ps + (row - NFR - 1) * t;
    fr acc = img[base];
#pragma unroll
    for (int k = 1; k < t; k++) { acc = fr_add(acc, img[base + k]); img[base + k] = acc; }
  }
  __syncthreads();
  if (!nx) return;
  // the S-box inputs of full layers 1-3, 5-7 (the mix after layer f - 1, full row (f - 1, j)) and of the partial
  // rounds (round 0: the P mix after layer 3, full row (3, 0); round r: the partial mix of round r - 1)
  for (int q = tid; q < NS; q += nt) {
    int src = -1, dst;
    if (q < 8 * t) {
      const int f = q / t, j = q - f * t;
      if (f != 0 && f != 4) src = I.fs + ((f - 1) * t + j) * t + t - 1;
      dst = I.in + q;
    } else {
      const int r = q - 8 * t;
      src = r == 0 ? I.fs + (3 * t) * t + t - 1 : I.ps + (r - 1) * t + t - 1;
      dst = I.pin + r * t;
    }
    if (src >= 0) img[dst] = img[src];
  }
  __syncthreads();
}

}  // namespace pzk
