// k_smt_chain4: the SMT chain of SMTVerifier(80) (merkleTree/SMTVerifier.circom:82-107) on quad-spread Fr (fq.hpp).
//
// One SMT proof is a chain of up to 79 dependent PoseidonHash(2) permutations (hasher/poseidon/poseidon.circom:
// 80-209): level i hashes Switcher(child, sibling) into the next child. There are only as many chains as witnesses
// in a call (2,048), so one lane group per witness leaves most of the chip idle and each product's latency sets the
// pace (round 5: 4 lanes per witness, 128 waves per 2,048 witnesses, 29 ms for proofs of depth 1-79). Here a witness
// takes one 16-lane DPP row: quad k (lanes 4k..4k+3) holds state element k of the width-3 permutation spread over its
// four lanes (two words each), quad 3 is the spare. A product is a row-wise CIOS pass over the quad (fq_dot), ~2.5x
// shorter than the one-lane product, and a call gets 4x the waves.
//
// Arithmetic: no value is reduced on the critical path. Every state value is the output of ONE lazily reduced sum of
// products (fq_dot: K + sum_r a_r b_r, one Montgomery reduction), so the round constants, the partial round's
// additions and the mix all fold into the reductions:
//   full round f:  st'_i = sum_k x5_k (x) Mat[k][i] + D_i,   D_i = sum_k Mat[k][i] (x) C[c0(f) + k]
//   partial round: st0' = x^3 (x) (S0 x^2) + st1 (x) S1 + st2 (x) S2 + S0 C
//                  stk' = x^3 (x) (S'k x^2) + stk (x) 1 + S'k C            (x^2 = st0 (x) st0, x^3 = x^2 (x) st0)
// ((x) is the Montgomery product; the constant terms enter as K = c * R mod p, so K * R^-1 = c.) With canonical
// constants every state stays below 2.2p (products of inputs < 2.2p are < 2.0p + the K term; R / p > 5.28), so the
// 256-bit digits never overflow. The level hashes and Switcher outputs leave the kernel canonicalised (two conditional
// subtractions); the round states of the Poseidon core leave as they are (< 2.2p, see pos2_perm_quad).
//
// The constant table (QC_*, Montgomery form, built once per instance by k_qc_build from the reference's constants
// poseidonConstants.circom, as PosConsts holds them) is staged in LDS per workgroup; every lane reads its own 8-byte
// digit of an entry.
#pragma once
#include "core_util.hpp"
#include "fq.hpp"
#include "layout.hpp"
#include "poseidon.hpp"

namespace pzk {

static_assert(QC_RP == pos_rp(3), "width-3 partial rounds");

// One thread per entry (k_qc_build<<<1, 256>>> loops; the layout QC_* is in layout.hpp). Reference constants: hasher/poseidon/poseidonConstants.circom
// (POSEIDON_C / M / P / S for t = 3) through PosConsts.
#ifndef PZK_TEMPLATE_KERNELS_ONLY
__global__ void __launch_bounds__(256) k_qc_build(PosConsts K, fr* qc) {
  constexpr int t = 3, RP = QC_RP;
  const fr R2 = fr_const(R2_);
  auto mont = [&](const fr& x) { return fr_mul(x, R2); };  // x * R: the K whose reduction is x
  for (int e = threadIdx.x; e < QC_SIZE; e += blockDim.x) {
    fr v = fr_zero();
    if (e < QC_FULL) {
      if (e < t) v = K.C(t, e);
    } else if (e < QC_PART) {
      const int f = (e - QC_FULL) / 16, quad = ((e - QC_FULL) % 16) / 4, k = (e - QC_FULL) % 4;
      if (f < 7 && quad < t) {
        const bool p = f == 3;  // full round 3 mixes with P (poseidon.circom:186-200)
        if (k < t) {
          v = p ? K.Pm(t, k, quad) : K.M(t, k, quad);
        } else {
          const int c0 = f < 4 ? (f + 1) * t : 5 * t + RP + (f - 4) * t;
          fr d = fr_zero();
          for (int kk = 0; kk < t; kk++) d = fr_add(d, fr_mul(p ? K.Pm(t, kk, quad) : K.M(t, kk, quad), K.C(t, c0 + kk)));
          v = mont(d);
        }
      } else if (f == 7 && k < t) {
        v = K.M(t, k, 0);  // the hash: sum_k M[k][0] x5_k, the same on every quad
      }
    } else if (e < QC_R2) {
      const int r = (e - QC_PART) / 10, k = (e - QC_PART) % 10, sb = (2 * t - 1) * r;
      switch (k) {
        case QC_P_S0: v = K.S(t, sb); break;
        case QC_P_SP1: v = K.S(t, sb + t); break;
        case QC_P_SP2: v = K.S(t, sb + t + 1); break;
        case QC_P_S1: v = K.S(t, sb + 1); break;
        case QC_P_S2: v = K.S(t, sb + 2); break;
        case QC_P_K0: v = mont(K.SC(t, sb)); break;
        case QC_P_K1: v = mont(K.SC(t, sb + t)); break;
        case QC_P_K2: v = mont(K.SC(t, sb + t + 1)); break;
        case QC_P_ONE: v = fr_mont_one(); break;
        default: break;
      }
    } else {
      v = R2;
    }
    qc[e] = v;
  }
}
#endif

// this lane's digit of table entry e (LDS)
__device__ __forceinline__ fq qc_digit(const fr* qc, int e, int q) {
  const uint2 d = reinterpret_cast<const uint2*>(qc + e)[q];
  return fq{d.x, d.y};
}
__device__ __forceinline__ fq fq_canon2(const fq& a, const QLane& c) { return fq_canon(fq_canon(a, c), c); }
// store this lane's digit of element `a` (8 bytes of the 32-byte element at dst)
__device__ __forceinline__ void fq_store(fr* dst, const fq& a, int q) {
  reinterpret_cast<uint2*>(dst)[q] = make_uint2(a.lo, a.hi);
}
__device__ __forceinline__ fq fq_load(const void* src, int q) {
  const uint2 d = reinterpret_cast<const uint2*>(src)[q];
  return fq{d.x, d.y};
}

// PoseidonHash(2) of the quads' inputs (quad 1: in_1, quad 2: in_2, quads 0 and 3: zero) on one 16-lane row;
// the round states go to out (canonical Montgomery, the k_pos_core layout X0..X3, Y0..Y_RP, Z1..Z3: element
// 3 * round + k), the hash comes back to every quad (canonical Montgomery). quad = this lane's quad in the row.
__device__ __forceinline__ fq pos2_perm_quad(const fr* qc, fq in, fr* out, int quad, const QLane& c) {
  fq st = fq_add_raw(in, qc_digit(qc, QC_INIT + quad, c.q));  // < 2p
  int o = 0;
  // the round states leave as they are, below 2.2p, not canonicalised: their only reader, the Poseidon image fill
  // (pos_img_fill), takes every core value through a FIPS product or a Montgomery -> normal conversion, and both give
  // the canonical result for inputs below 2.2p (fr_mul_fast: < (2.2p * 2.2p + R p) / R < 2p before its final
  // subtraction; fr_from_mont_fast: < p + 1)
  auto store = [&](const fq& v) {
    if (quad < 3) fq_store(out + o + quad, v, c.q);
    o += 3;
  };
  // full round f (f = 7: the hash): x5 = st^5 per quad, then the lazy mix over the three quads' x5
  auto full = [&](int f) {
    const fq x2 = fq_mulq(st, st, c);
    const fq x4 = fq_mulq(x2, x2, c);
    const fq x5 = fq_mulq(x4, st, c);
    const int rec = QC_FULL + 16 * f + 4 * quad;
    const fq b[3] = {qc_digit(qc, rec, c.q), qc_digit(qc, rec + 1, c.q), qc_digit(qc, rec + 2, c.q)};
    st = fq_dot<3>(
        [&](int r, auto J) {
          constexpr int j = decltype(J)::value;
          return r == 0 ? rword<0, j>(x5) : r == 1 ? rword<1, j>(x5) : rword<2, j>(x5);
        },
        b, qc_digit(qc, rec + 3, c.q), c);
  };
  // per-quad table offsets of the partial round's operands (quad 3: zeros; its step-2 operand is st0)
  const int o_b2 = quad == 0 ? QC_P_S0 : quad == 1 ? QC_P_SP1 : QC_P_SP2;
  const int o_r1 = quad == 0 ? QC_P_S1 : quad == 1 ? QC_P_ONE : QC_P_ZERO;
  const int o_r2 = quad == 0 ? QC_P_S2 : quad == 2 ? QC_P_ONE : QC_P_ZERO;
  const int o_k = quad == 0 ? QC_P_K0 : quad == 1 ? QC_P_K1 : quad == 2 ? QC_P_K2 : QC_P_ZERO;
#pragma unroll 1
  for (int f = 0; f < 8; f++) {  // full rounds 0..6 (the partial rounds before round 4), then Z3 and the hash
    if (f == 4) {
#pragma unroll 1
      for (int r = 0; r < QC_RP; r++) {
        store(st);
        const int rec = QC_PART + 10 * r;
        const fq st0 = fq_from_quad<3>(st);  // quad 3 <- quad 0
        // step 1: x^2 (quad 0's)
        const fq b1[1] = {st};
        const fq x2 = fq_dot<1>([&](int, auto J) { return rword<0, decltype(J)::value>(st); }, b1, fq_zero(), c);
        // step 2: quad 0 S0 x^2, quad 1 S'1 x^2, quad 2 S'2 x^2, quad 3 x^3
        const fq b2[1] = {quad == 3 ? st0 : qc_digit(qc, rec + o_b2, c.q)};
        const fq y = fq_dot<1>([&](int, auto J) { return rword<0, decltype(J)::value>(x2); }, b2, fq_zero(), c);
        // step 3: x^3 (quad 3) times the quad's y, plus the st1 / st2 rows and the constant
        const fq b3[3] = {y, qc_digit(qc, rec + o_r1, c.q), qc_digit(qc, rec + o_r2, c.q)};
        st = fq_dot<3>(
            [&](int r3, auto J) {
              constexpr int j = decltype(J)::value;
              return r3 == 0 ? rword<3, j>(y) : r3 == 1 ? rword<1, j>(st) : rword<2, j>(st);
            },
            b3, qc_digit(qc, rec + o_k, c.q), c);
      }
    }
    store(st);  // f = 7: Z3
    full(f);    // f = 7: the hash, on every quad
  }
  return fq_canon2(st, c);
}

// a^(p-2) (the inverse; 0 -> 0) on a quad: fr_inv_sw's 4-bit sliding window, 309 products
__device__ __forceinline__ fq fq_inv(const fq& a, const QLane& c) {
  static constexpr uint8_t SQ[49] = {7, 3, 7, 2, 5, 6, 1, 8, 1, 7, 10, 6, 2, 7, 6, 7, 5, 3, 8, 9, 3, 8, 3, 5, 7,
                                     6, 3, 8, 8, 6, 2, 6, 1, 8, 6, 8, 1, 8, 3, 3, 6, 4, 5, 4, 4, 4, 4, 4, 4};
  static constexpr uint8_t WV[49] = {3, 1, 9, 3, 7, 11, 1, 9, 1, 13, 5, 13, 3, 5, 1, 11, 13, 5, 3, 5, 3, 11, 5, 5, 3,
                                     15, 5, 9, 15, 13, 3, 11, 1, 9, 5, 15, 1, 15, 5, 3, 9, 15, 15, 15, 15, 15, 15, 15, 15};
  const fq a2 = fq_mulq(a, a, c);
  const fq t3 = fq_mulq(a, a2, c), t5 = fq_mulq(t3, a2, c), t7 = fq_mulq(t5, a2, c), t9 = fq_mulq(t7, a2, c),
           t11 = fq_mulq(t9, a2, c), t13 = fq_mulq(t11, a2, c), t15 = fq_mulq(t13, a2, c);
  fq r = t3;
#pragma unroll 1
  for (int s = 0; s < 49; s++) {
#pragma unroll 1
    for (int q = 0; q < SQ[s]; q++) r = fq_mulq(r, r, c);
    const int v = WV[s];
    auto pick = [&](uint32_t x1, uint32_t x3, uint32_t x5, uint32_t x7, uint32_t x9, uint32_t x11, uint32_t x13,
                    uint32_t x15) {
      return (x1 & (0u - (uint32_t)(v == 1))) | (x3 & (0u - (uint32_t)(v == 3))) | (x5 & (0u - (uint32_t)(v == 5))) |
             (x7 & (0u - (uint32_t)(v == 7))) | (x9 & (0u - (uint32_t)(v == 9))) | (x11 & (0u - (uint32_t)(v == 11))) |
             (x13 & (0u - (uint32_t)(v == 13))) | (x15 & (0u - (uint32_t)(v == 15)));
    };
    const fq t{pick(a.lo, t3.lo, t5.lo, t7.lo, t9.lo, t11.lo, t13.lo, t15.lo),
               pick(a.hi, t3.hi, t5.hi, t7.hi, t9.hi, t11.hi, t13.hi, t15.hi)};
    r = fq_mulq(r, t, c);
  }
  return r;
}

// The SMT chain of a call (the levels below each proof's insertion level, from the top down), then every level's
// root and the isEqual inverse of root_0 (SMTVerifier.circom:104-106, 112-119). 16 lanes per witness, 16 witnesses
// per 256-thread workgroup; witness groups take proofs in k_smt_order's depth order, so a wave's four proofs have
// (nearly) one depth. Outputs as k_smt_chain (regcore.hpp): the Switcher L / R and level hashes in the value store,
// the permutations' round states in the Poseidon core, roots and the inverse in the SMT core.
#ifndef PZK_TEMPLATE_KERNELS_ONLY  // defined once, in kernels.hip
__global__ void __launch_bounds__(256) k_smt_chain4(DevLayout L, PosConsts K, const int32_t* level_task,
                                                    const uint8_t* inputs, ValueStore vs, fr* pos_core, fr* smt_core,
                                                    const uint32_t* order, int32_t* status, uint32_t batch) {
  core_priority();
  constexpr int GW = 16, NGW = 256 / GW;
  __shared__ fr qc[QC_SIZE];
  __shared__ uint8_t lrs[NGW][SMT_LEVELS];
  __shared__ int32_t lv_core[SMT_LEVELS];
  for (int i = threadIdx.x; i < QC_SIZE; i += blockDim.x) qc[i] = K.qc[i];
  for (int i = threadIdx.x; i < SMT_LEVELS; i += blockDim.x) lv_core[i] = L.pos[level_task[i]].core_off;
  const uint32_t g = (blockIdx.x * blockDim.x + threadIdx.x) / GW;
  const int gi = (int)(threadIdx.x / GW), lq = (int)(threadIdx.x % GW), quad = lq >> 2;
  const bool live = g < batch;  // whole witness rows only; every thread takes part in the barrier
  const uint32_t w = live ? (order ? order[g] : g) : 0;
  const RegInfo& R = L.reg;
  const uint8_t* row = inputs + 32ull * (uint64_t)w * L.n_inputs;
  fr* core = smt_core + (size_t)w * L.smt_core_fr;
  const uint32_t* flags = reinterpret_cast<const uint32_t*>(core + 2 * SMT_LEVELS);
  const int jins = live ? (int)reinterpret_cast<const uint32_t*>(core + 3 * SMT_LEVELS)[0] : 0;
  const int top = jins < SMT_LEVELS ? jins : SMT_LEVELS;
  for (int i = lq; i < top; i += GW) lrs[gi][i] = (uint8_t)((flags[i] >> 4) & 1);
  __syncthreads();
  if (!live) return;
  const QLane c = QLane::make();
  fr* roots = core + SMT_LEVELS;
  const fq leaf = fq_load(&vs.at(R.v_leaf, w), c.q);
  fq child = leaf;  // root_j = leaf
  fr* pcore = pos_core + (size_t)w * L.pos_core_elems;
  const uint8_t* sib_row = row + 32ull * R.in_br;
  const fq r2 = qc_digit(qc, QC_R2, c.q);
  // the sibling in Montgomery form (canonical, every quad): sib (normal) (x) R^2
  auto to_mont = [&](const fq& raw) { return fq_canon2(fq_mulq(raw, r2, c), c); };
  fq sib = top > 0 ? to_mont(fq_load(sib_row + 32ull * (top - 1), c.q)) : fq_zero();
#pragma unroll 1
  for (int i = top - 1; i >= 0; i--) {
    const fq sib_next = i > 0 ? fq_load(sib_row + 32ull * (i - 1), c.q) : fq_zero();  // before this level's stores
    const bool lr = lrs[gi][i] != 0;
    const fq lv = lr ? sib : child, rv = lr ? child : sib;  // Switcher (SMTVerifier.circom): the level's L / R
    if (quad == 1) fq_store(&vs.at(R.v_smt_lr + 2 * i, w), lv, c.q);
    if (quad == 2) fq_store(&vs.at(R.v_smt_lr + 2 * i + 1, w), rv, c.q);
    child = pos2_perm_quad(qc, quad == 1 ? lv : quad == 2 ? rv : fq_zero(), pcore + lv_core[i], quad, c);
    if (quad == 0) {
      fq_store(&vs.at(R.v_smt_h + i, w), child, c.q);  // root_i = H_i (st_top = 1 below j)
      fq_store(roots + i, child, c.q);
    }
    if (i > 0) sib = to_mont(sib_next);
  }
  // roots of the levels at and above the insertion level: root_i = st_top_i * H_i + st_inew_i * leaf (those H_i are
  // the zero-child level hashes of k_pos_core1, written by an earlier kernel)
  const fr leaf_f = vs.at(R.v_leaf, w);
  for (int i = top + lq; i < SMT_LEVELS; i += GW) {
    const uint32_t f = flags[i];
    fr r = fr_zero();
    if (f & 4) r = vs.at(R.v_smt_h + i, w);
    if (f & 8) r = fr_add(r, leaf_f);
    roots[i] = r;
  }
  // isEqual(root_0, root): inverse of root - root_0
  fr root0;
  if (top > 0) {
    root0 = fq_gather(child);
  } else {
    const uint32_t f = flags[0];
    root0 = fr_zero();
    if (f & 4) root0 = vs.at(R.v_smt_h, w);
    if (f & 8) root0 = fr_add(root0, leaf_f);
  }
  const fr rin = fq_gather(to_mont(fq_load(row + 32ull * R.in_root, c.q)));
  const fr dlt = fr_sub(rin, root0);
  const fq inv = fq_canon2(fq_inv(fq_digit(dlt, c.q), c), c);
  if (quad == 0) fq_store(core + 3 * SMT_LEVELS + 1, inv, c.q);
  // smtVerifier.isVerified === 1 where the circuit asserts it (identityStateVerifier.circom:46; the register
  // circuit leaves it commented out, passportVerificationBuilder.circom:240)
  if (lq == 0 && R.smt_check && !fr_is_zero(dlt)) set_status(status ? status + w : nullptr, ST_ISV_ROOT);
}
#endif

}  // namespace pzk
