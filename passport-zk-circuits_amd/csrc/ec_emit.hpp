// Closed-form ECDSA regions emitted by the packed generic emitter (E_GENR, after k_ec_core):
// the selection logic of the two scalar multiplications (ec/curve.circom:356-494, 672-906) —
// Num2Bits / Bits2Num of the scalars, the IsEqual / GetSumOfNElements window selections, the
// dummy tests and switchers — read from the EC core (forwarded affine points, op records, the
// batch-inverted IsEqual differences).
#pragma once
#include "bufs.hpp"
#include "ec_common.hpp"
#include "fr.hpp"
#include "layout.hpp"

namespace pzk {

__device__ __forceinline__ uint64_t u64_mask(uint64_t v, int nb) { return nb >= 64 ? v : (v & ((1ull << nb) - 1ull)); }
// 4-limb integer: bit i / low nb bits (as an element)
__device__ __forceinline__ uint32_t limbs_bit(const uint64_t* x, int i) { return (uint32_t)((x[i >> 6] >> (i & 63)) & 1ull); }
__device__ __forceinline__ El limbs_mask(const uint64_t* x, int nb) {
  uint64_t m[4];
#pragma unroll
  for (int k = 0; k < 4; k++) m[k] = nb >= 64 * (k + 1) ? x[k] : nb <= 64 * k ? 0ull : u64_mask(x[k], nb - 64 * k);
  return El{make_uint4((uint32_t)m[0], (uint32_t)(m[0] >> 32), (uint32_t)m[1], (uint32_t)(m[1] >> 32)),
            make_uint4((uint32_t)m[2], (uint32_t)(m[2] >> 32), (uint32_t)m[3], (uint32_t)(m[3] >> 32))};
}
// Fr (normal form) of a - b, a, b < 2^64
__device__ __forceinline__ fr fr_sdiff(uint64_t a, uint64_t b) {
  return a >= b ? fr_u64(a - b) : fr_sub(fr_zero(), fr_u64(b - a));
}
// 1/d for a small signed d (|d| < 256); 0 -> 0
__device__ __forceinline__ fr inv_small_signed(const fr* T, int d) {
  if (d == 0) return fr_zero();
  return d > 0 ? T[d] : fr_sub(fr_zero(), T[-d]);
}
__device__ __forceinline__ fr fr_small_signed(int d) { return d >= 0 ? fr_u64((uint64_t)d) : fr_sub(fr_zero(), fr_u64((uint64_t)(-d))); }

// IsEqual (comparators.circom:24-33) block signal e: out | in[2] | IsZero(out, in = in1 - in0, inv)
__device__ __forceinline__ El iseq_sig(int e, uint64_t in0, uint64_t in1, const fr& inv) {
  const uint64_t eq = in0 == in1;
  switch (e) {
    case 0: case 3: return el_u64(eq);
    case 1: return el_u64(in0);
    case 2: return el_u64(in1);
    case 4: return el_fr(fr_sdiff(in1, in0));
    default: return el_fr(inv);
  }
}
// Switcher (switcher.circom:16-26) signal e: out[2] | bool, in[2] | aux = (in1 - in0) * bool
__device__ __forceinline__ El switcher_sig(int e, uint64_t bl, uint64_t in0, uint64_t in1) {
  switch (e) {
    case 0: return el_u64(bl ? in1 : in0);
    case 1: return el_u64(bl ? in0 : in1);
    case 2: return el_u64(bl);
    case 3: return el_u64(in0);
    case 4: return el_u64(in1);
    default: {
      fr d = fr_sdiff(in1, in0);
      return el_fr(bl == 0 ? fr_zero() : bl == 1 ? d : fr_add(d, d));
    }
  }
}

__device__ El ec_small(const DevLayout& L, const Bufs& B, const Region& R, uint32_t w, uint32_t s) {
  const uint64_t* C = B.ec_core + (size_t)w * EC_CORE_WORDS;
  const fr* I = B.ec_inv + (size_t)w * EC_N_INV;
  const uint8_t* row = B.inputs + 32ull * (uint64_t)w * L.n_inputs;
  auto rec_out = [&](int op) { return C + ECC_REC + ECC_REC_WORDS * op + 16; };
  const int cv = L.reg.ec_curve;  // this TU is curve-generic: constants by run-time curve id
  switch (R.kind) {
    case RK_EC_U64: return el_u64(C[R.a[0] + s]);
    case RK_EC_CONST: return el_u64(ec_k(cv, R.a[0], (int)s));
    case RK_EC_GM_RCC: {  // resultCoordinateComputation[i][j][a][k] = equal[i][j] * point  (curve.circom:724-749)
      const uint32_t i = s >> 11, j = (s >> 3) & 255u, q = s & 7u;
      const uint32_t b = (uint32_t)((C[ECC_U1 + (i >> 3)] >> (8 * (i & 7))) & 255);
      return el_u64(b == j ? C[ECC_GM_AP + 8 * i + q] : 0);
    }
    case RK_EC_GM_EQ: {  // equal[i][j]: in = (j, byte_i)
      const uint32_t blk = s / 6, e = s % 6, i = blk >> 8, j = blk & 255u;
      const uint32_t b = (uint32_t)((C[ECC_U1 + (i >> 3)] >> (8 * (i & 7))) & 255);
      return iseq_sig((int)e, j, b, inv_small_signed(B.inv_small, (int)b - (int)j));
    }
    case RK_EC_GM_SUM: {  // GetSumOfNElements(256) of column (i, a, k): out | in[256] | sum[255]
      const uint32_t blk = s >> 9, m = s & 511u, i = blk >> 3, q = blk & 7u;
      const uint32_t b = (uint32_t)((C[ECC_U1 + (i >> 3)] >> (8 * (i & 7))) & 255);
      const uint64_t v = C[ECC_GM_AP + 8 * i + q];
      if (m == 0) return el_u64(v);
      if (m <= 256) return el_u64(b == m - 1 ? v : 0);
      return el_u64(b <= m - 256 ? v : 0);
    }
    case RK_EC_GM_STEP: {  // isFirst/SecondDummyLeft/Right[i], then (switcherRight, switcherLeft)[a][k]
      const int i = R.a[0];
      const uint64_t* left = i == 0 ? C + ECC_GM_AP : C + ECC_GM_RP + 8 * (i - 1);
      const uint64_t* right = C + ECC_GM_AP + 8 * (i + 1);
      const uint64_t dx = ec_k(cv, EC_K_DUMMY, 0), sdx = rec_out(EC_OP_SD)[0];
      if (s < 24) {
        const int k = (int)s / 6, e = (int)s % 6;
        const uint64_t in0 = (k & 1) ? sdx : dx, in1 = k < 2 ? left[0] : right[0];
        return iseq_sig(e, in0, in1, I[ECI_GM + 4 * i + k]);
      }
      const uint32_t t = s - 24, q = t / 12, e = t % 12;
      const uint64_t br = (uint64_t)(right[0] == sdx) + (uint64_t)(right[0] == dx);
      const uint64_t bl = (uint64_t)(left[0] == sdx) + (uint64_t)(left[0] == dx);
      const uint64_t add = rec_out(ec_op_gm_add(i))[q];
      if (e < 6) return switcher_sig((int)e, br, add, left[q]);
      const uint64_t swr0 = br ? left[q] : add;
      return switcher_sig((int)e - 6, bl, right[q], swr0);
    }
    case RK_EC_N2B: {  // Num2Bits(64): out[64] | in | sum[64]
      const uint64_t v = R.a[0] == 0 ? C[R.a[1]] : *reinterpret_cast<const uint64_t*>(row + 32ull * R.a[1]);
      if (s < 64) return el_u64((v >> s) & 1);
      if (s == 64) return el_u64(v);
      return el_u64(u64_mask(v, (int)s - 64));
    }
    case RK_EC_B2N8: {  // bits2num[i] = Bits2Num(8) of scalar byte i: out | in[8] | sum[8]
      const uint32_t i = s / 17, e = s % 17;
      const uint64_t b = (C[R.a[0] + (i >> 3)] >> (8 * (i & 7))) & 255;
      if (e == 0) return el_u64(b);
      if (e <= 8) return el_u64((b >> (e - 1)) & 1);
      return el_u64(u64_mask(b, (int)e - 8));
    }
    case RK_EC_SBITS: return el_u64(limbs_bit(C + R.a[0], 255 - (int)s));  // scalarBits, MSB first
    case RK_EC_SM_W0: {  // bits2Num[w] (Bits2Num(4) of nibble w) | isZeroResult[w] (in = (rp[w].x0, D.x0))
      const int w4 = R.a[0], bb = 252 - 4 * w4;
      const uint64_t nib = (C[ECC_U2 + (bb >> 6)] >> (bb & 63)) & 15;
      if (s == 0) return el_u64(nib);
      if (s <= 4) return el_u64((nib >> (s - 1)) & 1);
      if (s <= 8) return el_u64(u64_mask(nib, (int)s - 4));
      return iseq_sig((int)s - 9, C[ECC_SM_RP + 8 * w4], ec_k(cv, EC_K_DUMMY, 0), I[ECI_SM_ZR + w4]);
    }
    case RK_EC_SM_DSW: {  // doubleSwitcher[w-1][a][k]: bool = isZeroResult[w], in = (D, rp[w])
      const int w4 = R.a[0];
      const uint32_t q = s / 6, e = s % 6;
      const uint64_t zr = C[ECC_SM_RP + 8 * w4] == ec_k(cv, EC_K_DUMMY, 0);
      return switcher_sig((int)e, zr, ec_k(cv, EC_K_DUMMY, (int)q), C[ECC_SM_RP + 8 * w4 + q]);
    }
    case RK_EC_SM_SEL: {  // getSum[w][a][k] (GetSum(16)) | partsEqual[w][k]
      const int w4 = R.a[0], bb = 252 - 4 * w4;
      const uint64_t nib = (C[ECC_U2 + (bb >> 6)] >> (bb & 63)) & 15;
      if (s < 256) {
        const uint32_t q = s >> 5, m = s & 31u;
        const uint64_t v = C[ECC_SM_AP + 8 * w4 + q];
        if (m == 0) return el_u64(v);
        if (m <= 16) return el_u64(nib == m - 1 ? v : 0);
        return el_u64(nib <= m - 16 ? v : 0);
      }
      const uint32_t t = s - 256, k = t / 6, e = t % 6;
      return iseq_sig((int)e, k, nib, inv_small_signed(B.inv_small, (int)nib - (int)k));
    }
    case RK_EC_SM_RSW: {  // isZeroAddition[w] | (resultSwitcherAddition, resultSwitcherDoubling)[w-1][a][k]
      const int w4 = R.a[0];
      const uint64_t* ap = C + ECC_SM_AP + 8 * w4;
      if (s < 6) return iseq_sig((int)s, ap[0], ec_k(cv, EC_K_DUMMY, 0), I[ECI_SM_ZA + w4 - 1]);
      const uint32_t t = s - 6, q = t / 12, e = t % 12;
      const uint64_t za = ap[0] == ec_k(cv, EC_K_DUMMY, 0), zr = C[ECC_SM_RP + 8 * w4] == ec_k(cv, EC_K_DUMMY, 0);
      const uint64_t addq = rec_out(ec_op_sm_add(w4 - 1))[q], dblq = rec_out(ec_op_sm_dbl(4 * w4 - 1))[q];
      if (e < 6) return switcher_sig((int)e, za, addq, dblq);
      const uint64_t rsa0 = za ? dblq : addq;
      return switcher_sig((int)e - 6, zr, ap[q], rsa0);
    }
    case RK_EC_PKBITS: {  // ecBitsX[k] = bit 255-k of x, then y (passportVerificationBuilder.circom:197-210)
      const uint32_t a = s >> 8, k = s & 255u;
      uint64_t x[4];
      for (int j = 0; j < 4; j++) x[j] = *reinterpret_cast<const uint64_t*>(row + 32ull * (R.a[0] + 4 * a + j));
      return el_u64(limbs_bit(x, 255 - (int)k));
    }
    case RK_EC_B2N248: {  // Bits2Num(248) of x mod 2^248: out | in[248] | sum[248]
      uint64_t x[4];
      for (int j = 0; j < 4; j++) x[j] = *reinterpret_cast<const uint64_t*>(row + 32ull * (R.a[0] + j));
      if (s == 0) return limbs_mask(x, 248);
      if (s <= 248) return el_u64(limbs_bit(x, (int)s - 1));
      return limbs_mask(x, (int)s - 248);
    }
    default: return el_u64(0);
  }
}

}  // namespace pzk
