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
// integer given as n chunks of cs bits (one per u64): bit i / low nb bits (as an element, nb <= 256)
__device__ __forceinline__ uint32_t chunks_bit(const uint64_t* x, int cs, int i) { return (uint32_t)((x[i / cs] >> (i % cs)) & 1ull); }
__device__ __forceinline__ El chunks_mask(const uint64_t* x, int n, int cs, int nb) {
  uint32_t m[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int k = 0; k < n && cs * k < nb; k++) {
    const uint64_t v = u64_mask(x[k], nb - cs * k);
    const int b = cs * k;
    m[b >> 5] |= (uint32_t)v;
    if (cs == 64 && (b >> 5) + 1 < 8) m[(b >> 5) + 1] |= (uint32_t)(v >> 32);
  }
  return El{make_uint4(m[0], m[1], m[2], m[3]), make_uint4(m[4], m[5], m[6], m[7])};
}
// byte i / nibble at bit b of a chunked scalar
__device__ __forceinline__ uint32_t sc8(const uint64_t* s, int cs, int i) { return (uint32_t)((s[(8 * i) / cs] >> ((8 * i) % cs)) & 255); }
__device__ __forceinline__ uint64_t sc4(const uint64_t* s, int cs, int b) { return (s[b / cs] >> (b % cs)) & 15; }
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

// The small ECDSA regions (one instance for every curve: the geometry comes from EC_GEO[curve]; the three big
// selection tables of the generator multiplication have their own per-curve emitter, k_emit_ecr in ec_core.hpp)
__device__ El ec_small(const DevLayout& L, const Bufs& B, const Region& R, uint32_t w, uint32_t s) {
  const int cv = L.reg.ec_curve;
  const EcGeo& G = EC_GEO[cv];
  const int N = G.nl, CS = G.cs, P2 = 2 * N;
  const uint64_t* C = B.ec_core + (size_t)w * G.core_words;
  const fr* I = B.ec_inv + (size_t)w * G.n_inv;
  const uint8_t* row = B.inputs + 32ull * (uint64_t)w * L.n_inputs;
  auto rec_out = [&](int op) { return C + G.c_rec + G.rec_words * op + 2 * P2; };
  const uint64_t dx = ec_k(cv, EC_K_DUMMY, 0);
  switch (R.kind) {
    case RK_EC_U64: return el_u64(C[R.a[0] + s]);
    case RK_EC_CONST: return el_u64(ec_k(cv, R.a[0], (int)s));
    case RK_EC_GM_STEP: {  // isFirst/SecondDummyLeft/Right[i], then (switcherRight, switcherLeft)[a][k]
      const int i = R.a[0];
      const uint64_t* left = i == 0 ? C + G.c_gm_ap : C + G.c_gm_rp + P2 * (i - 1);
      const uint64_t* right = C + G.c_gm_ap + P2 * (i + 1);
      const uint64_t sdx = rec_out(EC_OP_SD)[0];
      if (s < 24) {
        const int k = (int)s / 6, e = (int)s % 6;
        const uint64_t in0 = (k & 1) ? sdx : dx, in1 = k < 2 ? left[0] : right[0];
        return iseq_sig(e, in0, in1, I[4 * i + k]);
      }
      const uint32_t t = s - 24, q = t / 12, e = t % 12;
      const uint64_t br = (uint64_t)(right[0] == sdx) + (uint64_t)(right[0] == dx);
      const uint64_t bl = (uint64_t)(left[0] == sdx) + (uint64_t)(left[0] == dx);
      const uint64_t add = rec_out(ec_op_gm_add(i))[q];
      if (e < 6) return switcher_sig((int)e, br, add, left[q]);
      const uint64_t swr0 = br ? left[q] : add;
      return switcher_sig((int)e - 6, bl, right[q], swr0);
    }
    case RK_EC_N2B: {  // Num2Bits(cs): out[cs] | in | sum[cs]
      const int cs = R.a[2];
      const uint64_t v = R.a[0] == 0 ? C[R.a[1]] : *reinterpret_cast<const uint64_t*>(row + 32ull * R.a[1]);
      if ((int)s < cs) return el_u64((v >> s) & 1);
      if ((int)s == cs) return el_u64(v);
      return el_u64(u64_mask(v, (int)s - cs));
    }
    case RK_EC_B2N8: {  // bits2num[i] = Bits2Num(8) of scalar byte i: out | in[8] | sum[8]
      const uint32_t i = s / 17, e = s % 17;
      const uint64_t b = sc8(C + R.a[0], CS, (int)i);
      if (e == 0) return el_u64(b);
      if (e <= 8) return el_u64((b >> (e - 1)) & 1);
      return el_u64(u64_mask(b, (int)e - 8));
    }
    case RK_EC_SBITS: return el_u64(chunks_bit(C + R.a[0], CS, G.fb - 1 - (int)s));  // scalarBits, MSB first
    case RK_EC_SM_W0: {  // bits2Num[w] (Bits2Num(4) of nibble w) | isZeroResult[w] (in = (rp[w].x0, D.x0))
      const int w4 = R.a[0];
      const uint64_t nib = sc4(C + G.c_u2, CS, G.fb - 4 - 4 * w4);
      if (s == 0) return el_u64(nib);
      if (s <= 4) return el_u64((nib >> (s - 1)) & 1);
      if (s <= 8) return el_u64(u64_mask(nib, (int)s - 4));
      return iseq_sig((int)s - 9, C[G.c_sm_rp + P2 * w4], dx, I[G.i_sm_zr + w4]);
    }
    case RK_EC_SM_DSW: {  // doubleSwitcher[w-1][a][k]: bool = isZeroResult[w], in = (D, rp[w])
      const int w4 = R.a[0];
      const uint32_t q = s / 6, e = s % 6;
      const uint64_t zr = C[G.c_sm_rp + P2 * w4] == dx;
      return switcher_sig((int)e, zr, ec_k(cv, EC_K_DUMMY, (int)q), C[G.c_sm_rp + P2 * w4 + q]);
    }
    case RK_EC_SM_SEL: {  // getSum[w][a][k] (GetSum(16)) | partsEqual[w][k]
      const int w4 = R.a[0];
      const uint64_t nib = sc4(C + G.c_u2, CS, G.fb - 4 - 4 * w4);
      if (s < 32u * P2) {
        const uint32_t q = s >> 5, m = s & 31u;
        const uint64_t v = C[G.c_sm_ap + P2 * w4 + q];
        if (m == 0) return el_u64(v);
        if (m <= 16) return el_u64(nib == m - 1 ? v : 0);
        return el_u64(nib <= m - 16 ? v : 0);
      }
      const uint32_t t = s - 32u * P2, k = t / 6, e = t % 6;
      return iseq_sig((int)e, k, nib, inv_small_signed(B.inv_small, (int)nib - (int)k));
    }
    case RK_EC_SM_RSW: {  // isZeroAddition[w] | (resultSwitcherAddition, resultSwitcherDoubling)[w-1][a][k]
      const int w4 = R.a[0];
      const uint64_t* ap = C + G.c_sm_ap + P2 * w4;
      if (s < 6) return iseq_sig((int)s, ap[0], dx, I[G.i_sm_za + w4 - 1]);
      const uint32_t t = s - 6, q = t / 12, e = t % 12;
      const uint64_t za = ap[0] == dx, zr = C[G.c_sm_rp + P2 * w4] == dx;
      const uint64_t addq = rec_out(ec_op_sm_add(G, w4 - 1))[q], dblq = rec_out(ec_op_sm_dbl(G, 4 * w4 - 1))[q];
      if (e < 6) return switcher_sig((int)e, za, addq, dblq);
      const uint64_t rsa0 = za ? dblq : addq;
      return switcher_sig((int)e - 6, zr, ap[q], rsa0);
    }
    case RK_EC_PKBITS: {  // ecBitsX[k] = bit F-1-k of x, then y (passportVerificationBuilder.circom:197-210)
      const int n = R.a[1], cs = R.a[2], F = n * cs;
      const uint32_t a = s / F, k = s % F;
      uint64_t x[EC_MAXN];
      for (int j = 0; j < n; j++) x[j] = *reinterpret_cast<const uint64_t*>(row + 32ull * (R.a[0] + n * a + j));
      return el_u64(chunks_bit(x, cs, F - 1 - (int)k));
    }
    case RK_EC_B2N248: {  // Bits2Num(FD) of x mod 2^FD, FD = min(F, 248): out | in[FD] | sum[FD]
      const int n = R.a[1], cs = R.a[2], FD = R.a[3];
      uint64_t x[EC_MAXN];
      for (int j = 0; j < n; j++) x[j] = *reinterpret_cast<const uint64_t*>(row + 32ull * (R.a[0] + j));
      if (s == 0) return chunks_mask(x, n, cs, FD);
      if ((int)s <= FD) return el_u64(chunks_bit(x, cs, (int)s - 1));
      return chunks_mask(x, n, cs, (int)s - FD);
    }
    default: return el_u64(0);
  }
}
}  // namespace pzk
