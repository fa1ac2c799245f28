// Template walkers of the ECDSA table blocks: EllipticCurveDouble, EllipticCurveAdd
// (ec/curve.circom:281-345 with PointOnTangent / PointOnCurve / PointOnLine :110-245) and
// BigMultModP(64,4,4,4) (bigInt.circom:206-272).
//
// ONE source, two instantiations:
//   * host, C = EcProgCtx (builder_register.cpp): values are symbolic; every put() allocates the
//     next table entry and writes a COPY descriptor at the signal's offset; bits()/masks() write
//     BIT/MASK descriptors; the result is the per-type descriptor program;
//   * device, C = EcTabCtx (ec_core.hpp, k_ec_table): values are signed 256-bit integers
//     (two's complement; every value of these templates is an integer of magnitude < 2^210, or an
//     Fr inverse); every put() appends the value, Fr normal form, to the op's table.
// Both run the same statements in the same order, so entry numbering agrees by construction.
// Signal offsets follow the O0 layout exactly as oracle/ecdsa_p256.inc.c lays them
// out: a block = own signals (outputs, inputs, intermediates) then sub-blocks in creation order.
#pragma once
#include "ec_common.hpp"

namespace pzk {
inline namespace PZK_EC_NS {

// Every walker function is force-inlined, so on the device each k_ec_table<TYPE> holds only its own
// type's walk and no callable function exists. A callable walker (what hipcc chose on its own: one
// ~46 k-instruction function shared by the three types) needs long branches, and ROCm 7.2's branch
// relaxation may expand them with s[30:31] — the function's unsaved return address — as the scratch
// pair; the walker then "returns" into its own body (the round-2 P-256 hang / brainpool fault,
// DESIGN.md §4.8; tools/check_code_objects.py checks every built code object for this).
#define PZK_WALK __host__ __device__ __attribute__((always_inline)) inline

template <class C>
struct EcWalk {
  using V = typename C::V;
  C& c;
  PZK_WALK explicit EcWalk(C& ctx) : c(ctx) {}

  // Num2Bits(L) bitify.circom:10-32: out[L] | in | sum[L]   (v already in the table)
  PZK_WALK void n2b(uint32_t b, const V& v, int L) {
    c.bits(b, v, L);
    c.cp(b + L, v);
    c.masks(b + L + 1, v, L);
  }
  // Num2Bits(L) whose input is a fresh value
  PZK_WALK V n2b_new(uint32_t b, const V& x, int L) {
    V v = c.put(b + L, x);
    c.bits(b, v, L);
    c.masks(b + L + 1, v, L);
    return v;
  }

  // BigMultNonEqualOverflow(G,L) bigIntHelpers.circom:55-124:
  // out[G+L-1] | in1[G], in2[L] | tmpMults[G][L], tmpResult[G+L-1][L]
  // column i sums tmpMults[a][j] (a + j = i) with a descending; every product is materialised
  // in the column that consumes it.
  // f(i, out[i]) is called per output column, so callers can consume columns without an array
  template <class F>
  PZK_WALK void bmneq_cb(uint32_t b, int G, int L, const V* in1, const V* in2, F f) {
    const uint32_t i1 = b + G + L - 1, i2 = i1 + G, tm = i2 + L, tr = tm + G * L;
    for (int i = 0; i < G; i++) c.cp(i1 + i, in1[i]);
    for (int j = 0; j < L; j++) c.cp(i2 + j, in2[j]);
    for (int i = 0; i < G + L - 1; i++) {
      int j0 = i < G ? 0 : i - G + 1, j1 = i < L ? i : L - 1;  // in2 index range of column i
      V s{};
      for (int j = j0, k = 0; j <= j1; j++, k++) {
        const int a = i - j;
        V p = c.put(tm + a * L + j, c.mul(in1[a], in2[j]));
        if (k == 0) { c.cp(tr + i * L + 0, p); s = p; }
        else s = c.put(tr + i * L + k, c.add(s, p));
      }
      c.cp(b + i, s);
      f(i, s);
    }
  }
  PZK_WALK void bmneq(uint32_t b, int G, int L, const V* in1, const V* in2, V* out) {
    bmneq_cb(b, G, L, in1, in2, [&](int i, const V& s) { out[i] = s; });
  }
  // BigMultOverflow(G,L) bigIntOverflow.circom:38-72 (schoolbook for these sizes):
  // out[G+L-1] | in1[G], in2[L] | mult
  template <class F>
  PZK_WALK void bmo_cb(uint32_t b, int G, int L, const V* in1, const V* in2, F f) {
    for (int i = 0; i < G; i++) c.cp(b + G + L - 1 + i, in1[i]);
    for (int j = 0; j < L; j++) c.cp(b + 2 * G + L - 1 + j, in2[j]);
    bmneq_cb(b + 2 * G + 2 * L - 1, G, L, in1, in2, [&](int i, const V& s) { c.cp(b + i, s); f(i, s); });
  }
  PZK_WALK void bmo(uint32_t b, int G, int L, const V* in1, const V* in2, V* out) {
    bmo_cb(b, G, L, in1, in2, [&](int i, const V& s) { out[i] = s; });
  }
  // ScalarMultOverflow(N) bigIntOverflow.circom:101-111: out[N] | in[N], scalar
  PZK_WALK void smo(uint32_t b, int N, const V* in, uint64_t k, V* out) {
    for (int i = 0; i < N; i++) c.cp(b + N + i, in[i]);
    V kv = c.put(b + 2 * N, c.u64(k));
    for (int i = 0; i < N; i++) out[i] = c.put(b + i, c.mul(kv, in[i]));
  }
  // BigAddOverflow(G,L) bigIntOverflow.circom:22-35: out[G] | in1[G], in2[L]
  PZK_WALK void bao(uint32_t b, int G, int L, const V* in1, const V* in2, V* out) {
    for (int i = 0; i < G; i++) c.cp(b + G + i, in1[i]);
    for (int j = 0; j < L; j++) c.cp(b + 2 * G + j, in2[j]);
    for (int i = 0; i < G; i++) {
      out[i] = i < L ? c.put(b + i, c.add(in1[i], in2[i])) : in1[i];
      if (i >= L) c.cp(b + i, in1[i]);
    }
  }
  // BigSubModOverflow(N) bigIntOverflow.circom:78-98: out[N] | in1[N], in2[N], modulus[N]
  PZK_WALK void bsmo(uint32_t b, const V* in1, const V* in2, const V* mod, V* out) {
    for (int i = 0; i < 4; i++) { c.cp(b + 4 + i, in1[i]); c.cp(b + 8 + i, in2[i]); c.cp(b + 12 + i, mod[i]); }
    for (int i = 0; i < 4; i++) {
      V v = c.sub(c.add(mod[i], in1[i]), in2[i]);
      if (i != 3) v = c.add(v, c.pow2(64));
      if (i != 0) v = c.sub(v, c.u64(1));
      out[i] = c.put(b + i, v);
    }
  }
  // materialise 4 constant limbs
  PZK_WALK void consts4(const uint64_t* k, V* out) {
    for (int i = 0; i < 4; i++) out[i] = c.put_hidden(c.u64(k[i]));
  }

  // BigIntIsZero(64,MAX,K) bigIntComparators.circom:105-129: in[K] | carry[K-1] | carryRangeChecks[K-1]
  // (in already placed by the caller)
  PZK_WALK void bisz(uint32_t b, int MAX, int K, const V* in) {
    const int L = MAX + 3 - 64;
    const uint32_t carry = b + K, sub = carry + K - 1;
    V cy{};
    for (int i = 0; i < K - 1; i++) {
      V t = i == 0 ? in[0] : c.add(in[i], cy);
      cy = c.put(carry + i, c.shr64_exact(t));
      n2b_new(sub + i * ec_n2b(L), c.add(cy, c.pow2(L - 1)), L);
    }
    c.check_zero(c.add(in[K - 1], cy));  // bigIntComparators.circom:128
  }

  // BigIntIsZeroModP(64,MAX,CN,MCN,4) bigIntComparators.circom:158-212:
  // in[CN], modulus[4] | sign, k[DIV] | kRangeChecks[DIV], mult, isZero, swicher[CN]
  // The columns of mult = k * modulus feed the switchers, isZero.in and the carry chain of
  // BigIntIsZero (bigIntComparators.circom:105-129) as they are produced (no column arrays).
  PZK_WALK void bizmp(uint32_t b, int MAX, int CN, int MCN, const V* in, const V* mod) {
    const int DIV = MCN - 3, LB = MAX + 3 - 64;
    const uint32_t o_mod = b + CN, o_sign = o_mod + 4, o_k = o_sign + 1, o_krc = o_k + DIV,
                   o_mult = o_krc + DIV * ec_n2b(64), o_isz = o_mult + ec_bmo(DIV, 4), o_sw = o_isz + ec_bisz(MAX, MCN);
    const uint32_t o_carry = o_isz + MCN, o_rc = o_carry + MCN - 1;
    for (int i = 0; i < CN; i++) c.cp(b + i, in[i]);
    for (int i = 0; i < 4; i++) c.cp(o_mod + i, mod[i]);
    V sign, k[10];
    c.div_signed(in, CN, MCN, sign, k);  // reduce_overflow_signed + long_div (bigIntFunc.circom:646-694, 190-232)
    sign = c.put(o_sign, sign);
    for (int i = 0; i < DIV; i++) {
      k[i] = c.put(o_k + i, k[i]);
      n2b(o_krc + i * ec_n2b(64), k[i], 64);
    }
    V cy{};
    bmo_cb(o_mult, DIV, 4, k, mod, [&](int i, const V& m) {
      V iz;
      if (i < CN) {  // swicher[i]: out[2] | bool, in[2] | aux (switcher.circom:16-26), in = (x, -x), bool = sign
        const uint32_t s = o_sw + 6 * i;
        V neg = c.put(s + 4, c.neg(in[i]));
        c.cp(s + 2, sign);
        c.cp(s + 3, in[i]);
        c.put(s + 5, c.sel(sign, c.add(neg, neg), c.u64(0)));  // aux = (in1 - in0) * bool
        c.put(s + 0, c.sel(sign, neg, in[i]));
        V o1 = c.put(s + 1, c.sel(sign, in[i], neg));
        iz = c.put(o_isz + i, c.sub(m, o1));
      } else {
        iz = c.put(o_isz + i, m);
      }
      if (i < MCN - 1) {  // carry[i] = (in[i] + carry[i-1]) / 2^64, Num2Bits(LB)(carry + 2^(LB-1))
        V t = i == 0 ? iz : c.add(iz, cy);
        cy = c.put(o_carry + i, c.shr64_exact(t));
        n2b_new(o_rc + i * ec_n2b(LB), c.add(cy, c.pow2(LB - 1)), LB);
      } else {
        c.check_zero(c.add(iz, cy));  // bigIntComparators.circom:128
      }
    });
  }

  // PointOnCurve curve.circom:110-138: in[2][4] | squareX, cubeX, squareY, coefMult, isZeroModP
  PZK_WALK void poncurve(uint32_t b, const V* pt) {
    for (int i = 0; i < 8; i++) c.cp(b + i, pt[i]);
    const uint32_t sx = b + 8, cx = sx + ec_bmo(4, 4), sy = cx + ec_bmo(7, 4), cm = sy + ec_bmo(4, 4),
                   iz = cm + ec_bmo(4, 4);
    V in[10], A[4], Bc[4], P[4];
    {
      V sxo[7];
      bmo(sx, 4, 4, pt, pt, sxo);
      bmo(cx, 7, 4, sxo, pt, in);
    }
    bmo_cb(sy, 4, 4, pt + 4, pt + 4, [&](int i, const V& v) { in[i] = c.sub(in[i], v); });
    consts4(EC_A, A);
    bmo_cb(cm, 4, 4, pt, A, [&](int i, const V& v) { in[i] = c.add(in[i], v); });
    consts4(EC_B, Bc);
    for (int i = 0; i < 10; i++) {
      if (i < 4) in[i] = c.add(in[i], Bc[i]);
      in[i] = c.put(iz + i, in[i]);
    }
    consts4(EC_P, P);
    bizmp(iz, 200, 10, 12, in, P);
  }
  // PointOnTangent curve.circom:145-197: in1[2][4], in2[2][4] | squareX, scalarMult, bigAdd, bigSub,
  // rightMult, scalarMult2, bigAdd2, leftMult, isZeroModP
  PZK_WALK void pontangent(uint32_t b, const V* p1, const V* p2) {
    for (int i = 0; i < 8; i++) { c.cp(b + i, p1[i]); c.cp(b + 8 + i, p2[i]); }
    const uint32_t sx = b + 16, sm = sx + ec_bmo(4, 4), ba = sm + 15, bs = ba + 18, rm = bs + 16, sm2 = rm + ec_bmo(7, 4),
                   ba2 = sm2 + 9, lm = ba2 + 12, iz = lm + ec_bmo(4, 4);
    V t7[7], u7[7], A[4], P[4], d[4], in[10];
    bmo(sx, 4, 4, p1, p1, t7);
    smo(sm, 7, t7, 3, u7);
    consts4(EC_A, A);
    bao(ba, 7, 4, u7, A, t7);
    consts4(EC_P, P);
    bsmo(bs, p1, p2, P, d);
    bmo(rm, 7, 4, t7, d, in);
    V y2[4], ys[4];
    smo(sm2, 4, p1 + 4, 2, y2);
    bao(ba2, 4, 4, p1 + 4, p2 + 4, ys);
    bmo_cb(lm, 4, 4, ys, y2, [&](int i, const V& v) { in[i] = c.sub(in[i], v); });
    for (int i = 0; i < 10; i++) in[i] = c.put(iz + i, in[i]);
    bizmp(iz, 200, 10, 13, in, P);
  }
  // PointOnLine curve.circom:204-245: in1, in2, in3 | bigAdd, bigSub, bigSub2, bigSub3, leftMult,
  // rightMult, isZeroModP
  PZK_WALK void ponline(uint32_t b, const V* p1, const V* p2, const V* p3) {
    for (int i = 0; i < 8; i++) { c.cp(b + i, p1[i]); c.cp(b + 8 + i, p2[i]); c.cp(b + 16 + i, p3[i]); }
    const uint32_t ba = b + 24, s1 = ba + 12, s2 = s1 + 16, s3 = s2 + 16, lm = s3 + 16, rm = lm + ec_bmo(4, 4),
                   iz = rm + ec_bmo(4, 4);
    V P[4], ys[4], d1[4], d2[4], d3[4], l7[7];
    bao(ba, 4, 4, p1 + 4, p3 + 4, ys);
    consts4(EC_P, P);
    bsmo(s1, p2, p1, P, d1);
    bsmo(s2, p2 + 4, p1 + 4, P, d2);
    bsmo(s3, p1, p3, P, d3);
    bmo(lm, 4, 4, ys, d1, l7);
    bmo_cb(rm, 4, 4, d2, d3, [&](int i, const V& v) { l7[i] = c.put(iz + i, c.sub(l7[i], v)); });
    bizmp(iz, 136, 7, 9, l7, P);
  }

  // EllipticCurveDouble curve.circom:281-310: out[2][4] | in[2][4] | onTangentCheck, onCurveCheck
  PZK_WALK void dbl() {
    V in[8], out[8];
    for (int i = 0; i < 8; i++) in[i] = c.put(8 + i, c.rec(i));
    for (int i = 0; i < 8; i++) out[i] = c.put(i, c.rec(16 + i));
    pontangent(16, in, out);
    poncurve(16 + EC_SZ_PONTANGENT, out);
  }
  // EllipticCurveAdd curve.circom:314-345: out[2][4] | in1[2][4], in2[2][4] | onCurveCheck, onLineCheck
  PZK_WALK void add() {
    V in1[8], in2[8], out[8];
    for (int i = 0; i < 8; i++) in1[i] = c.put(8 + i, c.rec(i));
    for (int i = 0; i < 8; i++) in2[i] = c.put(16 + i, c.rec(8 + i));
    for (int i = 0; i < 8; i++) out[i] = c.put(i, c.rec(16 + i));
    poncurve(24, out);
    ponline(24 + EC_SZ_PONCURVE, in1, in2, out);
  }

  // IsEqual comparators.circom:24-33: out | in[2] | IsZero(out, in, inv)
  PZK_WALK V isequal(uint32_t b, const V& a, const V& bb) {
    c.cp(b + 1, a);
    c.cp(b + 2, bb);
    V d = c.put(b + 4, c.sub(bb, a));
    c.put(b + 5, c.inv_fr(d));
    V o = c.put(b + 3, c.is_zero(d));
    c.cp(b, o);
    return o;
  }
  // BigMultModP(64,4,4,4) bigInt.circom:206-272:
  // div[5], mod[4] | in1[4], in2[4], modulus[4] | mult, modChecks[4], greaterThan, mult2, isZero
  PZK_WALK void mm() {
    V x[4], y[4], n[4];
    for (int i = 0; i < 4; i++) x[i] = c.put(9 + i, c.rec(i));
    for (int i = 0; i < 4; i++) y[i] = c.put(13 + i, c.rec(4 + i));
    for (int i = 0; i < 4; i++) n[i] = c.put(17 + i, c.u64(EC_N[i]));
    const uint32_t o_mult = 21, o_chk = o_mult + ec_bmo(4, 4), o_gt = o_chk + 4 * ec_n2b(64), o_le = o_gt + 9,
                   o_m2 = o_le + EC_SZ_BLET, o_isz = o_m2 + ec_bmneq(5, 4);
    V mo[7], q[5], r[4];
    bmo(o_mult, 4, 4, x, y, mo);
    c.divmod_n(mo, q, r);  // reduce_overflow + long_div (bigIntFunc.circom:570-588, 190-232)
    for (int i = 0; i < 5; i++) q[i] = c.put(i, q[i]);
    for (int i = 0; i < 4; i++) r[i] = c.put(5 + i, r[i]);
    for (int i = 0; i < 4; i++) n2b(o_chk + i * ec_n2b(64), r[i], 64);
    // BigGreaterThan(64,4): out | in[2][4] | BigLessEqThan: out | in[2][4] | result[4] | (LessThan, IsEqual)[4]
    for (int i = 0; i < 4; i++) { c.cp(o_gt + 1 + i, n[i]); c.cp(o_gt + 5 + i, r[i]); }
    for (int i = 0; i < 4; i++) { c.cp(o_le + 1 + i, n[i]); c.cp(o_le + 5 + i, r[i]); }
    V res{};
    for (int i = 0; i < 4; i++) {
      const uint32_t lt = o_le + 13 + i * (3 + ec_n2b(65) + 6), eq = lt + 3 + ec_n2b(65);
      c.cp(lt + 1, n[i]);
      c.cp(lt + 2, r[i]);
      V v = n2b_new(lt + 3, c.sub(c.add(n[i], c.pow2(64)), r[i]), 65);
      V lto = c.put(lt, c.sub(c.u64(1), c.bit(v, 64)));
      V eqo = isequal(eq, n[i], r[i]);
      res = i == 0 ? c.put(o_le + 9 + i, c.add(lto, eqo)) : c.put(o_le + 9 + i, c.add(lto, c.mul(eqo, res)));
    }
    c.cp(o_le, res);
    V gt = c.put(o_gt, c.sub(c.u64(1), res));
    c.check_one(gt);  // bigInt.circom:245
    // mult2 = div * modulus; isZero.in[i] = mult[i] - mult2[i] - mod[i] (bigInt.circom:252-271)
    V iz[7];
    bmneq_cb(o_m2, 5, 4, q, n, [&](int i, const V& m2) {
      if (i < 7) {
        V v = c.sub(mo[i], m2);
        if (i < 4) v = c.sub(v, r[i]);
        iz[i] = c.put(o_isz + i, v);
      }
    });
    bisz(o_isz, 132, 7, iz);
  }

  PZK_WALK void run(int type) {
    if (type == ECT_DBL) dbl();
    else if (type == ECT_ADD) add();
    else mm();
  }
};

}  // namespace PZK_EC_NS
}  // namespace pzk
