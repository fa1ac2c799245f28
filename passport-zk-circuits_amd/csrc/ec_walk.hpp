// Template walkers of the ECDSA table blocks: EllipticCurveDouble, EllipticCurveAdd
// (ec/curve.circom:281-345 with PointOnTangent / PointOnCurve / PointOnLine :107-245) and
// BigMultModP(CS,N,N,N) (bigInt.circom:206-272), for the N x CS chunking of curve CV.
//
// ONE source, two instantiations:
//   * host, C = EcProgCtx (builder_ecdsa.cpp): values are symbolic; every put() allocates the
//     next table entry and writes a COPY descriptor at the signal's offset; bits()/masks() write
//     BIT/MASK descriptors; the result is the per-type descriptor program;
//   * device, C = EcTabCtx (ec_core.hpp, k_ec_table): values are signed 256-bit integers
//     (two's complement; every value of these templates is an integer of magnitude < 2^210, or an
//     Fr inverse); every put() appends the value, Fr normal form, to the op's table.
// Both run the same statements in the same order, so entry numbering agrees by construction.
// Signal offsets follow the O0 layout exactly as oracle/ecdsa.inc.c lays them
// out: a block = own signals (outputs, inputs, intermediates) then sub-blocks in creation order.
#pragma once
#include "ec_common.hpp"

namespace pzk {

// Every walker function is force-inlined, so on the device each k_ec_table<TYPE> holds only its own
// type's walk and no callable function exists. A callable walker (what hipcc chose on its own: one
// ~46 k-instruction function shared by the three types) needs long branches, and ROCm 7.2's branch
// relaxation may expand them with s[30:31] — the function's unsaved return address — as the scratch
// pair; the walker then "returns" into its own body (the round-2 P-256 hang / brainpool fault,
// DESIGN.md §4.8; tools/check_code_objects.py checks every built code object for this).
#define PZK_WALK __host__ __device__ __attribute__((always_inline)) inline

template <class C, int CV>
struct EcWalk {
  using V = typename C::V;
  static constexpr EcGeo G = EC_GEO[CV];
  static constexpr int N = G.nl, CS = G.cs;
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
  // BigSubModOverflow(CS,N) bigIntOverflow.circom:78-98: out[N] | in1[N], in2[N], modulus[N]
  PZK_WALK void bsmo(uint32_t b, const V* in1, const V* in2, const V* mod, V* out) {
    for (int i = 0; i < N; i++) { c.cp(b + N + i, in1[i]); c.cp(b + 2 * N + i, in2[i]); c.cp(b + 3 * N + i, mod[i]); }
    for (int i = 0; i < N; i++) {
      V v = c.sub(c.add(mod[i], in1[i]), in2[i]);
      if (i != N - 1) v = c.add(v, c.pow2(CS));
      if (i != 0) v = c.sub(v, c.u64(1));
      out[i] = c.put(b + i, v);
    }
  }
  // materialise N constant chunks
  PZK_WALK void constsN(const uint64_t* k, V* out) {
    for (int i = 0; i < N; i++) out[i] = c.put_hidden(c.u64(k[i]));
  }

  // BigIntIsZero(CS,MAX,K) bigIntComparators.circom:105-129: in[K] | carry[K-1] | carryRangeChecks[K-1]
  // (in already placed by the caller)
  PZK_WALK void bisz(uint32_t b, int MAX, int K, const V* in) {
    const int L = MAX + 3 - CS;
    const uint32_t carry = b + K, sub = carry + K - 1;
    V cy{};
    for (int i = 0; i < K - 1; i++) {
      V t = i == 0 ? in[0] : c.add(in[i], cy);
      cy = c.put(carry + i, c.shr_exact(t, CS));
      n2b_new(sub + i * ec_n2b(L), c.add(cy, c.pow2(L - 1)), L);
    }
    c.check_zero(c.add(in[K - 1], cy));  // bigIntComparators.circom:128
  }

  // BigIntIsZeroModP(CS,MAX,CN,MCN,N) bigIntComparators.circom:158-212:
  // in[CN], modulus[N] | sign, k[DIV] | kRangeChecks[DIV], mult, isZero, swicher[CN]
  // The columns of mult = k * modulus feed the switchers, isZero.in and the carry chain of
  // BigIntIsZero (bigIntComparators.circom:105-129) as they are produced (no column arrays).
  // DIV = MCN - N + 1 >= N for every instance here, so mult = BigMultOverflow(CS, DIV, N)(k, modulus).
  PZK_WALK void bizmp(uint32_t b, int MAX, int CN, int MCN, const V* in, const V* mod) {
    const int DIV = MCN - N + 1, LB = MAX + 3 - CS;
    const uint32_t o_mod = b + CN, o_sign = o_mod + N, o_k = o_sign + 1, o_krc = o_k + DIV,
                   o_mult = o_krc + DIV * ec_n2b(CS), o_isz = o_mult + ec_bmo(DIV, N), o_sw = o_isz + ec_bisz(CS, MAX, MCN);
    const uint32_t o_carry = o_isz + MCN, o_rc = o_carry + MCN - 1;
    for (int i = 0; i < CN; i++) c.cp(b + i, in[i]);
    for (int i = 0; i < N; i++) c.cp(o_mod + i, mod[i]);
    V sign, k[2 * N + 2];
    c.div_signed(in, CN, MCN, sign, k);  // reduce_overflow_signed + long_div (bigIntFunc.circom:646-694, 190-232)
    sign = c.put(o_sign, sign);
    for (int i = 0; i < DIV; i++) {
      k[i] = c.put(o_k + i, k[i]);
      n2b(o_krc + i * ec_n2b(CS), k[i], CS);
    }
    V cy{};
    bmo_cb(o_mult, DIV, N, k, mod, [&](int i, const V& m) {
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
      if (i < MCN - 1) {  // carry[i] = (in[i] + carry[i-1]) / 2^CS, Num2Bits(LB)(carry + 2^(LB-1))
        V t = i == 0 ? iz : c.add(iz, cy);
        cy = c.put(o_carry + i, c.shr_exact(t, CS));
        n2b_new(o_rc + i * ec_n2b(LB), c.add(cy, c.pow2(LB - 1)), LB);
      } else {
        c.check_zero(c.add(iz, cy));  // bigIntComparators.circom:128
      }
    });
  }

  // PointOnCurve curve.circom:107-137: in[2][N] | squareX, cubeX, squareY, coefMult,
  // isZeroModP(CS, 3 CS + 2N, 3N - 2, 3N, N)
  PZK_WALK void poncurve(uint32_t b, const V* pt) {
    for (int i = 0; i < 2 * N; i++) c.cp(b + i, pt[i]);
    const uint32_t sx = b + 2 * N, cx = sx + ec_bmo(N, N), sy = cx + ec_bmo(2 * N - 1, N), cm = sy + ec_bmo(N, N),
                   iz = cm + ec_bmo(N, N);
    V in[3 * N - 2], A[N], Bc[N], P[N];
    {
      V sxo[2 * N - 1];
      bmo(sx, N, N, pt, pt, sxo);
      bmo(cx, 2 * N - 1, N, sxo, pt, in);
    }
    bmo_cb(sy, N, N, pt + N, pt + N, [&](int i, const V& v) { in[i] = c.sub(in[i], v); });
    constsN(EC_CURVE_K[CV][EC_K_A], A);
    bmo_cb(cm, N, N, pt, A, [&](int i, const V& v) { in[i] = c.add(in[i], v); });
    constsN(EC_CURVE_K[CV][EC_K_B], Bc);
    for (int i = 0; i < 3 * N - 2; i++) {
      if (i < N) in[i] = c.add(in[i], Bc[i]);
      in[i] = c.put(iz + i, in[i]);
    }
    constsN(EC_CURVE_K[CV][EC_K_P], P);
    bizmp(iz, 3 * CS + 2 * N, 3 * N - 2, 3 * N, in, P);
  }
  // PointOnTangent curve.circom:144-190: in1[2][N], in2[2][N] | squareX, scalarMult, bigAdd, bigSub,
  // rightMult, scalarMult2, bigAdd2, leftMult, isZeroModP(CS, 3 CS + 2N, 3N - 2, 3N + 1, N)
  PZK_WALK void pontangent(uint32_t b, const V* p1, const V* p2) {
    constexpr int M = 2 * N - 1;
    for (int i = 0; i < 2 * N; i++) { c.cp(b + i, p1[i]); c.cp(b + 2 * N + i, p2[i]); }
    const uint32_t sx = b + 4 * N, sm = sx + ec_bmo(N, N), ba = sm + (2 * M + 1), bs = ba + (2 * M + N), rm = bs + 4 * N,
                   sm2 = rm + ec_bmo(M, N), ba2 = sm2 + (2 * N + 1), lm = ba2 + 3 * N, iz = lm + ec_bmo(N, N);
    V t7[M], u7[M], A[N], P[N], d[N], in[3 * N - 2];
    bmo(sx, N, N, p1, p1, t7);
    smo(sm, M, t7, 3, u7);
    constsN(EC_CURVE_K[CV][EC_K_A], A);
    bao(ba, M, N, u7, A, t7);
    constsN(EC_CURVE_K[CV][EC_K_P], P);
    bsmo(bs, p1, p2, P, d);
    bmo(rm, M, N, t7, d, in);
    V y2[N], ys[N];
    smo(sm2, N, p1 + N, 2, y2);
    bao(ba2, N, N, p1 + N, p2 + N, ys);
    bmo_cb(lm, N, N, ys, y2, [&](int i, const V& v) { in[i] = c.sub(in[i], v); });
    for (int i = 0; i < 3 * N - 2; i++) in[i] = c.put(iz + i, in[i]);
    bizmp(iz, 3 * CS + 2 * N, 3 * N - 2, 3 * N + 1, in, P);
  }
  // PointOnLine curve.circom:197-245: in1, in2, in3 | bigAdd, bigSub, bigSub2, bigSub3, leftMult,
  // rightMult, isZeroModP(CS, 2 CS + 2N, 2N - 1, 2N + 1, N)
  PZK_WALK void ponline(uint32_t b, const V* p1, const V* p2, const V* p3) {
    for (int i = 0; i < 2 * N; i++) { c.cp(b + i, p1[i]); c.cp(b + 2 * N + i, p2[i]); c.cp(b + 4 * N + i, p3[i]); }
    const uint32_t ba = b + 6 * N, s1 = ba + 3 * N, s2 = s1 + 4 * N, s3 = s2 + 4 * N, lm = s3 + 4 * N, rm = lm + ec_bmo(N, N),
                   iz = rm + ec_bmo(N, N);
    V P[N], ys[N], d1[N], d2[N], d3[N], l7[2 * N - 1];
    bao(ba, N, N, p1 + N, p3 + N, ys);
    constsN(EC_CURVE_K[CV][EC_K_P], P);
    bsmo(s1, p2, p1, P, d1);
    bsmo(s2, p2 + N, p1 + N, P, d2);
    bsmo(s3, p1, p3, P, d3);
    bmo(lm, N, N, ys, d1, l7);
    bmo_cb(rm, N, N, d2, d3, [&](int i, const V& v) { l7[i] = c.put(iz + i, c.sub(l7[i], v)); });
    bizmp(iz, 2 * CS + 2 * N, 2 * N - 1, 2 * N + 1, l7, P);
  }

  // EllipticCurveDouble curve.circom:281-310: out[2][N] | in[2][N] | onTangentCheck, onCurveCheck
  PZK_WALK void dbl() {
    V in[2 * N], out[2 * N];
    for (int i = 0; i < 2 * N; i++) in[i] = c.put(2 * N + i, c.rec(i));
    for (int i = 0; i < 2 * N; i++) out[i] = c.put(i, c.rec(4 * N + i));
    pontangent(4 * N, in, out);
    poncurve(4 * N + G.sz_pontangent, out);
  }
  // EllipticCurveAdd curve.circom:314-345: out[2][N] | in1[2][N], in2[2][N] | onCurveCheck, onLineCheck
  PZK_WALK void add() {
    V in1[2 * N], in2[2 * N], out[2 * N];
    for (int i = 0; i < 2 * N; i++) in1[i] = c.put(2 * N + i, c.rec(i));
    for (int i = 0; i < 2 * N; i++) in2[i] = c.put(4 * N + i, c.rec(2 * N + i));
    for (int i = 0; i < 2 * N; i++) out[i] = c.put(i, c.rec(4 * N + i));
    poncurve(6 * N, out);
    ponline(6 * N + G.sz_poncurve, in1, in2, out);
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
  // BigMultModP(CS,N,N,N) bigInt.circom:206-272:
  // div[N+1], mod[N] | in1[N], in2[N], modulus[N] | mult, modChecks[N], greaterThan, mult2, isZero
  PZK_WALK void mm() {
    V x[N], y[N], n[N];
    for (int i = 0; i < N; i++) x[i] = c.put(2 * N + 1 + i, c.rec(i));
    for (int i = 0; i < N; i++) y[i] = c.put(3 * N + 1 + i, c.rec(N + i));
    for (int i = 0; i < N; i++) n[i] = c.put(4 * N + 1 + i, c.u64(EC_CURVE_K[CV][EC_K_ORDER][i]));
    const uint32_t o_mult = 5 * N + 1, o_chk = o_mult + ec_bmo(N, N), o_gt = o_chk + N * ec_n2b(CS), o_le = o_gt + 1 + 2 * N,
                   o_m2 = o_le + G.sz_blet, o_isz = o_m2 + ec_bmneq(N + 1, N);
    V mo[2 * N - 1], q[N + 1], r[N];
    bmo(o_mult, N, N, x, y, mo);
    c.divmod_n(mo, q, r);  // reduce_overflow + long_div (bigIntFunc.circom:570-588, 190-232)
    for (int i = 0; i < N + 1; i++) q[i] = c.put(i, q[i]);
    for (int i = 0; i < N; i++) r[i] = c.put(N + 1 + i, r[i]);
    for (int i = 0; i < N; i++) n2b(o_chk + i * ec_n2b(CS), r[i], CS);
    // BigGreaterThan(CS,N): out | in[2][N] | BigLessEqThan: out | in[2][N] | result[N] | (LessThan(CS), IsEqual)[N]
    for (int i = 0; i < N; i++) { c.cp(o_gt + 1 + i, n[i]); c.cp(o_gt + 1 + N + i, r[i]); }
    for (int i = 0; i < N; i++) { c.cp(o_le + 1 + i, n[i]); c.cp(o_le + 1 + N + i, r[i]); }
    V res{};
    for (int i = 0; i < N; i++) {
      const uint32_t lt = o_le + 1 + 3 * N + i * (3 + ec_n2b(CS + 1) + 6), eq = lt + 3 + ec_n2b(CS + 1);
      c.cp(lt + 1, n[i]);
      c.cp(lt + 2, r[i]);
      V v = n2b_new(lt + 3, c.sub(c.add(n[i], c.pow2(CS)), r[i]), CS + 1);
      V lto = c.put(lt, c.sub(c.u64(1), c.bit(v, CS)));
      V eqo = isequal(eq, n[i], r[i]);
      res = i == 0 ? c.put(o_le + 1 + 2 * N + i, c.add(lto, eqo)) : c.put(o_le + 1 + 2 * N + i, c.add(lto, c.mul(eqo, res)));
    }
    c.cp(o_le, res);
    V gt = c.put(o_gt, c.sub(c.u64(1), res));
    c.check_one(gt);  // bigInt.circom:245
    // mult2 = div * modulus; isZero.in[i] = mult[i] - mult2[i] - mod[i] (bigInt.circom:252-271)
    V iz[2 * N - 1];
    bmneq_cb(o_m2, N + 1, N, q, n, [&](int i, const V& m2) {
      if (i < 2 * N - 1) {
        V v = c.sub(mo[i], m2);
        if (i < N) v = c.sub(v, r[i]);
        iz[i] = c.put(o_isz + i, v);
      }
    });
    bisz(o_isz, 2 * CS + ec_log_ceil(2 * N), 2 * N - 1, iz);
  }

  PZK_WALK void run(int type) {
    if (type == ECT_DBL) dbl();
    else if (type == ECT_ADD) add();
    else mm();
  }
};

}  // namespace pzk
