/* oracle/r1cs_check.c — constraint checker for RegisterIdentityBuilder witnesses.
 *
 * TEST INFRASTRUCTURE ONLY (like witness_oracle.c): loaded by tests/ as a checker; the shipped
 * library never links or loads it.
 *
 * What it restates: the CONSTRAINTS of every template on the hot path — each `<==` and `===` of
 * the .circom sources, as the quadratic relation A * B = C (or the linear A = C) it compiles to —
 * and checks them over a whole witness. This is the acceptance test the reference applies to a
 * witness (circom_tester's checkConstraints, test/automatisationTest.js:51), restated because the
 * reference's .r1cs cannot be compiled here. It is written from the templates
 * independently of the witness oracle: it walks the component tree itself, allocating every
 * component's signals in the --O0 numbering of DESIGN.md §2 (own outputs, inputs, intermediates in
 * declaration order, then subcomponents in creation order), and never computes a witness value —
 * it only evaluates constraints on the values it is given. `<--` assignments are not constraints:
 * the signals they set (bits, quotients, inverses) are pinned by the constraints that follow them.
 *
 * Coverage: every signal a constraint reads is marked; ck_report() returns how many witness
 * elements no constraint touches (declared-but-unconstrained signals of the templates, listed in
 * tests/test_r1cs.py).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "fr.h"

typedef struct {
  const fr_t *w;
  size_t n;
  uint8_t *cov;
  uint64_t n_cons, n_bad;
  int64_t first_bad;        /* index of the first failing constraint (in evaluation order) */
  const char *first_tmpl;   /* its template and reference file:line */
  int first_line;
  size_t first_at;          /* base offset of the component it belongs to */
  int oob;                  /* a signal index past the witness: allocation mismatch */
} ck_t;

/* structure trace (r1cs_shape.inc.c): while TR is set, every constraint also records the signals it reads and its
 * residual lhs - rhs */
typedef struct {
  uint32_t *sig; uint64_t n_sig, cap_sig;  /* signals read, constraint after constraint */
  uint64_t *off; fr_t *res; uint64_t n_cons, cap_cons, cap_res;  /* per constraint: end of its reads, residual */
  int nomem;
} ck_tr_t;
static ck_tr_t *TR = NULL;
static void tr_read(size_t i);
static void tr_cons(fr_t residual);

/* signal read: marks coverage */
static inline fr_t S(ck_t *c, size_t i) {
  if (i >= c->n) { c->oob = 1; return fr_zero(); }
  c->cov[i] = 1;
  if (TR) tr_read(i);
  return c->w[i];
}
static void req(ck_t *c, fr_t lhs, fr_t rhs, const char *tmpl, int line, size_t at) {
  if (TR) tr_cons(fr_sub(lhs, rhs));
  if (!fr_eq(lhs, rhs)) {
    if (!c->n_bad) { c->first_bad = (int64_t)c->n_cons; c->first_tmpl = tmpl; c->first_line = line; c->first_at = at; }
    c->n_bad++;
  }
  c->n_cons++;
}
#define EQ(lhs, rhs, T, L) req(c, (lhs), (rhs), T, L, b)
static inline fr_t KC(uint64_t v) { return fr_u64(v); }
static inline fr_t ADD(fr_t a, fr_t b) { return fr_add(a, b); }
static inline fr_t SUB(fr_t a, fr_t b) { return fr_sub(a, b); }
static inline fr_t MUL(fr_t a, fr_t b) { return fr_mul(a, b); }
static fr_t P2[256];

/* ============================================================ bitify / comparators */
static size_t ck_aliascheck(ck_t *c, size_t b);

/* Num2Bits(LEN) bitify.circom:10-32: out[LEN] | in | sum[LEN] | [AliasCheck] */
static size_t ck_num2bits(ck_t *c, size_t b, int L) {
  const char *T = "Num2Bits bitify.circom";
  size_t out = b, in = b + L, sum = b + L + 1;
  for (int i = 0; i < L; i++) EQ(MUL(S(c, out + i), SUB(S(c, out + i), KC(1))), fr_zero(), T, 18);
  EQ(MUL(S(c, out), S(c, out)), S(c, sum), T, 21);
  for (int i = 1; i < L; i++) EQ(ADD(MUL(P2[i], S(c, out + i)), S(c, sum + i - 1)), S(c, sum + i), T, 23);
  EQ(S(c, in), S(c, sum + L - 1), T, 26);
  size_t sz = 2 * (size_t)L + 1;
  if (L == 254) {
    size_t a = b + sz;  /* aliascheck.in <== out (:30) */
    for (int i = 0; i < 254; i++) EQ(S(c, a + i), S(c, out + i), T, 30);
    sz += ck_aliascheck(c, a);
  }
  return sz;
}

/* Bits2Num(LEN) bitify.circom:38-55: out | in[LEN] | sum[LEN] | [AliasCheck] */
static size_t ck_bits2num(ck_t *c, size_t b, int L) {
  const char *T = "Bits2Num bitify.circom";
  size_t out = b, in = b + 1, sum = b + 1 + L;
  EQ(MUL(S(c, in), S(c, in)), S(c, sum), T, 45);
  for (int i = 1; i < L; i++) EQ(ADD(MUL(P2[i], S(c, in + i)), S(c, sum + i - 1)), S(c, sum + i), T, 48);
  EQ(S(c, out), S(c, sum + L - 1), T, 50);
  size_t sz = 2 * (size_t)L + 1;
  if (L == 254) {
    size_t a = b + sz;
    for (int i = 0; i < 254; i++) EQ(S(c, a + i), S(c, in + i), T, 53);
    sz += ck_aliascheck(c, a);
  }
  return sz;
}

/* CompConstant(ct) compconstant.circom:7-55: out | in[254] | parts[127] | sout | Num2Bits(135) */
static size_t ck_compconst(ck_t *c, size_t b, fr_t ct) {
  const char *T = "CompConstant compconstant.circom";
  size_t out = b, in = b + 1, parts = b + 255, sout = b + 382, n2b = b + 383;
  fr_t bb = SUB(P2[128], KC(1)), a = KC(1), e = KC(1), sum = fr_zero();
  for (int i = 0; i < 127; i++) {
    int clsb = fr_bit(ct, 2 * i), cmsb = fr_bit(ct, 2 * i + 1);
    fr_t sl = S(c, in + 2 * i), sm = S(c, in + 2 * i + 1), sms = MUL(sm, sl), rhs;
    if (!cmsb && !clsb) rhs = ADD(ADD(fr_neg(MUL(bb, sms)), MUL(bb, sm)), MUL(bb, sl));
    else if (!cmsb && clsb) rhs = ADD(SUB(ADD(SUB(MUL(a, sms), MUL(a, sl)), MUL(bb, sm)), MUL(a, sm)), a);
    else if (cmsb && !clsb) rhs = ADD(SUB(MUL(bb, sms), MUL(a, sm)), a);
    else rhs = ADD(fr_neg(MUL(a, sms)), a);
    EQ(S(c, parts + i), rhs, T, 30);
    sum = ADD(sum, S(c, parts + i));
    bb = SUB(bb, e); a = ADD(a, e); e = ADD(e, e);
  }
  EQ(S(c, sout), sum, T, 46);
  EQ(S(c, n2b + 135), S(c, sout), T, 50);
  EQ(S(c, out), S(c, n2b + 127), T, 52);
  return 383 + ck_num2bits(c, n2b, 135);
}

/* AliasCheck aliascheck.circom:7-14: in[254] | CompConstant(-1) */
static size_t ck_aliascheck(ck_t *c, size_t b) {
  const char *T = "AliasCheck aliascheck.circom";
  size_t cc = b + 254;
  for (int i = 0; i < 254; i++) EQ(S(c, cc + 1 + i), S(c, b + i), T, 12);
  size_t sz = 254 + ck_compconst(c, cc, fr_neg(KC(1)));
  EQ(S(c, cc), fr_zero(), T, 14);
  return sz;
}

/* IsZero comparators.circom:11-21: out | in | inv */
static size_t ck_iszero(ck_t *c, size_t b) {
  const char *T = "IsZero comparators.circom";
  EQ(S(c, b), ADD(fr_neg(MUL(S(c, b + 1), S(c, b + 2))), KC(1)), T, 19);
  EQ(MUL(S(c, b + 1), S(c, b)), fr_zero(), T, 20);
  return 3;
}

/* IsEqual comparators.circom:24-33: out | in[2] | IsZero */
static size_t ck_isequal(ck_t *c, size_t b) {
  const char *T = "IsEqual comparators.circom";
  size_t z = b + 3;
  EQ(S(c, z + 1), SUB(S(c, b + 2), S(c, b + 1)), T, 30);
  ck_iszero(c, z);
  EQ(S(c, b), S(c, z), T, 32);
  return 6;
}

/* LessThan(LEN) comparators.circom:46-57: out | in[2] | Num2Bits(LEN+1) */
static size_t ck_lessthan(ck_t *c, size_t b, int L) {
  const char *T = "LessThan comparators.circom";
  size_t n = b + 3;
  EQ(S(c, n + L + 1), SUB(ADD(S(c, b + 1), P2[L]), S(c, b + 2)), T, 53);
  size_t sz = 3 + ck_num2bits(c, n, L + 1);
  EQ(S(c, b), SUB(KC(1), S(c, n + L)), T, 55);
  return sz;
}

/* ============================================================ int/arithmetic.circom */
/* GetLastBitUnsecure arithmetic.circom:161-171: bit, div | in */
static size_t ck_lastbit(ck_t *c, size_t b) {
  const char *T = "GetLastBitUnsecure int/arithmetic.circom";
  fr_t bit = S(c, b), div = S(c, b + 1);
  EQ(MUL(SUB(KC(1), bit), bit), fr_zero(), T, 169);
  EQ(ADD(MUL(div, KC(2)), MUL(bit, bit)), S(c, b + 2), T, 170);
  return 3;
}

/* GetLastNBits(N) arithmetic.circom:178-204: div, out[N] | in | check[N] | GetLastBitUnsecure[N] */
static size_t ck_lastnbits(ck_t *c, size_t b, int N) {
  const char *T = "GetLastNBits int/arithmetic.circom";
  size_t div = b, out = b + 1, in = b + 1 + N, chk = b + 2 + N, g = b + 2 + 2 * (size_t)N;
  for (int i = 0; i < N; i++) {
    size_t gi = g + 3 * (size_t)i;
    ck_lastbit(c, gi);
    EQ(S(c, gi + 2), i == 0 ? S(c, in) : S(c, gi - 3 + 1), T, i == 0 ? 188 : 190);
    EQ(S(c, out + i), S(c, gi), T, 192);
  }
  EQ(S(c, div), S(c, g + 3 * (size_t)(N - 1) + 1), T, 195);
  EQ(MUL(S(c, out), S(c, out)), S(c, chk), T, 198);
  for (int i = 1; i < N; i++) EQ(ADD(S(c, chk + i - 1), MUL(S(c, out + i), P2[i])), S(c, chk + i), T, 200);
  EQ(ADD(S(c, chk + N - 1), MUL(S(c, div), P2[N])), S(c, in), T, 203);
  return 5 * (size_t)N + 2;
}

/* GetSumOfNElements(N) arithmetic.circom:210-226: out | in[N] | sum[N-1] */
static size_t ck_getsum(ck_t *c, size_t b, int N) {
  const char *T = "GetSumOfNElements int/arithmetic.circom";
  size_t in = b + 1, sum = b + 1 + N;
  EQ(S(c, sum), ADD(S(c, in), S(c, in + 1)), T, 219);
  for (int i = 1; i < N - 1; i++) EQ(S(c, sum + i), ADD(S(c, sum + i - 1), S(c, in + i + 1)), T, 221);
  EQ(S(c, b), S(c, sum + N - 2), T, 224);
  return 2 * (size_t)N;
}

/* ============================================================ SHA-2 (224/256) */
/* XOR3_v2 sha2Common.circom:80-88: out | x, y, z | tmp */
static size_t ck_xor3(ck_t *c, size_t b) {
  const char *T = "XOR3_v2 hasher/sha2/sha2Common.circom";
  fr_t x = S(c, b + 1), y = S(c, b + 2), z = S(c, b + 3), tmp = S(c, b + 4);
  EQ(tmp, MUL(y, z), T, 86);
  fr_t f = ADD(SUB(SUB(KC(1), MUL(KC(2), y)), MUL(KC(2), z)), MUL(KC(4), tmp));
  EQ(S(c, b), SUB(ADD(ADD(MUL(x, f), y), z), MUL(KC(2), tmp)), T, 87);
  return 5;
}

/* Bits2 sha2Common.circom:57-68: lo, hi | xy */
static size_t ck_bits2(ck_t *c, size_t b) {
  const char *T = "Bits2 hasher/sha2/sha2Common.circom";
  fr_t lo = S(c, b), hi = S(c, b + 1);
  EQ(MUL(lo, SUB(KC(1), lo)), fr_zero(), T, 65);
  EQ(MUL(hi, SUB(KC(1), hi)), fr_zero(), T, 66);
  EQ(S(c, b + 2), ADD(MUL(KC(2), hi), lo), T, 68);
  return 3;
}

/* the (1 << i) * bit[i] inputs of a GetSumOfNElements(32) at g from 32 bits at `bits` (stride st) */
static void wire_sum32(ck_t *c, size_t b, size_t g, size_t bits, size_t st, const char *T, int line) {
  for (int i = 0; i < 32; i++) EQ(S(c, g + 1 + i), MUL(P2[i], S(c, bits + (size_t)i * st)), T, line);
}

/* Sha2_224_256Shedule sha256Schedule.circom:11-72:
 * outWords[64] | chunkBits[16][32] | outBits[64][32] | sumN[16], then per m: s0Sum, s1Sum, (s0Xor, s1Xor)[32], modulo, bits2Num */
static size_t ck_schedule(ck_t *c, size_t b) {
  const char *T = "Sha2_224_256Shedule hasher/sha2/sha256/sha256Schedule.circom";
  size_t ow = b, cb = b + 64, ob = b + 64 + 512, o = b + 64 + 512 + 2048;
  for (int k = 0; k < 16; k++) {
    o += ck_getsum(c, o, 32);
    size_t g = o - 64;
    wire_sum32(c, b, g, cb + 32 * (size_t)k, 1, T, 22);
    EQ(S(c, ow + k), S(c, g), T, 24);
    for (int i = 0; i < 32; i++) EQ(S(c, ob + 32 * (size_t)k + i), S(c, cb + 32 * (size_t)k + i), T, 25);
  }
  for (int m = 16; m < 64; m++) {
    size_t k = m - 15, l = m - 2;
    size_t s0 = o, s1 = o + 64;
    o += ck_getsum(c, s0, 32) + ck_getsum(c, s1, 32);
    for (int i = 0; i < 32; i++) {
      size_t x0 = o, x1 = o + 5;
      o += ck_xor3(c, x0) + ck_xor3(c, x1);
      EQ(S(c, x0 + 1), S(c, ob + 32 * k + (i + 7) % 32), T, 51);
      EQ(S(c, x0 + 2), S(c, ob + 32 * k + (i + 18) % 32), T, 52);
      EQ(S(c, x0 + 3), i < 29 ? S(c, ob + 32 * k + i + 3) : fr_zero(), T, 53);
      EQ(S(c, s0 + 1 + i), MUL(P2[i], S(c, x0)), T, 54);
      EQ(S(c, x1 + 1), S(c, ob + 32 * l + (i + 17) % 32), T, 57);
      EQ(S(c, x1 + 2), S(c, ob + 32 * l + (i + 19) % 32), T, 58);
      EQ(S(c, x1 + 3), i < 22 ? S(c, ob + 32 * l + i + 10) : fr_zero(), T, 59);
      EQ(S(c, s1 + 1 + i), MUL(P2[i], S(c, x1)), T, 60);
    }
    size_t md = o;
    o += ck_lastnbits(c, md, 32);
    EQ(S(c, md + 33), ADD(ADD(ADD(S(c, s1), S(c, ow + m - 7)), S(c, s0)), S(c, ow + m - 16)), T, 65);
    for (int i = 0; i < 32; i++) EQ(S(c, ob + 32 * (size_t)m + i), S(c, md + 1 + i), T, 66);
    size_t bn = o;
    o += ck_bits2num(c, bn, 32);
    for (int i = 0; i < 32; i++) EQ(S(c, bn + 1 + i), S(c, ob + 32 * (size_t)m + i), T, 68);
    EQ(S(c, ow + m), S(c, bn), T, 69);
  }
  return o - b;
}

static const uint32_t SHA256_K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

/* Sha2_224_256CompressInner sha256Compress.circom:11-96:
 * outA[32] outB[32] outC[32] outDD outE[32] outF[32] outG[32] outHH | inp key a[32] b[32] c[32] dd e[32] f[32] g[32] hh |
 * chb[32] overflowE overflowA | dSum hSum s0Sum s1Sum mjSum chSum (major, s0Xor, s1Xor)[32] decomposeE decomposeA */
static size_t ck_compress(ck_t *c, size_t b) {
  const char *T = "Sha2_224_256CompressInner hasher/sha2/sha256/sha256Compress.circom";
  size_t oA = b, oB = b + 32, oC = b + 64, oDD = b + 96, oE = b + 97, oF = b + 129, oG = b + 161, oHH = b + 193;
  size_t inp = b + 194, key = b + 195, a = b + 196, bb = b + 228, cc = b + 260, dd = b + 292, e = b + 293,
         f = b + 325, g = b + 357, hh = b + 389;
  size_t chb = b + 390, ovE = b + 422, ovA = b + 423, o = b + 424;
  for (int i = 0; i < 32; i++) {
    EQ(S(c, oG + i), S(c, f + i), T, 37);
    EQ(S(c, oF + i), S(c, e + i), T, 38);
    EQ(S(c, oC + i), S(c, bb + i), T, 39);
    EQ(S(c, oB + i), S(c, a + i), T, 40);
  }
  size_t dS = o, hS = o + 64, s0S = o + 128, s1S = o + 192, mjS = o + 256, chS = o + 320;
  for (int q = 0; q < 6; q++) o += ck_getsum(c, o, 32);
  wire_sum32(c, b, dS, cc, 1, T, 46);
  wire_sum32(c, b, hS, g, 1, T, 47);
  EQ(S(c, oDD), S(c, dS), T, 49);
  EQ(S(c, oHH), S(c, hS), T, 50);
  for (int i = 0; i < 32; i++) {
    size_t mj = o, x0 = o + 3, x1 = o + 8;
    o += ck_bits2(c, mj) + ck_xor3(c, x0) + ck_xor3(c, x1);
    EQ(S(c, chb + i), ADD(MUL(S(c, e + i), SUB(S(c, f + i), S(c, g + i))), S(c, g + i)), T, 65);
    EQ(S(c, chS + 1 + i), MUL(P2[i], S(c, chb + i)), T, 66);
    EQ(S(c, mj + 2), ADD(ADD(S(c, a + i), S(c, bb + i)), S(c, cc + i)), T, 70);
    EQ(S(c, mjS + 1 + i), MUL(P2[i], S(c, mj + 1)), T, 71);
    EQ(S(c, x0 + 1), S(c, a + (i + 2) % 32), T, 74);
    EQ(S(c, x0 + 2), S(c, a + (i + 13) % 32), T, 75);
    EQ(S(c, x0 + 3), S(c, a + (i + 22) % 32), T, 76);
    EQ(S(c, s0S + 1 + i), MUL(P2[i], S(c, x0)), T, 77);
    EQ(S(c, x1 + 1), S(c, e + (i + 6) % 32), T, 80);
    EQ(S(c, x1 + 2), S(c, e + (i + 11) % 32), T, 81);
    EQ(S(c, x1 + 3), S(c, e + (i + 25) % 32), T, 82);
    EQ(S(c, s1S + 1 + i), MUL(P2[i], S(c, x1)), T, 83);
  }
  fr_t t1 = ADD(ADD(ADD(S(c, s1S), S(c, chS)), S(c, key)), S(c, inp));
  EQ(S(c, ovE), ADD(ADD(S(c, dd), S(c, hh)), t1), T, 87);
  EQ(S(c, ovA), ADD(ADD(ADD(S(c, hh), t1), S(c, s0S)), S(c, mjS)), T, 88);
  size_t dE = o;
  o += ck_lastnbits(c, dE, 32);
  EQ(S(c, dE + 33), S(c, ovE), T, 91);
  for (int i = 0; i < 32; i++) EQ(S(c, oE + i), S(c, dE + 1 + i), T, 92);
  size_t dA = o;
  o += ck_lastnbits(c, dA, 32);
  EQ(S(c, dA + 33), S(c, ovA), T, 95);
  for (int i = 0; i < 32; i++) EQ(S(c, oA + i), S(c, dA + 1 + i), T, 96);
  return o - b;
}

/* Sha2_224_256Rounds(64) sha256Rounds.circom:12-125:
 * outHash[8][32] | words[64] inpHash[8][32] | a b c [65][32] dd[65] e f g [65][32] hh[65] ROUND_KEYS[64] hashWords[8] |
 * roundKeys sumDd sumHh sum[8] compress[64] modulo[8] sumA sumB sumC sumE sumF sumG */
static size_t ck_rounds(ck_t *c, size_t b) {
  const char *T = "Sha2_224_256Rounds hasher/sha2/sha256/sha256Rounds.circom";
  const int n = 64;
  size_t outH = b, words = b + 256, inH = b + 320;
  size_t A = b + 576, B = A + 65 * 32, C = B + 65 * 32, DD = C + 65 * 32, E = DD + 65, F = E + 65 * 32, G = F + 65 * 32,
         HH = G + 65 * 32, RK = HH + 65, HW = RK + 64, o = HW + 8;
  size_t rk = o;  /* Sha2_224_256RoundKeys sha256RoundConst.circom:6-25: out[64] */
  for (int j = 0; j < 64; j++) req(c, S(c, rk + j), KC(SHA256_K[j]), "Sha2_224_256RoundKeys sha256RoundConst.circom", 23, rk);
  o += 64;
  for (int j = 0; j < 64; j++) EQ(S(c, RK + j), S(c, rk + j), T, 38);
  for (int i = 0; i < 32; i++) {
    EQ(S(c, A + i), S(c, inH + i), T, 40);
    EQ(S(c, B + i), S(c, inH + 32 + i), T, 41);
    EQ(S(c, C + i), S(c, inH + 64 + i), T, 42);
    EQ(S(c, E + i), S(c, inH + 128 + i), T, 44);
    EQ(S(c, F + i), S(c, inH + 160 + i), T, 45);
    EQ(S(c, G + i), S(c, inH + 192 + i), T, 46);
  }
  size_t sDd = o, sHh = o + 64;
  o += ck_getsum(c, sDd, 32) + ck_getsum(c, sHh, 32);
  wire_sum32(c, b, sDd, inH + 96, 1, T, 51);
  wire_sum32(c, b, sHh, inH + 224, 1, T, 52);
  EQ(S(c, DD), S(c, sDd), T, 54);
  EQ(S(c, HH), S(c, sHh), T, 55);
  for (int j = 0; j < 8; j++) {
    size_t s = o;
    o += ck_getsum(c, s, 32);
    wire_sum32(c, b, s, inH + 32 * (size_t)j, 1, T, 62);
    EQ(S(c, HW + j), S(c, s), T, 64);
  }
  for (int k = 0; k < n; k++) {
    size_t ci = o;
    o += ck_compress(c, ci);
    EQ(S(c, ci + 194), S(c, words + k), T, 73);
    EQ(S(c, ci + 195), S(c, RK + k), T, 74);
    for (int i = 0; i < 32; i++) {
      EQ(S(c, ci + 196 + i), S(c, A + 32 * (size_t)k + i), T, 76);
      EQ(S(c, ci + 228 + i), S(c, B + 32 * (size_t)k + i), T, 77);
      EQ(S(c, ci + 260 + i), S(c, C + 32 * (size_t)k + i), T, 78);
      EQ(S(c, ci + 293 + i), S(c, E + 32 * (size_t)k + i), T, 80);
      EQ(S(c, ci + 325 + i), S(c, F + 32 * (size_t)k + i), T, 81);
      EQ(S(c, ci + 357 + i), S(c, G + 32 * (size_t)k + i), T, 82);
      EQ(S(c, A + 32 * (size_t)(k + 1) + i), S(c, ci + i), T, 85);
      EQ(S(c, B + 32 * (size_t)(k + 1) + i), S(c, ci + 32 + i), T, 86);
      EQ(S(c, C + 32 * (size_t)(k + 1) + i), S(c, ci + 64 + i), T, 87);
      EQ(S(c, E + 32 * (size_t)(k + 1) + i), S(c, ci + 97 + i), T, 89);
      EQ(S(c, F + 32 * (size_t)(k + 1) + i), S(c, ci + 129 + i), T, 90);
      EQ(S(c, G + 32 * (size_t)(k + 1) + i), S(c, ci + 161 + i), T, 91);
    }
    EQ(S(c, ci + 292), S(c, DD + k), T, 79);
    EQ(S(c, ci + 389), S(c, HH + k), T, 83);
    EQ(S(c, DD + k + 1), S(c, ci + 96), T, 88);
    EQ(S(c, HH + k + 1), S(c, ci + 193), T, 92);
  }
  size_t md = o;
  for (int j = 0; j < 8; j++) o += ck_lastnbits(c, o, 32);
  size_t sums[6], src[6] = {A, B, C, E, F, G};
  for (int q = 0; q < 6; q++) {
    sums[q] = o;
    o += ck_getsum(c, o, 32);
    wire_sum32(c, b, sums[q], src[q] + 32 * (size_t)n, 1, T, 106);
  }
  static const int which[8] = {0, 1, 2, -1, 3, 4, 5, -2};
  for (int j = 0; j < 8; j++) {
    size_t mj = md + 162 * (size_t)j;
    fr_t rhs = which[j] >= 0 ? S(c, sums[which[j]]) : which[j] == -1 ? S(c, DD + n) : S(c, HH + n);
    EQ(S(c, mj + 33), ADD(S(c, HW + j), rhs), T, 114);
    for (int i = 0; i < 32; i++) EQ(S(c, outH + 32 * (size_t)j + i), S(c, mj + 1 + i), T, 123);
  }
  return o - b;
}

static const uint32_t SHA256_IV[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                      0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
static const uint32_t SHA224_IV[8] = {0xc1059ed8, 0x367cd507, 0x3070dd17, 0xf70e5939,
                                      0xffc00b31, 0x68581511, 0x64f98fa7, 0xbefa4fa4};

/* Sha256HashChunks(B) sha256HashChunks.circom:8-48 (O = 256) / Sha224HashChunks(B) sha224/sha224HashChunks.circom
 * (O = 224, SHA-224 IV): out[O] | in[512B] | states[B+1][8][32] | iv, (sch, rds)[B] */
static size_t ck_sha2chunks(ck_t *c, size_t b, int B, int O) {
  const char *T = O == 256 ? "Sha256HashChunks hasher/sha2/sha256/sha256HashChunks.circom"
                           : "Sha224HashChunks hasher/sha2/sha224/sha224HashChunks.circom";
  size_t out = b, in = b + O, st = in + 512 * (size_t)B, o = st + (size_t)(B + 1) * 256;
  size_t iv = o;
  const uint32_t *IV = O == 256 ? SHA256_IV : SHA224_IV;
  for (int k = 0; k < 8; k++)
    for (int i = 0; i < 32; i++)
      req(c, S(c, iv + 32 * k + i), KC((IV[k] >> i) & 1), "Sha256InitialValue sha256InitialValue.circom", 24, iv);
  o += 256;
  for (int q = 0; q < 256; q++) EQ(S(c, st + q), S(c, iv + q), T, 21);
  for (int m = 0; m < B; m++) {
    size_t sch = o;
    o += ck_schedule(c, sch);
    size_t rds = o;
    o += ck_rounds(c, rds);
    for (int k = 0; k < 16; k++)
      for (int i = 0; i < 32; i++)
        EQ(S(c, sch + 64 + 32 * k + i), S(c, in + 512 * (size_t)m + 32 * k + 31 - i), T, 33);
    for (int q = 0; q < 64; q++) EQ(S(c, rds + 256 + q), S(c, sch + q), T, 38);
    for (int q = 0; q < 256; q++) {
      EQ(S(c, rds + 320 + q), S(c, st + 256 * (size_t)m + q), T, 40);
      EQ(S(c, st + 256 * (size_t)(m + 1) + q), S(c, rds + q), T, 41);
    }
  }
  for (int j = 0; j < O / 32; j++)
    for (int i = 0; i < 32; i++) EQ(S(c, out + 32 * j + i), S(c, st + 256 * (size_t)B + 32 * j + 31 - i), T, 46);
  return o - b;
}


/* ============================================================ SHA-2 (384/512) */
/* the (1 << i) * bit[i] inputs of a GetSumOfNElements(64) at g from 64 bits at `bits` */
static void wire_sum64(ck_t *c, size_t b, size_t g, size_t bits, const char *T, int line) {
  for (int i = 0; i < 64; i++) EQ(S(c, g + 1 + i), MUL(P2[i], S(c, bits + i)), T, line);
}

/* Sha2_384_512Schedule sha512/sha512Schedule.circom:11-74:
 * outWords[80] | chunkBits[16][64] | outBits[80][64] | sumN[16], then per m: s0Sum, s1Sum, (s0Xor, s1Xor)[64], modulo, bits2Num */
static size_t ck_schedule512(ck_t *c, size_t b) {
  const char *T = "Sha2_384_512Schedule hasher/sha2/sha512/sha512Schedule.circom";
  size_t ow = b, cb = b + 80, ob = cb + 1024, o = ob + 5120;
  for (int k = 0; k < 16; k++) {
    size_t g = o;
    o += ck_getsum(c, g, 64);
    wire_sum64(c, b, g, cb + 64 * (size_t)k, T, 25);
    EQ(S(c, ow + k), S(c, g), T, 27);
    for (int i = 0; i < 64; i++) EQ(S(c, ob + 64 * (size_t)k + i), S(c, cb + 64 * (size_t)k + i), T, 28);
  }
  for (int m = 16; m < 80; m++) {
    size_t k = m - 15, l = m - 2;
    size_t s0 = o, s1 = o + 128;
    o += ck_getsum(c, s0, 64) + ck_getsum(c, s1, 64);
    for (int i = 0; i < 64; i++) {
      size_t x0 = o, x1 = o + 5;
      o += ck_xor3(c, x0) + ck_xor3(c, x1);
      EQ(S(c, x0 + 1), S(c, ob + 64 * k + (i + 1) % 64), T, 54);
      EQ(S(c, x0 + 2), S(c, ob + 64 * k + (i + 8) % 64), T, 55);
      EQ(S(c, x0 + 3), i < 57 ? S(c, ob + 64 * k + i + 7) : fr_zero(), T, 56);
      EQ(S(c, s0 + 1 + i), MUL(P2[i], S(c, x0)), T, 57);
      EQ(S(c, x1 + 1), S(c, ob + 64 * l + (i + 19) % 64), T, 60);
      EQ(S(c, x1 + 2), S(c, ob + 64 * l + (i + 61) % 64), T, 61);
      EQ(S(c, x1 + 3), i < 58 ? S(c, ob + 64 * l + i + 6) : fr_zero(), T, 62);
      EQ(S(c, s1 + 1 + i), MUL(P2[i], S(c, x1)), T, 63);
    }
    size_t md = o;
    o += ck_lastnbits(c, md, 64);
    EQ(S(c, md + 65), ADD(ADD(ADD(S(c, s1), S(c, ow + m - 7)), S(c, s0)), S(c, ow + m - 16)), T, 68);
    for (int i = 0; i < 64; i++) EQ(S(c, ob + 64 * (size_t)m + i), S(c, md + 1 + i), T, 69);
    size_t bn = o;
    o += ck_bits2num(c, bn, 64);
    for (int i = 0; i < 64; i++) EQ(S(c, bn + 1 + i), S(c, ob + 64 * (size_t)m + i), T, 71);
    EQ(S(c, ow + m), S(c, bn), T, 72);
  }
  return o - b;
}

static const uint64_t SHA512_K[80] = {
    0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL, 0x3956c25bf348b538ULL,
    0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL, 0xd807aa98a3030242ULL, 0x12835b0145706fbeULL,
    0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL, 0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL,
    0xc19bf174cf692694ULL, 0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
    0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL, 0x983e5152ee66dfabULL,
    0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL, 0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL,
    0x06ca6351e003826fULL, 0x142929670a0e6e70ULL, 0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL,
    0x53380d139d95b3dfULL, 0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
    0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL, 0xd192e819d6ef5218ULL,
    0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL, 0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL,
    0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL, 0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL,
    0x682e6ff3d6b2b8a3ULL, 0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
    0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL, 0xca273eceea26619cULL,
    0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL, 0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL,
    0x113f9804bef90daeULL, 0x1b710b35131c471bULL, 0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL,
    0x431d67c49c100d4cULL, 0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL};

/* Sha2_384_512CompressInner sha512/sha512Compress.circom:11-96:
 * outA[64] outB[64] outC[64] outDD outE[64] outF[64] outG[64] outHH | inp key a[64] b[64] c[64] dd e[64] f[64] g[64] hh |
 * chb[64] overflowE overflowA | dSum hSum s0Sum s1Sum mjSum chSum (major, s0Xor, s1Xor)[64] decomposeE decomposeA */
static size_t ck_compress512(ck_t *c, size_t b) {
  const char *T = "Sha2_384_512CompressInner hasher/sha2/sha512/sha512Compress.circom";
  size_t oA = b, oB = b + 64, oC = b + 128, oDD = b + 192, oE = b + 193, oF = b + 257, oG = b + 321, oHH = b + 385;
  size_t inp = b + 386, key = b + 387, a = b + 388, bb = b + 452, cc = b + 516, dd = b + 580, e = b + 581,
         f = b + 645, g = b + 709, hh = b + 773;
  size_t chb = b + 774, ovE = b + 838, ovA = b + 839, o = b + 840;
  size_t dS = o, hS = o + 128, s0S = o + 256, s1S = o + 384, mjS = o + 512, chS = o + 640;
  for (int q = 0; q < 6; q++) o += ck_getsum(c, o, 64);
  wire_sum64(c, b, dS, cc, T, 43);
  wire_sum64(c, b, hS, g, T, 44);
  for (int i = 0; i < 64; i++) {
    EQ(S(c, oG + i), S(c, f + i), T, 39);
    EQ(S(c, oF + i), S(c, e + i), T, 40);
    EQ(S(c, oC + i), S(c, bb + i), T, 41);
    EQ(S(c, oB + i), S(c, a + i), T, 42);
  }
  EQ(S(c, oDD), S(c, dS), T, 46);
  EQ(S(c, oHH), S(c, hS), T, 47);
  for (int i = 0; i < 64; i++) {
    size_t mj = o, x0 = o + 3, x1 = o + 8;
    o += ck_bits2(c, mj) + ck_xor3(c, x0) + ck_xor3(c, x1);
    EQ(S(c, chb + i), ADD(MUL(S(c, e + i), SUB(S(c, f + i), S(c, g + i))), S(c, g + i)), T, 63);
    EQ(S(c, chS + 1 + i), MUL(P2[i], S(c, chb + i)), T, 64);
    EQ(S(c, mj + 2), ADD(ADD(S(c, a + i), S(c, bb + i)), S(c, cc + i)), T, 68);
    EQ(S(c, mjS + 1 + i), MUL(P2[i], S(c, mj + 1)), T, 69);
    EQ(S(c, x0 + 1), S(c, a + (i + 28) % 64), T, 72);
    EQ(S(c, x0 + 2), S(c, a + (i + 34) % 64), T, 73);
    EQ(S(c, x0 + 3), S(c, a + (i + 39) % 64), T, 74);
    EQ(S(c, s0S + 1 + i), MUL(P2[i], S(c, x0)), T, 75);
    EQ(S(c, x1 + 1), S(c, e + (i + 14) % 64), T, 78);
    EQ(S(c, x1 + 2), S(c, e + (i + 18) % 64), T, 79);
    EQ(S(c, x1 + 3), S(c, e + (i + 41) % 64), T, 80);
    EQ(S(c, s1S + 1 + i), MUL(P2[i], S(c, x1)), T, 81);
  }
  fr_t t1 = ADD(ADD(ADD(S(c, s1S), S(c, chS)), S(c, key)), S(c, inp));
  EQ(S(c, ovE), ADD(ADD(S(c, dd), S(c, hh)), t1), T, 85);
  EQ(S(c, ovA), ADD(ADD(ADD(S(c, hh), t1), S(c, s0S)), S(c, mjS)), T, 86);
  size_t dE = o;
  o += ck_lastnbits(c, dE, 64);
  EQ(S(c, dE + 65), S(c, ovE), T, 89);
  for (int i = 0; i < 64; i++) EQ(S(c, oE + i), S(c, dE + 1 + i), T, 90);
  size_t dA = o;
  o += ck_lastnbits(c, dA, 64);
  EQ(S(c, dA + 65), S(c, ovA), T, 93);
  for (int i = 0; i < 64; i++) EQ(S(c, oA + i), S(c, dA + 1 + i), T, 94);
  return o - b;
}

/* Sha2_384_512Rounds(80) sha512/sha512Rounds.circom:11-126:
 * outHash[8][64] | words[80] inpHash[8][64] | a b c [81][64] dd[81] e f g [81][64] hh[81] ROUND_KEYS[80] hashWords[8] |
 * roundKeys sumDd sumHh sum[8] compress[80] modulo[8] sumA sumB sumC sumE sumF sumG */
static size_t ck_rounds512(ck_t *c, size_t b) {
  const char *T = "Sha2_384_512Rounds hasher/sha2/sha512/sha512Rounds.circom";
  const int n = 80;
  size_t outH = b, words = b + 512, inH = b + 592;
  size_t A = b + 1104, B = A + 81 * 64, C = B + 81 * 64, DD = C + 81 * 64, E = DD + 81, F = E + 81 * 64, G = F + 81 * 64,
         HH = G + 81 * 64, RK = HH + 81, HW = RK + 80, o = HW + 8;
  size_t rk = o;  /* SHA2_384_512RoundKeys sha512RoundConst.circom:6-38: out[80] */
  for (int j = 0; j < 80; j++) req(c, S(c, rk + j), KC(SHA512_K[j]), "SHA2_384_512RoundKeys sha512RoundConst.circom", 35, rk);
  o += 80;
  for (int j = 0; j < 80; j++) EQ(S(c, RK + j), S(c, rk + j), T, 34);
  for (int i = 0; i < 64; i++) {
    EQ(S(c, A + i), S(c, inH + i), T, 36);
    EQ(S(c, B + i), S(c, inH + 64 + i), T, 37);
    EQ(S(c, C + i), S(c, inH + 128 + i), T, 38);
    EQ(S(c, E + i), S(c, inH + 256 + i), T, 40);
    EQ(S(c, F + i), S(c, inH + 320 + i), T, 41);
    EQ(S(c, G + i), S(c, inH + 384 + i), T, 42);
  }
  size_t sDd = o, sHh = o + 128;
  o += ck_getsum(c, sDd, 64) + ck_getsum(c, sHh, 64);
  wire_sum64(c, b, sDd, inH + 192, T, 47);
  wire_sum64(c, b, sHh, inH + 448, T, 48);
  EQ(S(c, DD), S(c, sDd), T, 50);
  EQ(S(c, HH), S(c, sHh), T, 51);
  for (int j = 0; j < 8; j++) {
    size_t sj = o;
    o += ck_getsum(c, sj, 64);
    wire_sum64(c, b, sj, inH + 64 * (size_t)j, T, 58);
    EQ(S(c, HW + j), S(c, sj), T, 60);
  }
  for (int k = 0; k < n; k++) {
    size_t ci = o;
    o += ck_compress512(c, ci);
    EQ(S(c, ci + 386), S(c, words + k), T, 69);
    EQ(S(c, ci + 387), S(c, RK + k), T, 70);
    for (int i = 0; i < 64; i++) {
      EQ(S(c, ci + 388 + i), S(c, A + 64 * (size_t)k + i), T, 73);
      EQ(S(c, ci + 452 + i), S(c, B + 64 * (size_t)k + i), T, 74);
      EQ(S(c, ci + 516 + i), S(c, C + 64 * (size_t)k + i), T, 75);
      EQ(S(c, ci + 581 + i), S(c, E + 64 * (size_t)k + i), T, 77);
      EQ(S(c, ci + 645 + i), S(c, F + 64 * (size_t)k + i), T, 78);
      EQ(S(c, ci + 709 + i), S(c, G + 64 * (size_t)k + i), T, 79);
      EQ(S(c, A + 64 * (size_t)(k + 1) + i), S(c, ci + i), T, 82);
      EQ(S(c, B + 64 * (size_t)(k + 1) + i), S(c, ci + 64 + i), T, 83);
      EQ(S(c, C + 64 * (size_t)(k + 1) + i), S(c, ci + 128 + i), T, 84);
      EQ(S(c, E + 64 * (size_t)(k + 1) + i), S(c, ci + 193 + i), T, 86);
      EQ(S(c, F + 64 * (size_t)(k + 1) + i), S(c, ci + 257 + i), T, 87);
      EQ(S(c, G + 64 * (size_t)(k + 1) + i), S(c, ci + 321 + i), T, 88);
    }
    EQ(S(c, ci + 580), S(c, DD + k), T, 76);
    EQ(S(c, ci + 773), S(c, HH + k), T, 80);
    EQ(S(c, DD + k + 1), S(c, ci + 192), T, 85);
    EQ(S(c, HH + k + 1), S(c, ci + 385), T, 89);
  }
  size_t md = o;
  for (int j = 0; j < 8; j++) o += ck_lastnbits(c, o, 64);
  size_t sums[6], src[6] = {A, B, C, E, F, G};
  for (int q = 0; q < 6; q++) {
    sums[q] = o;
    o += ck_getsum(c, o, 64);
    wire_sum64(c, b, sums[q], src[q] + 64 * (size_t)n, T, 105);
  }
  static const int which[8] = {0, 1, 2, -1, 3, 4, 5, -2};
  for (int j = 0; j < 8; j++) {
    size_t mj = md + 322 * (size_t)j;
    fr_t rhs = which[j] >= 0 ? S(c, sums[which[j]]) : which[j] == -1 ? S(c, DD + n) : S(c, HH + n);
    EQ(S(c, mj + 65), ADD(S(c, HW + j), rhs), T, 113);
    for (int i = 0; i < 64; i++) EQ(S(c, outH + 64 * (size_t)j + i), S(c, mj + 1 + i), T, 123);
  }
  return o - b;
}

static const uint64_t SHA512_IV64[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                                        0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                                        0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
static const uint64_t SHA384_IV64[8] = {0xcbbb9d5dc1059ed8ULL, 0x629a292a367cd507ULL, 0x9159015a3070dd17ULL,
                                        0x152fecd8f70e5939ULL, 0x67332667ffc00b31ULL, 0x8eb44a8768581511ULL,
                                        0xdb0c2e0d64f98fa7ULL, 0x47b5481dbefa4fa4ULL};

/* Sha384HashChunks(B) sha384/sha384HashChunks.circom:8-47 (O = 384) / Sha512HashChunks(B) sha512/sha512HashChunks.circom
 * (O = 512): out[O] | in[1024B] | states[B+1][8][64] | iv, (sch, rds)[B] */
static size_t ck_sha5chunks(ck_t *c, size_t b, int B, int O) {
  const char *T = O == 384 ? "Sha384HashChunks hasher/sha2/sha384/sha384HashChunks.circom"
                           : "Sha512HashChunks hasher/sha2/sha512/sha512HashChunks.circom";
  const int d = O == 384 ? 1 : 0;  /* Sha512HashChunks' lines are one above Sha384HashChunks' */
  size_t out = b, in = b + O, st = in + 1024 * (size_t)B, o = st + (size_t)(B + 1) * 512;
  size_t iv = o;
  const uint64_t *IV = O == 384 ? SHA384_IV64 : SHA512_IV64;
  for (int k = 0; k < 8; k++)
    for (int i = 0; i < 64; i++)
      req(c, S(c, iv + 64 * k + i), KC((IV[k] >> i) & 1),
          O == 384 ? "Sha384InitialValues sha384InitialValue.circom" : "Sha512InitialValues sha512InitialValue.circom", 24, iv);
  o += 512;
  for (int q = 0; q < 512; q++) EQ(S(c, st + q), S(c, iv + q), T, 19 + d);
  for (int m = 0; m < B; m++) {
    size_t sch = o;
    o += ck_schedule512(c, sch);
    size_t rds = o;
    o += ck_rounds512(c, rds);
    for (int k = 0; k < 16; k++)
      for (int i = 0; i < 64; i++)
        EQ(S(c, sch + 80 + 64 * k + i), S(c, in + 1024 * (size_t)m + 64 * k + 63 - i), T, 31 + d);
    for (int q = 0; q < 80; q++) EQ(S(c, rds + 512 + q), S(c, sch + q), T, 35 + d);
    for (int q = 0; q < 512; q++) {
      EQ(S(c, rds + 592 + q), S(c, st + 512 * (size_t)m + q), T, 37 + d);
      EQ(S(c, st + 512 * (size_t)(m + 1) + q), S(c, rds + q), T, 38 + d);
    }
  }
  for (int j = 0; j < O / 64; j++)
    for (int i = 0; i < 64; i++) EQ(S(c, out + 64 * j + i), S(c, st + 512 * (size_t)B + 64 * j + 63 - i), T, 43 + d);
  return o - b;
}

/* ============================================================ SHA-1 (hasher/sha1) */
/* RotL(32, L) rotate.circom: out[32] | in[32] */
static size_t ck_rotl(ck_t *c, size_t b, int L) {
  for (int i = 31; i >= 0; i--) EQ(S(c, b + i), S(c, b + 32 + (i + L) % 32), "RotL hasher/sha1/rotate.circom", 8);
  return 64;
}
/* H(x) / K(t) constants.circom: out[32] | bitify (Num2Bits(32)) */
static size_t ck_sha1const(ck_t *c, size_t b, uint32_t v, int line) {
  const char *T = "H / K hasher/sha1/constants.circom";
  size_t n = b + 32;
  size_t sz = 32 + ck_num2bits(c, n, 32);
  EQ(S(c, n + 32), KC(v), T, line);
  for (int k = 0; k < 32; k++) EQ(S(c, b + k), S(c, n + 31 - k), T, line + 2);
  return sz;
}
/* Xor4(n) xor4.circom: out[n] | a b c d | mid[n] aTemp[n] */
static size_t ck_xor4(ck_t *c, size_t b) {
  const char *T = "Xor4 hasher/sha1/xor4.circom";
  size_t out = b, a = b + 32, bb = b + 64, cc = b + 96, d = b + 128, mid = b + 160, at = b + 192;
  for (int k = 0; k < 32; k++) {
    fr_t B = S(c, bb + k), C = S(c, cc + k), M = S(c, mid + k), A = S(c, at + k), D = S(c, d + k);
    EQ(M, MUL(B, C), T, 15);
    EQ(A, SUB(ADD(ADD(MUL(S(c, a + k), ADD(SUB(SUB(KC(1), MUL(KC(2), B)), MUL(KC(2), C)), MUL(KC(4), M))), B), C), MUL(KC(2), M)), T, 16);
    EQ(S(c, out + k), ADD(SUB(A, MUL(MUL(KC(2), D), A)), D), T, 17);
  }
  return 224;
}
/* BinSum(NUM, LEN) bitify/operations.circom:9-29: out[LEN+NUM-1] | in[NUM][LEN] | sumN bits2Num[NUM] num2Bits */
static size_t ck_binsum(ck_t *c, size_t b, int N, int L) {
  const char *T = "BinSum bitify/operations.circom";
  int OL = L + N - 1;
  size_t out = b, in = b + OL, sn = in + (size_t)N * L, o = sn;
  o += ck_getsum(c, sn, N);
  for (int i = 0; i < N; i++) {
    size_t bn = o;
    o += ck_bits2num(c, bn, L);
    for (int k = 0; k < L; k++) EQ(S(c, bn + 1 + k), S(c, in + (size_t)i * L + k), T, 22);
    EQ(S(c, sn + 1 + i), S(c, bn), T, 23);
  }
  size_t nb = o;
  o += ck_num2bits(c, nb, OL);
  EQ(S(c, nb + OL), S(c, sn), T, 26);
  for (int k = 0; k < OL; k++) EQ(S(c, out + k), S(c, nb + k), T, 28);
  return o - b;
}
/* fT(t) f.circom: out[32] | b c d | maj (MajT) parity (ParityT -> XOR3_v3) ch (ChT) */
static size_t ck_ft(ck_t *c, size_t b, int t) {
  const char *T = "fT hasher/sha1/f.circom";
  size_t out = b, ib = b + 32, ic = b + 64, id = b + 96;
  size_t mj = b + 128;               /* MajT: out | a b c | mid : 160 */
  size_t pa = mj + 160;              /* ParityT: out | a b c | xor3 (XOR3_v3: out | a b c | mid : 160) : 128 + 160 */
  size_t x3 = pa + 128;
  size_t ch = x3 + 160;              /* ChT: out | a b c : 128 */
  for (int k = 0; k < 32; k++) {
    fr_t A, B, C;
    /* ChT :5-14 */
    EQ(S(c, ch + 32 + k), S(c, ib + k), T, 31); EQ(S(c, ch + 64 + k), S(c, ic + k), T, 32); EQ(S(c, ch + 96 + k), S(c, id + k), T, 33);
    A = S(c, ch + 32 + k); B = S(c, ch + 64 + k); C = S(c, ch + 96 + k);
    req(c, S(c, ch + k), ADD(MUL(A, SUB(B, C)), C), "ChT hasher/sha1/f.circom", 12, ch);
    /* ParityT parity.circom -> XOR3_v3 sha2Common.circom:102-113 */
    EQ(S(c, pa + 32 + k), S(c, ib + k), T, 38); EQ(S(c, pa + 64 + k), S(c, ic + k), T, 39); EQ(S(c, pa + 96 + k), S(c, id + k), T, 40);
    req(c, S(c, x3 + 32 + k), S(c, pa + 32 + k), "ParityT hasher/sha1/parity.circom", 13, pa);
    req(c, S(c, x3 + 64 + k), S(c, pa + 64 + k), "ParityT hasher/sha1/parity.circom", 14, pa);
    req(c, S(c, x3 + 96 + k), S(c, pa + 96 + k), "ParityT hasher/sha1/parity.circom", 15, pa);
    A = S(c, x3 + 32 + k); B = S(c, x3 + 64 + k); C = S(c, x3 + 96 + k);
    fr_t M = S(c, x3 + 128 + k);
    req(c, M, MUL(B, C), "XOR3_v3 hasher/sha2/sha2Common.circom", 110, x3);
    req(c, S(c, x3 + k), SUB(ADD(ADD(MUL(A, ADD(SUB(SUB(KC(1), MUL(KC(2), B)), MUL(KC(2), C)), MUL(KC(4), M))), B), C), MUL(KC(2), M)),
        "XOR3_v3 hasher/sha2/sha2Common.circom", 111, x3);
    req(c, S(c, pa + k), S(c, x3 + k), "ParityT hasher/sha1/parity.circom", 19, pa);
    /* MajT :16-27 */
    EQ(S(c, mj + 32 + k), S(c, ib + k), T, 45); EQ(S(c, mj + 64 + k), S(c, ic + k), T, 46); EQ(S(c, mj + 96 + k), S(c, id + k), T, 47);
    A = S(c, mj + 32 + k); B = S(c, mj + 64 + k); C = S(c, mj + 96 + k);
    M = S(c, mj + 128 + k);
    req(c, M, MUL(B, C), "MajT hasher/sha1/f.circom", 24, mj);
    req(c, S(c, mj + k), ADD(MUL(A, SUB(ADD(B, C), MUL(KC(2), M))), M), "MajT hasher/sha1/f.circom", 25, mj);
    size_t src = t <= 19 ? ch : (t <= 39 || t >= 60) ? pa : mj;
    EQ(S(c, out + k), S(c, src + k), T, t <= 19 ? 52 : (t <= 39 || t >= 60) ? 57 : 61);
  }
  return ch + 128 - b;
}
/* T(t) t.circom:8-57: out[32] | a b c d e kT w | rotatel5 f sumBinary (BinSum(5,32)) sum (Bits2Num(35)) getLastNBits(32) */
static size_t ck_sha1t(ck_t *c, size_t b, int t) {
  const char *T = "T hasher/sha1/t.circom";
  size_t out = b, a = b + 32, bb = b + 64, cc = b + 96, d = b + 128, e = b + 160, kt = b + 192, w = b + 224, o = b + 256;
  size_t r5 = o;
  o += ck_rotl(c, r5, 5);
  size_t f = o;
  o += ck_ft(c, f, t);
  for (int k = 0; k < 32; k++) {
    EQ(S(c, r5 + 32 + k), S(c, a + k), T, 27);
    EQ(S(c, f + 32 + k), S(c, bb + k), T, 28);
    EQ(S(c, f + 64 + k), S(c, cc + k), T, 29);
    EQ(S(c, f + 96 + k), S(c, d + k), T, 30);
  }
  size_t bs = o;
  o += ck_binsum(c, bs, 5, 32);
  for (int k = 0; k < 32; k++) {
    size_t in = bs + 36;
    EQ(S(c, in + k), S(c, r5 + 31 - k), T, 37);
    EQ(S(c, in + 32 + k), S(c, f + 31 - k), T, 38);
    EQ(S(c, in + 64 + k), S(c, e + 31 - k), T, 39);
    EQ(S(c, in + 96 + k), S(c, kt + 31 - k), T, 40);
    EQ(S(c, in + 128 + k), S(c, w + 31 - k), T, 41);
  }
  size_t sm = o;
  o += ck_bits2num(c, sm, 35);
  for (int k = 0; k < 35; k++) EQ(S(c, sm + 1 + k), S(c, bs + k), T, 46);
  size_t gl = o;
  o += ck_lastnbits(c, gl, 32);
  EQ(S(c, gl + 33), S(c, sm), T, 51);
  for (int k = 0; k < 32; k++) EQ(S(c, out + k), S(c, gl + 1 + 31 - k), T, 54);
  return o - b;
}
/* Sha1compression sha1compression.circom:7-132: out[160] | hin[160] inp[512] | a b c d e [81][32] w[80][32] |
 * rotl1[64] xor4[64] rotl30[80] kT[80] tTmp[80] fSum[5] */
static const uint32_t SHA1_K[4] = {0x5a827999, 0x6ed9eba1, 0x8f1bbcdc, 0xca62c1d6};
static size_t ck_sha1comp(ck_t *c, size_t b) {
  const char *T = "Sha1compression hasher/sha1/sha1compression.circom";
  size_t out = b, hin = b + 160, inp = hin + 160, A = inp + 512, B = A + 81 * 32, C = B + 81 * 32, D = C + 81 * 32,
         E = D + 81 * 32, Wd = E + 81 * 32, o = Wd + 80 * 32;
  size_t r1 = o; o += 64 * 64;
  size_t x4 = o; o += 64 * 224;
  size_t r30 = o; o += 80 * 64;
  size_t kt = o;
  size_t kt_at[80];
  for (int i = 0; i < 80; i++) { kt_at[i] = o; o += ck_sha1const(c, o, SHA1_K[i / 20], 29); }
  (void)kt;
  size_t tt[80];
  for (int i = 0; i < 80; i++) { tt[i] = o; o += ck_sha1t(c, o, i); }
  size_t fs[5];
  for (int i = 0; i < 5; i++) { fs[i] = o; o += ck_binsum(c, o, 2, 32); }
  for (int i = 0; i < 64; i++) { ck_rotl(c, r1 + 64 * (size_t)i, 1); ck_xor4(c, x4 + 224 * (size_t)i); ck_rotl(c, r30 + 64 * (size_t)i, 30); }
  for (int i = 64; i < 80; i++) ck_rotl(c, r30 + 64 * (size_t)i, 30);
#define WB(t, k) (Wd + 32 * (size_t)(t) + (k))
  for (int t = 0; t < 16; t++)
    for (int k = 0; k < 32; k++) EQ(S(c, WB(t, k)), S(c, inp + t * 32 + k), T, 60);
  for (int t = 16; t < 80; t++) {
    size_t X = x4 + 224 * (size_t)(t - 16), R = r1 + 64 * (size_t)(t - 16);
    for (int k = 0; k < 32; k++) {
      EQ(S(c, X + 32 + k), S(c, WB(t - 3, k)), T, 66);
      EQ(S(c, X + 64 + k), S(c, WB(t - 8, k)), T, 67);
      EQ(S(c, X + 96 + k), S(c, WB(t - 14, k)), T, 68);
      EQ(S(c, X + 128 + k), S(c, WB(t - 16, k)), T, 69);
      EQ(S(c, R + 32 + k), S(c, X + k), T, 72);
      EQ(S(c, WB(t, k)), S(c, R + k), T, 75);
    }
  }
#define AB(arr, t, k) ((arr) + 32 * (size_t)(t) + (k))
  for (int k = 0; k < 32; k++) {
    EQ(S(c, AB(A, 0, k)), S(c, hin + k), T, 81);
    EQ(S(c, AB(B, 0, k)), S(c, hin + 32 + k), T, 82);
    EQ(S(c, AB(C, 0, k)), S(c, hin + 64 + k), T, 83);
    EQ(S(c, AB(D, 0, k)), S(c, hin + 96 + k), T, 84);
    EQ(S(c, AB(E, 0, k)), S(c, hin + 128 + k), T, 85);
  }
  for (int t = 0; t < 80; t++) {
    size_t Tt = tt[t], R = r30 + 64 * (size_t)t;
    for (int k = 0; k < 32; k++) {
      EQ(S(c, Tt + 32 + k), S(c, AB(A, t, k)), T, 90);
      EQ(S(c, Tt + 64 + k), S(c, AB(B, t, k)), T, 91);
      EQ(S(c, Tt + 96 + k), S(c, AB(C, t, k)), T, 92);
      EQ(S(c, Tt + 128 + k), S(c, AB(D, t, k)), T, 93);
      EQ(S(c, Tt + 160 + k), S(c, AB(E, t, k)), T, 94);
      EQ(S(c, Tt + 192 + k), S(c, kt_at[t] + k), T, 95);
      EQ(S(c, Tt + 224 + k), S(c, WB(t, k)), T, 96);
      EQ(S(c, R + 32 + k), S(c, AB(B, t, k)), T, 98);
      EQ(S(c, AB(E, t + 1, k)), S(c, AB(D, t, k)), T, 102);
      EQ(S(c, AB(D, t + 1, k)), S(c, AB(C, t, k)), T, 103);
      EQ(S(c, AB(C, t + 1, k)), S(c, R + k), T, 104);
      EQ(S(c, AB(B, t + 1, k)), S(c, AB(A, t, k)), T, 105);
      EQ(S(c, AB(A, t + 1, k)), S(c, Tt + k), T, 106);
    }
  }
  size_t arr[5] = {A, B, C, D, E};
  for (int q = 0; q < 5; q++)
    for (int k = 0; k < 32; k++) {
      size_t in = fs[q] + 33;  /* BinSum(2,32): out[33] | in[2][32] */
      EQ(S(c, in + k), S(c, hin + 31 * (q + 1) - k + q), T, 111);
      EQ(S(c, in + 32 + k), S(c, AB(arr[q], 80, 31 - k)), T, 112);
      EQ(S(c, out + 32 * q + k), S(c, fs[q] + k), T, 127);
    }
#undef WB
#undef AB
  return o - b;
}
/* Sha1HashChunks(B) sha1.circom:7-57: out[160] | in[512B] | ha0..he0 sha1Compression[B] */
static const uint32_t SHA1_H[5] = {0x67452301, 0xefcdab89, 0x98badcfe, 0x10325476, 0xc3d2e1f0};
static size_t ck_sha1chunks(ck_t *c, size_t b, int Bn) {
  const char *T = "Sha1HashChunks hasher/sha1/sha1.circom";
  size_t out = b, in = b + 160, o = in + 512 * (size_t)Bn, h[5];
  for (int i = 0; i < 5; i++) { h[i] = o; o += ck_sha1const(c, o, SHA1_H[i], 15); }
  size_t prev = 0;
  for (int i = 0; i < Bn; i++) {
    size_t sc = o;
    o += ck_sha1comp(c, sc);
    for (int q = 0; q < 5; q++)
      for (int k = 0; k < 32; k++)
        EQ(S(c, sc + 160 + 32 * q + k), i == 0 ? S(c, h[q] + k) : S(c, prev + 32 * q + 31 - k), T, i == 0 ? 26 : 34);
    for (int k = 0; k < 512; k++) EQ(S(c, sc + 320 + k), S(c, in + (size_t)i * 512 + k), T, 42);
    prev = sc;
  }
  for (int i = 0; i < 5; i++)
    for (int k = 0; k < 32; k++) EQ(S(c, out + (31 - k) + 32 * i), S(c, prev + k + 32 * i), T, 49);
  return o - b;
}

/* ============================================================ Poseidon (hasher/poseidon/poseidon.circom) */
typedef struct { int t, nRP; fr_t *C, *M, *P, *S; } pos_t;
static pos_t POS[7];
static int pos_loaded = 0;

int ck_load_poseidon(const char *path) {
  FILE *fp = fopen(path, "rb");
  if (!fp) return -1;
  char magic[8]; uint32_t nt;
  if (fread(magic, 1, 8, fp) != 8 || memcmp(magic, "PZKPOS01", 8) || fread(&nt, 4, 1, fp) != 1) { fclose(fp); return -2; }
  for (uint32_t q = 0; q < nt; q++) {
    uint32_t h[4];
    if (fread(h, 4, 4, fp) != 4 || h[0] < 2 || h[0] > 6) { fclose(fp); return -3; }
    int t = (int)h[0];
    pos_t *pp = &POS[t];
    pp->t = t; pp->nRP = (int)h[1];
    pp->C = malloc(32 * h[2]); pp->M = malloc(32 * t * t); pp->P = malloc(32 * t * t); pp->S = malloc(32 * h[3]);
    if (fread(pp->C, 32, h[2], fp) != h[2] || fread(pp->M, 32, (size_t)t * t, fp) != (size_t)t * t ||
        fread(pp->P, 32, (size_t)t * t, fp) != (size_t)t * t || fread(pp->S, 32, h[3], fp) != h[3]) {
      fclose(fp); return -4;
    }
  }
  fclose(fp);
  pos_loaded = 1;
  return 0;
}

/* Sigma :10-21: out | in | in2, in4 */
static size_t ck_sigma(ck_t *c, size_t b) {
  const char *T = "Sigma hasher/poseidon/poseidon.circom";
  fr_t in = S(c, b + 1), in2 = S(c, b + 2), in4 = S(c, b + 3);
  EQ(in2, MUL(in, in), T, 17);
  EQ(in4, MUL(in2, in2), T, 18);
  EQ(S(c, b), MUL(in4, in), T, 20);
  return 4;
}
/* Ark(t, C, r) :23-30: out[t] | in[t] */
static size_t ck_ark(ck_t *c, size_t b, int t, const fr_t *C, int r) {
  for (int i = 0; i < t; i++) EQ(S(c, b + i), ADD(S(c, b + t + i), C[i + r]), "Ark hasher/poseidon/poseidon.circom", 28);
  return 2 * (size_t)t;
}
/* Mix(t, M) :32-46: out[t] | in[t] | sum[t] */
static size_t ck_mix(ck_t *c, size_t b, int t, const fr_t *M) {
  const char *T = "Mix hasher/poseidon/poseidon.circom";
  size_t o = b + 2 * t;
  for (int i = 0; i < t; i++) {
    size_t s = o;
    o += ck_getsum(c, s, t);
    for (int j = 0; j < t; j++) EQ(S(c, s + 1 + j), MUL(M[j * t + i], S(c, b + t + j)), T, 42);
    EQ(S(c, b + i), S(c, s), T, 44);
  }
  return o - b;
}
/* MixLast(t, M, s) :48-58: out | in[t] | sum */
static size_t ck_mixlast(ck_t *c, size_t b, int t, const fr_t *M, int s_) {
  const char *T = "MixLast hasher/poseidon/poseidon.circom";
  size_t s = b + 1 + t;
  for (int j = 0; j < t; j++) EQ(S(c, s + 1 + j), MUL(M[j * t + s_], S(c, b + 1 + j)), T, 55);
  EQ(S(c, b), S(c, s), T, 57);
  return 1 + (size_t)t + ck_getsum(c, s, t);
}
/* MixS(t, S, r) :60-78: out[t] | in[t] | sum */
static size_t ck_mixs(ck_t *c, size_t b, int t, const fr_t *Sc, int r) {
  const char *T = "MixS hasher/poseidon/poseidon.circom";
  size_t s = b + 2 * t;
  for (int i = 0; i < t; i++) EQ(S(c, s + 1 + i), MUL(Sc[(t * 2 - 1) * r + i], S(c, b + t + i)), T, 71);
  EQ(S(c, b), S(c, s), T, 73);
  for (int i = 1; i < t; i++)
    EQ(S(c, b + i), ADD(S(c, b + t + i), MUL(S(c, b + t), Sc[(t * 2 - 1) * r + t + i - 1])), T, 76);
  return 2 * (size_t)t + ck_getsum(c, s, t);
}

/* PoseidonEx(nIn, 1) :80-209: out[1] | in[nIn] initialState | components in creation order */
static size_t ck_poseidonex(ck_t *c, size_t b, int nIn) {
  const char *T = "PoseidonEx hasher/poseidon/poseidon.circom";
  const int t = nIn + 1, F = 8;
  const pos_t *pp = &POS[t];
  const int RP = pp->nRP;
  size_t out = b, in = b + 1, init = b + 1 + nIn, o = b + 2 + nIn;
  size_t ark = o;  /* ark[0] */
  o += ck_ark(c, ark, t, pp->C, 0);
  for (int j = 0; j < t; j++) EQ(S(c, ark + t + j), j > 0 ? S(c, in + j - 1) : S(c, init), T, j > 0 ? 127 : 129);
  size_t prev = ark;  /* block whose out[0..t) feeds the next sigma layer */
  for (int r = 0; r < F / 2; r++) {
    size_t sg = o;
    for (int j = 0; j < t; j++) {
      o += ck_sigma(c, o);
      EQ(S(c, sg + 4 * j + 1), S(c, prev + j), T, r == 0 ? 137 : 139);
    }
    size_t ak = o;
    o += ck_ark(c, ak, t, pp->C, (r + 1) * t);
    for (int j = 0; j < t; j++) EQ(S(c, ak + t + j), S(c, sg + 4 * j), T, 145);
    size_t mx = o;
    o += ck_mix(c, mx, t, r < F / 2 - 1 ? pp->M : pp->P);
    for (int j = 0; j < t; j++) EQ(S(c, mx + t + j), S(c, ak + j), T, 150);
    prev = mx;
  }
  size_t mixP = prev, ms = 0;
  for (int r = 0; r < RP; r++) {
    size_t sp = o;
    o += ck_sigma(c, sp);
    EQ(S(c, sp + 1), r == 0 ? S(c, mixP) : S(c, ms), T, r == 0 ? 178 : 180);
    size_t m = o;
    o += ck_mixs(c, m, t, pp->S, r);
    for (int j = 0; j < t; j++) {
      if (j == 0) EQ(S(c, m + t), ADD(S(c, sp), pp->C[(F / 2 + 1) * t + r]), T, 186);
      else EQ(S(c, m + t + j), r == 0 ? S(c, mixP + j) : S(c, ms + j), T, r == 0 ? 189 : 191);
    }
    ms = m;
  }
  prev = ms;
  for (int r = 0; r < F / 2 - 1; r++) {
    size_t sg = o;
    for (int j = 0; j < t; j++) {
      o += ck_sigma(c, o);
      EQ(S(c, sg + 4 * j + 1), S(c, prev + j), T, r == 0 ? 201 : 203);
    }
    size_t ak = o;
    o += ck_ark(c, ak, t, pp->C, (F / 2 + 1) * t + RP + r * t);
    for (int j = 0; j < t; j++) EQ(S(c, ak + t + j), S(c, sg + 4 * j), T, 209);
    size_t mx = o;
    o += ck_mix(c, mx, t, pp->M);
    for (int j = 0; j < t; j++) EQ(S(c, mx + t + j), S(c, ak + j), T, 214);
    prev = mx;
  }
  size_t sg = o;
  for (int j = 0; j < t; j++) {
    o += ck_sigma(c, o);
    EQ(S(c, sg + 4 * j + 1), S(c, prev + j), T, 221);
  }
  size_t ml = o;
  o += ck_mixlast(c, ml, t, pp->M, 0);
  for (int j = 0; j < t; j++) EQ(S(c, ml + 1 + j), S(c, sg + 4 * j), T, 227);
  EQ(S(c, out), S(c, ml), T, 229);
  return o - b;
}

/* PoseidonHash(n) :214-226: out | in[n] | pEx */
static size_t ck_poseidon(ck_t *c, size_t b, int n) {
  const char *T = "PoseidonHash hasher/poseidon/poseidon.circom";
  size_t px = b + 1 + n;
  size_t sz = 1 + (size_t)n + ck_poseidonex(c, px, n);
  EQ(S(c, px + 1 + n), fr_zero(), T, 221);
  for (int i = 0; i < n; i++) EQ(S(c, px + 1 + i), S(c, b + 1 + i), T, 223);
  EQ(S(c, b), S(c, px), T, 225);
  return sz;
}

/* ============================================================ SMT (merkleTree/SMTVerifier.circom) */
/* Switcher utils/switcher.circom:16-26: out[2] | bool in[2] | aux */
static size_t ck_switcher(ck_t *c, size_t b) {
  const char *T = "Switcher utils/switcher.circom";
  fr_t bo = S(c, b + 2), i0 = S(c, b + 3), i1 = S(c, b + 4), aux = S(c, b + 5);
  EQ(aux, MUL(SUB(i1, i0), bo), T, 23);
  EQ(S(c, b), ADD(aux, i0), T, 24);
  EQ(S(c, b + 1), ADD(fr_neg(aux), i1), T, 25);
  return 6;
}

/* SMTLevIns(N) :39-65: levIns[N] | siblings[N] | done[N-1] | isZero[N] */
static size_t ck_smtlevins(ck_t *c, size_t b, int N) {
  const char *T = "SMTLevIns merkleTree/SMTVerifier.circom";
  size_t lev = b, sib = b + N, done = b + 2 * (size_t)N, z = b + 3 * (size_t)N - 1;
  for (int i = 0; i < N; i++) {
    ck_iszero(c, z + 3 * (size_t)i);
    EQ(S(c, z + 3 * (size_t)i + 1), S(c, sib + i), T, 51);
  }
#define ZO(i) S(c, z + 3 * (size_t)(i))
  EQ(SUB(ZO(N - 1), KC(1)), fr_zero(), T, 54);
  EQ(S(c, lev + N - 1), SUB(KC(1), ZO(N - 2)), T, 56);
  EQ(S(c, done + N - 2), S(c, lev + N - 1), T, 57);
  for (int i = N - 2; i > 0; i--) {
    EQ(S(c, lev + i), MUL(SUB(KC(1), S(c, done + i)), SUB(KC(1), ZO(i - 1))), T, 60);
    EQ(S(c, done + i - 1), ADD(S(c, lev + i), S(c, done + i)), T, 61);
  }
  EQ(S(c, lev), SUB(KC(1), S(c, done)), T, 64);
#undef ZO
  return 3 * (size_t)N - 1 + 3 * (size_t)N;
}

/* SMTVerifierLevel :82-107: root | st_top st_inew sibling new1leaf lrbit child | fromProof | proofHash(SMTHash2) switcher */
static size_t ck_smtlevel(ck_t *c, size_t b) {
  const char *T = "SMTVerifierLevel merkleTree/SMTVerifier.circom";
  size_t root = b, top = b + 1, inew = b + 2, sib = b + 3, leaf = b + 4, lr = b + 5, child = b + 6, fp = b + 7;
  size_t ph = b + 8;           /* SMTHash2: out | L R | h = PoseidonHash(2) */
  size_t h = ph + 3;
  size_t sz_ph = 3 + ck_poseidon(c, h, 2);
  EQ(S(c, h + 1), S(c, ph + 1), "SMTHash2 merkleTree/SMTVerifier.circom", 28);
  EQ(S(c, h + 2), S(c, ph + 2), "SMTHash2 merkleTree/SMTVerifier.circom", 29);
  EQ(S(c, ph), S(c, h), "SMTHash2 merkleTree/SMTVerifier.circom", 31);
  size_t sw = ph + sz_ph;
  ck_switcher(c, sw);
  EQ(S(c, sw + 3), S(c, child), T, 96);
  EQ(S(c, sw + 4), S(c, sib), T, 97);
  EQ(S(c, sw + 2), S(c, lr), T, 99);
  EQ(S(c, ph + 1), S(c, sw), T, 100);
  EQ(S(c, ph + 2), S(c, sw + 1), T, 101);
  EQ(S(c, fp), MUL(S(c, ph), S(c, top)), T, 103);
  EQ(S(c, root), ADD(S(c, fp), MUL(S(c, leaf), S(c, inew))), T, 105);
  return 8 + sz_ph + 6;
}

/* SMTVerifier(N) :109-176: isVerified | root leaf key siblings[N] | value |
 * hash1New(SMTHash1) n2bNew(Num2Bits(254)) smtLevIns sm[0..N) levels[N-1..0] isEqual */
static size_t ck_smt(ck_t *c, size_t b, int N) {
  const char *T = "SMTVerifier merkleTree/SMTVerifier.circom";
  size_t isv = b, root = b + 1, leaf = b + 2, key = b + 3, sib = b + 4, value = b + 4 + N, o = b + 5 + N;
  EQ(S(c, value), S(c, leaf), T, 118);
  size_t h1 = o, h = h1 + 3;   /* SMTHash1: out | key value | h = PoseidonHash(3) */
  o += 3 + ck_poseidon(c, h, 3);
  EQ(S(c, h + 1), S(c, h1 + 1), "SMTHash1 merkleTree/SMTVerifier.circom", 16);
  EQ(S(c, h + 2), S(c, h1 + 2), "SMTHash1 merkleTree/SMTVerifier.circom", 17);
  EQ(S(c, h + 3), KC(1), "SMTHash1 merkleTree/SMTVerifier.circom", 18);
  EQ(S(c, h1), S(c, h), "SMTHash1 merkleTree/SMTVerifier.circom", 20);
  EQ(S(c, h1 + 1), S(c, key), T, 121);
  EQ(S(c, h1 + 2), S(c, value), T, 122);
  size_t n2b = o;
  o += ck_num2bits(c, n2b, 254);
  EQ(S(c, n2b + 254), S(c, key), T, 126);
  size_t li = o;
  o += ck_smtlevins(c, li, N);
  for (int i = 0; i < N; i++) EQ(S(c, li + N + i), S(c, sib + i), T, 131);
  size_t sm = o;  /* SMTVerifierSM :71-80: st_top st_inew | levIns prev_top */
  for (int i = 0; i < N; i++) {
    size_t q = sm + 4 * (size_t)i;
    const char *TS = "SMTVerifierSM merkleTree/SMTVerifier.circom";
    req(c, S(c, q + 1), MUL(S(c, q + 3), S(c, q + 2)), TS, 78, q);
    req(c, S(c, q), SUB(S(c, q + 3), S(c, q + 1)), TS, 79, q);
    EQ(S(c, q + 3), i == 0 ? KC(1) : S(c, q - 4), T, i == 0 ? 140 : 142);
    EQ(S(c, q + 2), S(c, li + i), T, 145);
  }
  o += 4 * (size_t)N;
  size_t lvl_at[128];
  for (int i = N - 1; i >= 0; i--) {
    size_t L = o;
    lvl_at[i] = L;
    o += ck_smtlevel(c, L);
    size_t q = sm + 4 * (size_t)i;
    EQ(S(c, L + 1), S(c, q), T, 153);
    EQ(S(c, L + 2), S(c, q + 1), T, 154);
    EQ(S(c, L + 3), S(c, sib + i), T, 156);
    EQ(S(c, L + 4), S(c, h1), T, 157);
    EQ(S(c, L + 5), S(c, n2b + i), T, 159);
    EQ(S(c, L + 6), i == N - 1 ? fr_zero() : S(c, lvl_at[i + 1]), T, i == N - 1 ? 162 : 164);
  }
  size_t ie = o;
  o += ck_isequal(c, ie);
  EQ(S(c, ie + 1), S(c, lvl_at[0]), T, 171);
  EQ(S(c, ie + 2), S(c, root), T, 172);
  EQ(S(c, isv), S(c, ie), T, 173);
  return o - b;
}

/* ============================================================ BabyJubJub (babyjubjub/curve.circom) */
/* BabyjubjubAdd :71-105: out[2] | in1[2] in2[2] | beta gamma delta tau */
static size_t ck_bjjadd(ck_t *c, size_t b) {
  const char *T = "BabyjubjubAdd babyjubjub/curve.circom";
  const fr_t a = KC(168700), d = KC(168696);
  fr_t x1 = S(c, b + 2), y1 = S(c, b + 3), x2 = S(c, b + 4), y2 = S(c, b + 5);
  fr_t be = S(c, b + 6), ga = S(c, b + 7), de = S(c, b + 8), ta = S(c, b + 9);
  EQ(be, MUL(x1, y2), T, 83);
  EQ(ga, MUL(y1, x2), T, 86);
  EQ(de, MUL(SUB(y1, MUL(a, x1)), ADD(x2, y2)), T, 89);
  EQ(ta, MUL(be, ga), T, 92);
  EQ(MUL(ADD(KC(1), MUL(d, ta)), S(c, b)), ADD(be, ga), T, 96);
  EQ(MUL(SUB(KC(1), MUL(d, ta)), S(c, b + 1)), SUB(ADD(de, MUL(a, be)), ga), T, 100);
  return 10;
}
/* BabyjubjubDouble :109-118: out[2] | in[2] | adder */
static size_t ck_bjjdouble(ck_t *c, size_t b) {
  const char *T = "BabyjubjubDouble babyjubjub/curve.circom";
  size_t ad = b + 4;
  ck_bjjadd(c, ad);
  for (int i = 0; i < 2; i++) {
    EQ(S(c, ad + 2 + i), S(c, b + 2 + i), T, 114);
    EQ(S(c, ad + 4 + i), S(c, b + 2 + i), T, 115);
    EQ(S(c, b + i), S(c, ad + i), T, 117);
  }
  return 14;
}
/* addZeroBabyjub :19-58: out[2] | in1[2] in2[2] | isZeroIn1 isZeroIn2 adder (switcherLeft[i], switcherRight[i])[2] */
static size_t ck_addzero(ck_t *c, size_t b) {
  const char *T = "addZeroBabyjub babyjubjub/curve.circom";
  size_t z1 = b + 6, z2 = b + 9, ad = b + 12, sw = b + 22;
  ck_iszero(c, z1);
  EQ(S(c, z1 + 1), S(c, b + 2), T, 25);
  ck_iszero(c, z2);
  EQ(S(c, z2 + 1), S(c, b + 4), T, 27);
  ck_bjjadd(c, ad);
  for (int i = 0; i < 2; i++) {
    EQ(S(c, ad + 2 + i), S(c, b + 2 + i), T, 31);
    EQ(S(c, ad + 4 + i), S(c, b + 4 + i), T, 32);
  }
  for (int i = 0; i < 2; i++) {
    size_t L = sw + 12 * (size_t)i, R = L + 6;
    ck_switcher(c, L);
    EQ(S(c, L + 2), S(c, z2), T, 47);
    EQ(S(c, L + 3), S(c, ad + i), T, 48);
    EQ(S(c, L + 4), S(c, b + 2 + i), T, 49);
    ck_switcher(c, R);
    EQ(S(c, R + 2), S(c, z1), T, 52);
    EQ(S(c, R + 3), S(c, L), T, 53);
    EQ(S(c, R + 4), S(c, b + 4 + i), T, 54);
  }
  EQ(S(c, b), S(c, sw + 6), T, 57);
  EQ(S(c, b + 1), S(c, sw + 18), T, 58);
  return 46;
}

/* BabyjubjubBase8Multiplication :143-171: out[2] | scalar | getBase8 num2Bits adders[0] (doublers[i-1] adders[i])[i=1..253] */
static size_t ck_bjjmul(ck_t *c, size_t b) {
  const char *T = "BabyjubjubBase8Multiplication babyjubjub/curve.circom";
  static const uint64_t B8X[4] = {0x2893f3f6bb957051ULL, 0x2ab8d8010534e0b6ULL, 0x4eacb2e09d6277c1ULL, 0x0bb77a6ad63e739bULL};
  static const uint64_t B8Y[4] = {0x4b3c257a872d7d8bULL, 0xfce0051fb9e13377ULL, 0x25572e1cd16bf9edULL, 0x25797203f7a0b249ULL};
  fr_t bx, by;
  memcpy(bx.l, B8X, 32); memcpy(by.l, B8Y, 32);
  size_t g8 = b + 3, n2b = b + 5, o = b + 5;
  req(c, S(c, g8), bx, "GetBabyjubjubBase8 babyjubjub/get.circom", 9, g8);
  req(c, S(c, g8 + 1), by, "GetBabyjubjubBase8 babyjubjub/get.circom", 10, g8);
  o += ck_num2bits(c, n2b, 254);
  EQ(S(c, n2b + 254), S(c, b + 2), T, 150);
  size_t prev = 0;
  for (int i = 0; i < 254; i++) {  /* adders[i] is created before doublers[i - 1] (:153-160) */
    size_t ad = o;
    o += ck_addzero(c, ad);
    size_t dbl = 0;
    if (i > 0) {
      dbl = o;
      o += ck_bjjdouble(c, dbl);
      EQ(S(c, dbl + 2), S(c, prev), T, 162);
      EQ(S(c, dbl + 3), S(c, prev + 1), T, 162);
    }
    fr_t bit = S(c, n2b + 253 - i);
    EQ(S(c, ad + 2), i == 0 ? fr_zero() : S(c, dbl), T, i == 0 ? 157 : 163);
    EQ(S(c, ad + 3), i == 0 ? fr_zero() : S(c, dbl + 1), T, i == 0 ? 157 : 163);
    EQ(S(c, ad + 4), MUL(S(c, g8), bit), T, i == 0 ? 158 : 164);
    EQ(S(c, ad + 5), MUL(S(c, g8 + 1), bit), T, i == 0 ? 159 : 165);
    prev = ad;
  }
  EQ(S(c, b), S(c, prev), T, 169);
  EQ(S(c, b + 1), S(c, prev + 1), T, 169);
  return o - b;
}

/* ============================================================ big integers (lib/circuits/bigInt) */
/* KaratsubaOverflow(N) bigIntHelpers.circom:11-53: out[2N] | in[2][N] | A1B1 A2B2 A1A2B1B2 */
static size_t ck_karatsuba(ck_t *c, size_t b, int N) {
  const char *T = "KaratsubaOverflow bigInt/bigIntHelpers.circom";
  size_t out = b, in0 = b + 2 * (size_t)N, in1 = in0 + N;
  if (N == 1) {
    EQ(S(c, out), MUL(S(c, in0), S(c, in1)), T, 16);
    return 4;  /* out[1] is declared and never assigned */
  }
  int h = N / 2;
  size_t k1 = b + 4 * (size_t)N, o = k1;
  o += ck_karatsuba(c, k1, h);
  size_t k2 = o;
  o += ck_karatsuba(c, k2, h);
  size_t k3 = o;
  o += ck_karatsuba(c, k3, h);
#define KI(k, j, i) ((k) + 2 * (size_t)h + (size_t)(j) * h + (i))
  for (int i = 0; i < h; i++) {
    EQ(S(c, KI(k1, 0, i)), S(c, in0 + i), T, 23);
    EQ(S(c, KI(k1, 1, i)), S(c, in1 + i), T, 24);
    EQ(S(c, KI(k2, 0, i)), S(c, in0 + i + h), T, 25);
    EQ(S(c, KI(k2, 1, i)), S(c, in1 + i + h), T, 26);
    EQ(S(c, KI(k3, 0, i)), ADD(S(c, in0 + i), S(c, in0 + i + h)), T, 27);
    EQ(S(c, KI(k3, 1, i)), ADD(S(c, in1 + i), S(c, in1 + i + h)), T, 28);
  }
#undef KI
  for (int i = 0; i < 2 * N; i++) {
    fr_t rhs;
    int mid = h <= i && i < 3 * h;
    if (i < N) rhs = mid ? SUB(SUB(ADD(S(c, k1 + i), S(c, k3 + i - h)), S(c, k1 + i - h)), S(c, k2 + i - h)) : S(c, k1 + i);
    else rhs = mid ? SUB(SUB(ADD(S(c, k2 + i - N), S(c, k3 + i - h)), S(c, k1 + i - h)), S(c, k2 + i - h)) : S(c, k2 + i - N);
    EQ(S(c, out + i), rhs, T, i < N ? (mid ? 34 : 39) : (mid ? 43 : 48));
  }
  return o - b;
}

/* BigMultNonEqualOverflow(n, G, L) bigIntHelpers.circom:55-124: out[G+L-1] | in1[G] in2[L] | tmpMults[G][L] tmpResult[G+L-1][L] */
static size_t ck_bmneq(ck_t *c, size_t b, int G, int L) {
  const char *T = "BigMultNonEqualOverflow bigInt/bigIntHelpers.circom";
  size_t out = b, in1 = b + G + L - 1, in2 = in1 + G, tm = in2 + L, tr = tm + (size_t)G * L;
#define TM(i, j) S(c, tm + (size_t)(i) * L + (j))
#define TR(i, j) (tr + (size_t)(i) * L + (j))
  for (int i = 0; i < G; i++)
    for (int j = 0; j < L; j++) EQ(TM(i, j), MUL(S(c, in1 + i), S(c, in2 + j)), T, 69);
  for (int i = 0; i < G + L - 1; i++) {
    int n;
    if (i < L) n = i + 1;
    else if (i < G) n = L;
    else n = G + L - 1 - i;
    for (int j = 0; j < n; j++) {
      fr_t m = (i < G) ? TM(i - j, j) : TM(G - 1 - j, i + j - G + 1);
      EQ(S(c, TR(i, j)), j == 0 ? m : ADD(m, S(c, TR(i, j - 1))), T, i < L ? 91 : i < G ? 101 : 111);
    }
    EQ(S(c, out + i), S(c, TR(i, n - 1)), T, i < L ? 95 : i < G ? 104 : 115);
  }
#undef TM
#undef TR
  return (size_t)(G + L - 1) + G + L + (size_t)G * L + (size_t)(G + L - 1) * L;
}

static int karatsuba_path(int G, int L) {
  /* BigMultOverflow bigIntOverflow.circom:43-53: power-of-two G and is_karatsuba_optimal(G, L)
   * (bigIntFunc.circom:617-629: G >= 8 and get_a_coeff(G) <= G L, dontOpenPlease.circom: 70, 211, 640, 1940 for
   * G = 8, 16, 32, 64). The instances here: G = L in {32, 48, 64} (RSA; optimal for 32 and 64), and the EC
   * templates' G in {N, N+2, 2N-1, 2N+1, 2N+2} x L = N for N = 4, 6, 7 (G = 8 x 6 and 16 x 7 are powers of two
   * but not optimal) */
  if ((G & (G - 1)) != 0 || G < 8) return 0;
  const int a = G == 8 ? 70 : G == 16 ? 211 : G == 32 ? 640 : G == 64 ? 1940 : -1;
  if (a < 0) {
    fprintf(stderr, "r1cs_check: BigMultOverflow(%d,%d) unsupported\n", G, L);
    abort();
  }
  return a <= G * L;
}

/* BigMultOverflow(n, G, L) bigIntOverflow.circom:38-72: out[G+L-1] | in1[G] in2[L] | karatsuba or mult */
static size_t ck_bmo(ck_t *c, size_t b, int G, int L) {
  const char *T = "BigMultOverflow bigInt/bigIntOverflow.circom";
  size_t out = b, in1 = b + G + L - 1, in2 = in1 + G, sub = in2 + L, sz;
  if (karatsuba_path(G, L)) {
    sz = ck_karatsuba(c, sub, G);
    for (int i = 0; i < G; i++) {
      EQ(S(c, sub + 2 * G + i), S(c, in1 + i), T, 56);
      EQ(S(c, sub + 3 * G + i), i < L ? S(c, in2 + i) : fr_zero(), T, i < L ? 58 : 61);
    }
    for (int i = 0; i < G + L - 1; i++) EQ(S(c, out + i), S(c, sub + i), T, 64);
  } else {
    sz = ck_bmneq(c, sub, G, L);
    for (int i = 0; i < G; i++) EQ(S(c, sub + G + L - 1 + i), S(c, in1 + i), T, 68);
    for (int i = 0; i < L; i++) EQ(S(c, sub + G + L - 1 + G + i), S(c, in2 + i), T, 69);
    for (int i = 0; i < G + L - 1; i++) EQ(S(c, out + i), S(c, sub + i), T, 70);
  }
  return (size_t)(G + L - 1) + G + L + sz;
}

/* BigLessEqThan(n, K) bigIntComparators.circom:50-75: out | in[2][K] | result[K] | (lessThan[i] isEqual[i])[K] */
static size_t ck_blet(ck_t *c, size_t b, int n, int K) {
  const char *T = "BigLessEqThan bigInt/bigIntComparators.circom";
  size_t in0 = b + 1, in1 = in0 + K, res = in1 + K, o = res + K;
  for (int i = 0; i < K; i++) {
    size_t lt = o;
    o += ck_lessthan(c, lt, n);
    EQ(S(c, lt + 1), S(c, in0 + i), T, 60);
    EQ(S(c, lt + 2), S(c, in1 + i), T, 61);
    size_t eq = o;
    o += ck_isequal(c, eq);
    EQ(S(c, eq + 1), S(c, in0 + i), T, 64);
    EQ(S(c, eq + 2), S(c, in1 + i), T, 65);
    EQ(S(c, res + i), i == 0 ? ADD(S(c, lt), S(c, eq)) : ADD(S(c, lt), MUL(S(c, eq), S(c, res + i - 1))), T, i == 0 ? 70 : 72);
  }
  EQ(S(c, b), S(c, res + K - 1), T, 76);
  return o - b;
}

/* BigGreaterThan(n, K) bigIntComparators.circom:79-87: out | in[2][K] | lessEqThan */
static size_t ck_bgt(ck_t *c, size_t b, int n, int K) {
  const char *T = "BigGreaterThan bigInt/bigIntComparators.circom";
  size_t le = b + 1 + 2 * (size_t)K;
  size_t sz = 1 + 2 * (size_t)K + ck_blet(c, le, n, K);
  for (int i = 0; i < 2 * K; i++) EQ(S(c, le + 1 + i), S(c, b + 1 + i), T, 85);
  EQ(S(c, b), SUB(KC(1), S(c, le)), T, 86);
  return sz;
}

/* BigIntIsZero(n, MAX, K) bigIntComparators.circom:105-129: in[K] | carry[K-1] | carryRangeChecks[K-1] */
static fr_t INV2_64;
static size_t ck_bisz(ck_t *c, size_t b, int n, int MAX, int K) {
  const char *T = "BigIntIsZero bigInt/bigIntComparators.circom";
  int L = MAX + 3 - n;
  size_t in = b, carry = b + K, o = carry + K - 1;
  for (int i = 0; i < K - 1; i++) {
    size_t rc = o;
    o += ck_num2bits(c, rc, L);
    /* carry <== (in + carry_prev) / 2^n: the linear constraint carry * 2^n = in + carry_prev */
    EQ(MUL(S(c, carry + i), P2[n]), i == 0 ? S(c, in) : ADD(S(c, in + i), S(c, carry + i - 1)), T, i == 0 ? 120 : 123);
    EQ(S(c, rc + L), ADD(S(c, carry + i), P2[L - 1]), T, 126);
  }
  EQ(ADD(S(c, in + K - 1), S(c, carry + K - 2)), fr_zero(), T, 129);
  return o - b;
}

static int log_ceil(int n) { int i = 0; while (n) { n /= 2; i++; } return i; }  /* bigIntFunc.circom:20-29 */

/* BigMultModP(n, K, K, K) bigInt.circom:206-272: div[K+1] mod[K] | in1[K] in2[K] modulus[K] |
 * mult modChecks[K] greaterThan mult2 isZero */
static size_t ck_bmm_n(ck_t *c, size_t b, int n, int K) {
  const char *T = "BigMultModP bigInt/bigInt.circom";
  const int BASE = 2 * K, DIV = K + 1;
  size_t div = b, mod = b + DIV, in1 = mod + K, in2 = in1 + K, md = in2 + K, o = md + K;
  size_t mult = o;
  o += ck_bmo(c, mult, K, K);
  for (int i = 0; i < K; i++) {
    EQ(S(c, mult + BASE - 1 + i), S(c, in1 + i), T, 218);
    EQ(S(c, mult + BASE - 1 + K + i), S(c, in2 + i), T, 219);
  }
  for (int i = 0; i < K; i++) {
    size_t mc = o;
    o += ck_num2bits(c, mc, n);
    EQ(S(c, mc + n), S(c, mod + i), T, 233);
  }
  size_t gt = o;
  o += ck_bgt(c, gt, n, K);
  for (int i = 0; i < K; i++) {
    EQ(S(c, gt + 1 + i), S(c, md + i), T, 240);
    EQ(S(c, gt + 1 + K + i), S(c, mod + i), T, 241);
  }
  EQ(S(c, gt), KC(1), T, 242);
  size_t m2 = o;  /* DIV >= K: BigMultNonEqualOverflow(n, DIV, K)(div, modulus) */
  o += ck_bmneq(c, m2, DIV, K);
  for (int i = 0; i < DIV; i++) EQ(S(c, m2 + DIV + K - 1 + i), S(c, div + i), T, 252);
  for (int i = 0; i < K; i++) EQ(S(c, m2 + DIV + K - 1 + DIV + i), S(c, md + i), T, 253);
  size_t iz = o;
  o += ck_bisz(c, iz, n, 2 * n + log_ceil(K + DIV - 1), BASE - 1);
  for (int i = 0; i < BASE - 1; i++) {
    fr_t v = SUB(S(c, mult + i), S(c, m2 + i));
    EQ(S(c, iz + i), i < K ? SUB(v, S(c, mod + i)) : v, T, i < K ? 266 : 269);
  }
  return o - b;
}

static size_t ck_bmm(ck_t *c, size_t b, int K) { return ck_bmm_n(c, b, 64, K); }

/* exp_to_bits bigIntFunc.circom:590-616 (result_counter starts at 0, circom's default for a var) */
static void exp_to_bits(uint32_t e, int *idx) {
  int mul_num = 0, res_num = 0, rc = 0, counter = 0;
  while (e > 0) {
    int bit = e & 1;
    e >>= 1;
    if (bit) { res_num++; idx[rc + 2] = counter; rc++; }
    mul_num++; counter++;
  }
  idx[0] = mul_num - 1;
  idx[1] = res_num;
}

/* PowerMod(n, K, EXP) bigInt.circom:280-340: out[K] | base[K] modulus[K] | muls[e0] resultMuls[e1-1] */
static size_t ck_powermod(ck_t *c, size_t b, int K, uint32_t EXP) {
  const char *T = "PowerMod bigInt/bigInt.circom";
  int ep[40] = {0};
  exp_to_bits(EXP, ep);
  size_t out = b, base = b + K, modl = base + K, o = modl + K;
  size_t muls[40], rm[40];
  for (int i = 0; i < ep[0]; i++) { muls[i] = o; o += ck_bmm(c, o, K); }
  for (int i = 0; i < ep[1] - 1; i++) { rm[i] = o; o += ck_bmm(c, o, K); }
#define BIN1(m) ((m) + 2 * (size_t)K + 1)
#define BIN2(m) (BIN1(m) + K)
#define BMOD(m) (BIN2(m) + K)
#define BOUT(m) ((m) + (size_t)K + 1)
  for (int i = 0; i < ep[0]; i++)
    for (int j = 0; j < K; j++) EQ(S(c, BMOD(muls[i]) + j), S(c, modl + j), T, 307);
  for (int i = 0; i < ep[1] - 1; i++)
    for (int j = 0; j < K; j++) EQ(S(c, BMOD(rm[i]) + j), S(c, modl + j), T, 312);
  for (int j = 0; j < K; j++) {
    EQ(S(c, BIN1(muls[0]) + j), S(c, base + j), T, 316);
    EQ(S(c, BIN2(muls[0]) + j), S(c, base + j), T, 317);
  }
  for (int i = 1; i < ep[0]; i++)
    for (int j = 0; j < K; j++) {
      EQ(S(c, BIN1(muls[i]) + j), S(c, BOUT(muls[i - 1]) + j), T, 320);
      EQ(S(c, BIN2(muls[i]) + j), S(c, BOUT(muls[i - 1]) + j), T, 321);
    }
  for (int i = 0; i < ep[1] - 1; i++)
    for (int j = 0; j < K; j++) {
      fr_t in1;
      if (i == 0) in1 = ep[2] == 0 ? S(c, base + j) : S(c, BOUT(muls[ep[2] - 1]) + j);
      else in1 = S(c, BOUT(rm[i - 1]) + j);
      EQ(S(c, BIN1(rm[i]) + j), in1, T, i == 0 ? 328 : 334);
      EQ(S(c, BIN2(rm[i]) + j), S(c, BOUT(muls[ep[i + 3] - 1]) + j), T, i == 0 ? 332 : 335);
    }
  for (int j = 0; j < K; j++)
    EQ(S(c, out + j), ep[1] == 1 ? S(c, BOUT(muls[ep[0] - 1]) + j) : S(c, BOUT(rm[ep[1] - 2]) + j), T, 338);
#undef BIN1
#undef BIN2
#undef BMOD
#undef BOUT
  return o - b;
}

/* RsaVerifyPkcs1v15(64, K, EXP, 256) signatures/rsa.circom:16-72:
 * signature[K] pubkey[K] hashed[256] | hashed_chunks[4] | pm bits2num[3..0] num2bits_6 */
static size_t ck_rsa_pkcs256(ck_t *c, size_t b, int K, uint32_t EXP) {
  const char *T = "RsaVerifyPkcs1v15 signatures/rsa.circom";
  size_t sig = b, pk = b + K, hs = pk + K, hc = hs + 256, o = hc + 4;
  size_t pm = o;
  o += ck_powermod(c, pm, K, EXP);
  for (int i = 0; i < K; i++) {
    EQ(S(c, pm + K + i), S(c, sig + i), T, 29);
    EQ(S(c, pm + 2 * K + i), S(c, pk + i), T, 30);
  }
  for (int i = 0; i < 4; i++) {  /* bits2num[3 - i] created in this order */
    size_t bn = o;
    o += ck_bits2num(c, bn, 64);
    for (int j = 0; j < 64; j++) EQ(S(c, bn + 1 + j), S(c, hs + i * 64 + 63 - j), T, 39);
    EQ(S(c, hc + 3 - i), S(c, bn), T, 41);
  }
  for (int i = 0; i < 4; i++) EQ(S(c, hc + i), S(c, pm + i), T, 46);
  EQ(S(c, pm + 4), KC(217300885422736416ULL), T, 50);
  EQ(S(c, pm + 5), KC(938447882527703397ULL), T, 51);
  size_t n6 = o;
  o += ck_num2bits(c, n6, 64);
  EQ(S(c, n6 + 64), S(c, pm + 6), T, 55);
  static const int rb[32] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 0, 0, 0, 0, 0, 0, 1, 1, 0, 0, 0, 1, 0, 0, 1, 1, 0, 0, 0, 0};
  for (int i = 0; i < 32; i++) EQ(S(c, n6 + i), KC(rb[31 - i]), T, 58);
  for (int i = 32; i < 64; i++) EQ(S(c, n6 + i), KC(1), T, 63);
  for (int i = 7; i < K - 1; i++) EQ(S(c, pm + i), KC(18446744073709551615ULL), T, 67);
  return o - b;
}

/* ============================================================ RSA-PSS (signatures/rsaPss.circom, mgf1.circom) */
static size_t ck_shahash(ck_t *c, size_t b, int B, int algo);
/* Mgf1Sha256 / Mgf1Sha384(SEED_LEN, MASK_LEN) mgf1.circom:5-133 (H = 256 / 384):
 * out[8 MASK] | seed[8 SEED] | hashed[H ITER] | (shaH[i] num2Bits[i])[ITER], ITER = MASK / (H/8) + 1; block i hashes
 * seed | counter i (MSB first) | the padding of an (8 SEED + 32)-bit message to one BS-bit block */
static size_t ck_mgf1(ck_t *c, size_t b, int SEED, int MASK, int H) {
  const int h384 = H == 384;
  const char *T = h384 ? "Mgf1Sha384 signatures/mgf1.circom" : "Mgf1Sha256 signatures/mgf1.circom";
  int SB = SEED * 8, MB = MASK * 8, IT = MASK / (H / 8) + 1, BS = H > 256 ? 1024 : 512, LM = SB + 32;
  size_t out = b, seed = b + MB, hs = seed + SB, o = hs + (size_t)H * IT;
  for (int i = 0; i < IT; i++) {
    size_t sh = o;
    o += ck_shahash(c, sh, 1, H);
    size_t nb = o;
    o += ck_num2bits(c, nb, 32);
    EQ(S(c, nb + 32), KC((uint64_t)i), T, h384 ? 35 : 99);
    size_t in = sh + H;
    for (int j = 0; j < BS; j++) {
      fr_t v;
      if (j < SB) v = S(c, seed + j);
      else if (j < LM) v = S(c, nb + 31 - (j - SB));
      else v = KC(j == LM || (j >= BS - 11 && ((LM >> (BS - 1 - j)) & 1)));  /* padding (:42-55, :106-117) */
      EQ(S(c, in + j), v, T, h384 ? 58 : 120);
    }
    for (int j = 0; j < H; j++) EQ(S(c, hs + (size_t)i * H + j), S(c, sh + j), T, h384 ? 61 : 123);
  }
  for (int i = 0; i < MB; i++) EQ(S(c, out + i), S(c, hs + i), T, h384 ? 66 : 128);
  return o - b;
}

/* VerifyRsaPssSig(64, K, SALT, EXP, 256) rsaPss.circom:18-254: pubkey[K] signature[K] hashed[256] |
 * eM[EM] eMsgInBits[8 EM] encoded[K] dbMask db salt maskedDB hash mDash[1024] |
 * powerMod num2Bits[K] bits2Num[EM] MGF1_256 xor hDash256 */
static size_t ck_pss(ck_t *c, size_t b, int K, int SALT, uint32_t EXP, int H) {
  const char *T = "VerifyRsaPssSig signatures/rsaPss.circom";
  const int EM = 8 * K, EMB = 64 * K, HL = H / 8, DBL = EM - HL - 1, SB = SALT * 8, h384 = H == 384;
  size_t pk = b, sig = b + K, hd = sig + K, eM = hd + H, bits = eM + EM, enc = bits + EMB, dbm = enc + K,
         db = dbm + 8 * (size_t)DBL, salt = db + 8 * (size_t)DBL, mdb = salt + SB, hash = mdb + 8 * (size_t)DBL,
         md = hash + H, o = md + 1024;
  size_t pm = o;
  o += ck_powermod(c, pm, K, EXP);
  for (int i = 0; i < K; i++) {
    EQ(S(c, pm + K + i), S(c, sig + i), T, 43);
    EQ(S(c, pm + 2 * K + i), S(c, pk + i), T, 44);
    EQ(S(c, enc + i), S(c, pm + i), T, 48);
  }
  for (int i = 0; i < K; i++) {
    size_t nb = o;
    o += ck_num2bits(c, nb, 64);
    EQ(S(c, nb + 64), S(c, enc + K - 1 - i), T, 53);
    for (int j = 0; j < 64; j++) EQ(S(c, bits + (size_t)i * 64 + j), S(c, nb + 63 - j), T, 56);
  }
  for (int i = 0; i < EM; i++) {
    size_t bn = o;
    o += ck_bits2num(c, bn, 8);
    for (int j = 0; j < 8; j++) EQ(S(c, bn + 1 + 7 - j), S(c, bits + (size_t)i * 8 + j), T, 64);
    EQ(S(c, eM + EM - i - 1), S(c, bn), T, 66);
  }
  for (int i = 0; i < 8 * DBL; i++) EQ(S(c, mdb + i), S(c, bits + i), T, 86);
  for (int i = 0; i < H; i++) EQ(S(c, hash + i), S(c, bits + EMB - H - 8 + i), T, 89);
  size_t mg = o;
  o += ck_mgf1(c, mg, HL, DBL, H);
  for (int i = 0; i < H; i++) EQ(S(c, mg + 8 * (size_t)DBL + i), S(c, hash + i), T, h384 ? 105 : 96);
  for (int i = 0; i < 8 * DBL; i++) EQ(S(c, dbm + i), S(c, mg + i), T, h384 ? 108 : 99);
  size_t xr = o;  /* Xor2(n) bitify/bitGates.circom:232-240: out[n] | in1[n] in2[n] */
  o += 3 * 8 * (size_t)DBL;
  for (int i = 0; i < 8 * DBL; i++) {
    size_t n8 = 8 * (size_t)DBL;
    fr_t a = S(c, xr + n8 + i), bb = S(c, xr + 2 * n8 + i);
    req(c, S(c, xr + i), SUB(ADD(a, bb), MUL(MUL(KC(2), a), bb)), "Xor2 bitify/bitGates.circom", 238, xr);
    EQ(a, S(c, mdb + i), T, 129);
    EQ(bb, S(c, dbm + i), T, 130);
    EQ(S(c, db + i), i == 0 ? fr_zero() : S(c, xr + i), T, i == 0 ? 135 : 137);
  }
  for (int i = 0; i < SB; i++) EQ(S(c, salt + SB - 1 - i), S(c, db + 8 * (size_t)DBL - 1 - i), T, 143);
  for (int i = 0; i < 64; i++) EQ(S(c, md + i), fr_zero(), T, 149);
  for (int i = 0; i < H; i++) EQ(S(c, md + 64 + i), S(c, hd + i), T, 153);
  for (int i = 0; i < SB; i++) EQ(S(c, md + 64 + H + i), S(c, salt + i), T, 157);
  /* padding of M' to 1024 bits (576 bits for salt 32, 832 for SHA-256 salt 64 and SHA-384 salt 48): two SHA-256
   * blocks (64-bit length) or one SHA-384 block (128-bit length); the length fits the last 11 bits */
  int L = 64 + H + SB;
  const int lp = h384 ? 210 : SALT == 32 ? 167 : 188;
  for (int i = L; i < 1024; i++) {
    int v = (i == L);
    if (i >= 1013) v = (L >> (1023 - i)) & 1;  /* the length field: L < 2^11 */
    EQ(S(c, md + i), KC((uint64_t)v), T, lp);
  }
  size_t hh = o;
  o += ck_shahash(c, hh, h384 ? 1 : 2, H);
  for (int i = 0; i < 1024; i++) EQ(S(c, hh + H + i), S(c, md + i), T, h384 ? 224 : SALT == 32 ? 181 : 200);
  for (int i = 0; i < H; i++) EQ(S(c, hh + i), S(c, hash + i), T, h384 ? 225 : SALT == 32 ? 182 : 201);
  return o - b;
}

/* ============================================================ ECDSA (signatures/ecdsa.circom, ec/curve.circom, ec/get.circom) */
/* curve constants as EK chunks of EB bits, little-endian (signatureVerification.circom:177-263, ec/get.circom):
 * SIG 20 secp256r1 and 21 brainpoolP256r1 (4 x 64), 24 secp224r1 (7 x 32), 25 brainpoolP384r1 (6 x 64) */
typedef struct { int nl, cs; uint64_t A[7], B[7], P[7], order[7], dummy[2][7]; uint64_t *gpow; } ec_curve_t;
static ec_curve_t EC[4] = {
    {4, 64,
     {18446744073709551612ULL, 4294967295ULL, 0ULL, 18446744069414584321ULL},
     {4309448131093880907ULL, 7285987128567378166ULL, 12964664127075681980ULL, 6540974713487397863ULL},
     {18446744073709551615ULL, 4294967295ULL, 0ULL, 18446744069414584321ULL},
     {17562291160714782033ULL, 13611842547513532036ULL, 18446744073709551615ULL, 18446744069414584320ULL},
     {{4148137498610012746ULL, 51237685452122967ULL, 6555942389409504868ULL, 799804747332166731ULL},
      {13395177781894339167ULL, 1107697421929919296ULL, 6228258783500845564ULL, 11862546499924939746ULL}}, NULL},
    {4, 64,
     {16810331318623712729ULL, 18122579188607900780ULL, 17219079075415130087ULL, 9032542404991529047ULL},
     {7767825457231955894ULL, 10773760575486288334ULL, 17523706096862592191ULL, 2800214691157789508ULL},
     {2311270323689771895ULL, 7943213001558335528ULL, 4496292894210231666ULL, 12248480212390422972ULL},
     {10384753744809580199ULL, 10104242082523752183ULL, 4496292894210231665ULL, 12248480212390422972ULL},
     {{5870538370169240658ULL, 13064052279558318326ULL, 1032222391323187885ULL, 10478252910764369874ULL},
      {9125809427693782222ULL, 4479624720887462683ULL, 4313457861005768495ULL, 11848267593595748038ULL}}, NULL},
    {7, 32,
     {4294967294ULL, 4294967295ULL, 4294967295ULL, 4294967294ULL, 4294967295ULL, 4294967295ULL, 4294967295ULL},
     {592838580ULL, 655046979ULL, 3619674298ULL, 1346678967ULL, 4114690646ULL, 201634731ULL, 3020229253ULL},
     {1ULL, 0ULL, 0ULL, 4294967295ULL, 4294967295ULL, 4294967295ULL, 4294967295ULL},
     {1549543997ULL, 333261125ULL, 3770216510ULL, 4294907554ULL, 4294967295ULL, 4294967295ULL, 4294967295ULL},
     {{2477436510ULL, 406882550ULL, 2884834286ULL, 2269163287ULL, 3636783260ULL, 3699382582ULL, 912817446ULL},
      {582933619ULL, 1778719645ULL, 3780674687ULL, 3008581200ULL, 3586474874ULL, 866709652ULL, 3566930607ULL}}, NULL},
    {6, 64,
     {335737924824737830ULL, 9990533504564909291ULL, 1410020238645393679ULL, 14032832221039175559ULL,
      4355552632119865248ULL, 8918115475071440140ULL},
     {4230998357940653073ULL, 8985869839777909140ULL, 3352946025465340629ULL, 3438355245973688998ULL,
      10032249017711215740ULL, 335737924824737830ULL},
     {9747760000893709395ULL, 12453481191562877553ULL, 1347097566612230435ULL, 1526563086152259252ULL,
      1107163671716839903ULL, 10140169582434348328ULL},
     {4289733633151100261ULL, 14932448379039367952ULL, 2240099277684876711ULL, 1526563086152259251ULL,
      1107163671716839903ULL, 10140169582434348328ULL},
     {{522720248942821492ULL, 13227018843434759032ULL, 17067096815187998133ULL, 8957183796380674257ULL,
       7544165743263758981ULL, 6159107397665645433ULL},
      {9174881270872499347ULL, 7148726877058227897ULL, 1584493337432922624ULL, 1438582915076653591ULL,
       16161625210166602047ULL, 946254366129831718ULL}}, NULL}};
static int ec_curve_of(int sig) { return sig == 20 ? 0 : sig == 21 ? 1 : sig == 24 ? 2 : sig == 25 ? 3 : -1; }
static const ec_curve_t *CV;  /* the curve of the witness being checked */
static int EK = 4, EB = 64;   /* its CHUNK_NUMBER, CHUNK_SIZE */

int ck_load_ec_table(int curve, const char *path) {
  if (curve < 0 || curve > 3) return -3;
  const size_t n = (size_t)(EC[curve].nl * EC[curve].cs / 8) * 256 * 2 * EC[curve].nl;
  FILE *fp = fopen(path, "rb");
  if (!fp) return -1;
  uint64_t *t = malloc(8 * n);
  size_t got = fread(t, 8, n, fp);
  fclose(fp);
  if (got != n) { free(t); return -2; }
  free(EC[curve].gpow);
  EC[curve].gpow = t;
  return 0;
}
#define GPOW(i, j, a, k) CV->gpow[((((size_t)(i) * 256 + (j)) * 2 + (a)) * EK) + (k)]

/* ScalarMultOverflow(N) bigIntOverflow.circom:101-110: out[N] | in[N] scalar */
static size_t ck_smo(ck_t *c, size_t b, int N) {
  for (int i = 0; i < N; i++)
    EQ(S(c, b + i), MUL(S(c, b + 2 * N), S(c, b + N + i)), "ScalarMultOverflow bigInt/bigIntOverflow.circom", 108);
  return 2 * (size_t)N + 1;
}
/* BigAddOverflow(G, L) bigIntOverflow.circom:22-35: out[G] | in1[G] in2[L] */
static size_t ck_bao(ck_t *c, size_t b, int G, int L) {
  for (int i = 0; i < G; i++)
    EQ(S(c, b + i), i < L ? ADD(S(c, b + G + i), S(c, b + 2 * G + i)) : S(c, b + G + i), "BigAddOverflow bigInt/bigIntOverflow.circom",
       i < L ? 30 : 33);
  return 2 * (size_t)G + L;
}
/* BigSubModOverflow(EB, K) bigIntOverflow.circom:78-98: out[K] | in1[K] in2[K] modulus[K] */
static size_t ck_bsmo(ck_t *c, size_t b, int K) {
  const char *T = "BigSubModOverflow bigInt/bigIntOverflow.circom";
  for (int i = 0; i < K; i++) {
    fr_t v = SUB(ADD(S(c, b + 3 * K + i), S(c, b + K + i)), S(c, b + 2 * K + i));
    if (i == 0) v = ADD(v, P2[EB]);
    else if (i == K - 1) v = SUB(v, KC(1));
    else v = SUB(ADD(v, P2[EB]), KC(1));
    EQ(S(c, b + i), v, T, i == 0 ? 89 : i == K - 1 ? 92 : 94);
  }
  return 4 * (size_t)K;
}
/* BigIntIsZeroModP(EB, MAX, N, MAXN, NM) bigIntComparators.circom:158-212:
 * in[N] modulus[NM] | sign k[DIV] | kRangeChecks[DIV] mult isZero swicher[N]  (kRangeChecks.in is set by `<--`) */
static size_t ck_biszmp(ck_t *c, size_t b, int N, int MAX, int MAXN, int NM) {
  const char *T = "BigIntIsZeroModP bigInt/bigIntComparators.circom";
  const int DIV = MAXN - NM + 1;
  size_t in = b, md = b + N, sign = md + NM, k = sign + 1, o = k + DIV;
  EQ(MUL(S(c, sign), SUB(KC(1), S(c, sign))), fr_zero(), T, 167);
  for (int i = 0; i < DIV; i++) o += ck_num2bits(c, o, EB);
  size_t mult = o;
  int G = DIV >= NM ? DIV : NM, L = DIV >= NM ? NM : DIV;
  o += ck_bmo(c, mult, G, L);
  size_t m1 = mult + G + L - 1, m2 = m1 + G;
  for (int i = 0; i < NM; i++) EQ(S(c, (DIV >= NM ? m2 : m1) + i), S(c, md + i), T, DIV >= NM ? 185 : 189);
  for (int i = 0; i < DIV; i++) EQ(S(c, (DIV >= NM ? m1 : m2) + i), S(c, k + i), T, DIV >= NM ? 186 : 190);
  size_t iz = o;
  o += ck_bisz(c, iz, EB, MAX, MAXN);
  for (int i = 0; i < N; i++) {
    size_t sw = o;
    o += ck_switcher(c, sw);
    EQ(S(c, sw + 3), S(c, in + i), T, 197);
    EQ(S(c, sw + 4), fr_neg(S(c, in + i)), T, 198);
    EQ(S(c, sw + 2), S(c, sign), T, 199);
    EQ(S(c, iz + i), SUB(S(c, mult + i), S(c, sw + 1)), T, 201);
  }
  for (int i = N; i < MAXN; i++) EQ(S(c, iz + i), S(c, mult + i), T, 204);
  return o - b;
}

static fr_t L64(uint64_t v) { return fr_u64(v); }

/* PointOnCurve curve.circom:107-138: in[2][K] | squareX cubeX squareY coefMult isZeroModP(EB, 3 EB + 2K, 3K - 2, 3K, K) */
static size_t ck_ponc(ck_t *c, size_t b) {
  const char *T = "PointOnCurve ec/curve.circom";
  const int K = EK, K2 = 2 * K - 1, K3 = 3 * K - 2;
  size_t x = b, y = b + K, o = b + 2 * K;
  size_t sx = o; o += ck_bmo(c, sx, K, K);
  size_t cx = o; o += ck_bmo(c, cx, K2, K);
  size_t sy = o; o += ck_bmo(c, sy, K, K);
  size_t cm = o; o += ck_bmo(c, cm, K, K);
  size_t iz = o; o += ck_biszmp(c, iz, K3, 3 * EB + 2 * K, 3 * K, K);
  for (int i = 0; i < K; i++) {
    EQ(S(c, sx + K2 + i), S(c, x + i), T, 111); EQ(S(c, sx + K2 + K + i), S(c, x + i), T, 112);
    EQ(S(c, cx + K3 + K2 + i), S(c, x + i), T, 116);
    EQ(S(c, sy + K2 + i), S(c, y + i), T, 119); EQ(S(c, sy + K2 + K + i), S(c, y + i), T, 120);
    EQ(S(c, cm + K2 + i), S(c, x + i), T, 123); EQ(S(c, cm + K2 + K + i), L64(CV->A[i]), T, 124);
    EQ(S(c, iz + K3 + i), L64(CV->P[i]), T, 137);
  }
  for (int i = 0; i < K2; i++) EQ(S(c, cx + K3 + i), S(c, sx + i), T, 115);
  for (int i = 0; i < K3; i++) {
    fr_t v = S(c, cx + i);
    if (i < K2) v = SUB(ADD(v, S(c, cm + i)), S(c, sy + i));
    if (i < K) v = ADD(v, L64(CV->B[i]));
    EQ(S(c, iz + i), v, T, i < K ? 128 : i < K2 ? 131 : 134);
  }
  return o - b;
}

/* PointOnTangent curve.circom:144-190: in1[2][K] in2[2][K] | squareX scalarMult bigAdd bigSub rightMult scalarMult2
 * bigAdd2 leftMult isZeroModP(EB, 3 EB + 2K, 3K - 2, 3K + 1, K) */
static size_t ck_pont(ck_t *c, size_t b) {
  const char *T = "PointOnTangent ec/curve.circom";
  const int K = EK, K2 = 2 * K - 1, K3 = 3 * K - 2;
  size_t x1 = b, y1 = b + K, x3 = b + 2 * K, y3 = b + 3 * K, o = b + 4 * K;
  size_t sx = o; o += ck_bmo(c, sx, K, K);
  size_t sm = o; o += ck_smo(c, sm, K2);
  size_t ba = o; o += ck_bao(c, ba, K2, K);
  size_t bs = o; o += ck_bsmo(c, bs, K);
  size_t rm = o; o += ck_bmo(c, rm, K2, K);
  size_t sm2 = o; o += ck_smo(c, sm2, K);
  size_t ba2 = o; o += ck_bao(c, ba2, K, K);
  size_t lm = o; o += ck_bmo(c, lm, K, K);
  size_t iz = o; o += ck_biszmp(c, iz, K3, 3 * EB + 2 * K, 3 * K + 1, K);
  for (int i = 0; i < K; i++) {
    EQ(S(c, sx + K2 + i), S(c, x1 + i), T, 148); EQ(S(c, sx + K2 + K + i), S(c, x1 + i), T, 149);
    EQ(S(c, ba + 2 * K2 + i), L64(CV->A[i]), T, 157);
    EQ(S(c, bs + K + i), S(c, x1 + i), T, 161); EQ(S(c, bs + 2 * K + i), S(c, x3 + i), T, 162);
    EQ(S(c, bs + 3 * K + i), L64(CV->P[i]), T, 163);
    EQ(S(c, rm + K3 + K2 + i), S(c, bs + i), T, 167);
    EQ(S(c, sm2 + K + i), S(c, y1 + i), T, 170);
    EQ(S(c, ba2 + K + i), S(c, y1 + i), T, 174); EQ(S(c, ba2 + 2 * K + i), S(c, y3 + i), T, 175);
    EQ(S(c, lm + K2 + i), S(c, ba2 + i), T, 178); EQ(S(c, lm + K2 + K + i), S(c, sm2 + i), T, 179);
    EQ(S(c, iz + K3 + i), L64(CV->P[i]), T, 189);
  }
  for (int i = 0; i < K2; i++) {
    EQ(S(c, sm + K2 + i), S(c, sx + i), T, 152);
    EQ(S(c, ba + K2 + i), S(c, sm + i), T, 156);
    EQ(S(c, rm + K3 + i), S(c, ba + i), T, 166);
  }
  EQ(S(c, sm + 2 * K2), KC(3), T, 153);
  EQ(S(c, sm2 + 2 * K), KC(2), T, 171);
  for (int i = 0; i < K3; i++) EQ(S(c, iz + i), i < K2 ? SUB(S(c, rm + i), S(c, lm + i)) : S(c, rm + i), T, i < K2 ? 182 : 185);
  return o - b;
}

/* PointOnLine curve.circom:198-238: in1 in2 in3 [2][K] | bigAdd bigSub bigSub2 bigSub3 leftMult rightMult
 * isZeroModP(EB, 2 EB + 2K, 2K - 1, 2K + 1, K) */
static size_t ck_ponl(ck_t *c, size_t b) {
  const char *T = "PointOnLine ec/curve.circom";
  const int K = EK, K2 = 2 * K - 1;
  size_t x1 = b, y1 = b + K, x2 = b + 2 * K, y2 = b + 3 * K, x3 = b + 4 * K, y3 = b + 5 * K, o = b + 6 * K;
  size_t ba = o; o += ck_bao(c, ba, K, K);
  size_t s1 = o; o += ck_bsmo(c, s1, K);
  size_t s2 = o; o += ck_bsmo(c, s2, K);
  size_t s3 = o; o += ck_bsmo(c, s3, K);
  size_t lm = o; o += ck_bmo(c, lm, K, K);
  size_t rm = o; o += ck_bmo(c, rm, K, K);
  size_t iz = o; o += ck_biszmp(c, iz, K2, 2 * EB + 2 * K, 2 * K + 1, K);
  for (int i = 0; i < K; i++) {
    EQ(S(c, ba + K + i), S(c, y1 + i), T, 204); EQ(S(c, ba + 2 * K + i), S(c, y3 + i), T, 205);
    EQ(S(c, s1 + K + i), S(c, x2 + i), T, 208); EQ(S(c, s1 + 2 * K + i), S(c, x1 + i), T, 209);
    EQ(S(c, s2 + K + i), S(c, y2 + i), T, 213); EQ(S(c, s2 + 2 * K + i), S(c, y1 + i), T, 214);
    EQ(S(c, s3 + K + i), S(c, x1 + i), T, 218); EQ(S(c, s3 + 2 * K + i), S(c, x3 + i), T, 219);
    EQ(S(c, s1 + 3 * K + i), L64(CV->P[i]), T, 210); EQ(S(c, s2 + 3 * K + i), L64(CV->P[i]), T, 215);
    EQ(S(c, s3 + 3 * K + i), L64(CV->P[i]), T, 220);
    EQ(S(c, lm + K2 + i), S(c, ba + i), T, 223); EQ(S(c, lm + K2 + K + i), S(c, s1 + i), T, 224);
    EQ(S(c, rm + K2 + i), S(c, s2 + i), T, 227); EQ(S(c, rm + K2 + K + i), S(c, s3 + i), T, 228);
    EQ(S(c, iz + K2 + i), L64(CV->P[i]), T, 236);
  }
  for (int i = 0; i < K2; i++) EQ(S(c, iz + i), SUB(S(c, lm + i), S(c, rm + i)), T, 233);
  return o - b;
}

/* EllipticCurveDouble curve.circom:281-313: out[2][K] | in[2][K] | onTangentCheck onCurveCheck */
static size_t ck_ecdbl(ck_t *c, size_t b) {
  const char *T = "EllipticCurveDouble ec/curve.circom";
  const int PT = 2 * EK;
  size_t o = b + 2 * PT, tg = o;
  o += ck_pont(c, tg);
  size_t oc = o;
  o += ck_ponc(c, oc);
  for (int i = 0; i < PT; i++) {
    EQ(S(c, tg + i), S(c, b + PT + i), T, 301);
    EQ(S(c, tg + PT + i), S(c, b + i), T, 302);
    EQ(S(c, oc + i), S(c, b + i), T, 305);
  }
  return o - b;
}
/* EllipticCurveAdd curve.circom:316-350: out[2][K] | in1 in2 | onCurveCheck onLineCheck */
static size_t ck_ecadd(ck_t *c, size_t b) {
  const char *T = "EllipticCurveAdd ec/curve.circom";
  const int PT = 2 * EK;
  size_t o = b + 3 * PT, oc = o;
  o += ck_ponc(c, oc);
  size_t ln = o;
  o += ck_ponl(c, ln);
  for (int i = 0; i < PT; i++) {
    EQ(S(c, oc + i), S(c, b + i), T, 339);
    EQ(S(c, ln + i), S(c, b + PT + i), T, 342);
    EQ(S(c, ln + PT + i), S(c, b + 2 * PT + i), T, 343);
    EQ(S(c, ln + 2 * PT + i), S(c, b + i), T, 344);
  }
  return o - b;
}
/* EllipticCurveGetDummy ec/get.circom:79-140: dummyPoint[2][K] */
static size_t ck_getdummy(ck_t *c, size_t b) {
  for (int a = 0; a < 2; a++)
    for (int i = 0; i < EK; i++) EQ(S(c, b + EK * a + i), L64(CV->dummy[a][i]), "EllipticCurveGetDummy ec/get.circom", 92 + a);
  return 2 * (size_t)EK;
}

/* EllipticCurvePrecomputePipinger(.., 4) curve.circom:242-278: out[16][2][K] | in[2][K] | getDummy (doublers, adders) */
static size_t ck_precompute(ck_t *c, size_t b) {
  const char *T = "EllipticCurvePrecomputePipinger ec/curve.circom";
  const size_t PT = 2 * (size_t)EK;
  size_t out = b, in = b + 16 * PT, o = in + PT;
  size_t gd = o;
  o += ck_getdummy(c, gd);
  for (size_t i = 0; i < PT; i++) {
    EQ(S(c, out + i), S(c, gd + i), T, 253);
    EQ(S(c, out + PT + i), S(c, in + i), T, 255);
  }
  for (int i = 2; i < 16; i++) {
    size_t x = o;
    if (i % 2 == 0) {
      o += ck_ecdbl(c, x);
      for (size_t q = 0; q < PT; q++) {
        EQ(S(c, x + PT + q), S(c, out + PT * (size_t)(i / 2) + q), T, 263);
        EQ(S(c, out + PT * (size_t)i + q), S(c, x + q), T, 264);
      }
    } else {
      o += ck_ecadd(c, x);
      for (size_t q = 0; q < PT; q++) {
        EQ(S(c, x + PT + q), S(c, out + PT + q), T, 269);
        EQ(S(c, x + 2 * PT + q), S(c, out + PT * (size_t)(i - 1) + q), T, 270);
        EQ(S(c, out + PT * (size_t)i + q), S(c, x + q), T, 271);
      }
    }
  }
  return o - b;
}

/* EllipticCurveScalarMult(.., 4) curve.circom:359-512 (F = K EB bits, F / 4 windows): out[2][K] | in[2][K] scalar[K] |
 * scalarBits[F] resultingPoints[F/4+1][2][K] additionPoints[F/4][2][K] | precompute getDummy num2Bits[K], then per
 * window: bits2Num isZeroResult [doublers (doubleSwitcher x2K after the first) ] getSum x2K partsEqual x16
 * [adders isZeroAddition (resultSwitcherAddition resultSwitcherDoubling) x2K] */
static size_t ck_ecmul(ck_t *c, size_t b) {
  const char *T = "EllipticCurveScalarMult ec/curve.circom";
  const int F = EK * EB, NW = F / 4;
  const size_t PT = 2 * (size_t)EK;
  size_t out = b, in = b + PT, sc = in + PT, bits = sc + EK, rp = bits + F, ap = rp + (NW + 1) * PT, o = ap + NW * PT;
  size_t pc = o;
  o += ck_precompute(c, pc);
  for (size_t i = 0; i < PT; i++) EQ(S(c, pc + 16 * PT + i), S(c, in + i), T, 368);
  size_t gd = o;
  o += ck_getdummy(c, gd);
  for (int i = 0; i < EK; i++) {
    size_t nb = o;
    o += ck_num2bits(c, nb, EB);
    EQ(S(c, nb + EB), S(c, sc + i), T, 387);
    for (int j = 0; j < EB; j++) EQ(S(c, bits + F - EB * (i + 1) + j), S(c, nb + EB - 1 - j), T, 389);
  }
  for (size_t q = 0; q < PT; q++) EQ(S(c, rp + q), S(c, pc + q), T, 409);
  size_t *dbl_at = malloc(sizeof(size_t) * F);
  for (int i = 0; i < F; i += 4) {
    int w = i / 4;
    size_t bn = o;
    o += ck_bits2num(c, bn, 4);
    for (int j = 0; j < 4; j++) EQ(S(c, bn + 1 + j), S(c, bits + i + 3 - j), T, 414);
    size_t izr = o;
    o += ck_isequal(c, izr);
    EQ(S(c, izr + 1), S(c, rp + PT * (size_t)w), T, 418);
    EQ(S(c, izr + 2), S(c, gd), T, 419);
    if (i != 0) {
      for (int j = 0; j < 4; j++) {
        size_t d = o;
        dbl_at[i + j - 4] = d;
        o += ck_ecdbl(c, d);
        if (j == 0) {
          for (size_t q = 0; q < PT; q++) {
            size_t sw = o;
            o += ck_switcher(c, sw);
            EQ(S(c, sw + 2), S(c, izr), T, 431);
            EQ(S(c, sw + 3), S(c, gd + q), T, 432);
            EQ(S(c, sw + 4), S(c, rp + PT * (size_t)w + q), T, 433);
            EQ(S(c, d + PT + q), S(c, sw + 1), T, 435);
          }
        } else {
          for (size_t q = 0; q < PT; q++) EQ(S(c, d + PT + q), S(c, dbl_at[i + j - 5] + q), T, 440);
        }
      }
    }
    size_t gs = o;
    for (size_t q = 0; q < PT; q++) o += ck_getsum(c, o, 16);
    for (int pt = 0; pt < 16; pt++) {
      size_t pe = o;
      o += ck_isequal(c, pe);
      EQ(S(c, pe + 1), KC((uint64_t)pt), T, 457);
      EQ(S(c, pe + 2), S(c, bn), T, 458);
      for (size_t q = 0; q < PT; q++) EQ(S(c, gs + 32 * q + 1 + pt), MUL(S(c, pe), S(c, pc + PT * (size_t)pt + q)), T, 461);
    }
    for (size_t q = 0; q < PT; q++) EQ(S(c, ap + PT * (size_t)w + q), S(c, gs + 32 * q), T, 470);
    if (i == 0) {
      for (size_t q = 0; q < PT; q++) EQ(S(c, rp + PT + q), S(c, ap + q), T, 476);
    } else {
      size_t ad = o;
      o += ck_ecadd(c, ad);
      for (size_t q = 0; q < PT; q++) {
        EQ(S(c, ad + PT + q), S(c, dbl_at[i - 1] + q), T, 482);
        EQ(S(c, ad + 2 * PT + q), S(c, ap + PT * (size_t)w + q), T, 483);
      }
      size_t iza = o;
      o += ck_isequal(c, iza);
      EQ(S(c, iza + 1), S(c, ap + PT * (size_t)w), T, 486);
      EQ(S(c, iza + 2), S(c, gd), T, 487);
      for (size_t q = 0; q < PT; q++) {
        size_t sa = o, sd = o + 6;
        o += 12;
        ck_switcher(c, sa);
        ck_switcher(c, sd);
        EQ(S(c, sa + 2), S(c, iza), T, 500);
        EQ(S(c, sa + 3), S(c, ad + q), T, 501);
        EQ(S(c, sa + 4), S(c, dbl_at[i - 1] + q), T, 502);
        EQ(S(c, sd + 2), S(c, izr), T, 504);
        EQ(S(c, sd + 3), S(c, ap + PT * (size_t)w + q), T, 505);
        EQ(S(c, sd + 4), S(c, sa), T, 506);
        EQ(S(c, rp + PT * (size_t)(w + 1) + q), S(c, sd + 1), T, 508);
      }
    }
  }
  free(dbl_at);
  for (size_t q = 0; q < PT; q++) EQ(S(c, out + q), S(c, rp + (size_t)NW * PT + q), T, 513);
  return o - b;
}

/* EllipicCurveScalarGeneratorMult curve.circom:680-906 (NP = K EB / 8 parts): out[2][K] | scalar[K] |
 * resultCoordinateComputation[NP][256][2][K] additionPoints[NP][2][K] resultingPointsLeft/Left2/Right/Right2 (never
 * assigned) resultingPoints[NP][2][K] | num2bits[K] bits2num[NP] getDummy getSecondDummy equal[NP][256]
 * getSumOfNElements[NP][2][K] (adders isFirstDummyLeft isSecondDummyLeft isFirstDummyRight isSecondDummyRight
 * (switcherRight switcherLeft) x2K)[NP-1] */
static size_t ck_ecgen(ck_t *c, size_t b) {
  const char *T = "EllipicCurveScalarGeneratorMult ec/curve.circom";
  const size_t NP = (size_t)EK * EB / 8, PT = 2 * (size_t)EK;
  size_t out = b, sc = b + PT, rcc = sc + EK, ap = rcc + NP * 256 * PT, unused = ap + NP * PT, rp = unused + 4 * NP * PT,
         o = rp + NP * PT;
  size_t n2b[7];
  for (int i = 0; i < EK; i++) {
    n2b[i] = o;
    o += ck_num2bits(c, o, EB);
    EQ(S(c, n2b[i] + EB), S(c, sc + i), T, 733);
  }
  size_t *b2n = malloc(sizeof(size_t) * NP);
  for (size_t i = 0; i < NP; i++) {
    b2n[i] = o;
    o += ck_bits2num(c, o, 8);
    for (int j = 0; j < 8; j++) EQ(S(c, b2n[i] + 1 + j), S(c, n2b[(i * 8 + j) / EB] + (i * 8 + j) % EB), T, 739);
  }
  size_t gd = o;
  o += ck_getdummy(c, gd);
  size_t g2 = o;
  o += ck_ecdbl(c, g2);
  for (size_t q = 0; q < PT; q++) EQ(S(c, g2 + PT + q), S(c, gd + q), T, 745);
  for (size_t i = 0; i < NP; i++)
    for (int j = 0; j < 256; j++) {
      size_t e = o;
      o += ck_isequal(c, e);
      EQ(S(c, e + 1), KC((uint64_t)j), T, 751);
      EQ(S(c, e + 2), S(c, b2n[i]), T, 752);
      for (size_t q = 0; q < PT; q++) {
        fr_t v;
        if (j == 0) v = (i % 2 == 0) ? S(c, gd + q) : S(c, g2 + q);
        else v = L64(GPOW(i, j, q / EK, q % EK));
        EQ(S(c, rcc + (i * 256 + j) * PT + q), MUL(S(c, e), v), T, j == 0 ? (i % 2 == 0 ? 756 : 764) : 772);
      }
    }
  for (size_t i = 0; i < NP; i++)
    for (size_t q = 0; q < PT; q++) {
      size_t g = o;
      o += ck_getsum(c, g, 256);
      for (int j = 0; j < 256; j++) EQ(S(c, g + 1 + j), S(c, rcc + (i * 256 + j) * PT + q), T, 787);
      EQ(S(c, ap + i * PT + q), S(c, g), T, 797);
    }
  free(b2n);
  for (size_t i = 0; i + 1 < NP; i++) {
    size_t ad = o;
    o += ck_ecadd(c, ad);
    size_t fl = o, sl = o + 6, fr = o + 12, sr = o + 18;
    o += 24;
    ck_isequal(c, fl); ck_isequal(c, sl); ck_isequal(c, fr); ck_isequal(c, sr);
    EQ(S(c, fl + 1), S(c, gd), T, 826);
    EQ(S(c, sl + 1), S(c, g2), T, 828);
    EQ(S(c, fr + 1), S(c, gd), T, 831);
    EQ(S(c, sr + 1), S(c, g2), T, 833);
    fr_t left0 = i == 0 ? S(c, ap) : S(c, rp + (i - 1) * PT);
    EQ(S(c, fl + 2), left0, T, i == 0 ? 838 : 866);
    EQ(S(c, sl + 2), left0, T, i == 0 ? 839 : 867);
    EQ(S(c, fr + 2), S(c, ap + (i + 1) * PT), T, i == 0 ? 840 : 868);
    EQ(S(c, sr + 2), S(c, ap + (i + 1) * PT), T, i == 0 ? 841 : 869);
    for (size_t q = 0; q < PT; q++) {
      EQ(S(c, ad + PT + q), i == 0 ? S(c, ap + q) : S(c, rp + (i - 1) * PT + q), T, i == 0 ? 842 : 871);
      EQ(S(c, ad + 2 * PT + q), S(c, ap + (i + 1) * PT + q), T, i == 0 ? 843 : 872);
    }
    for (size_t q = 0; q < PT; q++) {
      size_t swr = o, swl = o + 6;
      o += 12;
      ck_switcher(c, swr);
      ck_switcher(c, swl);
      EQ(S(c, swr + 2), ADD(S(c, sr), S(c, fr)), T, 853);
      EQ(S(c, swr + 3), S(c, ad + q), T, 854);
      EQ(S(c, swr + 4), i == 0 ? S(c, ap + q) : S(c, rp + (i - 1) * PT + q), T, i == 0 ? 855 : 883);
      EQ(S(c, swl + 2), ADD(S(c, sl), S(c, fl)), T, 858);
      EQ(S(c, swl + 3), S(c, ap + (i + 1) * PT + q), T, 859);
      EQ(S(c, swl + 4), S(c, swr), T, 860);
      EQ(S(c, rp + i * PT + q), S(c, swl + 1), T, 862);
    }
  }
  for (size_t q = 0; q < PT; q++) EQ(S(c, out + q), S(c, rp + (NP - 2) * PT + q), T, 905);
  return o - b;
}

/* BigModInv(EB, K) bigInt.circom:344-368: out[K] | in[K] modulus[K] | mult */
static size_t ck_bminv(ck_t *c, size_t b, int K) {
  const char *T = "BigModInv bigInt/bigInt.circom";
  size_t m = b + 3 * (size_t)K;
  size_t sz = 3 * (size_t)K + ck_bmm_n(c, m, EB, K);
  size_t md_out = m + K + 1, in1 = md_out + K, in2 = in1 + K, modl = in2 + K;
  for (int i = 0; i < K; i++) {
    EQ(S(c, in1 + i), S(c, b + K + i), T, 357);
    EQ(S(c, in2 + i), S(c, b + i), T, 358);
    EQ(S(c, modl + i), S(c, b + 2 * K + i), T, 359);
    EQ(S(c, md_out + i), KC(i == 0), T, i == 0 ? 362 : 364);
  }
  return sz;
}

/* verifyECDSABits(EB, K, A, B, P, K EB) signatures/ecdsa.circom:18-87: pubkey[2][K] signature[2][K] hashed[K EB] |
 * hashedChunked[K] one[K] order[K] sinv[K] | bits2Num[K] getOrder modInv mult mult2 scalarMult1 scalarMult2 add modOrder */
static size_t ck_ecdsa(ck_t *c, size_t b) {
  const char *T = "verifyECDSABits signatures/ecdsa.circom";
  const int K = EK, PT = 2 * EK;
  size_t pk = b, sig = b + PT, hs = sig + PT, hc = hs + (size_t)K * EB, one = hc + K, ord = one + K, sinv = ord + K, o = sinv + K;
  EQ(S(c, one), KC(1), T, 27);
  for (int i = 1; i < K; i++) EQ(S(c, one + i), fr_zero(), T, 29);
  for (int i = 0; i < K; i++) {
    size_t bn = o;
    o += ck_bits2num(c, bn, EB);
    for (int j = 0; j < EB; j++) EQ(S(c, bn + 1 + EB - 1 - j), S(c, hs + (size_t)i * EB + j), T, 36);
    EQ(S(c, hc + K - 1 - i), S(c, bn), T, 38);
  }
  size_t go = o;  /* EllipicCurveGetOrder ec/get.circom:146: order[K] */
  for (int i = 0; i < K; i++) req(c, S(c, go + i), L64(CV->order[i]), "EllipicCurveGetOrder ec/get.circom", 156, go);
  o += K;
  for (int i = 0; i < K; i++) EQ(S(c, ord + i), S(c, go + i), T, 43);
  size_t mi = o;
  o += ck_bminv(c, mi, K);
  for (int i = 0; i < K; i++) {
    EQ(S(c, mi + K + i), S(c, sig + K + i), T, 50);
    EQ(S(c, mi + 2 * K + i), S(c, ord + i), T, 51);
    EQ(S(c, sinv + i), S(c, mi + i), T, 52);
  }
  size_t m1 = o;
  o += ck_bmm_n(c, m1, EB, K);
  size_t m2 = o;
  o += ck_bmm_n(c, m2, EB, K);
#define BI1(m) ((m) + 2 * (size_t)K + 1)
  for (int i = 0; i < K; i++) {
    EQ(S(c, BI1(m1) + i), S(c, sinv + i), T, 56);
    EQ(S(c, BI1(m1) + K + i), S(c, hc + i), T, 57);
    EQ(S(c, BI1(m1) + 2 * K + i), S(c, ord + i), T, 58);
    EQ(S(c, BI1(m2) + i), S(c, sinv + i), T, 62);
    EQ(S(c, BI1(m2) + K + i), S(c, sig + i), T, 63);
    EQ(S(c, BI1(m2) + 2 * K + i), S(c, ord + i), T, 64);
  }
  size_t g = o;
  o += ck_ecgen(c, g);
  for (int i = 0; i < K; i++) EQ(S(c, g + PT + i), S(c, m1 + K + 1 + i), T, 68);
  size_t sm = o;
  o += ck_ecmul(c, sm);
  for (int i = 0; i < K; i++) EQ(S(c, sm + 2 * PT + i), S(c, m2 + K + 1 + i), T, 72);
  for (int i = 0; i < PT; i++) EQ(S(c, sm + PT + i), S(c, pk + i), T, 73);
  size_t ad = o;
  o += ck_ecadd(c, ad);
  for (int i = 0; i < PT; i++) {
    EQ(S(c, ad + PT + i), S(c, g + i), T, 77);
    EQ(S(c, ad + 2 * PT + i), S(c, sm + i), T, 78);
  }
  size_t mo = o;
  o += ck_bmm_n(c, mo, EB, K);
  for (int i = 0; i < K; i++) {
    EQ(S(c, BI1(mo) + i), S(c, ad + i), T, 83);
    EQ(S(c, BI1(mo) + K + i), S(c, one + i), T, 84);
    EQ(S(c, BI1(mo) + 2 * K + i), S(c, ord + i), T, 85);
    EQ(S(c, mo + K + 1 + i), S(c, sig + i), T, 89);
  }
#undef BI1
  return o - b;
}

/* ============================================================ passport verification */
/* PassportVerificationFlow(ECS, H, EHT, DG1S, DG15S, SAS, DG15V) passportVerificationFlow.circom:6-109:
 * flowResult | dg1Hash[H] dg15Hash[H] encapsulatedContent[ECS] encapsulatedContentHash[EHT] signedAttributes[1024] |
 * verifyAllChecksPassed[3H+8] | dg1Eq[H] dg15Eq[H] encEq[H] prefix[8] */
static size_t ck_flow(ck_t *c, size_t b, int ECS, int H, int EHT, int DG1S, int DG15S, int SAS, int DG15V) {
  const char *T = "PassportVerificationFlow passportVerification/passportVerificationFlow.circom";
  size_t fr_ = b, d1 = b + 1, d15 = d1 + H, ec = d15 + H, ech = ec + ECS, sa = ech + EHT, v = sa + 1024,
         o = v + 3 * (size_t)H + 8;
  fr_t aa = KC((uint64_t)DG15V);
  size_t eq0 = o;
  for (int i = 0; i < 3 * H + 8; i++) o += ck_isequal(c, o);
#define EQB(i) (eq0 + 6 * (size_t)(i))
  for (int i = 0; i < H; i++) {
    EQ(S(c, EQB(i) + 1), S(c, d1 + i), T, 30);
    EQ(S(c, EQB(i) + 2), S(c, ec + DG1S + i), T, 31);
    EQ(S(c, EQB(H + i) + 1), MUL(S(c, d15 + i), aa), T, 45);
    EQ(S(c, EQB(H + i) + 2), MUL(S(c, ec + DG15S + i), aa), T, 46);
    EQ(S(c, EQB(2 * H + i) + 1), S(c, ech + i), T, 59);
    EQ(S(c, EQB(2 * H + i) + 2), S(c, sa + SAS + i), T, 60);
  }
  static const int pre[8] = {0, 0, 0, 0, 1, 1, 1, 1};
  for (int i = 0; i < 8; i++) {
    EQ(S(c, EQB(3 * H + i) + 1), MUL(KC(pre[i]), aa), T, 74);
    EQ(S(c, EQB(3 * H + i) + 2), MUL(S(c, ec + DG15S - 24 + i), aa), T, 75);
  }
  EQ(S(c, v), S(c, EQB(0)), T, 84);
  for (int i = 1; i < 3 * H + 8; i++) EQ(S(c, v + i), MUL(S(c, v + i - 1), S(c, EQB(i))), T, 87);
#undef EQB
  EQ(S(c, fr_), S(c, v + 3 * H + 7), T, 108);
  return o - b;
}

/* ShaHashChunks(B, ALGO) hasher/hash.circom:32-68: out[ALGO] | in[BS x B] | hashALGO (BS = 512, or 1024 above 256) */
static size_t ck_shahash(ck_t *c, size_t b, int B, int algo) {
  const char *T = "ShaHashChunks hasher/hash.circom";
  const size_t BS = algo > 256 ? 1024 : 512;
  size_t out = b, in = b + algo, h = in + BS * (size_t)B;
  size_t sz = (size_t)algo + BS * (size_t)B +
              (algo == 160 ? ck_sha1chunks(c, h, B) : algo > 256 ? ck_sha5chunks(c, h, B, algo) : ck_sha2chunks(c, h, B, algo));
  int l0 = algo == 160 ? 46 : algo == 224 ? 51 : algo == 256 ? 56 : algo == 384 ? 60 : 65;
  for (size_t i = 0; i < BS * B; i++) EQ(S(c, h + algo + i), S(c, in + i), T, l0);
  for (int i = 0; i < algo; i++) EQ(S(c, out + i), S(c, h + i), T, l0 + 1);
  return sz;
}

/* RsaVerifyPkcs1v15(64, K, EXP, 160) signatures/rsa.circom:73-109:
 * signature[K] pubkey[K] hashed[160] | hashed_chunks[2] | pm bits2num[0] bits2num[1] getBits getDiv */
static size_t ck_rsa_pkcs160(ck_t *c, size_t b, int K, uint32_t EXP) {
  const char *T = "RsaVerifyPkcs1v15 signatures/rsa.circom";
  size_t sig = b, pk = b + K, hs = pk + K, o = hs + 160 + 2;  /* hashed_chunks[2] are never assigned */
  size_t pm = o;
  o += ck_powermod(c, pm, K, EXP);
  for (int i = 0; i < K; i++) {
    EQ(S(c, pm + K + i), S(c, sig + i), T, 76);
    EQ(S(c, pm + 2 * K + i), S(c, pk + i), T, 77);
  }
  for (int i = 0; i < 2; i++) {
    size_t bn = o;
    o += ck_bits2num(c, bn, 64);
    for (int j = 0; j < 64; j++) EQ(S(c, bn + 1 + j), S(c, hs + 159 - j - i * 64), T, 86);
  }
  size_t gb = o;
  o += ck_num2bits(c, gb, 64);
  size_t gd = o;
  o += ck_bits2num(c, gd, 32);
  EQ(S(c, gb + 64), S(c, pm + 2), T, 92);
  for (int i = 0; i < 32; i++) EQ(S(c, gb + i), S(c, hs + 31 - i), T, 95);
  for (int i = 32; i < 64; i++) EQ(S(c, gd + 1 + i - 32), S(c, gb + i), T, 99);
  EQ(S(c, gd), KC(83887124), T, 101);
  EQ(S(c, pm + 3), KC(650212878678426138ULL), T, 104);
  EQ(S(c, pm + 4), KC(18446744069417738544ULL), T, 105);
  for (int i = 5; i < K - 1; i++) EQ(S(c, pm + i), KC(18446744073709551615ULL), T, 107);
  EQ(S(c, pm + K - 1), KC(562949953421311ULL), T, 110);
  return o - b;
}

typedef struct { int sig, dg_hash, doc, ec_blocks, ec_shift, dg1_shift, aa, dg15_shift, dg15_blocks, aa_shift; } ck_params;

static int sig_K(int sig) {
  return sig == 2 ? 64 : (sig == 4 || sig == 14) ? 48 : sig >= 20 ? (ec_curve_of(sig) >= 0 ? EC[ec_curve_of(sig)].nl : 4) : 32;
}
/* HASH_TYPE of the SA hasher (passportVerificationBuilder.circom:16-59) and EC_HASH_TYPE of the EC hasher (:53: the
 * HASH_TYPE before SIG 24 sets 224) */
static int sig_hash(int sig) { return (sig == 3 || sig == 4) ? 160 : (sig == 13 || sig == 25) ? 384 : sig == 24 ? 224 : 256; }
static int ec_hash_t(int sig) { return sig == 24 ? 256 : sig_hash(sig); }

/* PassportVerificationBuilder(...) passportVerificationBuilder.circom:11-246 (RSA PKCS#1 v1.5 over SHA-2):
 * passportHash | encapsulatedContent dg1 dg15 signedAttributes signature pubkey slaveMerkleInclusionBranches[80]
 * slaveMerkleRoot | dg1Hash dg15Hash encapsulatedContentHash signedAttributesHash pubkeyHash tempModulus[5] |
 * dg1PassportHasher [dg15PassportHasher] ecPassportHasher saPassportHasher passportVerificationFlow
 * signatureVerification signedAttributesNum pubkeyHasherRsa smtVerifier signedAttributesHashHasher */
static size_t ck_pvb(ck_t *c, size_t b, const ck_params *P) {
  const char *T = "PassportVerificationBuilder passportVerification/passportVerificationBuilder.circom";
  const int K = sig_K(P->sig), DGH = P->dg_hash, HT = sig_hash(P->sig), EHT = ec_hash_t(P->sig), HBS = HT > 256 ? 1024 : 512,
            DBS = DGH > 256 ? 1024 : 512, ECL = P->ec_blocks * HBS, D15L = P->dg15_blocks * HBS, ecdsa = P->sig >= 20,
            PKL = ecdsa ? 2 * K : K;
  size_t ph = b, ec = b + 1, dg1 = ec + ECL, dg15 = dg1 + 1024, sa = dg15 + D15L, sig = sa + 1024, pk = sig + PKL,
         br = pk + PKL, root = br + 80;
  /* intermediates: ..., pubkeyHash, then tempModulus[5] (RSA, :170) or ecBitsX[F] ecBitsY[F] (ECDSA, :188-189) */
  const int EF = ecdsa ? K * EB : 0;
  size_t d1h = root + 1, d15h = d1h + DGH, ech = d15h + DGH, sah = ech + EHT, pkh = sah + HT, tmod = pkh + 1,
         ebx = pkh + 1, eby = ebx + EF, o = ecdsa ? eby + EF : tmod + 5;
  size_t hs = o;
  o += ck_shahash(c, hs, 1024 / DBS, DGH);
  for (int j = 0; j < 1024; j++) EQ(S(c, hs + DGH + j), S(c, dg1 + j), T, 104);
  for (int j = 0; j < DGH; j++) EQ(S(c, d1h + j), S(c, hs + j), T, 98);
  if (P->aa) {
    hs = o;
    o += ck_shahash(c, hs, P->dg15_blocks, DGH);
    for (int j = 0; j < DBS * P->dg15_blocks; j++) EQ(S(c, hs + DGH + j), S(c, dg15 + j), T, 119);
    for (int j = 0; j < DGH; j++) EQ(S(c, d15h + j), S(c, hs + j), T, 113);
  } else {
    for (int j = 0; j < DGH; j++) EQ(S(c, d15h + j), fr_zero(), T, 118);
  }
  hs = o;
  o += ck_shahash(c, hs, P->ec_blocks, EHT);
  for (int j = 0; j < ECL; j++) EQ(S(c, hs + EHT + j), S(c, ec + j), T, 124);
  for (int j = 0; j < EHT; j++) EQ(S(c, ech + j), S(c, hs + j), T, 126);
  hs = o;
  o += ck_shahash(c, hs, 1024 / HBS, HT);
  for (int j = 0; j < 1024; j++) EQ(S(c, hs + HT + j), S(c, sa + j), T, 137);
  for (int j = 0; j < HT; j++) EQ(S(c, sah + j), S(c, hs + j), T, 130);
  size_t fl = o;
  o += ck_flow(c, fl, ECL, DGH, EHT, P->dg1_shift, P->aa ? P->dg15_shift : DGH, P->ec_shift, P->aa);
  for (int j = 0; j < DGH; j++) {
    EQ(S(c, fl + 1 + j), S(c, d1h + j), T, 140);
    EQ(S(c, fl + 1 + DGH + j), S(c, d15h + j), T, 141);
  }
  for (int j = 0; j < ECL; j++) EQ(S(c, fl + 1 + 2 * DGH + j), S(c, ec + j), T, 142);
  for (int j = 0; j < EHT; j++) EQ(S(c, fl + 1 + 2 * DGH + ECL + j), S(c, ech + j), T, 143);
  for (int j = 0; j < 1024; j++) EQ(S(c, fl + 1 + 2 * DGH + ECL + EHT + j), S(c, sa + j), T, 144);
  EQ(S(c, fl), KC(1), T, 146);
  size_t sv = o;  /* VerifySignature(SIG) signatureVerification.circom: pubkey[PK] signature[PK] hashed[HT] | verifier */
  const char *TV = "VerifySignature signatureVerifier/signatureVerification.circom";
  const int PK = ecdsa ? 2 * K : K;
  size_t rsa = sv + 2 * (size_t)PK + HT;
  const int pss = P->sig >= 10 && P->sig <= 14;
  if (ecdsa) {    /* verifyECDSABits: pubkey[2][K], signature[2][K], hashed */
    o += 2 * (size_t)PK + HT + ck_ecdsa(c, rsa);
    for (int i = 0; i < 2 * K; i++) {
      req(c, S(c, rsa + i), S(c, sv + i), TV, 184, sv);
      req(c, S(c, rsa + 2 * K + i), S(c, sv + PK + i), TV, 186, sv);
    }
  } else if (pss) {  /* VerifyRsaPssSig: pubkey, signature, hashed */
    o += 2 * (size_t)K + HT + ck_pss(c, rsa, K, P->sig == 12 ? 64 : P->sig == 13 ? 48 : 32, P->sig == 10 ? 3 : 65537, HT);
    for (int i = 0; i < K; i++) {
      req(c, S(c, rsa + i), S(c, sv + i), TV, 147, sv);
      req(c, S(c, rsa + K + i), S(c, sv + K + i), TV, 148, sv);
    }
  } else {    /* RsaVerifyPkcs1v15: signature, pubkey, hashed */
    o += 2 * (size_t)K + HT + (HT == 256 ? ck_rsa_pkcs256(c, rsa, K, 65537) : ck_rsa_pkcs160(c, rsa, K, P->sig == 4 ? 37187 : 65537));
    for (int i = 0; i < K; i++) {
      req(c, S(c, rsa + K + i), S(c, sv + i), TV, 124, sv);
      req(c, S(c, rsa + i), S(c, sv + K + i), TV, 125, sv);
    }
  }
  for (int i = 0; i < HT; i++) req(c, S(c, rsa + 2 * PK + i), S(c, sv + 2 * PK + i), TV, ecdsa ? 189 : pss ? 149 : 126, sv);
  for (int i = 0; i < PK; i++) {
    EQ(S(c, sv + PK + i), S(c, sig + i), T, 150);
    EQ(S(c, sv + i), S(c, pk + i), T, 151);
  }
  for (int i = 0; i < HT; i++) EQ(S(c, sv + 2 * PK + i), S(c, sah + i), T, 152);
  size_t san = o;
  o += ck_bits2num(c, san, 252);
  if (HT >= 252) {
    for (int i = 0; i < 252; i++) EQ(S(c, san + 1 + i), S(c, sah + i), T, 159);
  } else {
    for (int i = 0; i < 252 - HT; i++) EQ(S(c, san + 1 + i), fr_zero(), T, 163);
    for (int i = 0; i < HT; i++) EQ(S(c, san + 1 + 252 - HT + i), S(c, sah + i), T, 166);
  }
  if (!ecdsa) {
    size_t pkr = o;
    o += ck_poseidon(c, pkr, 5);
    for (int i = 0; i < 5; i++) {
      EQ(S(c, tmod + i), ADD(MUL(S(c, pk + 3 * i), P2[128]), MUL(S(c, pk + 3 * i + 1), P2[64])), T, 176);
      EQ(S(c, pkr + 1 + i), ADD(S(c, tmod + i), S(c, pk + 3 * i + 2)), T, 177);
    }
    EQ(S(c, pkh), S(c, pkr), T, 179);
  } else {  /* :184-218, EC_FIELD_SIZE EF = K x EB, DIFF = EF - 248 above 248 bits */
    const int DF = EF > 248 ? EF - 248 : 0, NB = EF - DF;
    for (int i = 0; i < K; i++) {
      size_t nx = o;
      o += ck_num2bits(c, nx, EB);
      size_t ny = o;
      o += ck_num2bits(c, ny, EB);
      EQ(S(c, nx + EB), S(c, pk + i), T, 195);
      EQ(S(c, ny + EB), S(c, pk + i + K), T, 196);
      for (int j = 0; j < EB; j++) {
        EQ(S(c, ebx + EF - 1 - j - EB * i), S(c, nx + j), T, 199);
        EQ(S(c, eby + EF - 1 - j - EB * i), S(c, ny + j), T, 200);
      }
    }
    size_t xn = o;
    o += ck_bits2num(c, xn, NB);
    size_t yn = o;
    o += ck_bits2num(c, yn, NB);
    for (int i = 0; i < NB; i++) {
      EQ(S(c, xn + 1 + NB - 1 - i), S(c, ebx + i + DF), T, 212);
      EQ(S(c, yn + 1 + NB - 1 - i), S(c, eby + i + DF), T, 213);
    }
    size_t h = o;
    o += ck_poseidon(c, h, 2);
    EQ(S(c, h + 1), S(c, xn), T, 218);
    EQ(S(c, h + 2), S(c, yn), T, 219);
    EQ(S(c, pkh), S(c, h), T, 221);
  }
  size_t smt = o;
  o += ck_smt(c, smt, 80);
  EQ(S(c, smt + 1), S(c, root), T, 226);
  EQ(S(c, smt + 2), S(c, pkh), T, 227);
  EQ(S(c, smt + 3), S(c, pkh), T, 228);
  for (int i = 0; i < 80; i++) EQ(S(c, smt + 4 + i), S(c, br + i), T, 229);
  size_t sh = o;
  o += ck_poseidon(c, sh, 1);
  EQ(S(c, sh + 1), S(c, san), T, 234);
  EQ(S(c, ph), S(c, sh), T, 235);
  return o - b;
}

/* RegisterIdentity(DG15_SIZE, HBS, SIG, DOC, AA, AA_SHIFT) identityManagement/identity.circom:6-121:
 * dg15PubKeyHash dg1Commitment pkIdentityHash | dg1[1024] dg15[..] skIdentity | AA key hashing components,
 * dg1Hasher dg1Chunking[4] skIndentityHasher pkIdentityCalc pkIdentityHasher */
static size_t ck_regid(ck_t *c, size_t b, const ck_params *P) {
  const char *T = "RegisterIdentity identityManagement/identity.circom";
  const int D15L = P->dg15_blocks * (P->dg_hash > 256 ? 1024 : 512);  /* DG15_SIZE x DG_HASH_BLOCK_SIZE */
  size_t d15ph = b, d1c = b + 1, pkih = b + 2, dg1 = b + 3, dg15 = dg1 + 1024, sk = dg15 + D15L, o = sk + 1;
  if (P->aa && P->aa < 20) {
    size_t ch[5];
    for (int j = 0; j < 5; j++) {
      int L = j < 4 ? 200 : 224;
      ch[j] = o;
      o += ck_bits2num(c, o, L);
      for (int i = 0; i < L; i++) EQ(S(c, ch[j] + 1 + L - 1 - i), S(c, dg15 + P->aa_shift + j * 200 + i), T, j < 4 ? 34 : 40);
    }
    size_t h = o;
    o += ck_poseidon(c, h, 5);
    for (int i = 0; i < 5; i++) EQ(S(c, h + 1 + i), S(c, ch[i]), T, 46);
    EQ(S(c, d15ph), S(c, h), T, 49);
  } else if (P->aa >= 20) {
    int HS = 248, EFS = 256;
    if (P->aa == 22) EFS = 320;
    if (P->aa == 23) { EFS = 192; HS = 192; }
    int XY = EFS - HS;
    size_t xn = o;
    o += ck_bits2num(c, xn, HS);
    size_t yn = o;
    o += ck_bits2num(c, yn, HS);
    for (int i = 0; i < HS; i++) {
      EQ(S(c, xn + 1 + HS - 1 - i), S(c, dg15 + P->aa_shift + i + XY), T, 73);
      EQ(S(c, yn + 1 + HS - 1 - i), S(c, dg15 + P->aa_shift + EFS + i + XY), T, 74);
    }
    size_t h = o;
    o += ck_poseidon(c, h, 2);
    EQ(S(c, h + 1), S(c, xn), T, 79);
    EQ(S(c, h + 2), S(c, yn), T, 80);
    EQ(S(c, d15ph), S(c, h), T, 82);
  } else {
    EQ(S(c, d15ph), fr_zero(), T, 86);
  }
  size_t dh = o;
  o += ck_poseidon(c, dh, 5);
  const int CS = P->doc == 1 ? 190 : 186;
  for (int i = 0; i < 4; i++) {
    size_t ch = o;
    o += ck_bits2num(c, ch, CS);
    for (int j = 0; j < CS; j++) EQ(S(c, ch + 1 + j), S(c, dg1 + i * CS + j), T, 99);
    EQ(S(c, dh + 1 + i), S(c, ch), T, 101);
  }
  size_t skh = o;
  o += ck_poseidon(c, skh, 1);
  EQ(S(c, skh + 1), S(c, sk), T, 105);
  EQ(S(c, dh + 5), S(c, skh), T, 106);
  EQ(S(c, d1c), S(c, dh), T, 108);
  size_t pc = o;
  o += ck_bjjmul(c, pc);
  EQ(S(c, pc + 2), S(c, sk), T, 113);
  size_t ph = o;
  o += ck_poseidon(c, ph, 2);
  EQ(S(c, ph + 1), S(c, pc), T, 116);
  EQ(S(c, ph + 2), S(c, pc + 1), T, 117);
  EQ(S(c, pkih), S(c, ph), T, 119);
  return o - b;
}

/* RegisterIdentityBuilder(...) identityManagement/registerIdentityBuilder.circom:41-196, main (public
 * slaveMerkleRoot): [1] dg15PubKeyHash passportHash dg1Commitment pkIdentityHash | slaveMerkleRoot
 * encapsulatedContent dg1 dg15 signedAttributes signature pubkey slaveMerkleInclusionBranches skIdentity |
 * passportVerifier registerIdentity */
static size_t ck_builder(ck_t *c, size_t b, const ck_params *P) {
  const char *T = "RegisterIdentityBuilder identityManagement/registerIdentityBuilder.circom";
  const int HBS = sig_hash(P->sig) > 256 ? 1024 : 512;
  const int K = sig_K(P->sig) * (P->sig >= 20 ? 2 : 1), ECL = P->ec_blocks * HBS, D15L = P->dg15_blocks * HBS;
  size_t d15ph = b, ph = b + 1, d1c = b + 2, pkih = b + 3, root = b + 4, ec = b + 5, dg1 = ec + ECL, dg15 = dg1 + 1024,
         sa = dg15 + D15L, sig = sa + 1024, pk = sig + K, br = pk + K, sk = br + 80, o = sk + 1;
  size_t pv = o;
  o += ck_pvb(c, pv, P);
  size_t pv_ec = pv + 1, pv_dg1 = pv_ec + ECL, pv_dg15 = pv_dg1 + 1024, pv_sa = pv_dg15 + D15L, pv_sig = pv_sa + 1024,
         pv_pk = pv_sig + K, pv_br = pv_pk + K, pv_root = pv_br + 80;
  for (int i = 0; i < ECL; i++) EQ(S(c, pv_ec + i), S(c, ec + i), T, 174);
  for (int i = 0; i < 1024; i++) EQ(S(c, pv_dg1 + i), S(c, dg1 + i), T, 175);
  for (int i = 0; i < D15L; i++) EQ(S(c, pv_dg15 + i), S(c, dg15 + i), T, 176);
  for (int i = 0; i < 1024; i++) EQ(S(c, pv_sa + i), S(c, sa + i), T, 177);
  for (int i = 0; i < K; i++) {
    EQ(S(c, pv_sig + i), S(c, sig + i), T, 178);
    EQ(S(c, pv_pk + i), S(c, pk + i), T, 179);
  }
  for (int i = 0; i < 80; i++) EQ(S(c, pv_br + i), S(c, br + i), T, 180);
  EQ(S(c, pv_root), S(c, root), T, 181);
  EQ(S(c, ph), S(c, pv), T, 182);
  size_t ri = o;
  o += ck_regid(c, ri, P);
  for (int i = 0; i < 1024; i++) EQ(S(c, ri + 3 + i), S(c, dg1 + i), T, 193);
  for (int i = 0; i < D15L; i++) EQ(S(c, ri + 3 + 1024 + i), S(c, dg15 + i), T, 194);
  EQ(S(c, ri + 3 + 1024 + D15L), S(c, sk), T, 195);
  EQ(S(c, d15ph), S(c, ri), T, 196);
  EQ(S(c, d1c), S(c, ri + 1), T, 197);
  EQ(S(c, pkih), S(c, ri + 2), T, 198);
  return o - b;
}

#include "r1cs_query.inc.c"

/* ============================================================ entry points */
static int ck_ready = 0;
static void ck_init(void) {
  if (ck_ready) return;
  for (int i = 0; i < 254; i++) P2[i] = fr_pow2(i);
  INV2_64 = fr_inv(P2[64]);
  ck_ready = 1;
}

typedef struct {
  uint64_t n_constraints, n_failed, n_uncovered, size_walked;
  int64_t first_failed;
  int32_t first_line, oob;
  char first_template[96];
  uint64_t first_component;
  int64_t first_uncovered;
  uint64_t n_uncovered_nonzero;  /* uncovered signals holding a non-zero value (an unassigned signal is 0) */
} ck_report;

static ck_t ck_begin(const uint8_t *wit, size_t n) {
  ck_init();
  ck_t c;
  memset(&c, 0, sizeof c);
  c.w = (const fr_t *)wit;
  c.n = n;
  c.cov = calloc(n, 1);
  c.first_bad = -1;
  return c;
}

static int ck_end(ck_t *c, size_t walked, ck_report *r) {
  memset(r, 0, sizeof *r);
  r->n_constraints = c->n_cons;
  r->n_failed = c->n_bad;
  r->first_failed = c->first_bad;
  r->first_line = c->first_line;
  r->first_component = c->first_at;
  r->oob = c->oob;
  r->size_walked = walked;
  if (c->first_tmpl) snprintf(r->first_template, sizeof r->first_template, "%s", c->first_tmpl);
  r->first_uncovered = -1;
  c->cov[0] = 1;  /* the constant 1 */
  for (size_t i = 0; i < c->n; i++)
    if (!c->cov[i]) {
      if (r->first_uncovered < 0) r->first_uncovered = (int64_t)i;
      r->n_uncovered++;
      if (!fr_is_zero(c->w[i])) r->n_uncovered_nonzero++;
    }
  free(c->cov);
  return (c->n_bad || c->oob || walked != c->n || r->n_uncovered_nonzero) ? 1 : 0;
}

int ck_sha256(int B, const uint8_t *wit, size_t n, ck_report *r) {
  ck_t c = ck_begin(wit, n);
  size_t walked = 1 + ck_sha2chunks(&c, 1, B, 256);
  return ck_end(&c, walked, r);
}

int ck_poseidon_circuit(int n, const uint8_t *wit, size_t nw, ck_report *r) {
  if (!pos_loaded) return -1;
  ck_t c = ck_begin(wit, nw);
  size_t walked = 1 + ck_poseidon(&c, 1, n);
  return ck_end(&c, walked, r);
}

/* RegisterIdentityBuilder as main: RSA PKCS#1 v1.5 (SIG 1-4), RSA-PSS (SIG 10-14), ECDSA P-256 / brainpoolP256r1 /
 * P-224 / brainpoolP384r1 (SIG 20 / 21 / 24 / 25), DG hash 160 / 224 / 256 / 384 */
int ck_register(const ck_params *P, const uint8_t *wit, size_t nw, ck_report *r) {
  if (!pos_loaded) return -1;
  if (!((P->sig >= 1 && P->sig <= 4) || (P->sig >= 10 && P->sig <= 14) || ec_curve_of(P->sig) >= 0) ||
      !(P->dg_hash == 256 || P->dg_hash == 224 || P->dg_hash == 160 || P->dg_hash == 384))
    return -2;
  if (P->sig >= 20) {
    CV = &EC[ec_curve_of(P->sig)];
    EK = CV->nl; EB = CV->cs;
    if (!CV->gpow) return -3;
  }
  ck_t c = ck_begin(wit, nw);
  size_t walked = 1 + ck_builder(&c, 1, P);
  req(&c, S(&c, 0), KC(1), "witness[0] = 1", 0, 0);
  return ck_end(&c, walked, r);
}

int ck_sha512(int B, int O, const uint8_t *wit, size_t n, ck_report *r) {
  ck_t c = ck_begin(wit, n);
  size_t walked = 1 + ck_sha5chunks(&c, 1, B, O);
  return ck_end(&c, walked, r);
}

int ck_sha1(int B, const uint8_t *wit, size_t n, ck_report *r) {
  ck_t c = ck_begin(wit, n);
  size_t walked = 1 + ck_sha1chunks(&c, 1, B);
  return ck_end(&c, walked, r);
}

/* QueryIdentity(80) as main (oracle/r1cs_query.inc.c); td1: QueryIdentityTD1 */
int ck_query(int td1, const uint8_t *wit, size_t nw, ck_report *r) {
  if (!pos_loaded) return -1;
  CKQ_TD1 = td1 != 0;
  ck_t c = ck_begin(wit, nw);
  size_t walked = 1 + ck_queryid(&c, 1);
  req(&c, S(&c, 0), KC(1), "witness[0] = 1", 0, 0);
  return ck_end(&c, walked, r);
}

#include "r1cs_shape.inc.c"
