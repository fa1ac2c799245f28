/* oracle/witness_oracle.c — CPU restatement of the reference's witness semantics.
 *
 * TEST INFRASTRUCTURE ONLY. This is the parity checker and the CPU baseline
 * ("kind": "port") for the MI355X witness generator: tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it; the shipped library never does.
 *
 * What it restates: circom 2.1.6 witness evaluation of the RegisterIdentityBuilder
 * circuit family (SURVEY.md §8a rows a1–a22) statement by statement, emitting EVERY
 * signal of every component instance (the unsimplified, "--O0" signal set) in the
 * layout documented in DESIGN.md §3:
 *   witness[0] = 1; then the main component; each component instance occupies one
 *   contiguous block = its own signals (outputs, inputs, intermediates — each group
 *   in declaration order, arrays row-major) followed by the blocks of its
 *   subcomponents in creation order (pre-order DFS). Main's inputs are ordered
 *   public-first. Declared-but-never-assigned signals hold 0.
 * circom's own numbering / O1-O2 elimination cannot be run here:
 * .wtns parity vs circom's WASM is UNPINNED; values per signal follow the templates.
 *
 * `<--` integer semantics: `%`, `\`, `>>`, `&` act on the canonical representative
 * in [0,p); `/` on signals is field division; `1/in` of IsZero uses inv(0)=0.
 * Every `===` / `assert` on the hot path is checked; the first failure sets a
 * check-site id (enum pzk_site below, mirrored in include/pzkwit.h).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "fr.h"

/* ------------------------------------------------------------------ context */
typedef struct {
  fr_t *w;
  int err;  /* first failing check site (0 = none) */
} ctx_t;

#define W(i) (c->w[(i)])

/* check sites (reference file:line of the `===`) — keep in sync with include/pzkwit.h */
enum {
  S_OK = 0,
  S_NUM2BITS = 1,        /* bitify.circom:26  in === sum */
  S_ALIAS = 2,           /* aliascheck.circom:14 */
  S_ISZERO = 3,          /* comparators.circom:20 */
  S_LASTBIT = 4,         /* arithmetic.circom:169-170 */
  S_LASTNBITS = 5,       /* arithmetic.circom:203 */
  S_BITS2 = 6,           /* sha2Common.circom:65-68 */
  S_FLOW = 7,            /* passportVerificationBuilder.circom:155 */
  S_RSA_HASH = 8,        /* rsa.circom:48 */
  S_RSA_PREFIX = 9,      /* rsa.circom:53-54 */
  S_RSA_PAD = 10,        /* rsa.circom:57-71 */
  S_BIGMOD_GT = 11,      /* bigInt.circom:245 */
  S_BIGISZERO = 12,      /* bigIntComparators.circom:128 */
  S_SMT_LAST = 13,       /* SMTVerifier.circom:54 */
  S_BJJ_ADD = 14,        /* babyjubjub/curve.circom:98,102 */
  S_ECDSA_INV = 15,      /* bigInt.circom:364-368  in * inv mod n === 1 */
  S_ECDSA_R = 16,        /* ecdsa.circom:81-83  x1 mod n === r */
  S_PSS_TRAILER = 17,    /* rsaPss.circom:73  assert(eM[0] == 188) */
  S_PSS_HASH = 18,       /* rsaPss.circom:182,201  hDash256.out === hash */
  S_QUERY = 19,          /* comparators.circom:42  (1 - isEqual.out) * enabled === 0 (QueryIdentity bounds) */
  S_DATE = 20,           /* dateDecoder.circom:22  dateEncoder.encoded === dateEncoded */
  S_CIT_BLACKLIST = 21,  /* citizenshipCheck.circom:271  isEqual[i].out * isEqual2[i].out === 0 */
  S_CIT_LIST = 22,       /* citizenshipCheck.circom:274  validCheck[COUNTRY_COUNT] === 1 */
  S_ISV_ROOT = 23,       /* identityStateVerifier.circom:46  smtVerifier.isVerified === 1 */
};

/* ------------------------------------------------------------- fr helpers */
static fr_t POW2[256];
static void init_pow2(void) { for (int i = 0; i < 254; i++) POW2[i] = fr_pow2(i); }

/* x * bit-or-general y */
static inline fr_t mulg(fr_t a, fr_t b) {
  if (fr_is_zero(a) || fr_is_zero(b)) return fr_zero();
  if (b.l[0] == 1 && !(b.l[1] | b.l[2] | b.l[3])) return a;
  if (a.l[0] == 1 && !(a.l[1] | a.l[2] | a.l[3])) return b;
  return fr_mul(a, b);
}
static inline fr_t ONE(void) { return fr_u64(1); }
static inline uint64_t small(fr_t a) { return a.l[0]; }

/* ================================================================ bitify */
static size_t sz_aliascheck(void);
static void run_aliascheck(ctx_t *c, size_t b);

/* Num2Bits(L) bitify.circom:10-32: out[L] | in | sum[L] | [AliasCheck] */
static size_t sz_num2bits(int L) { return 2 * (size_t)L + 1 + (L == 254 ? sz_aliascheck() : 0); }
static void run_num2bits(ctx_t *c, size_t b, int L) {
  fr_t in = W(b + L);
  for (int i = 0; i < L; i++) W(b + i) = fr_u64((uint64_t)fr_bit(in, i));
  fr_t s = W(b);  /* out[0]*out[0] == out[0] for a bit */
  W(b + L + 1) = s;
  for (int i = 1; i < L; i++) {
    if (fr_bit(in, i)) s = fr_add(s, POW2[i]);
    W(b + L + 1 + i) = s;
  }
  if (!fr_eq(in, s) && !c->err) c->err = S_NUM2BITS;
  if (L == 254) {
    size_t a = b + 2 * L + 1;
    for (int i = 0; i < 254; i++) W(a + i) = W(b + i);
    run_aliascheck(c, a);
  }
}

/* Bits2Num(L) bitify.circom:38-55: out | in[L] | sum[L] | [AliasCheck] */
static size_t sz_bits2num(int L) { return 2 * (size_t)L + 1 + (L == 254 ? sz_aliascheck() : 0); }
static void run_bits2num(ctx_t *c, size_t b, int L) {
  fr_t s = mulg(W(b + 1), W(b + 1));
  W(b + L + 1) = s;
  for (int i = 1; i < L; i++) {
    s = fr_add(mulg(POW2[i], W(b + 1 + i)), s);
    W(b + L + 1 + i) = s;
  }
  W(b) = s;
  if (L == 254) {
    size_t a = b + 2 * L + 1;
    for (int i = 0; i < 254; i++) W(a + i) = W(b + 1 + i);
    run_aliascheck(c, a);
  }
}

/* CompConstant(ct) compconstant.circom:7-55: out | in[254] | parts[127] | sout | Num2Bits(135) */
static size_t sz_compconst(void) { return 1 + 254 + 127 + 1 + sz_num2bits(135); }
static void run_compconst(ctx_t *c, size_t b, fr_t ct) {
  fr_t bb = fr_sub(fr_pow2(128), ONE()), a = ONE(), e = ONE(), sum = fr_zero();
  for (int i = 0; i < 127; i++) {
    int clsb = fr_bit(ct, 2 * i), cmsb = fr_bit(ct, 2 * i + 1);
    fr_t slsb = W(b + 1 + 2 * i), smsb = W(b + 1 + 2 * i + 1);
    fr_t sl = mulg(smsb, slsb), part;
    if (!cmsb && !clsb) part = fr_add(fr_add(fr_neg(mulg(bb, sl)), mulg(bb, smsb)), mulg(bb, slsb));
    else if (!cmsb && clsb)
      part = fr_add(fr_sub(fr_add(fr_sub(mulg(a, sl), mulg(a, slsb)), mulg(bb, smsb)), mulg(a, smsb)), a);
    else if (cmsb && !clsb) part = fr_add(fr_sub(mulg(bb, sl), mulg(a, smsb)), a);
    else part = fr_add(fr_neg(mulg(a, sl)), a);
    W(b + 255 + i) = part;
    sum = fr_add(sum, part);
    bb = fr_sub(bb, e); a = fr_add(a, e); e = fr_add(e, e);
  }
  W(b + 382) = sum;
  size_t n = b + 383;
  W(n + 135) = sum;
  run_num2bits(c, n, 135);
  W(b) = W(n + 127);
}

/* AliasCheck aliascheck.circom:7-14: in[254] | CompConstant(-1) */
static size_t sz_aliascheck(void) { return 254 + sz_compconst(); }
static void run_aliascheck(ctx_t *c, size_t b) {
  size_t cc = b + 254;
  for (int i = 0; i < 254; i++) W(cc + 1 + i) = W(b + i);
  fr_t pm1 = FR_P; pm1.l[0] -= 1;
  run_compconst(c, cc, pm1);
  if (!fr_is_zero(W(cc)) && !c->err) c->err = S_ALIAS;
}

/* IsZero comparators.circom:11-21: out | in | inv */
static void run_iszero(ctx_t *c, size_t b) {
  fr_t in = W(b + 1);
  fr_t inv = fr_inv(in);
  W(b + 2) = inv;
  W(b) = fr_add(fr_neg(mulg(in, inv)), ONE());
  if (!fr_is_zero(mulg(in, W(b))) && !c->err) c->err = S_ISZERO;
}
/* IsEqual comparators.circom:24-33: out | in[2] | IsZero */
static void run_isequal(ctx_t *c, size_t b) {
  W(b + 4) = fr_sub(W(b + 2), W(b + 1));
  run_iszero(c, b + 3);
  W(b) = W(b + 3);
}
/* LessThan(L) comparators.circom:46-57: out | in[2] | Num2Bits(L+1) */
static size_t sz_lessthan(int L) { return 3 + sz_num2bits(L + 1); }
static void run_lessthan(ctx_t *c, size_t b, int L) {
  size_t n = b + 3;
  W(n + L + 1) = fr_sub(fr_add(W(b + 1), POW2[L]), W(b + 2));
  run_num2bits(c, n, L + 1);
  W(b) = fr_sub(ONE(), W(n + L));
}

/* Switcher switcher.circom:16-26: out[2] | bool, in[2] | aux */
static void run_switcher(ctx_t *c, size_t b) {
  fr_t aux = mulg(fr_sub(W(b + 4), W(b + 3)), W(b + 2));
  W(b + 5) = aux;
  W(b) = fr_add(aux, W(b + 3));
  W(b + 1) = fr_add(fr_neg(aux), W(b + 4));
}

/* ============================================================== arithmetic */
/* GetSumOfNElements(N) arithmetic.circom:210-226: out | in[N] | sum[N-1] */
static void run_getsum(ctx_t *c, size_t b, int n) {
  fr_t s = fr_add(W(b + 1), W(b + 2));
  W(b + n + 1) = s;
  for (int i = 1; i < n - 1; i++) {
    s = fr_add(s, W(b + 2 + i));
    W(b + n + 1 + i) = s;
  }
  W(b) = s;
}
/* GetLastBitUnsecure arithmetic.circom:161-171: bit, div | in */
static void run_lastbit(ctx_t *c, size_t b) {
  fr_t in = W(b + 2);
  fr_t bit = fr_u64(in.l[0] & 1), div = fr_shr(in, 1);
  W(b) = bit; W(b + 1) = div;
  if (!fr_eq(fr_add(fr_add(div, div), mulg(bit, bit)), in) && !c->err) c->err = S_LASTBIT;
}
/* GetLastNBits(N) arithmetic.circom:178-204: div, out[N] | in | check[N] | GetLastBitUnsecure[N] */
static size_t sz_lastnbits(int N) { return 5 * (size_t)N + 2; }
static void run_lastnbits(ctx_t *c, size_t b, int N) {
  fr_t cur = W(b + N + 1);
  size_t s0 = b + 2 * (size_t)N + 2;
  for (int i = 0; i < N; i++) {
    size_t s = s0 + 3 * (size_t)i;
    W(s + 2) = cur;
    run_lastbit(c, s);
    W(b + 1 + i) = W(s);
    cur = W(s + 1);
  }
  W(b) = cur;
  fr_t chk = mulg(W(b + 1), W(b + 1));
  W(b + N + 2) = chk;
  for (int i = 1; i < N; i++) {
    chk = fr_add(chk, mulg(W(b + 1 + i), POW2[i]));
    W(b + N + 2 + i) = chk;
  }
  if (!fr_eq(fr_add(chk, mulg(cur, POW2[N])), W(b + N + 1)) && !c->err) c->err = S_LASTNBITS;
}

/* ================================================================= SHA-256 */
/* XOR3_v2 sha2Common.circom:80-88: out | x, y, z | tmp */
static void run_xor3(ctx_t *c, size_t b) {
  int64_t x = (int64_t)small(W(b + 1)), y = (int64_t)small(W(b + 2)), z = (int64_t)small(W(b + 3));
  int64_t tmp = y * z;
  W(b + 4) = fr_i64(tmp);
  W(b) = fr_i64(x * (1 - 2 * y - 2 * z + 4 * tmp) + y + z - 2 * tmp);
}
/* Bits2 sha2Common.circom:57-68: lo, hi | xy */
static void run_bits2(ctx_t *c, size_t b) {
  fr_t xy = W(b + 2);
  W(b) = fr_u64(xy.l[0] & 1);
  W(b + 1) = fr_shr(xy, 1); W(b + 1).l[0] &= 1; W(b + 1).l[1] = W(b + 1).l[2] = W(b + 1).l[3] = 0;
  if (!fr_eq(fr_add(fr_add(W(b + 1), W(b + 1)), W(b)), xy) && !c->err) c->err = S_BITS2;
}

static const uint32_t SHA_IV[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                   0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
static const uint32_t SHA_K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

/* Sha2_224_256Shedule sha256Schedule.circom:11-72
 * outWords[64] | chunkBits[16][32] | outBits[64][32] | sumN[16], {s0Sum,s1Sum,(s0Xor,s1Xor)x32,modulo,bits2Num}x48 */
#define SCH_OWN (64 + 512 + 2048)
#define SCH_PER_M (64 + 64 + 32 * 10 + 162 + 65)
static size_t sz_schedule(void) { return SCH_OWN + 16 * 64 + 48 * SCH_PER_M; }
static void run_schedule(ctx_t *c, size_t b) {
  size_t outWords = b, chunk = b + 64, outBits = b + 576;
  size_t sub = b + SCH_OWN;
  for (int k = 0; k < 16; k++) {
    size_t s = sub + 64 * (size_t)k;
    for (int i = 0; i < 32; i++) W(s + 1 + i) = mulg(POW2[i], W(chunk + 32 * k + i));
    run_getsum(c, s, 32);
    W(outWords + k) = W(s);
    for (int i = 0; i < 32; i++) W(outBits + 32 * k + i) = W(chunk + 32 * k + i);
  }
  sub += 16 * 64;
  for (int m = 16; m < 64; m++) {
    int r = m - 16, k = m - 15, l = m - 2;
    size_t s0Sum = sub + (size_t)r * SCH_PER_M, s1Sum = s0Sum + 64, xo = s1Sum + 64;
    size_t modulo = xo + 320, b2n = modulo + 162;
    for (int i = 0; i < 32; i++) {
      size_t x0 = xo + 10 * (size_t)i, x1 = x0 + 5;
      W(x0 + 1) = W(outBits + 32 * k + (i + 7) % 32);
      W(x0 + 2) = W(outBits + 32 * k + (i + 18) % 32);
      W(x0 + 3) = (i < 29) ? W(outBits + 32 * k + i + 3) : fr_zero();
      run_xor3(c, x0);
      W(s0Sum + 1 + i) = mulg(POW2[i], W(x0));
      W(x1 + 1) = W(outBits + 32 * l + (i + 17) % 32);
      W(x1 + 2) = W(outBits + 32 * l + (i + 19) % 32);
      W(x1 + 3) = (i < 22) ? W(outBits + 32 * l + i + 10) : fr_zero();
      run_xor3(c, x1);
      W(s1Sum + 1 + i) = mulg(POW2[i], W(x1));
    }
    run_getsum(c, s0Sum, 32);
    run_getsum(c, s1Sum, 32);
    W(modulo + 33) = fr_add(fr_add(fr_add(W(s1Sum), W(outWords + m - 7)), W(s0Sum)), W(outWords + m - 16));
    run_lastnbits(c, modulo, 32);
    for (int i = 0; i < 32; i++) W(outBits + 32 * m + i) = W(modulo + 1 + i);
    for (int i = 0; i < 32; i++) W(b2n + 1 + i) = W(outBits + 32 * m + i);
    run_bits2num(c, b2n, 32);
    W(outWords + m) = W(b2n);
  }
}

/* Sha2_224_256CompressInner sha256Compress.circom:11-96
 * outA..outHH (194) | inp,key,a,b,c,dd,e,f,g,hh (196) | chb[32],overflowE,overflowA |
 * dSum,hSum,s0Sum,s1Sum,mjSum,chSum, (major,s0Xor,s1Xor)x32, decomposeE, decomposeA */
#define CI_OWN 424
static size_t sz_compress(void) { return CI_OWN + 6 * 64 + 32 * 13 + 2 * 162; }
static void run_compress(ctx_t *c, size_t b) {
  size_t oA = b, oB = b + 32, oC = b + 64, oDD = b + 96, oE = b + 97, oF = b + 129, oG = b + 161, oHH = b + 193;
  size_t inp = b + 194, key = b + 195, A = b + 196, B = b + 228, C = b + 260, DD = b + 292, E = b + 293,
         F = b + 325, G = b + 357, HH = b + 389, chb = b + 390, ovE = b + 422, ovA = b + 423;
  size_t dSum = b + CI_OWN, hSum = dSum + 64, s0Sum = hSum + 64, s1Sum = s0Sum + 64, mjSum = s1Sum + 64,
         chSum = mjSum + 64, loop = chSum + 64, decE = loop + 32 * 13, decA = decE + 162;
  for (int i = 0; i < 32; i++) {
    W(oG + i) = W(F + i); W(oF + i) = W(E + i); W(oC + i) = W(B + i); W(oB + i) = W(A + i);
  }
  for (int i = 0; i < 32; i++) {
    W(dSum + 1 + i) = mulg(POW2[i], W(C + i));
    W(hSum + 1 + i) = mulg(POW2[i], W(G + i));
  }
  run_getsum(c, dSum, 32); run_getsum(c, hSum, 32);
  W(oDD) = W(dSum); W(oHH) = W(hSum);
  for (int i = 0; i < 32; i++) {
    int64_t e = (int64_t)small(W(E + i)), f = (int64_t)small(W(F + i)), g = (int64_t)small(W(G + i));
    W(chb + i) = fr_i64(e * (f - g) + g);
    W(chSum + 1 + i) = mulg(POW2[i], W(chb + i));
    size_t mj = loop + 13 * (size_t)i, x0 = mj + 3, x1 = x0 + 5;
    W(mj + 2) = fr_add(fr_add(W(A + i), W(B + i)), W(C + i));
    run_bits2(c, mj);
    W(mjSum + 1 + i) = mulg(POW2[i], W(mj + 1));
    W(x0 + 1) = W(A + (i + 2) % 32); W(x0 + 2) = W(A + (i + 13) % 32); W(x0 + 3) = W(A + (i + 22) % 32);
    run_xor3(c, x0);
    W(s0Sum + 1 + i) = mulg(POW2[i], W(x0));
    W(x1 + 1) = W(E + (i + 6) % 32); W(x1 + 2) = W(E + (i + 11) % 32); W(x1 + 3) = W(E + (i + 25) % 32);
    run_xor3(c, x1);
    W(s1Sum + 1 + i) = mulg(POW2[i], W(x1));
  }
  run_getsum(c, s0Sum, 32); run_getsum(c, s1Sum, 32); run_getsum(c, mjSum, 32); run_getsum(c, chSum, 32);
  fr_t t1 = fr_add(fr_add(fr_add(fr_add(W(HH), W(s1Sum)), W(chSum)), W(key)), W(inp));
  W(ovE) = fr_add(fr_add(W(DD), W(HH)), fr_add(fr_add(fr_add(W(s1Sum), W(chSum)), W(key)), W(inp)));
  W(ovA) = fr_add(fr_add(t1, W(s0Sum)), W(mjSum));
  W(decE + 33) = W(ovE); run_lastnbits(c, decE, 32);
  W(decA + 33) = W(ovA); run_lastnbits(c, decA, 32);
  for (int i = 0; i < 32; i++) { W(oE + i) = W(decE + 1 + i); W(oA + i) = W(decA + 1 + i); }
}

/* Sha2_224_256Rounds(64) sha256Rounds.circom:12-125
 * outHash[8][32] | words[64], inpHash[8][32] | a,b,c[65][32], dd[65], e,f,g[65][32], hh[65], ROUND_KEYS[64],
 * hashWords[8] | roundKeys, sumDd, sumHh, sum[8], compress[64], modulo[8], sumA,sumB,sumC,sumE,sumF,sumG */
#define RD_N 64
#define RD_OWN (256 + 64 + 256 + 6 * 65 * 32 + 2 * 65 + 64 + 8)
static size_t sz_rounds(void) { return RD_OWN + 64 + 2 * 64 + 8 * 64 + RD_N * sz_compress() + 8 * 162 + 6 * 64; }
static void run_rounds(ctx_t *c, size_t b) {
  const size_t n1 = RD_N + 1;
  size_t outHash = b, words = b + 256, inpHash = b + 320;
  size_t a = b + 576, bb = a + n1 * 32, cc = bb + n1 * 32, dd = cc + n1 * 32, e = dd + n1, f = e + n1 * 32,
         g = f + n1 * 32, hh = g + n1 * 32, RK = hh + n1, hashWords = RK + 64;
  size_t roundKeys = b + RD_OWN, sumDd = roundKeys + 64, sumHh = sumDd + 64, sum = sumHh + 64,
         comp = sum + 8 * 64, modulo = comp + RD_N * sz_compress(), sumA = modulo + 8 * 162;
  for (int j = 0; j < 64; j++) W(roundKeys + j) = fr_u64(SHA_K[j]);
  for (int j = 0; j < 64; j++) W(RK + j) = W(roundKeys + j);
  for (int i = 0; i < 32; i++) {
    W(a + i) = W(inpHash + 0 * 32 + i); W(bb + i) = W(inpHash + 1 * 32 + i); W(cc + i) = W(inpHash + 2 * 32 + i);
    W(e + i) = W(inpHash + 4 * 32 + i); W(f + i) = W(inpHash + 5 * 32 + i); W(g + i) = W(inpHash + 6 * 32 + i);
  }
  for (int i = 0; i < 32; i++) {
    W(sumDd + 1 + i) = mulg(W(inpHash + 3 * 32 + i), POW2[i]);
    W(sumHh + 1 + i) = mulg(W(inpHash + 7 * 32 + i), POW2[i]);
  }
  run_getsum(c, sumDd, 32); run_getsum(c, sumHh, 32);
  W(dd) = W(sumDd); W(hh) = W(sumHh);
  for (int j = 0; j < 8; j++) {
    size_t s = sum + 64 * (size_t)j;
    for (int i = 0; i < 32; i++) W(s + 1 + i) = mulg(POW2[i], W(inpHash + 32 * j + i));
    run_getsum(c, s, 32);
    W(hashWords + j) = W(s);
  }
  for (int k = 0; k < RD_N; k++) {
    size_t cp = comp + (size_t)k * sz_compress();
    W(cp + 194) = W(words + k); W(cp + 195) = W(RK + k);
    for (int i = 0; i < 32; i++) {
      W(cp + 196 + i) = W(a + 32 * k + i); W(cp + 228 + i) = W(bb + 32 * k + i); W(cp + 260 + i) = W(cc + 32 * k + i);
      W(cp + 293 + i) = W(e + 32 * k + i); W(cp + 325 + i) = W(f + 32 * k + i); W(cp + 357 + i) = W(g + 32 * k + i);
    }
    W(cp + 292) = W(dd + k); W(cp + 389) = W(hh + k);
    run_compress(c, cp);
    for (int i = 0; i < 32; i++) {
      W(a + 32 * (k + 1) + i) = W(cp + i); W(bb + 32 * (k + 1) + i) = W(cp + 32 + i);
      W(cc + 32 * (k + 1) + i) = W(cp + 64 + i); W(e + 32 * (k + 1) + i) = W(cp + 97 + i);
      W(f + 32 * (k + 1) + i) = W(cp + 129 + i); W(g + 32 * (k + 1) + i) = W(cp + 161 + i);
    }
    W(dd + k + 1) = W(cp + 96); W(hh + k + 1) = W(cp + 193);
  }
  size_t srcs[6] = {a, bb, cc, e, f, g};
  for (int q = 0; q < 6; q++) {
    size_t s = sumA + 64 * (size_t)q;
    for (int i = 0; i < 32; i++) W(s + 1 + i) = mulg(POW2[i], W(srcs[q] + 32 * RD_N + i));
    run_getsum(c, s, 32);
  }
  fr_t add[8] = {W(sumA), W(sumA + 64), W(sumA + 128), W(dd + RD_N), W(sumA + 192), W(sumA + 256), W(sumA + 320),
                 W(hh + RD_N)};
  for (int j = 0; j < 8; j++) {
    size_t md = modulo + 162 * (size_t)j;
    W(md + 33) = fr_add(W(hashWords + j), add[j]);
    run_lastnbits(c, md, 32);
    for (int i = 0; i < 32; i++) W(outHash + 32 * j + i) = W(md + 1 + i);
  }
}

/* Sha256HashChunks(B) sha256HashChunks.circom:8-48 / Sha224HashChunks(B) sha224/sha224HashChunks.circom:8-51
 * (O = 256 / 224): out[O] | in[512B] | states[B+1][8][32] | iv, (sch[m], rds[m]) x B; the SHA-224 IV
 * sha224InitialValue.circom:10-20 */
static const uint32_t SHA224_IV[8] = {0xc1059ed8, 0x367cd507, 0x3070dd17, 0xf70e5939,
                                      0xffc00b31, 0x68581511, 0x64f98fa7, 0xbefa4fa4};
static size_t sz_sha2chunks(int O, int B) {
  return (size_t)O + 512 * (size_t)B + 256 * (size_t)(B + 1) + 256 + (size_t)B * (sz_schedule() + sz_rounds());
}
static size_t sz_sha256chunks(int B) { return sz_sha2chunks(256, B); }
static void run_sha2chunks(ctx_t *c, size_t b, int B, int O) {
  size_t out = b, in = b + O, states = in + 512 * (size_t)B, iv = states + 256 * (size_t)(B + 1);
  const uint32_t *IV = O == 224 ? SHA224_IV : SHA_IV;
  for (int k = 0; k < 8; k++)
    for (int i = 0; i < 32; i++) W(iv + 32 * k + i) = fr_u64((IV[k] >> i) & 1);
  for (int q = 0; q < 256; q++) W(states + q) = W(iv + q);
  size_t blk = iv + 256;
  for (int m = 0; m < B; m++) {
    size_t sch = blk + (size_t)m * (sz_schedule() + sz_rounds()), rds = sch + sz_schedule();
    for (int k = 0; k < 16; k++)
      for (int i = 0; i < 32; i++) W(sch + 64 + 32 * k + i) = W(in + 512 * (size_t)m + 32 * k + (31 - i));
    run_schedule(c, sch);
    for (int k = 0; k < 64; k++) W(rds + 256 + k) = W(sch + k);
    for (int q = 0; q < 256; q++) W(rds + 320 + q) = W(states + 256 * (size_t)m + q);
    run_rounds(c, rds);
    for (int q = 0; q < 256; q++) W(states + 256 * (size_t)(m + 1) + q) = W(rds + q);
  }
  for (int j = 0; j < O / 32; j++)
    for (int i = 0; i < 32; i++) W(out + 32 * j + i) = W(states + 256 * (size_t)B + 32 * j + 31 - i);
}
static void run_sha256chunks(ctx_t *c, size_t b, int B) { run_sha2chunks(c, b, B, 256); }

/* ShaHashChunks(B, 256) hash.circom:32-68: out[256] | in[512B] | hash256 */
static size_t sz_shahash(int B) { return 256 + 512 * (size_t)B + sz_sha256chunks(B); }
static void run_shahash(ctx_t *c, size_t b, int B) {
  size_t in = b + 256, h = in + 512 * (size_t)B;
  for (size_t q = 0; q < 512 * (size_t)B; q++) W(h + 256 + q) = W(in + q);
  run_sha256chunks(c, h, B);
  for (int q = 0; q < 256; q++) W(b + q) = W(h + q);
}

/* ============================================================ SHA-384 / SHA-512
 * Sha384HashChunks(B) / Sha512HashChunks(B) (sha2/sha384/sha384HashChunks.circom:8-49,
 * sha2/sha512/sha512HashChunks.circom:8-46) over Sha2_384_512Schedule (sha512Schedule.circom:11-75),
 * Sha2_384_512Rounds(80) (sha512Rounds.circom:11-126) and Sha2_384_512CompressInner
 * (sha512Compress.circom:11-96): the SHA-256 templates above with 64-bit words, 80 rounds, the
 * FIPS 180-4 SHA-512 rotations and constants (sha512RoundConst.circom, sha512InitialValue.circom,
 * sha384InitialValue.circom). Word sums exceed 64 bits (overflowA < 7 * 2^64): fr arithmetic. */
static const uint64_t SHA512_IV[8] = {0x6a09e667f3bcc908ull, 0xbb67ae8584caa73bull, 0x3c6ef372fe94f82bull,
                                      0xa54ff53a5f1d36f1ull, 0x510e527fade682d1ull, 0x9b05688c2b3e6c1full,
                                      0x1f83d9abfb41bd6bull, 0x5be0cd19137e2179ull};
static const uint64_t SHA384_IV[8] = {0xcbbb9d5dc1059ed8ull, 0x629a292a367cd507ull, 0x9159015a3070dd17ull,
                                      0x152fecd8f70e5939ull, 0x67332667ffc00b31ull, 0x8eb44a8768581511ull,
                                      0xdb0c2e0d64f98fa7ull, 0x47b5481dbefa4fa4ull};
static const uint64_t SHA512_K[80] = {
    0x428a2f98d728ae22ull, 0x7137449123ef65cdull, 0xb5c0fbcfec4d3b2full, 0xe9b5dba58189dbbcull, 0x3956c25bf348b538ull,
    0x59f111f1b605d019ull, 0x923f82a4af194f9bull, 0xab1c5ed5da6d8118ull, 0xd807aa98a3030242ull, 0x12835b0145706fbeull,
    0x243185be4ee4b28cull, 0x550c7dc3d5ffb4e2ull, 0x72be5d74f27b896full, 0x80deb1fe3b1696b1ull, 0x9bdc06a725c71235ull,
    0xc19bf174cf692694ull, 0xe49b69c19ef14ad2ull, 0xefbe4786384f25e3ull, 0x0fc19dc68b8cd5b5ull, 0x240ca1cc77ac9c65ull,
    0x2de92c6f592b0275ull, 0x4a7484aa6ea6e483ull, 0x5cb0a9dcbd41fbd4ull, 0x76f988da831153b5ull, 0x983e5152ee66dfabull,
    0xa831c66d2db43210ull, 0xb00327c898fb213full, 0xbf597fc7beef0ee4ull, 0xc6e00bf33da88fc2ull, 0xd5a79147930aa725ull,
    0x06ca6351e003826full, 0x142929670a0e6e70ull, 0x27b70a8546d22ffcull, 0x2e1b21385c26c926ull, 0x4d2c6dfc5ac42aedull,
    0x53380d139d95b3dfull, 0x650a73548baf63deull, 0x766a0abb3c77b2a8ull, 0x81c2c92e47edaee6ull, 0x92722c851482353bull,
    0xa2bfe8a14cf10364ull, 0xa81a664bbc423001ull, 0xc24b8b70d0f89791ull, 0xc76c51a30654be30ull, 0xd192e819d6ef5218ull,
    0xd69906245565a910ull, 0xf40e35855771202aull, 0x106aa07032bbd1b8ull, 0x19a4c116b8d2d0c8ull, 0x1e376c085141ab53ull,
    0x2748774cdf8eeb99ull, 0x34b0bcb5e19b48a8ull, 0x391c0cb3c5c95a63ull, 0x4ed8aa4ae3418acbull, 0x5b9cca4f7763e373ull,
    0x682e6ff3d6b2b8a3ull, 0x748f82ee5defb2fcull, 0x78a5636f43172f60ull, 0x84c87814a1f0ab72ull, 0x8cc702081a6439ecull,
    0x90befffa23631e28ull, 0xa4506cebde82bde9ull, 0xbef9a3f7b2c67915ull, 0xc67178f2e372532bull, 0xca273eceea26619cull,
    0xd186b8c721c0c207ull, 0xeada7dd6cde0eb1eull, 0xf57d4f7fee6ed178ull, 0x06f067aa72176fbaull, 0x0a637dc5a2c898a6ull,
    0x113f9804bef90daeull, 0x1b710b35131c471bull, 0x28db77f523047d84ull, 0x32caab7b40c72493ull, 0x3c9ebe0a15c9bebcull,
    0x431d67c49c100d4cull, 0x4cc5d4becb3e42b6ull, 0x597f299cfc657e2aull, 0x5fcb6fab3ad6faecull, 0x6c44198c4a475817ull};

/* GetSumOfNElements(64) fed with (1 << i) * bits[i]: out | in[64] | sum[63] (128 signals) */
static void run_wordsum64(ctx_t *c, size_t s, size_t bits) {
  for (int i = 0; i < 64; i++) W(s + 1 + i) = mulg(POW2[i], W(bits + i));
  run_getsum(c, s, 64);
}

/* Sha2_384_512Schedule sha512Schedule.circom:11-75
 * outWords[80] | chunkBits[16][64] | outBits[80][64] | sumN[16], {s0Sum,s1Sum,(s0Xor,s1Xor)x64,modulo,bits2Num}x64 */
#define SCH5_OWN (80 + 1024 + 5120)
#define SCH5_PER_M (128 + 128 + 64 * 10 + 322 + 129)
static size_t sz_schedule512(void) { return SCH5_OWN + 16 * 128 + 64 * SCH5_PER_M; }
static void run_schedule512(ctx_t *c, size_t b) {
  size_t outWords = b, chunk = b + 80, outBits = b + 1104;
  size_t sub = b + SCH5_OWN;
  for (int k = 0; k < 16; k++) {
    size_t s = sub + 128 * (size_t)k;
    run_wordsum64(c, s, chunk + 64 * k);
    W(outWords + k) = W(s);
    for (int i = 0; i < 64; i++) W(outBits + 64 * k + i) = W(chunk + 64 * k + i);
  }
  sub += 16 * 128;
  for (int m = 16; m < 80; m++) {
    int r = m - 16, k = m - 15, l = m - 2;
    size_t s0Sum = sub + (size_t)r * SCH5_PER_M, s1Sum = s0Sum + 128, xo = s1Sum + 128;
    size_t modulo = xo + 640, b2n = modulo + 322;
    for (int i = 0; i < 64; i++) {
      size_t x0 = xo + 10 * (size_t)i, x1 = x0 + 5;
      W(x0 + 1) = W(outBits + 64 * k + (i + 1) % 64);
      W(x0 + 2) = W(outBits + 64 * k + (i + 8) % 64);
      W(x0 + 3) = (i < 64 - 7) ? W(outBits + 64 * k + i + 7) : fr_zero();
      run_xor3(c, x0);
      W(s0Sum + 1 + i) = mulg(POW2[i], W(x0));
      W(x1 + 1) = W(outBits + 64 * l + (i + 19) % 64);
      W(x1 + 2) = W(outBits + 64 * l + (i + 61) % 64);
      W(x1 + 3) = (i < 64 - 6) ? W(outBits + 64 * l + i + 6) : fr_zero();
      run_xor3(c, x1);
      W(s1Sum + 1 + i) = mulg(POW2[i], W(x1));
    }
    run_getsum(c, s0Sum, 64);
    run_getsum(c, s1Sum, 64);
    W(modulo + 65) = fr_add(fr_add(fr_add(W(s1Sum), W(outWords + m - 7)), W(s0Sum)), W(outWords + m - 16));
    run_lastnbits(c, modulo, 64);
    for (int i = 0; i < 64; i++) W(outBits + 64 * m + i) = W(modulo + 1 + i);
    for (int i = 0; i < 64; i++) W(b2n + 1 + i) = W(outBits + 64 * m + i);
    run_bits2num(c, b2n, 64);
    W(outWords + m) = W(b2n);
  }
}

/* Sha2_384_512CompressInner sha512Compress.circom:11-96
 * outA,outB,outC[64],outDD,outE,outF,outG[64],outHH (386) | inp,key,a,b,c,dd,e,f,g,hh (388) |
 * chb[64],overflowE,overflowA | dSum,hSum,s0Sum,s1Sum,mjSum,chSum, (major,s0Xor,s1Xor)x64, decomposeE, decomposeA */
#define CI5_OWN 840
static size_t sz_compress512(void) { return CI5_OWN + 6 * 128 + 64 * 13 + 2 * 322; }
static void run_compress512(ctx_t *c, size_t b) {
  size_t oA = b, oB = b + 64, oC = b + 128, oDD = b + 192, oE = b + 193, oF = b + 257, oG = b + 321, oHH = b + 385;
  size_t inp = b + 386, key = b + 387, A = b + 388, B = b + 452, C = b + 516, DD = b + 580, E = b + 581,
         F = b + 645, G = b + 709, HH = b + 773, chb = b + 774, ovE = b + 838, ovA = b + 839;
  size_t dSum = b + CI5_OWN, hSum = dSum + 128, s0Sum = hSum + 128, s1Sum = s0Sum + 128, mjSum = s1Sum + 128,
         chSum = mjSum + 128, loop = chSum + 128, decE = loop + 64 * 13, decA = decE + 322;
  for (int i = 0; i < 64; i++) {
    W(oG + i) = W(F + i); W(oF + i) = W(E + i); W(oC + i) = W(B + i); W(oB + i) = W(A + i);
  }
  run_wordsum64(c, dSum, C); run_wordsum64(c, hSum, G);
  W(oDD) = W(dSum); W(oHH) = W(hSum);
  for (int i = 0; i < 64; i++) {
    int64_t e = (int64_t)small(W(E + i)), f = (int64_t)small(W(F + i)), g = (int64_t)small(W(G + i));
    W(chb + i) = fr_i64(e * (f - g) + g);
    W(chSum + 1 + i) = mulg(POW2[i], W(chb + i));
    size_t mj = loop + 13 * (size_t)i, x0 = mj + 3, x1 = x0 + 5;
    W(mj + 2) = fr_add(fr_add(W(A + i), W(B + i)), W(C + i));
    run_bits2(c, mj);
    W(mjSum + 1 + i) = mulg(POW2[i], W(mj + 1));
    W(x0 + 1) = W(A + (i + 28) % 64); W(x0 + 2) = W(A + (i + 34) % 64); W(x0 + 3) = W(A + (i + 39) % 64);
    run_xor3(c, x0);
    W(s0Sum + 1 + i) = mulg(POW2[i], W(x0));
    W(x1 + 1) = W(E + (i + 14) % 64); W(x1 + 2) = W(E + (i + 18) % 64); W(x1 + 3) = W(E + (i + 41) % 64);
    run_xor3(c, x1);
    W(s1Sum + 1 + i) = mulg(POW2[i], W(x1));
  }
  run_getsum(c, s0Sum, 64); run_getsum(c, s1Sum, 64); run_getsum(c, mjSum, 64); run_getsum(c, chSum, 64);
  fr_t t1 = fr_add(fr_add(fr_add(fr_add(W(HH), W(s1Sum)), W(chSum)), W(key)), W(inp));
  W(ovE) = fr_add(fr_add(W(DD), W(HH)), fr_add(fr_add(fr_add(W(s1Sum), W(chSum)), W(key)), W(inp)));
  W(ovA) = fr_add(fr_add(t1, W(s0Sum)), W(mjSum));
  W(decE + 65) = W(ovE); run_lastnbits(c, decE, 64);
  W(decA + 65) = W(ovA); run_lastnbits(c, decA, 64);
  for (int i = 0; i < 64; i++) { W(oE + i) = W(decE + 1 + i); W(oA + i) = W(decA + 1 + i); }
}

/* Sha2_384_512Rounds(80) sha512Rounds.circom:11-126
 * outHash[8][64] | words[80], inpHash[8][64] | a,b,c[81][64], dd[81], e,f,g[81][64], hh[81], ROUND_KEYS[80],
 * hashWords[8] | roundKeys, sumDd, sumHh, sum[8], compress[80], modulo[8], sumA,sumB,sumC,sumE,sumF,sumG */
#define RD5_N 80
#define RD5_OWN (512 + 80 + 512 + 6 * 81 * 64 + 2 * 81 + 80 + 8)
static size_t sz_rounds512(void) { return RD5_OWN + 80 + 2 * 128 + 8 * 128 + RD5_N * sz_compress512() + 8 * 322 + 6 * 128; }
static void run_rounds512(ctx_t *c, size_t b) {
  const size_t n1 = RD5_N + 1;
  size_t outHash = b, words = b + 512, inpHash = b + 592;
  size_t a = b + 1104, bb = a + n1 * 64, cc = bb + n1 * 64, dd = cc + n1 * 64, e = dd + n1, f = e + n1 * 64,
         g = f + n1 * 64, hh = g + n1 * 64, RK = hh + n1, hashWords = RK + 80;
  size_t roundKeys = b + RD5_OWN, sumDd = roundKeys + 80, sumHh = sumDd + 128, sum = sumHh + 128,
         comp = sum + 8 * 128, modulo = comp + RD5_N * sz_compress512(), sumA = modulo + 8 * 322;
  for (int j = 0; j < 80; j++) W(roundKeys + j) = fr_u64(SHA512_K[j]);
  for (int j = 0; j < 80; j++) W(RK + j) = W(roundKeys + j);
  for (int i = 0; i < 64; i++) {
    W(a + i) = W(inpHash + 0 * 64 + i); W(bb + i) = W(inpHash + 1 * 64 + i); W(cc + i) = W(inpHash + 2 * 64 + i);
    W(e + i) = W(inpHash + 4 * 64 + i); W(f + i) = W(inpHash + 5 * 64 + i); W(g + i) = W(inpHash + 6 * 64 + i);
  }
  run_wordsum64(c, sumDd, inpHash + 3 * 64); run_wordsum64(c, sumHh, inpHash + 7 * 64);
  W(dd) = W(sumDd); W(hh) = W(sumHh);
  for (int j = 0; j < 8; j++) {
    size_t s = sum + 128 * (size_t)j;
    run_wordsum64(c, s, inpHash + 64 * j);
    W(hashWords + j) = W(s);
  }
  for (int k = 0; k < RD5_N; k++) {
    size_t cp = comp + (size_t)k * sz_compress512();
    W(cp + 386) = W(words + k); W(cp + 387) = W(RK + k);
    for (int i = 0; i < 64; i++) {
      W(cp + 388 + i) = W(a + 64 * k + i); W(cp + 452 + i) = W(bb + 64 * k + i); W(cp + 516 + i) = W(cc + 64 * k + i);
      W(cp + 581 + i) = W(e + 64 * k + i); W(cp + 645 + i) = W(f + 64 * k + i); W(cp + 709 + i) = W(g + 64 * k + i);
    }
    W(cp + 580) = W(dd + k); W(cp + 773) = W(hh + k);
    run_compress512(c, cp);
    for (int i = 0; i < 64; i++) {
      W(a + 64 * (k + 1) + i) = W(cp + i); W(bb + 64 * (k + 1) + i) = W(cp + 64 + i);
      W(cc + 64 * (k + 1) + i) = W(cp + 128 + i); W(e + 64 * (k + 1) + i) = W(cp + 193 + i);
      W(f + 64 * (k + 1) + i) = W(cp + 257 + i); W(g + 64 * (k + 1) + i) = W(cp + 321 + i);
    }
    W(dd + k + 1) = W(cp + 192); W(hh + k + 1) = W(cp + 385);
  }
  size_t srcs[6] = {a, bb, cc, e, f, g};
  for (int q = 0; q < 6; q++) run_wordsum64(c, sumA + 128 * (size_t)q, srcs[q] + 64 * RD5_N);
  fr_t add[8] = {W(sumA), W(sumA + 128), W(sumA + 256), W(dd + RD5_N), W(sumA + 384), W(sumA + 512), W(sumA + 640),
                 W(hh + RD5_N)};
  for (int j = 0; j < 8; j++) {
    size_t md = modulo + 322 * (size_t)j;
    W(md + 65) = fr_add(W(hashWords + j), add[j]);
    run_lastnbits(c, md, 64);
    for (int i = 0; i < 64; i++) W(outHash + 64 * j + i) = W(md + 1 + i);
  }
}

/* Sha384HashChunks(B) / Sha512HashChunks(B) (O = 384 / 512):
 * out[O] | in[1024B] | states[B+1][8][64] | iv (512), (sch[m], rds[m]) x B */
static size_t sz_sha5chunks(int O, int B) {
  return (size_t)O + 1024 * (size_t)B + 512 * (size_t)(B + 1) + 512 + (size_t)B * (sz_schedule512() + sz_rounds512());
}
static void run_sha5chunks(ctx_t *c, size_t b, int B, int O) {
  size_t out = b, in = b + O, states = in + 1024 * (size_t)B, iv = states + 512 * (size_t)(B + 1);
  const uint64_t *IV = O == 384 ? SHA384_IV : SHA512_IV;
  for (int k = 0; k < 8; k++)
    for (int i = 0; i < 64; i++) W(iv + 64 * k + i) = fr_u64((IV[k] >> i) & 1);
  for (int q = 0; q < 512; q++) W(states + q) = W(iv + q);
  size_t blk = iv + 512;
  for (int m = 0; m < B; m++) {
    size_t sch = blk + (size_t)m * (sz_schedule512() + sz_rounds512()), rds = sch + sz_schedule512();
    for (int k = 0; k < 16; k++)
      for (int i = 0; i < 64; i++) W(sch + 80 + 64 * k + i) = W(in + 1024 * (size_t)m + 64 * k + (63 - i));
    run_schedule512(c, sch);
    for (int k = 0; k < 80; k++) W(rds + 512 + k) = W(sch + k);
    for (int q = 0; q < 512; q++) W(rds + 592 + q) = W(states + 512 * (size_t)m + q);
    run_rounds512(c, rds);
    for (int q = 0; q < 512; q++) W(states + 512 * (size_t)(m + 1) + q) = W(rds + q);
  }
  for (int j = 0; j < O / 64; j++)
    for (int i = 0; i < 64; i++) W(out + 64 * j + i) = W(states + 512 * (size_t)B + 64 * j + 63 - i);
}

/* =================================================================== SHA-1
 * Sha1HashChunks(B) hasher/sha1/sha1.circom:7-57 and its templates (sha1compression.circom,
 * t.circom, f.circom, parity.circom, rotate.circom, xor4.circom, constants.circom; BinSum
 * bitify/operations.circom:9-29; XOR3_v3 sha2/sha2Common.circom:102-113). Bit arrays named
 * "MSB-first" hold bit 31 of the word at index 0. */
static const uint32_t SHA1_H[5] = {0x67452301, 0xefcdab89, 0x98badcfe, 0x10325476, 0xc3d2e1f0};
static const uint32_t SHA1_K[4] = {0x5a827999, 0x6ed9eba1, 0x8f1bbcdc, 0xca62c1d6};

/* RotL(32, L) rotate.circom: out[32] | in[32]; out[i] = in[(i + L) % 32] */
static void run_rotl(ctx_t *c, size_t b, int L) {
  for (int i = 0; i < 32; i++) W(b + i) = W(b + 32 + (i + L) % 32);
}
/* H(x) / K(t) constants.circom: out[32] (MSB first) | Num2Bits(32)(constant) */
static size_t sz_sha1const(void) { return 32 + sz_num2bits(32); }
static void run_sha1const(ctx_t *c, size_t b, uint32_t v) {
  size_t n = b + 32;
  W(n + 32) = fr_u64(v);
  run_num2bits(c, n, 32);
  for (int k = 0; k < 32; k++) W(b + k) = W(n + 31 - k);
}
/* Xor4(32) xor4.circom: out | a | b | c | d | mid | aTemp */
static void run_xor4(ctx_t *c, size_t b) {
  for (int k = 0; k < 32; k++) {
    uint64_t a = small(W(b + 32 + k)), bb = small(W(b + 64 + k)), cc = small(W(b + 96 + k)), d = small(W(b + 128 + k));
    uint64_t mid = bb * cc, at = a ^ bb ^ cc;
    W(b + 160 + k) = fr_u64(mid);
    W(b + 192 + k) = fr_u64(at);
    W(b + k) = fr_u64(at ^ d);
  }
}
/* BinSum(N, L) operations.circom:9-29: out[L+N-1] | in[N][L] | sumN, bits2Num[N], num2Bits(L+N-1) */
static size_t sz_binsum(int N, int L) { return (size_t)(L + N - 1) + (size_t)N * L + 2 * (size_t)N + (size_t)N * sz_bits2num(L) + sz_num2bits(L + N - 1); }
static void run_binsum(ctx_t *c, size_t b, int N, int L) {
  int O = L + N - 1;
  size_t in = b + O, gs = in + (size_t)N * L, b2n = gs + 2 * (size_t)N, n2b = b2n + (size_t)N * sz_bits2num(L);
  for (int i = 0; i < N; i++) {
    size_t bn = b2n + (size_t)i * sz_bits2num(L);
    for (int k = 0; k < L; k++) W(bn + 1 + k) = W(in + (size_t)i * L + k);
    run_bits2num(c, bn, L);
    W(gs + 1 + i) = W(bn);
  }
  run_getsum(c, gs, N);
  W(n2b + O) = W(gs);
  run_num2bits(c, n2b, O);
  for (int k = 0; k < O; k++) W(b + k) = W(n2b + k);
}
/* fT(t) f.circom:34-74: out | b | c | d | maj (MajT: out|a|b|c|mid), parity (ParityT: out|a|b|c |
 * XOR3_v3: out|a|b|c|mid), ch (ChT: out|a|b|c) */
static size_t sz_ft(void) { return 128 + 160 + (128 + 160) + 128; }
static void run_ft(ctx_t *c, size_t b, int t) {
  size_t maj = b + 128, par = maj + 160, x3 = par + 128, ch = x3 + 160;
  for (int k = 0; k < 32; k++) {
    uint64_t x = small(W(b + 32 + k)), y = small(W(b + 64 + k)), z = small(W(b + 96 + k));
    W(maj + 32 + k) = W(b + 32 + k); W(maj + 64 + k) = W(b + 64 + k); W(maj + 96 + k) = W(b + 96 + k);
    W(maj + 128 + k) = fr_u64(y * z);
    W(maj + k) = fr_u64((x & y) | (x & z) | (y & z));
    W(par + 32 + k) = W(b + 32 + k); W(par + 64 + k) = W(b + 64 + k); W(par + 96 + k) = W(b + 96 + k);
    W(x3 + 32 + k) = W(b + 32 + k); W(x3 + 64 + k) = W(b + 64 + k); W(x3 + 96 + k) = W(b + 96 + k);
    W(x3 + 128 + k) = fr_u64(y * z);
    W(x3 + k) = fr_u64(x ^ y ^ z);
    W(par + k) = W(x3 + k);
    W(ch + 32 + k) = W(b + 32 + k); W(ch + 64 + k) = W(b + 64 + k); W(ch + 96 + k) = W(b + 96 + k);
    W(ch + k) = fr_u64(x ? y : z);
    W(b + k) = t <= 19 ? W(ch + k) : (t <= 39 || t >= 60) ? W(par + k) : W(maj + k);
  }
}
/* T(t) t.circom:8-57: out | a | b | c | d | e | kT | w | rotatel5, f, sumBinary (BinSum(5,32)),
 * sum (Bits2Num(35)), getLastNBits(32) */
static size_t sz_sha1t(void) { return 256 + 64 + sz_ft() + sz_binsum(5, 32) + sz_bits2num(35) + sz_lastnbits(32); }
static void run_sha1t(ctx_t *c, size_t b, int t) {
  size_t a = b + 32, bb = a + 32, cc = bb + 32, dd = cc + 32, e = dd + 32, kt = e + 32, w = kt + 32;
  size_t r5 = b + 256, f = r5 + 64, bs = f + sz_ft(), sm = bs + sz_binsum(5, 32), ln = sm + sz_bits2num(35);
  for (int k = 0; k < 32; k++) {
    W(r5 + 32 + k) = W(a + k);
    W(f + 32 + k) = W(bb + k); W(f + 64 + k) = W(cc + k); W(f + 96 + k) = W(dd + k);
  }
  run_rotl(c, r5, 5);
  run_ft(c, f, t);
  size_t bin = bs + 36;
  for (int k = 0; k < 32; k++) {
    W(bin + k) = W(r5 + 31 - k);
    W(bin + 32 + k) = W(f + 31 - k);
    W(bin + 64 + k) = W(e + 31 - k);
    W(bin + 96 + k) = W(kt + 31 - k);
    W(bin + 128 + k) = W(w + 31 - k);
  }
  run_binsum(c, bs, 5, 32);
  for (int k = 0; k < 35; k++) W(sm + 1 + k) = W(bs + k);
  run_bits2num(c, sm, 35);
  W(ln + 33) = W(sm);
  run_lastnbits(c, ln, 32);
  for (int k = 0; k < 32; k++) W(b + k) = W(ln + 1 + 31 - k);
}
/* Sha1compression sha1compression.circom:7-132: out[160] | hin[160] | inp[512] | a, b, c, d, e [81][32] |
 * w[80][32] | rotl1[64], xor4[64], rotl30[80], kT[80], tTmp[80], fSum[5] (BinSum(2,32)) */
static size_t sz_sha1comp(void) {
  return 160 + 160 + 512 + 5 * 81 * 32 + 80 * 32 + 64 * 64 + 64 * 224 + 80 * 64 + 80 * sz_sha1const() + 80 * sz_sha1t() +
         5 * sz_binsum(2, 32);
}
static void run_sha1comp(ctx_t *c, size_t b) {
  size_t hin = b + 160, inp = hin + 160, A = inp + 512, Bv = A + 81 * 32, Cv = Bv + 81 * 32, Dv = Cv + 81 * 32,
         Ev = Dv + 81 * 32, Wv = Ev + 81 * 32, r1 = Wv + 80 * 32, x4 = r1 + 64 * 64, r30 = x4 + 64 * 224,
         kk = r30 + 80 * 64, tt = kk + 80 * sz_sha1const(), fs = tt + 80 * sz_sha1t();
  for (int t = 0; t < 16; t++)
    for (int k = 0; k < 32; k++) W(Wv + 32 * t + k) = W(inp + 32 * t + k);
  for (int t = 16; t < 80; t++) {
    size_t x = x4 + (size_t)(t - 16) * 224, r = r1 + (size_t)(t - 16) * 64;
    for (int k = 0; k < 32; k++) {
      W(x + 32 + k) = W(Wv + 32 * (t - 3) + k); W(x + 64 + k) = W(Wv + 32 * (t - 8) + k);
      W(x + 96 + k) = W(Wv + 32 * (t - 14) + k); W(x + 128 + k) = W(Wv + 32 * (t - 16) + k);
    }
    run_xor4(c, x);
    for (int k = 0; k < 32; k++) W(r + 32 + k) = W(x + k);
    run_rotl(c, r, 1);
    for (int k = 0; k < 32; k++) W(Wv + 32 * t + k) = W(r + k);
  }
  for (int k = 0; k < 32; k++) {
    W(A + k) = W(hin + k); W(Bv + k) = W(hin + 32 + k); W(Cv + k) = W(hin + 64 + k);
    W(Dv + k) = W(hin + 96 + k); W(Ev + k) = W(hin + 128 + k);
  }
  for (int t = 0; t < 80; t++) {
    size_t K = kk + (size_t)t * sz_sha1const(), T = tt + (size_t)t * sz_sha1t(), r = r30 + (size_t)t * 64;
    run_sha1const(c, K, SHA1_K[t / 20]);
    for (int k = 0; k < 32; k++) {
      W(T + 32 + k) = W(A + 32 * t + k); W(T + 64 + k) = W(Bv + 32 * t + k); W(T + 96 + k) = W(Cv + 32 * t + k);
      W(T + 128 + k) = W(Dv + 32 * t + k); W(T + 160 + k) = W(Ev + 32 * t + k); W(T + 192 + k) = W(K + k);
      W(T + 224 + k) = W(Wv + 32 * t + k);
      W(r + 32 + k) = W(Bv + 32 * t + k);
    }
    run_sha1t(c, T, t);
    run_rotl(c, r, 30);
    for (int k = 0; k < 32; k++) {
      W(Ev + 32 * (t + 1) + k) = W(Dv + 32 * t + k);
      W(Dv + 32 * (t + 1) + k) = W(Cv + 32 * t + k);
      W(Cv + 32 * (t + 1) + k) = W(r + k);
      W(Bv + 32 * (t + 1) + k) = W(A + 32 * t + k);
      W(A + 32 * (t + 1) + k) = W(T + k);
    }
  }
  const size_t regs[5] = {A, Bv, Cv, Dv, Ev};
  for (int i = 0; i < 5; i++) {
    size_t f = fs + (size_t)i * sz_binsum(2, 32), in = f + 33;
    for (int k = 0; k < 32; k++) {
      W(in + k) = W(hin + 32 * i + 31 - k);
      W(in + 32 + k) = W(regs[i] + 80 * 32 + 31 - k);
    }
    run_binsum(c, f, 2, 32);
    for (int k = 0; k < 32; k++) W(b + 32 * i + k) = W(f + k);
  }
}
/* Sha1HashChunks(B) sha1.circom:7-57: out[160] | in[512B] | ha0..he0 (H(0..4)), sha1Compression[B] */
static size_t sz_sha1chunks(int B) { return 160 + 512 * (size_t)B + 5 * sz_sha1const() + (size_t)B * sz_sha1comp(); }
static void run_sha1chunks(ctx_t *c, size_t b, int B) {
  size_t in = b + 160, hs = in + 512 * (size_t)B, cp = hs + 5 * sz_sha1const();
  for (int j = 0; j < 5; j++) run_sha1const(c, hs + (size_t)j * sz_sha1const(), SHA1_H[j]);
  for (int m = 0; m < B; m++) {
    size_t q = cp + (size_t)m * sz_sha1comp(), hin = q + 160, inp = hin + 160;
    for (int w = 0; w < 5; w++)
      for (int k = 0; k < 32; k++)
        W(hin + 32 * w + k) = m == 0 ? W(hs + (size_t)w * sz_sha1const() + k) : W(q - sz_sha1comp() + 32 * w + 31 - k);
    for (int k = 0; k < 512; k++) W(inp + k) = W(in + 512 * (size_t)m + k);
    run_sha1comp(c, q);
  }
  size_t last = cp + (size_t)(B - 1) * sz_sha1comp();
  for (int i = 0; i < 5; i++)
    for (int k = 0; k < 32; k++) W(b + (31 - k) + 32 * i) = W(last + k + 32 * i);
}

/* ShaHashChunks(B, ALGO) hash.circom:32-68: out[ALGO] | in[BS x B] | Sha1 / Sha224 / Sha256 / Sha384 / Sha512HashChunks(B),
 * BS = 512 bits for ALGO <= 256, 1024 above */
static size_t sz_hashc(int algo, int B) {
  if (algo > 256) return (size_t)algo + 1024 * (size_t)B + sz_sha5chunks(algo, B);
  return algo == 160 ? 160 + 512 * (size_t)B + sz_sha1chunks(B) : algo == 224 ? 224 + 512 * (size_t)B + sz_sha2chunks(224, B)
                                                                  : sz_shahash(B);
}
static void run_hashc(ctx_t *c, size_t b, int algo, int B) {
  if (algo > 256) {
    size_t in = b + algo, h = in + 1024 * (size_t)B;
    for (size_t q = 0; q < 1024 * (size_t)B; q++) W(h + algo + q) = W(in + q);
    run_sha5chunks(c, h, B, algo);
    for (int q = 0; q < algo; q++) W(b + q) = W(h + q);
    return;
  }
  if (algo == 224) {
    size_t in = b + 224, h = in + 512 * (size_t)B;
    for (size_t q = 0; q < 512 * (size_t)B; q++) W(h + 224 + q) = W(in + q);
    run_sha2chunks(c, h, B, 224);
    for (int q = 0; q < 224; q++) W(b + q) = W(h + q);
    return;
  }
  if (algo != 160) { run_shahash(c, b, B); return; }
  size_t in = b + 160, h = in + 512 * (size_t)B;
  for (size_t q = 0; q < 512 * (size_t)B; q++) W(h + 160 + q) = W(in + q);
  run_sha1chunks(c, h, B);
  for (int q = 0; q < 160; q++) W(b + q) = W(h + q);
}

/* ================================================================ Poseidon */
typedef struct { int t, nRP; fr_t *C, *M, *P, *S; } pos_params_t;
static pos_params_t POS[18];
static int pos_loaded = 0;

int orc_load_poseidon(const char *path) {
  FILE *fp = fopen(path, "rb");
  if (!fp) return -1;
  char magic[8]; uint32_t nt;
  if (fread(magic, 1, 8, fp) != 8 || memcmp(magic, "PZKPOS01", 8) || fread(&nt, 4, 1, fp) != 1) { fclose(fp); return -2; }
  for (uint32_t q = 0; q < nt; q++) {
    uint32_t h[4];
    if (fread(h, 4, 4, fp) != 4) { fclose(fp); return -3; }
    int t = (int)h[0];
    pos_params_t *pp = &POS[t];
    pp->t = t; pp->nRP = (int)h[1];
    pp->C = malloc(sizeof(fr_t) * h[2]); pp->M = malloc(sizeof(fr_t) * t * t);
    pp->P = malloc(sizeof(fr_t) * t * t); pp->S = malloc(sizeof(fr_t) * h[3]);
    if (fread(pp->C, 32, h[2], fp) != h[2] || fread(pp->M, 32, (size_t)t * t, fp) != (size_t)t * t ||
        fread(pp->P, 32, (size_t)t * t, fp) != (size_t)t * t || fread(pp->S, 32, h[3], fp) != h[3]) {
      fclose(fp); return -4;
    }
  }
  fclose(fp);
  pos_loaded = 1;
  return 0;
}

/* Sigma poseidon.circom:10-21: out | in | in2, in4 */
static void run_sigma(ctx_t *c, size_t b) {
  fr_t in = W(b + 1), in2 = fr_mul(in, in), in4 = fr_mul(in2, in2);
  W(b + 2) = in2; W(b + 3) = in4; W(b) = fr_mul(in4, in);
}
/* Ark poseidon.circom:23-30: out[t] | in[t] */
static void run_ark(ctx_t *c, size_t b, int t, const fr_t *C, int r) {
  for (int i = 0; i < t; i++) W(b + i) = fr_add(W(b + t + i), C[i + r]);
}
/* Mix poseidon.circom:32-46: out[t] | in[t] | sum[t] (GetSumOfNElements(t)) */
static void run_mix(ctx_t *c, size_t b, int t, const fr_t *M) {
  for (int i = 0; i < t; i++) {
    size_t s = b + 2 * t + (size_t)i * 2 * t;
    for (int j = 0; j < t; j++) W(s + 1 + j) = fr_mul(M[j * t + i], W(b + t + j));
    run_getsum(c, s, t);
    W(b + i) = W(s);
  }
}
/* MixLast poseidon.circom:48-58: out | in[t] | sum */
static void run_mixlast(ctx_t *c, size_t b, int t, const fr_t *M, int s_) {
  size_t s = b + 1 + t;
  for (int j = 0; j < t; j++) W(s + 1 + j) = fr_mul(M[j * t + s_], W(b + 1 + j));
  run_getsum(c, s, t);
  W(b) = W(s);
}
/* MixS poseidon.circom:60-78: out[t] | in[t] | sum */
static void run_mixs(ctx_t *c, size_t b, int t, const fr_t *S, int r) {
  size_t s = b + 2 * t;
  for (int i = 0; i < t; i++) W(s + 1 + i) = fr_mul(S[(t * 2 - 1) * r + i], W(b + t + i));
  run_getsum(c, s, t);
  W(b) = W(s);
  for (int i = 1; i < t; i++) W(b + i) = fr_add(W(b + t + i), fr_mul(W(b + t), S[(t * 2 - 1) * r + t + i - 1]));
}

/* PoseidonEx(nIn,1) poseidon.circom:80-209: out[1] | in[nIn], initialState | subcomponents in creation order */
static size_t sz_poseidonex(int nIn) {
  int t = nIn + 1, RP = POS[t].nRP;
  return (size_t)(1 + nIn + 1) + 8 * (2 * t) + 8 * t * 4 + 7 * (2 * t + 2 * t * t) + (size_t)RP * (4 + 4 * t) + (3 * t + 1);
}
static void run_poseidonex(ctx_t *c, size_t b, int nIn) {
  int t = nIn + 1;
  const pos_params_t *pp = &POS[t];
  int RP = pp->nRP;
  size_t p = b + 2 + nIn;
  size_t szArk = 2 * t, szMix = 2 * t + 2 * (size_t)t * t;
  /* ark[0] */
  size_t ark = p; p += szArk;
  for (int j = 0; j < t; j++) W(ark + t + j) = (j > 0) ? W(b + 1 + j - 1) : W(b + 1 + nIn);
  run_ark(c, ark, t, pp->C, 0);
  size_t prev = ark; /* block whose out[0..t-1] feeds the next sigma layer */
  for (int r = 0; r < 3; r++) {
    size_t sg = p; p += 4 * (size_t)t;
    for (int j = 0; j < t; j++) { W(sg + 4 * j + 1) = W(prev + j); run_sigma(c, sg + 4 * j); }
    size_t ak = p; p += szArk;
    for (int j = 0; j < t; j++) W(ak + t + j) = W(sg + 4 * j);
    run_ark(c, ak, t, pp->C, (r + 1) * t);
    size_t mx = p; p += szMix;
    for (int j = 0; j < t; j++) W(mx + t + j) = W(ak + j);
    run_mix(c, mx, t, pp->M);
    prev = mx;
  }
  size_t sg = p; p += 4 * (size_t)t;
  for (int j = 0; j < t; j++) { W(sg + 4 * j + 1) = W(prev + j); run_sigma(c, sg + 4 * j); }
  size_t ak = p; p += szArk;
  for (int j = 0; j < t; j++) W(ak + t + j) = W(sg + 4 * j);
  run_ark(c, ak, t, pp->C, 4 * t);
  size_t mxP = p; p += szMix;
  for (int j = 0; j < t; j++) W(mxP + t + j) = W(ak + j);
  run_mix(c, mxP, t, pp->P);
  size_t prevS = mxP; /* out[] of mix[3] or mixS[r-1] */
  for (int r = 0; r < RP; r++) {
    size_t sp = p; p += 4;
    W(sp + 1) = W(prevS);
    run_sigma(c, sp);
    size_t ms = p; p += 4 * (size_t)t;
    W(ms + t) = fr_add(W(sp), pp->C[5 * t + r]);
    for (int j = 1; j < t; j++) W(ms + t + j) = W(prevS + j);
    run_mixs(c, ms, t, pp->S, r);
    prevS = ms;
  }
  prev = prevS;
  for (int r = 0; r < 3; r++) {
    size_t sg2 = p; p += 4 * (size_t)t;
    for (int j = 0; j < t; j++) { W(sg2 + 4 * j + 1) = W(prev + j); run_sigma(c, sg2 + 4 * j); }
    size_t ak2 = p; p += szArk;
    for (int j = 0; j < t; j++) W(ak2 + t + j) = W(sg2 + 4 * j);
    run_ark(c, ak2, t, pp->C, 5 * t + RP + r * t);
    size_t mx = p; p += szMix;
    for (int j = 0; j < t; j++) W(mx + t + j) = W(ak2 + j);
    run_mix(c, mx, t, pp->M);
    prev = mx;
  }
  size_t sgL = p; p += 4 * (size_t)t;
  for (int j = 0; j < t; j++) { W(sgL + 4 * j + 1) = W(prev + j); run_sigma(c, sgL + 4 * j); }
  size_t ml = p; p += 3 * (size_t)t + 1;
  for (int j = 0; j < t; j++) W(ml + 1 + j) = W(sgL + 4 * j);
  run_mixlast(c, ml, t, pp->M, 0);
  W(b) = W(ml);
}

/* PoseidonHash(n) poseidon.circom:214-226: out | in[n] | pEx */
static size_t sz_poseidon(int n) { return 1 + (size_t)n + sz_poseidonex(n); }
static void run_poseidon(ctx_t *c, size_t b, int n) {
  size_t px = b + 1 + n;
  W(px + 1 + n) = fr_zero();
  for (int i = 0; i < n; i++) W(px + 1 + i) = W(b + 1 + i);
  run_poseidonex(c, px, n);
  W(b) = W(px);
}

/* ============================================================= BabyJubJub */
static const char *BASE8X = "5299619240641551281634865583518297030282874472190772894086521144482721001553";
static const char *BASE8Y = "16950150798460657717958625567821834550301663161624707787222815936182638968203";
static fr_t fr_from_dec(const char *s) {
  fr_t r = fr_zero(), ten = fr_u64(10);
  for (; *s; s++) r = fr_add(fr_mul(r, ten), fr_u64((uint64_t)(*s - '0')));
  return r;
}

/* BabyjubjubAdd curve.circom:71-105: out[2] | in1[2], in2[2] | beta, gamma, delta, tau */
static void run_bjjadd(ctx_t *c, size_t b) {
  fr_t x1 = W(b + 2), y1 = W(b + 3), x2 = W(b + 4), y2 = W(b + 5);
  fr_t A = fr_u64(168700), D = fr_u64(168696);
  fr_t beta = fr_mul(x1, y2), gamma = fr_mul(y1, x2);
  fr_t delta = fr_mul(fr_sub(y1, fr_mul(A, x1)), fr_add(x2, y2));
  fr_t tau = fr_mul(beta, gamma);
  W(b + 6) = beta; W(b + 7) = gamma; W(b + 8) = delta; W(b + 9) = tau;
  fr_t dt = fr_mul(D, tau);
  fr_t den0 = fr_add(ONE(), dt), den1 = fr_sub(ONE(), dt);
  fr_t num0 = fr_add(beta, gamma), num1 = fr_sub(fr_add(delta, fr_mul(A, beta)), gamma);
  W(b) = fr_div(num0, den0);
  W(b + 1) = fr_div(num1, den1);
  if ((!fr_eq(fr_mul(den0, W(b)), num0) || !fr_eq(fr_mul(den1, W(b + 1)), num1)) && !c->err) c->err = S_BJJ_ADD;
}
/* BabyjubjubDouble curve.circom:109-118: out[2] | in[2] | adder */
static void run_bjjdouble(ctx_t *c, size_t b) {
  size_t ad = b + 4;
  W(ad + 2) = W(b + 2); W(ad + 3) = W(b + 3); W(ad + 4) = W(b + 2); W(ad + 5) = W(b + 3);
  run_bjjadd(c, ad);
  W(b) = W(ad); W(b + 1) = W(ad + 1);
}
/* addZeroBabyjub curve.circom:19-58: out[2] | in1[2], in2[2] | isZeroIn1, isZeroIn2, adder, (swL, swR) x 2 */
static void run_addzero(ctx_t *c, size_t b) {
  size_t z1 = b + 6, z2 = b + 9, ad = b + 12, sw = b + 22;
  W(z1 + 1) = W(b + 2); run_iszero(c, z1);
  W(z2 + 1) = W(b + 4); run_iszero(c, z2);
  for (int q = 0; q < 4; q++) W(ad + 2 + q) = W(b + 2 + q);
  run_bjjadd(c, ad);
  for (int i = 0; i < 2; i++) {
    size_t L = sw + 12 * (size_t)i, R = L + 6;
    W(L + 2) = W(z2); W(L + 3) = W(ad + i); W(L + 4) = W(b + 2 + i);
    run_switcher(c, L);
    W(R + 2) = W(z1); W(R + 3) = W(L); W(R + 4) = W(b + 4 + i);
    run_switcher(c, R);
  }
  /* out[c] <== switcherRight[c].out[0] (curve.circom:56-57); blocks are L0, R0, L1, R1 */
  W(b) = W(sw + 6); W(b + 1) = W(sw + 18);
}
/* BabyjubjubBase8Multiplication curve.circom:143-171:
 * out[2] | scalar | getBase8, num2Bits(254), adders[0], (adders[i], doublers[i-1]) i=1..253 */
static size_t sz_bjjmul(void) { return 3 + 2 + sz_num2bits(254) + 254 * 46 + 253 * 14; }
static void run_bjjmul(ctx_t *c, size_t b) {
  size_t gb = b + 3, nb = gb + 2, p = nb + sz_num2bits(254);
  W(gb) = fr_from_dec(BASE8X); W(gb + 1) = fr_from_dec(BASE8Y);
  W(nb + 254) = W(b + 2);
  run_num2bits(c, nb, 254);
  size_t prev_add = 0;
  for (int i = 0; i < 254; i++) {
    size_t ad = p; p += 46;
    size_t db = 0;
    if (i > 0) { db = p; p += 14; }
    fr_t bit = W(nb + 253 - i);
    if (i == 0) { W(ad + 2) = fr_zero(); W(ad + 3) = fr_zero(); }
    else {
      W(db + 2) = W(prev_add); W(db + 3) = W(prev_add + 1);
      run_bjjdouble(c, db);
      W(ad + 2) = W(db); W(ad + 3) = W(db + 1);
    }
    W(ad + 4) = mulg(W(gb), bit); W(ad + 5) = mulg(W(gb + 1), bit);
    run_addzero(c, ad);
    prev_add = ad;
  }
  W(b) = W(prev_add); W(b + 1) = W(prev_add + 1);
}

/* ================================================================== BigInt */
static int log_ceil(int n) { int i = 0; while (n) { n >>= 1; i++; } return i; }
static int is_pow2(int n) { return n > 0 && (n & (n - 1)) == 0; }
static int get_a_coeff(int a);
static int karatsuba_optimal(int a, int b) { return a < 8 ? 0 : (get_a_coeff(a) > a * b ? 0 : 1); }

/* KaratsubaOverflow(N) bigIntHelpers.circom:11-53: out[2N] | in[2][N] | A1B1, A2B2, A1A2B1B2 */
static size_t sz_karatsuba(int N) { return N == 1 ? 4 : 4 * (size_t)N + 3 * sz_karatsuba(N / 2); }
static void run_karatsuba(ctx_t *c, size_t b, int N) {
  size_t in0 = b + 2 * N, in1 = in0 + N;
  if (N == 1) { W(b) = fr_mul(W(in0), W(in1)); W(b + 1) = fr_zero(); return; }
  int h = N / 2;
  size_t s = sz_karatsuba(h), k1 = b + 4 * N, k2 = k1 + s, k3 = k2 + s;
  for (int i = 0; i < h; i++) {
    W(k1 + 2 * h + i) = W(in0 + i); W(k1 + 3 * h + i) = W(in1 + i);
    W(k2 + 2 * h + i) = W(in0 + i + h); W(k2 + 3 * h + i) = W(in1 + i + h);
    W(k3 + 2 * h + i) = fr_add(W(in0 + i), W(in0 + i + h));
    W(k3 + 3 * h + i) = fr_add(W(in1 + i), W(in1 + i + h));
  }
  run_karatsuba(c, k1, h); run_karatsuba(c, k2, h); run_karatsuba(c, k3, h);
  for (int i = 0; i < 2 * N; i++) {
    int mid = (h <= i && i < 3 * h);
    fr_t base = (i < N) ? W(k1 + i) : W(k2 + i - N);
    if (mid) base = fr_sub(fr_sub(fr_add(base, W(k3 + i - h)), W(k1 + i - h)), W(k2 + i - h));
    W(b + i) = base;
  }
}

/* BigMultNonEqualOverflow(n,G,L) bigIntHelpers.circom:55-124:
 * out[G+L-1] | in1[G], in2[L] | tmpMults[G][L], tmpResult[G+L-1][L] */
static size_t sz_bmneq(int G, int L) { return (size_t)(G + L - 1) + G + L + (size_t)G * L + (size_t)(G + L - 1) * L; }
static void run_bmneq(ctx_t *c, size_t b, int G, int L) {
  size_t in1 = b + G + L - 1, in2 = in1 + G, tm = in2 + L, tr = tm + (size_t)G * L;
  for (int i = 0; i < G; i++)
    for (int j = 0; j < L; j++) W(tm + (size_t)i * L + j) = fr_mul(W(in1 + i), W(in2 + j));
#define TM(i, j) W(tm + (size_t)(i) * L + (j))
#define TR(i, j) W(tr + (size_t)(i) * L + (j))
  for (int i = 0; i < G + L - 1; i++) {
    if (i < L) {
      for (int j = 0; j < i + 1; j++) TR(i, j) = j == 0 ? TM(i - j, j) : fr_add(TM(i - j, j), TR(i, j - 1));
      W(b + i) = TR(i, i);
    } else if (i < G) {
      for (int j = 0; j < L; j++) TR(i, j) = j == 0 ? TM(i - j, j) : fr_add(TM(i - j, j), TR(i, j - 1));
      W(b + i) = TR(i, L - 1);
    } else {
      for (int j = 0; j < G + L - 1 - i; j++)
        TR(i, j) = j == 0 ? TM(G - 1 - j, i + j - G + 1) : fr_add(TM(G - 1 - j, i + j - G + 1), TR(i, j - 1));
      W(b + i) = TR(i, G + L - 2 - i);
    }
  }
#undef TM
#undef TR
}

/* BigMultOverflow(n,G,L) bigIntOverflow.circom:38-72: out[G+L-1] | in1[G], in2[L] | karatsuba | mult */
static int bmo_kara(int G, int L) { return is_pow2(G) && karatsuba_optimal(G, L); }
static size_t sz_bmo(int G, int L) {
  return (size_t)(G + L - 1) + G + L + (bmo_kara(G, L) ? sz_karatsuba(G) : sz_bmneq(G, L));
}
static void run_bmo(ctx_t *c, size_t b, int G, int L) {
  size_t in1 = b + G + L - 1, in2 = in1 + G, sub = in2 + L;
  if (bmo_kara(G, L)) {
    for (int i = 0; i < G; i++) W(sub + 2 * G + i) = W(in1 + i);
    for (int i = 0; i < G; i++) W(sub + 3 * G + i) = i < L ? W(in2 + i) : fr_zero();
    run_karatsuba(c, sub, G);
  } else {
    for (int i = 0; i < G; i++) W(sub + G + L - 1 + i) = W(in1 + i);
    for (int i = 0; i < L; i++) W(sub + G + L - 1 + G + i) = W(in2 + i);
    run_bmneq(c, sub, G, L);
  }
  for (int i = 0; i < G + L - 1; i++) W(b + i) = W(sub + i);
}

/* BigLessEqThan(n,K) bigIntComparators.circom:50-75: out | in[2][K] | result[K] | (lessThan[i], isEqual[i]) */
static size_t sz_blet(int n, int K) { return 1 + 2 * (size_t)K + K + (size_t)K * (sz_lessthan(n) + 6); }
static void run_blet(ctx_t *c, size_t b, int n, int K) {
  size_t in0 = b + 1, in1 = in0 + K, res = in1 + K, sub = res + K, per = sz_lessthan(n) + 6;
  for (int i = 0; i < K; i++) {
    size_t lt = sub + (size_t)i * per, eq = lt + sz_lessthan(n);
    W(lt + 1) = W(in0 + i); W(lt + 2) = W(in1 + i);
    run_lessthan(c, lt, n);
    W(eq + 1) = W(in0 + i); W(eq + 2) = W(in1 + i);
    run_isequal(c, eq);
    W(res + i) = i == 0 ? fr_add(W(lt), W(eq)) : fr_add(W(lt), mulg(W(eq), W(res + i - 1)));
  }
  W(b) = W(res + K - 1);
}
/* BigGreaterThan(n,K) bigIntComparators.circom:78-87: out | in[2][K] | lessEqThan */
static size_t sz_bgt(int n, int K) { return 1 + 2 * (size_t)K + sz_blet(n, K); }
static void run_bgt(ctx_t *c, size_t b, int n, int K) {
  size_t le = b + 1 + 2 * K;
  for (int i = 0; i < 2 * K; i++) W(le + 1 + i) = W(b + 1 + i);
  run_blet(c, le, n, K);
  W(b) = fr_sub(ONE(), W(le));
}

/* BigIntIsZero(n,MAX,K) bigIntComparators.circom:105-129: in[K] | carry[K-1] | carryRangeChecks[K-1] */
static size_t sz_bisz(int n, int MAX, int K) { return (size_t)K + (K - 1) + (size_t)(K - 1) * sz_num2bits(MAX + 3 - n); }
static fr_t INV2_64, INV2_N[65];
static void run_bisz(ctx_t *c, size_t b, int n, int MAX, int K) {
  int L = MAX + 3 - n;
  size_t in = b, carry = b + K, sub = carry + K - 1, per = sz_num2bits(L);
  if (n != 64 && fr_is_zero(INV2_N[n])) INV2_N[n] = fr_inv(POW2[n]);
  fr_t inv = (n == 64) ? INV2_64 : INV2_N[n];
  for (int i = 0; i < K - 1; i++) {
    fr_t v = i == 0 ? W(in) : fr_add(W(in + i), W(carry + i - 1));
    W(carry + i) = fr_mul(v, inv);
    size_t rc = sub + (size_t)i * per;
    W(rc + L) = fr_add(W(carry + i), POW2[L - 1]);
    run_num2bits(c, rc, L);
  }
  if (!fr_is_zero(fr_add(W(in + K - 1), W(carry + K - 2))) && !c->err) c->err = S_BIGISZERO;
}

/* multiprecision helpers for the witness-time functions of bigIntFunc.circom */
typedef struct { uint64_t d[140]; int n; } mp_t;

/* reduce_overflow bigIntFunc.circom:570-588 over non-negative overflowed limbs (< 2^192 each) */
static void reduce_overflow(const fr_t *N, int k, int m, uint64_t *M) {
  uint64_t ov[3] = {0, 0, 0};
  for (int i = 0; i < m; i++) {
    uint64_t v[3] = {0, 0, 0};
    if (i < k) { v[0] = N[i].l[0]; v[1] = N[i].l[1]; v[2] = N[i].l[2]; }
    u128 s = (u128)v[0] + ov[0];
    uint64_t r0 = (uint64_t)s; uint64_t cy = (uint64_t)(s >> 64);
    s = (u128)v[1] + ov[1] + cy; uint64_t r1 = (uint64_t)s; cy = (uint64_t)(s >> 64);
    s = (u128)v[2] + ov[2] + cy; uint64_t r2 = (uint64_t)s;
    M[i] = r0; ov[0] = r1; ov[1] = r2; ov[2] = 0;
  }
}

/* Floor division a / b on 64-bit limbs (Knuth D). a: na limbs, b: nb limbs (top non-zero).
 * Quotient q[na-nb+1], remainder r[nb]. Same (unique) result as long_div
 * (bigIntFunc.circom:190-232) whenever that function's output passes the template's checks. */
static void mp_divmod(const uint64_t *a, int na, const uint64_t *b, int nb, uint64_t *q, uint64_t *r) {
  uint64_t u[160], v[80];
  int s = __builtin_clzll(b[nb - 1]);
  for (int i = nb - 1; i > 0; i--) v[i] = (b[i] << s) | (s ? b[i - 1] >> (64 - s) : 0);
  v[0] = b[0] << s;
  u[na] = s ? a[na - 1] >> (64 - s) : 0;
  for (int i = na - 1; i > 0; i--) u[i] = (a[i] << s) | (s ? a[i - 1] >> (64 - s) : 0);
  u[0] = a[0] << s;
  for (int j = na - nb; j >= 0; j--) {
    u128 num = ((u128)u[j + nb] << 64) | u[j + nb - 1];
    u128 qhat = num / v[nb - 1], rhat = num % v[nb - 1];
    while (qhat >> 64 || (nb > 1 && qhat * v[nb - 2] > ((rhat << 64) | u[j + nb - 2]))) {
      qhat--; rhat += v[nb - 1];
      if (rhat >> 64) break;
    }
    int64_t borrow = 0; uint64_t carry = 0;
    for (int i = 0; i < nb; i++) {
      u128 p = qhat * v[i] + carry;
      carry = (uint64_t)(p >> 64);
      u128 t = (u128)u[i + j] - (uint64_t)p - (uint64_t)borrow;
      u[i + j] = (uint64_t)t; borrow = (t >> 64) ? 1 : 0;
    }
    u128 t = (u128)u[j + nb] - carry - (uint64_t)borrow;
    u[j + nb] = (uint64_t)t;
    if (t >> 64) { /* add back */
      qhat--; uint64_t cy = 0;
      for (int i = 0; i < nb; i++) {
        u128 s2 = (u128)u[i + j] + v[i] + cy;
        u[i + j] = (uint64_t)s2; cy = (uint64_t)(s2 >> 64);
      }
      u[j + nb] += cy;
    }
    q[j] = (uint64_t)qhat;
  }
  for (int i = 0; i < nb; i++) r[i] = (u[i] >> s) | (s && i + 1 <= nb ? u[i + 1] << (64 - s) : 0);
}

/* acc (AW words, two's complement) += / -= mag (4 words) << sh bits */
static void acc_shifted(uint64_t *acc, int AW, const uint64_t *mag, int sh, int neg) {
  uint64_t t[6] = {0};
  int s = sh & 63, w0 = sh >> 6;
  for (int w = 0; w < 4; w++) {
    t[w] |= mag[w] << s;
    if (s) t[w + 1] |= mag[w] >> (64 - s);
  }
  uint64_t cy = 0;
  for (int w = 0; w + w0 < AW; w++) {
    uint64_t v = w < 6 ? t[w] : 0;
    if (!neg) {
      u128 x = (u128)acc[w + w0] + v + cy;
      acc[w + w0] = (uint64_t)x; cy = (uint64_t)(x >> 64);
    } else {
      u128 x = (u128)acc[w + w0] - v - cy;
      acc[w + w0] = (uint64_t)x; cy = (uint64_t)(x >> 64) & 1;
    }
  }
}
/* chunk j (n bits) of the word array a */
static uint64_t word_chunk(const uint64_t *a, int n, int j) {
  int off = n * j;
  uint64_t v = a[off >> 6] >> (off & 63);
  if ((off & 63) + n > 64) v |= a[(off >> 6) + 1] << (64 - (off & 63));
  return n == 64 ? v : v & ((1ULL << n) - 1);
}

/* BigMultModP(n,G,L,M) bigInt.circom:206-272:
 * div[DIV], mod[M] | in1[G], in2[L], modulus[M] | mult, modChecks[M], greaterThan, mult2, isZero */
static size_t sz_bmmp(int n, int G, int L, int M) {
  int BASE = G + L, DIV = BASE - M + 1;
  size_t m2 = DIV >= M ? sz_bmneq(DIV, M) : sz_bmneq(M, DIV);
  return (size_t)DIV + M + G + L + M + sz_bmo(G, L) + (size_t)M * sz_num2bits(n) + sz_bgt(n, M) + m2 +
         sz_bisz(n, 2 * n + log_ceil(M + DIV - 1), BASE - 1);
}
static void run_bmmp(ctx_t *c, size_t b, int n, int G, int L, int M) {
  int BASE = G + L, DIV = BASE - M + 1, MAX = 2 * n + log_ceil(M + DIV - 1);
  size_t dv = b, md = b + DIV, in1 = md + M, in2 = in1 + G, mo = in2 + L;
  size_t mult = mo + M, mchk = mult + sz_bmo(G, L), gt = mchk + (size_t)M * sz_num2bits(n), m2 = gt + sz_bgt(n, M);
  int m2big = DIV >= M;
  size_t isz = m2 + (m2big ? sz_bmneq(DIV, M) : sz_bmneq(M, DIV));
  /* mult = in1 * in2 (overflowed) */
  for (int i = 0; i < G; i++) W(mult + BASE - 1 + i) = W(in1 + i);
  for (int i = 0; i < L; i++) W(mult + BASE - 1 + G + i) = W(in2 + i);
  run_bmo(c, mult, G, L);
  /* witness-time reduce_overflow + long_div (unconstrained) */
  uint64_t red[160], modl[80], q[90], r[80];
  memset(q, 0, sizeof q); memset(r, 0, sizeof r);
  if (n == 64) {
    reduce_overflow(&W(mult), BASE - 1, BASE, red);
    for (int i = 0; i < M; i++) modl[i] = W(mo + i).l[0];
    int nb = M;
    while (nb > 1 && modl[nb - 1] == 0) nb--;
    mp_divmod(red, BASE, modl, nb, q, r);
  } else { /* n < 64 chunks: the same quotient / remainder computed on words, then re-chunked */
    uint64_t qw[90] = {0}, rw[80] = {0};
    int aw = (n * BASE + 63) / 64 + 4;
    memset(red, 0, sizeof red); memset(modl, 0, sizeof modl);
    for (int i = 0; i < BASE - 1; i++) acc_shifted(red, aw, W(mult + i).l, n * i, 0);
    for (int i = 0; i < M; i++) modl[(n * i) >> 6] |= W(mo + i).l[0] << ((n * i) & 63);
    int nb = (n * M + 63) / 64;
    while (nb > 1 && modl[nb - 1] == 0) nb--;
    mp_divmod(red, aw, modl, nb, qw, rw);
    for (int i = 0; i < DIV; i++) q[i] = word_chunk(qw, n, i);
    for (int i = 0; i < M; i++) r[i] = word_chunk(rw, n, i);
  }
  for (int i = 0; i < DIV; i++) W(dv + i) = fr_u64(q[i]);
  for (int i = 0; i < M; i++) W(md + i) = fr_u64(r[i]);
  for (int i = 0; i < M; i++) {
    size_t nc = mchk + (size_t)i * sz_num2bits(n);
    W(nc + n) = W(md + i);
    run_num2bits(c, nc, n);
  }
  for (int i = 0; i < M; i++) { W(gt + 1 + i) = W(mo + i); W(gt + 1 + M + i) = W(md + i); }
  run_bgt(c, gt, n, M);
  if (!fr_eq(W(gt), ONE()) && !c->err) c->err = S_BIGMOD_GT;
  if (m2big) {
    size_t a1 = m2 + DIV + M - 1;
    for (int i = 0; i < DIV; i++) W(a1 + i) = W(dv + i);
    for (int i = 0; i < M; i++) W(a1 + DIV + i) = W(mo + i);
    run_bmneq(c, m2, DIV, M);
  } else {
    size_t a1 = m2 + DIV + M - 1;
    for (int i = 0; i < M; i++) W(a1 + i) = W(mo + i);
    for (int i = 0; i < DIV; i++) W(a1 + M + i) = W(dv + i);
    run_bmneq(c, m2, M, DIV);
  }
  for (int i = 0; i < BASE - 1; i++) {
    fr_t v = fr_sub(W(mult + i), W(m2 + i));
    if (i < M) v = fr_sub(v, W(md + i));
    W(isz + i) = v;
  }
  run_bisz(c, isz, n, MAX, BASE - 1);
}

/* exp_to_bits bigIntFunc.circom:590-616 */
static void exp_to_bits(long exp, int *idx) {
  int mul_num = 0, res_num = 0, counter = 0, rc = 0;
  while (exp > 0) {
    int bit = (int)(exp & 1); exp >>= 1;
    if (bit) { res_num++; idx[rc + 2] = counter; rc++; }
    mul_num++; counter++;
  }
  idx[0] = mul_num - 1; idx[1] = res_num;
}

/* PowerMod(n,K,EXP) bigInt.circom:280-340: out[K] | base[K], modulus[K] | muls[e0], resultMuls[e1-1] */
static size_t sz_powermod(int n, int K, long EXP) {
  int idx[260]; exp_to_bits(EXP, idx);
  return 3 * (size_t)K + (size_t)(idx[0] + idx[1] - 1) * sz_bmmp(n, K, K, K);
}
static void run_powermod(ctx_t *c, size_t b, int n, int K, long EXP) {
  int idx[260]; exp_to_bits(EXP, idx);
  size_t base = b + K, mod = base + K, per = sz_bmmp(n, K, K, K), muls = mod + K, res = muls + (size_t)idx[0] * per;
  /* BigMultModP input offsets: in1 @ DIV+M, in2 @ +G, modulus @ +L */
  int DIV = K + 1;
  size_t o_in1 = DIV + K, o_in2 = o_in1 + K, o_mod = o_in2 + K, o_mod_out = DIV;
  for (int i = 0; i < idx[0]; i++) {
    size_t m = muls + (size_t)i * per;
    for (int j = 0; j < K; j++) W(m + o_mod + j) = W(mod + j);
    for (int j = 0; j < K; j++) {
      fr_t v = i == 0 ? W(base + j) : W(muls + (size_t)(i - 1) * per + o_mod_out + j);
      W(m + o_in1 + j) = v; W(m + o_in2 + j) = v;
    }
    run_bmmp(c, m, n, K, K, K);
  }
  for (int i = 0; i < idx[1] - 1; i++) {
    size_t m = res + (size_t)i * per;
    for (int j = 0; j < K; j++) W(m + o_mod + j) = W(mod + j);
    for (int j = 0; j < K; j++) {
      fr_t a;
      if (i == 0) a = idx[2] == 0 ? W(base + j) : W(muls + (size_t)(idx[2] - 1) * per + o_mod_out + j);
      else a = W(res + (size_t)(i - 1) * per + o_mod_out + j);
      W(m + o_in1 + j) = a;
      W(m + o_in2 + j) = W(muls + (size_t)(idx[i + 3] - 1) * per + o_mod_out + j);
    }
    run_bmmp(c, m, n, K, K, K);
  }
  size_t src = idx[1] == 1 ? muls + (size_t)(idx[0] - 1) * per : res + (size_t)(idx[1] - 2) * per;
  for (int j = 0; j < K; j++) W(b + j) = W(src + o_mod_out + j);
}

/* RsaVerifyPkcs1v15(64,K,EXP,256) rsa.circom:16-72:
 * signature[K], pubkey[K], hashed[256] | hashed_chunks[4] | pm, bits2num[3..0], num2bits_6 */
static size_t sz_rsa(int K, long EXP) { return 2 * (size_t)K + 256 + 4 + sz_powermod(64, K, EXP) + 4 * sz_bits2num(64) + sz_num2bits(64); }
static void run_rsa(ctx_t *c, size_t b, int K, long EXP) {
  size_t sig = b, pk = b + K, hashed = pk + K, hc = hashed + 256, pm = hc + 4, b2n = pm + sz_powermod(64, K, EXP),
         n6 = b2n + 4 * sz_bits2num(64);
  for (int i = 0; i < K; i++) { W(pm + K + i) = W(sig + i); W(pm + 2 * K + i) = W(pk + i); }
  run_powermod(c, pm, 64, K, EXP);
  for (int i = 0; i < 4; i++) {
    size_t bn = b2n + (size_t)i * sz_bits2num(64); /* creation order: bits2num[3], [2], [1], [0] */
    int idx = 3 - i;
    for (int j = 0; j < 64; j++) W(bn + 1 + j) = W(hashed + i * 64 + 63 - j);
    run_bits2num(c, bn, 64);
    W(hc + idx) = W(bn);
  }
  for (int i = 0; i < 4; i++)
    if (!fr_eq(W(hc + i), W(pm + i)) && !c->err) c->err = S_RSA_HASH;
  if ((!fr_eq(W(pm + 4), fr_u64(217300885422736416ULL)) || !fr_eq(W(pm + 5), fr_u64(938447882527703397ULL))) && !c->err)
    c->err = S_RSA_PREFIX;
  W(n6 + 64) = W(pm + 6);
  run_num2bits(c, n6, 64);
  static const int remains[32] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 0, 0, 0, 0,
                                  0, 0, 1, 1, 0, 0, 0, 1, 0, 0, 1, 1, 0, 0, 0, 0};
  int bad = 0;
  for (int i = 0; i < 32; i++) bad |= !fr_eq(W(n6 + i), fr_u64((uint64_t)remains[31 - i]));
  for (int i = 32; i < 64; i++) bad |= !fr_eq(W(n6 + i), ONE());
  for (int i = 7; i < K - 1; i++) bad |= !fr_eq(W(pm + i), fr_u64(0xFFFFFFFFFFFFFFFFULL));
  if (bad && !c->err) c->err = S_RSA_PAD;
}

/* RsaVerifyPkcs1v15(64,K,EXP,160) rsa.circom:73-109 (SHA-1 DigestInfo):
 * signature[K], pubkey[K], hashed[160] | hashed_chunks[2] (never assigned) | pm, bits2num[0..1], getBits, getDiv.
 * The bits2num outputs are not constrained against EM (rsa.circom:82-88): only the first digest word is checked. */
static size_t sz_rsa160(int K, long EXP) {
  return 2 * (size_t)K + 160 + 2 + sz_powermod(64, K, EXP) + 2 * sz_bits2num(64) + sz_num2bits(64) + sz_bits2num(32);
}
static void run_rsa160(ctx_t *c, size_t b, int K, long EXP) {
  size_t sig = b, pk = b + K, hashed = pk + K, hc = hashed + 160, pm = hc + 2, b2n = pm + sz_powermod(64, K, EXP),
         gb = b2n + 2 * sz_bits2num(64), gd = gb + sz_num2bits(64);
  for (int i = 0; i < K; i++) { W(pm + K + i) = W(sig + i); W(pm + 2 * K + i) = W(pk + i); }
  run_powermod(c, pm, 64, K, EXP);
  W(hc) = fr_zero(); W(hc + 1) = fr_zero();
  for (int i = 0; i < 2; i++) {
    size_t bn = b2n + (size_t)i * sz_bits2num(64);
    for (int j = 0; j < 64; j++) W(bn + 1 + j) = W(hashed + 159 - j - i * 64);
    run_bits2num(c, bn, 64);
  }
  W(gb + 64) = W(pm + 2);
  run_num2bits(c, gb, 64);
  int bad = 0;
  for (int i = 0; i < 32; i++) bad |= !fr_eq(W(gb + i), W(hashed + 31 - i));
  if (bad && !c->err) c->err = S_RSA_HASH;  /* rsa.circom:95-97 */
  for (int i = 32; i < 64; i++) W(gd + 1 + i - 32) = W(gb + i);
  run_bits2num(c, gd, 32);
  if ((!fr_eq(W(gd), fr_u64(83887124ULL)) || !fr_eq(W(pm + 3), fr_u64(650212878678426138ULL)) ||
       !fr_eq(W(pm + 4), fr_u64(18446744069417738544ULL))) && !c->err)
    c->err = S_RSA_PREFIX;  /* rsa.circom:102-106 */
  bad = 0;
  for (int i = 5; i < K - 1; i++) bad |= !fr_eq(W(pm + i), fr_u64(0xFFFFFFFFFFFFFFFFULL));
  bad |= !fr_eq(W(pm + K - 1), fr_u64(562949953421311ULL));
  if (bad && !c->err) c->err = S_RSA_PAD;  /* rsa.circom:107-111 */
}

/* VerifySignature(SIG 1|2|3) signatureVerification.circom:9-145: pubkey[K], signature[K], hashed[HT] | rsa */
static size_t sz_verifysig(int K, int HT, long EXP) { return 2 * (size_t)K + HT + (HT == 160 ? sz_rsa160(K, EXP) : sz_rsa(K, EXP)); }
static void run_verifysig(ctx_t *c, size_t b, int K, int HT, long EXP) {
  size_t rsa = b + 2 * K + HT;
  for (int i = 0; i < K; i++) { W(rsa + i) = W(b + K + i); W(rsa + K + i) = W(b + i); }
  for (int i = 0; i < HT; i++) W(rsa + 2 * K + i) = W(b + 2 * K + i);
  if (HT == 160) run_rsa160(c, rsa, K, EXP);
  else run_rsa(c, rsa, K, EXP);
}

/* ================================================= RSA-PSS (SIGNATURE_TYPE 10-14)
 * VerifyRsaPssSig(64, K, SALT, EXP, H) rsaPss.circom:18-254 with Mgf1Sha256 / Mgf1Sha384 mgf1.circom:5-133.
 * SIG 10: e = 3, salt 32; SIG 11: e = 65537, salt 32; SIG 12: e = 65537, salt 64; SIG 13: SHA-384, salt 48;
 * SIG 14: RSA-3072 (signatureVerification.circom:46-75). EM = PowerMod.out, 8K bytes; DB = EM_LEN - H/8 - 1 bytes. */
static int is_pss(int sig) { return sig >= 10 && sig <= 14; }
static int pss_salt(int sig) { return sig == 12 ? 64 : sig == 13 ? 48 : 32; }
static int pss_hash(int sig) { return sig == 13 ? 384 : 256; }
static long sig_exp(int sig) { return sig == 10 ? 3 : sig == 4 ? 37187 : 65537; }

/* Mgf1ShaH(H/8, DBL): out[8 DBL] | seed[H] | hashed[H IT] | (ShaHashChunks(1, H), Num2Bits(32)) x IT, IT = DBL / (H/8) + 1;
 * each block hashes seed | counter (MSB first) | the padding of an (H + 32)-bit message in one BS-bit block */
static int mgf_iters(int DBL, int H) { return DBL / (H / 8) + 1; }
static size_t sz_mgf1(int DBL, int H) {
  int IT = mgf_iters(DBL, H);
  return 8 * (size_t)DBL + H + (size_t)H * IT + (size_t)IT * (sz_hashc(H, 1) + sz_num2bits(32));
}
static void run_mgf1(ctx_t *c, size_t b, int DBL, int H) {
  const int IT = mgf_iters(DBL, H), BS = H > 256 ? 1024 : 512, LM = H + 32;
  size_t out = b, seed = out + 8 * (size_t)DBL, hashed = seed + H, sub = hashed + (size_t)H * IT;
  for (int i = 0; i < IT; i++) {
    size_t sh = sub + (size_t)i * (sz_hashc(H, 1) + sz_num2bits(32)), nb = sh + sz_hashc(H, 1), in = sh + H;
    W(nb + 32) = fr_u64((uint64_t)i);
    run_num2bits(c, nb, 32);
    /* concated (mgf1.circom:30-58, 95-121) */
    for (int j = 0; j < H; j++) W(in + j) = W(seed + j);
    for (int j = 0; j < 32; j++) W(in + H + j) = W(nb + 31 - j);
    for (int j = LM; j < BS; j++) W(in + j) = fr_zero();
    W(in + LM) = ONE();
    for (int k = 0; k < 11; k++)
      if ((LM >> k) & 1) W(in + BS - 1 - k) = ONE();
    run_hashc(c, sh, H, 1);
    for (int j = 0; j < H; j++) W(hashed + (size_t)H * i + j) = W(sh + j);
  }
  for (int i = 0; i < 8 * DBL; i++) W(out + i) = W(hashed + i);
}

/* own: pubkey[K], signature[K], hashed[H] | eM[EML], eMsgInBits[64K], encoded[K], dbMask[DB8], db[DB8],
 *      salt[S8], maskedDB[DB8], hash[H], mDash[1024]
 * subcomponents: powerMod, num2Bits[K] (Num2Bits(64)), bits2Num[EML] (Bits2Num(8)), MGF1_H, xor (Xor2(DB8):
 * out | in1 | in2), hDash (ShaHashChunks(2, 256) or ShaHashChunks(1, 384): M' is 1024 bits either way) */
static size_t sz_pss(int K, int S, long EXP, int H) {
  size_t EML = 8 * (size_t)K, DBL = EML - H / 8 - 1, DB8 = 8 * DBL;
  return 2 * (size_t)K + H + EML + 64 * (size_t)K + K + 3 * DB8 + 8 * (size_t)S + H + 1024 + sz_powermod(64, K, EXP) +
         (size_t)K * sz_num2bits(64) + EML * sz_bits2num(8) + sz_mgf1((int)DBL, H) + 3 * DB8 + sz_hashc(H, 1024 / (H > 256 ? 1024 : 512));
}
static void run_pss(ctx_t *c, size_t b, int K, int S, long EXP, int H) {
  const int EMB = 64 * K, EML = 8 * K, DBL = EML - H / 8 - 1, DB8 = 8 * DBL, S8 = 8 * S, MB = H > 256 ? 1 : 2;
  size_t pk = b, sig = pk + K, hashed = sig + K, eM = hashed + H, bits = eM + EML, enc = bits + EMB,
         dbMask = enc + K, db = dbMask + DB8, salt = db + DB8, masked = salt + S8, hash = masked + DB8,
         mDash = hash + H, pm = mDash + 1024, n2b = pm + sz_powermod(64, K, EXP),
         b2n = n2b + (size_t)K * sz_num2bits(64), mgf = b2n + (size_t)EML * sz_bits2num(8), xr = mgf + sz_mgf1(DBL, H),
         hd = xr + 3 * (size_t)DB8;
  for (int i = 0; i < K; i++) { W(pm + K + i) = W(sig + i); W(pm + 2 * K + i) = W(pk + i); }
  run_powermod(c, pm, 64, K, EXP);
  for (int i = 0; i < K; i++) W(enc + i) = W(pm + i);
  for (int i = 0; i < K; i++) { /* rsaPss.circom:45-53: eMsgInBits = EM bits, most significant first */
    size_t nb = n2b + (size_t)i * sz_num2bits(64);
    W(nb + 64) = W(enc + K - 1 - i);
    run_num2bits(c, nb, 64);
    for (int j = 0; j < 64; j++) W(bits + 64 * (size_t)i + j) = W(nb + 63 - j);
  }
  for (int i = 0; i < EML; i++) { /* :55-61: eM[EML-1-i] = byte i (big-endian) */
    size_t bn = b2n + (size_t)i * sz_bits2num(8);
    for (int j = 0; j < 8; j++) W(bn + 1 + 7 - j) = W(bits + 8 * (size_t)i + j);
    run_bits2num(c, bn, 8);
    W(eM + EML - 1 - i) = W(bn);
  }
  if (!fr_eq(W(eM), fr_u64(188)) && !c->err) c->err = S_PSS_TRAILER;
  for (int i = 0; i < DB8; i++) W(masked + i) = W(bits + i);
  for (int i = 0; i < H; i++) W(hash + i) = W(bits + EMB - H - 8 + i);
  for (int i = 0; i < H; i++) W(mgf + DB8 + i) = W(hash + i);
  run_mgf1(c, mgf, DBL, H);
  for (int i = 0; i < DB8; i++) W(dbMask + i) = W(mgf + i);
  for (int i = 0; i < DB8; i++) { /* Xor2 (bitGates.circom:232-240) */
    fr_t x = W(masked + i), y = W(dbMask + i);
    W(xr + DB8 + i) = x; W(xr + 2 * (size_t)DB8 + i) = y;
    W(xr + i) = fr_sub(fr_add(x, y), fr_add(mulg(x, y), mulg(x, y)));
  }
  W(db) = fr_zero();
  for (int i = 1; i < DB8; i++) W(db + i) = W(xr + i);
  for (int i = 0; i < S8; i++) W(salt + S8 - 1 - i) = W(db + DB8 - 1 - i);
  /* mDash = 0^64 | hashed | salt | padding of a (64 + H + S8)-bit message to 1024 bits (:146-226) */
  const int LM = 64 + H + S8;
  for (int i = 0; i < 1024; i++) W(mDash + i) = fr_zero();
  for (int i = 0; i < H; i++) W(mDash + 64 + i) = W(hashed + i);
  for (int i = 0; i < S8; i++) W(mDash + 64 + H + i) = W(salt + i);
  W(mDash + LM) = ONE();
  for (int k = 0; k < 11; k++)
    if ((LM >> k) & 1) W(mDash + 1023 - k) = ONE();
  for (int i = 0; i < 1024; i++) W(hd + H + i) = W(mDash + i);
  run_hashc(c, hd, H, MB);
  int bad = 0;
  for (int i = 0; i < H; i++) bad |= !fr_eq(W(hd + i), W(hash + i));
  if (bad && !c->err) c->err = S_PSS_HASH;
}

/* VerifySignature(SIG 10-14): pubkey[K], signature[K], hashed[H] | VerifyRsaPssSig */
static size_t sz_verifysig_pss(int K, int sig) {
  return 2 * (size_t)K + pss_hash(sig) + sz_pss(K, pss_salt(sig), sig_exp(sig), pss_hash(sig));
}
static void run_verifysig_pss(ctx_t *c, size_t b, int K, int sig) {
  const int H = pss_hash(sig);
  size_t v = b + 2 * K + H;
  for (int i = 0; i < 2 * K + H; i++) W(v + i) = W(b + i);
  run_pss(c, v, K, pss_salt(sig), sig_exp(sig), H);
}

#include "ecdsa.inc.c"

/* ======================================================== SMT (depth 80) */
static size_t sz_smthash1(void) { return 3 + sz_poseidon(3); }
static size_t sz_smthash2(void) { return 3 + sz_poseidon(2); }
static size_t sz_levins(int N) { return (size_t)N + N + (N - 1) + (size_t)N * 3; }
static size_t sz_smtlevel(void) { return 8 + sz_smthash2() + 6; }
static size_t sz_smt(int N) {
  return 1 + 3 + (size_t)N + 1 + sz_smthash1() + sz_num2bits(254) + sz_levins(N) + (size_t)N * 4 + (size_t)N * sz_smtlevel() + 6;
}
static void run_smt(ctx_t *c, size_t b, int N) {
  size_t root = b + 1, leaf = b + 2, key = b + 3, sib = b + 4, value = sib + N;
  size_t h1 = value + 1, n2b = h1 + sz_smthash1(), li = n2b + sz_num2bits(254), sm = li + sz_levins(N),
         lv = sm + (size_t)N * 4, eq = lv + (size_t)N * sz_smtlevel();
  W(value) = W(leaf);
  /* hash1New: SMTHash1 out | key, value | h(PoseidonHash(3)) */
  W(h1 + 1) = W(key); W(h1 + 2) = W(value);
  W(h1 + 3 + 1) = W(key); W(h1 + 3 + 2) = W(value); W(h1 + 3 + 3) = ONE();
  run_poseidon(c, h1 + 3, 3);
  W(h1) = W(h1 + 3);
  W(n2b + 254) = W(key);
  run_num2bits(c, n2b, 254);
  /* SMTLevIns: levIns[N] | siblings[N] | done[N-1] | isZero[N] */
  size_t lvi = li, lsib = li + N, done = lsib + N, iz = done + N - 1;
  for (int i = 0; i < N; i++) {
    W(lsib + i) = W(sib + i);
    W(iz + 3 * (size_t)i + 1) = W(sib + i);
    run_iszero(c, iz + 3 * (size_t)i);
  }
#define IZ(i) W(iz + 3 * (size_t)(i))
  if (!fr_eq(IZ(N - 1), ONE()) && !c->err) c->err = S_SMT_LAST;
  W(lvi + N - 1) = fr_sub(ONE(), IZ(N - 2));
  W(done + N - 2) = W(lvi + N - 1);
  for (int i = N - 2; i > 0; i--) {
    W(lvi + i) = mulg(fr_sub(ONE(), W(done + i)), fr_sub(ONE(), IZ(i - 1)));
    W(done + i - 1) = fr_add(W(lvi + i), W(done + i));
  }
  W(lvi) = fr_sub(ONE(), W(done));
#undef IZ
  /* sm[i]: st_top, st_inew | levIns, prev_top */
  for (int i = 0; i < N; i++) {
    size_t s = sm + 4 * (size_t)i;
    W(s + 3) = i == 0 ? ONE() : W(sm + 4 * (size_t)(i - 1));
    W(s + 2) = W(lvi + i);
    W(s + 1) = mulg(W(s + 3), W(s + 2));
    W(s) = fr_sub(W(s + 3), W(s + 1));
  }
  /* levels created i = N-1 .. 0: level block for i at lv + (N-1-i)*sz */
  for (int i = N - 1; i >= 0; i--) {
    size_t L = lv + (size_t)(N - 1 - i) * sz_smtlevel();
    size_t ph = L + 8, sw = ph + sz_smthash2();
    W(L + 1) = W(sm + 4 * (size_t)i); W(L + 2) = W(sm + 4 * (size_t)i + 1);
    W(L + 3) = W(sib + i); W(L + 4) = W(h1); W(L + 5) = W(n2b + i);
    W(L + 6) = i == N - 1 ? fr_zero() : W(lv + (size_t)(N - 2 - i) * sz_smtlevel());
    W(sw + 3) = W(L + 6); W(sw + 4) = W(L + 3); W(sw + 2) = W(L + 5);
    run_switcher(c, sw);
    W(ph + 1) = W(sw); W(ph + 2) = W(sw + 1);
    W(ph + 3 + 1) = W(ph + 1); W(ph + 3 + 2) = W(ph + 2);
    run_poseidon(c, ph + 3, 2);
    W(ph) = W(ph + 3);
    W(L + 7) = mulg(W(ph), W(L + 1));
    W(L) = fr_add(W(L + 7), mulg(W(L + 4), W(L + 2)));
  }
  W(eq + 1) = W(lv + (size_t)(N - 1) * sz_smtlevel()); W(eq + 2) = W(root);
  run_isequal(c, eq);
  W(b) = W(eq);
}

/* ================================================================ Flow */
typedef struct {
  int sig, dg_hash, doc, ec_blocks, ec_shift, dg1_shift, aa, dg15_shift, dg15_blocks, aa_shift;
} orc_params;

/* PassportVerificationFlow(ecLen, H = DG hash bits, EH = EC hash bits, ...) passportVerificationFlow.circom:6-109:
 * flowResult | dg1Hash[H], dg15Hash[H], encapsulatedContent[ecLen], encapsulatedContentHash[EH], signedAttributes[1024]
 * | verifyAllChecksPassed[3H+8] | IsEqual x (3H + 8) */
static size_t sz_flow(int ecLen, int H, int EH) {
  return 1 + 2 * (size_t)H + (size_t)ecLen + EH + 1024 + (3 * (size_t)H + 8) * 7;
}
static void run_flow(ctx_t *c, size_t b, int ecLen, int H, int EH, int dg1s, int dg15s, int ecs, int V) {
  const int NC = 3 * H + 8;
  size_t h1 = b + 1, h15 = h1 + H, ec = h15 + H, ech = ec + ecLen, sa = ech + EH, v = sa + 1024, eq = v + NC;
  fr_t Vf = fr_u64((uint64_t)V);
  for (int i = 0; i < H; i++) {
    size_t e = eq + 6 * (size_t)i;
    W(e + 1) = W(h1 + i); W(e + 2) = W(ec + dg1s + i); run_isequal(c, e);
  }
  for (int i = 0; i < H; i++) {
    size_t e = eq + 6 * (size_t)(H + i);
    W(e + 1) = mulg(W(h15 + i), Vf); W(e + 2) = mulg(W(ec + dg15s + i), Vf); run_isequal(c, e);
  }
  for (int i = 0; i < H; i++) {  /* :36-40 reads encapsulatedContentHash[i] for i < HASH_SIZE */
    size_t e = eq + 6 * (size_t)(2 * H + i);
    W(e + 1) = W(ech + i); W(e + 2) = W(sa + ecs + i); run_isequal(c, e);
  }
  static const int prefix[8] = {0, 0, 0, 0, 1, 1, 1, 1};
  for (int i = 0; i < 8; i++) {
    size_t e = eq + 6 * (size_t)(3 * H + i);
    W(e + 1) = mulg(fr_u64((uint64_t)prefix[i]), Vf); W(e + 2) = mulg(W(ec + dg15s - 24 + i), Vf);
    run_isequal(c, e);
  }
  W(v) = W(eq);
  for (int i = 1; i < NC; i++) W(v + i) = mulg(W(v + i - 1), W(eq + 6 * (size_t)i));
  W(b) = W(v + NC - 1);
}

/* ============================================ PassportVerificationBuilder */
static int sig_chunks(int sig) { return sig == 2 ? 64 : (sig == 14 || sig == 4) ? 48 : 32; }
/* signature / pubkey input lengths (registerIdentityBuilder.circom:131-140): 2 x CHUNK_NUMBER chunks for ECDSA */
static int sig_len(int sig) { return sig >= 20 ? 2 * (ec_index(sig) >= 0 ? EC_CURVES[ec_index(sig)].nl : 4) : sig_chunks(sig); }

/* HASH_TYPE of the signed attributes (passportVerificationBuilder.circom:16-59): 160 for SIG 3 / 4, 384 for SIG 13 / 25,
 * 224 for SIG 24; inputs hashed with it come in HASH_BLOCK_SIZE = 512 / 1024-bit blocks (:65-68) */
static int sig_hash(int sig) { return (sig == 3 || sig == 4) ? 160 : (sig == 13 || sig == 25) ? 384 : sig == 24 ? 224 : 256; }
/* EC_HASH_TYPE, the encapsulated content's hash (:53-59): HASH_TYPE before SIG 24 sets it to 224, so 256 there */
static int ec_hash(int sig) { return sig == 24 ? 256 : sig_hash(sig); }
/* EC_FIELD_SIZE = CHUNK_NUMBER x CHUNK_SIZE bits of the ECDSA pubkey hash (:196), and its DIFF (:214-217) */
static int ec_field(int sig) { const ec_curve_t *C = &EC_CURVES[ec_index(sig)]; return C->nl * C->cs; }
static int ec_diff(int sig) { return ec_field(sig) > 248 ? ec_field(sig) - 248 : 0; }
static int hblock(int algo) { return algo > 256 ? 1024 : 512; }
static size_t sz_pvb(const orc_params *P) {
  int DG = P->dg_hash, HT = sig_hash(P->sig), EH = ec_hash(P->sig);
  int K = sig_len(P->sig), ecLen = P->ec_blocks * hblock(HT), dg15Len = P->dg15_blocks * hblock(HT), ec = P->sig >= 20;
  /* own: ..., dg1Hash[DG], dg15Hash[DG], ecHash[EH], saHash[HT], pubkeyHash, then tempModulus[5] (RSA, :184) or
   * ecBitsX[F], ecBitsY[F] (ECDSA, :197-198) */
  const int F = ec ? ec_field(P->sig) : 0;
  size_t own = 1 + (size_t)ecLen + 1024 + dg15Len + 1024 + K + K + 80 + 1 + 2 * (size_t)DG + EH + HT + 1 + (ec ? 2 * (size_t)F : 5);
  size_t pkh = ec ? (size_t)K * sz_num2bits(EC_CURVES[ec_index(P->sig)].cs) + 2 * sz_bits2num(F - ec_diff(P->sig)) + sz_poseidon(2)
                  : sz_poseidon(5);
  return own + sz_hashc(DG, 1024 / hblock(DG)) + (P->aa ? sz_hashc(DG, P->dg15_blocks) : 0) + sz_hashc(EH, P->ec_blocks) +
         sz_hashc(HT, 1024 / hblock(HT)) +
         sz_flow(ecLen, DG, EH) + (ec ? sz_verifysig_ec() : is_pss(P->sig) ? sz_verifysig_pss(K, P->sig) : sz_verifysig(K, HT, sig_exp(P->sig))) +
         sz_bits2num(252) + pkh + sz_smt(80) + sz_poseidon(1);
}
static void run_pvb(ctx_t *c, size_t b, const orc_params *P) {
  int DG = P->dg_hash, HT = sig_hash(P->sig), EH = ec_hash(P->sig);
  int K = sig_len(P->sig), ecLen = P->ec_blocks * hblock(HT), dg15Len = P->dg15_blocks * hblock(HT), isec = P->sig >= 20;
  const int dg1B = 1024 / hblock(DG), saB = 1024 / hblock(HT), dg15HB = P->dg15_blocks * hblock(DG);
  size_t ec = b + 1, dg1 = ec + ecLen, dg15 = dg1 + 1024, sa = dg15 + dg15Len, sig = sa + 1024, pk = sig + K,
         br = pk + K, root = br + 80, dg1H = root + 1, dg15H = dg1H + DG, ecH = dg15H + DG, saH = ecH + EH,
         pkHash = saH + HT, tmpMod = pkHash + 1;
  const int F = isec ? ec_field(P->sig) : 0, FD = isec ? F - ec_diff(P->sig) : 0, CS = isec ? F / (K / 2) : 64;
  size_t p = tmpMod + (isec ? 2 * (size_t)F : 5);
  size_t hDg1 = p; p += sz_hashc(DG, dg1B);
  size_t hDg15 = 0; if (P->aa) { hDg15 = p; p += sz_hashc(DG, P->dg15_blocks); }
  size_t hEc = p; p += sz_hashc(EH, P->ec_blocks);
  size_t hSa = p; p += sz_hashc(HT, saB);
  size_t flow = p; p += sz_flow(ecLen, DG, EH);
  size_t vs = p; p += isec ? sz_verifysig_ec() : is_pss(P->sig) ? sz_verifysig_pss(K, P->sig) : sz_verifysig(K, HT, sig_exp(P->sig));
  size_t saNum = p; p += sz_bits2num(252);
  size_t pkH = p; p += isec ? (size_t)K * sz_num2bits(CS) + 2 * sz_bits2num(FD) + sz_poseidon(2) : sz_poseidon(5);
  size_t smt = p; p += sz_smt(80);
  size_t saHH = p;
  /* hashes */
  for (int i = 0; i < 1024; i++) W(hDg1 + DG + i) = W(dg1 + i);
  run_hashc(c, hDg1, DG, dg1B);
  for (int i = 0; i < DG; i++) W(dg1H + i) = W(hDg1 + i);
  if (P->aa) {
    /* dg15PassportHasher.in[j] <== dg15[j] for j < DG_HASH_BLOCK_SIZE * DG15_BLOCK_NUMBER (:117-120) */
    for (int i = 0; i < dg15HB; i++) W(hDg15 + DG + i) = W(dg15 + i);
    run_hashc(c, hDg15, DG, P->dg15_blocks);
    for (int i = 0; i < DG; i++) W(dg15H + i) = W(hDg15 + i);
  } else {
    for (int i = 0; i < DG; i++) W(dg15H + i) = fr_zero();
  }
  for (int i = 0; i < ecLen; i++) W(hEc + EH + i) = W(ec + i);
  run_hashc(c, hEc, EH, P->ec_blocks);
  for (int i = 0; i < EH; i++) W(ecH + i) = W(hEc + i);
  for (int i = 0; i < 1024; i++) W(hSa + HT + i) = W(sa + i);
  run_hashc(c, hSa, HT, saB);
  for (int i = 0; i < HT; i++) W(saH + i) = W(hSa + i);
  /* flow */
  {
    size_t h1 = flow + 1, h15 = h1 + DG, fec = h15 + DG, fech = fec + ecLen, fsa = fech + EH;
    for (int i = 0; i < DG; i++) { W(h1 + i) = W(dg1H + i); W(h15 + i) = W(dg15H + i); }
    for (int i = 0; i < EH; i++) W(fech + i) = W(ecH + i);
    for (int i = 0; i < ecLen; i++) W(fec + i) = W(ec + i);
    for (int i = 0; i < 1024; i++) W(fsa + i) = W(sa + i);
    int dg15shift = P->aa ? P->dg15_shift : DG;
    run_flow(c, flow, ecLen, DG, EH, P->dg1_shift, dg15shift, P->ec_shift, P->aa);
    if (!fr_eq(W(flow), ONE()) && !c->err) c->err = S_FLOW;
  }
  /* signature */
  for (int i = 0; i < K; i++) { W(vs + K + i) = W(sig + i); W(vs + i) = W(pk + i); }
  for (int i = 0; i < HT; i++) W(vs + 2 * K + i) = W(saH + i);
  if (isec) run_verifysig_ec(c, vs);
  else if (is_pss(P->sig)) run_verifysig_pss(c, vs, K, P->sig);
  else run_verifysig(c, vs, K, HT, sig_exp(P->sig));
  /* passportHash bits (:164-177): the hash's first 252 bits, or all HT < 252 bits shifted up by 252 - HT */
  for (int i = 0; i < 252; i++) W(saNum + 1 + i) = HT >= 252 ? W(saH + i) : i < 252 - HT ? fr_zero() : W(saH + i - (252 - HT));
  run_bits2num(c, saNum, 252);
  if (!isec) { /* RSA pubkey hash (:182-191) */
    for (int i = 0; i < 5; i++) {
      W(tmpMod + i) = fr_add(fr_mul(W(pk + 3 * i), POW2[128]), fr_mul(W(pk + 3 * i + 1), POW2[64]));
      W(pkH + 1 + i) = fr_add(W(tmpMod + i), W(pk + 3 * i + 2));
    }
    run_poseidon(c, pkH, 5);
    W(pkHash) = W(pkH);
  } else { /* ECDSA pubkey hash (:193-230): Poseidon2 of the low F - DIFF = min(F, 248) bits of x and y */
    const int N = K / 2, D = F - FD;
    size_t bx = tmpMod, by = bx + F, n2b = pkH, per = sz_num2bits(CS);
    size_t xn = n2b + (size_t)K * per, yn = xn + sz_bits2num(FD), ph = yn + sz_bits2num(FD);
    for (int i = 0; i < N; i++) {
      size_t nx = n2b + (size_t)(2 * i) * per, ny = nx + per;
      W(nx + CS) = W(pk + i); run_num2bits(c, nx, CS);
      W(ny + CS) = W(pk + N + i); run_num2bits(c, ny, CS);
      for (int j = 0; j < CS; j++) { W(bx + F - 1 - j - CS * i) = W(nx + j); W(by + F - 1 - j - CS * i) = W(ny + j); }
    }
    for (int i = 0; i < FD; i++) { W(xn + 1 + FD - 1 - i) = W(bx + i + D); W(yn + 1 + FD - 1 - i) = W(by + i + D); }
    run_bits2num(c, xn, FD); run_bits2num(c, yn, FD);
    W(ph + 1) = W(xn); W(ph + 2) = W(yn);
    run_poseidon(c, ph, 2);
    W(pkHash) = W(ph);
  }
  /* SMT */
  W(smt + 1) = W(root); W(smt + 2) = W(pkHash); W(smt + 3) = W(pkHash);
  for (int i = 0; i < 80; i++) W(smt + 4 + i) = W(br + i);
  run_smt(c, smt, 80);
  /* passportHash */
  W(saHH + 1) = W(saNum);
  run_poseidon(c, saHH, 1);
  W(b) = W(saHH);
}

/* ======================================================= RegisterIdentity */
/* AA_SIGNATURE_ALGO >= 20: elliptic-curve AA key (identity.circom:51-84): x, y of EC_FIELD_SIZE bits
 * each at AA_SHIFT, hashed as Poseidon2 of their low HASH_SIZE bits; 1..19: RSA-1024 key chunks */
static int aa_is_ec(int aa) { return aa >= 20; }
static int aa_field(int aa) { return aa == 22 ? 320 : aa == 23 ? 192 : 256; }
static int aa_hsize(int aa) { return aa == 23 ? 192 : 248; }
/* RegisterIdentity(DG15_SIZE, DG_HASH_BLOCK_SIZE, ...): dg15[DG15_SIZE x DG_HASH_BLOCK_SIZE] (identity.circom:6-23) */
static size_t sz_regid(const orc_params *P) {
  int dg15Len = P->dg15_blocks * hblock(P->dg_hash), ch = P->doc == 1 ? 190 : 186;
  size_t own = 3 + 1024 + (size_t)dg15Len + 1;
  size_t aa = !P->aa ? 0 : aa_is_ec(P->aa) ? 2 * sz_bits2num(aa_hsize(P->aa)) + sz_poseidon(2)
                                           : 4 * sz_bits2num(200) + sz_bits2num(224) + sz_poseidon(5);
  return own + aa + sz_poseidon(5) + 4 * sz_bits2num(ch) + sz_poseidon(1) + sz_bjjmul() + sz_poseidon(2);
}
static void run_regid(ctx_t *c, size_t b, const orc_params *P) {
  int dg15Len = P->dg15_blocks * hblock(P->dg_hash), ch = P->doc == 1 ? 190 : 186;
  size_t dg1 = b + 3, dg15 = dg1 + 1024, sk = dg15 + dg15Len, p = sk + 1;
  if (P->aa && aa_is_ec(P->aa)) {
    int F = aa_field(P->aa), HS = aa_hsize(P->aa), XY = F - HS;
    size_t xn = p, yn = xn + sz_bits2num(HS), h = yn + sz_bits2num(HS);
    p = h + sz_poseidon(2);
    for (int i = 0; i < HS; i++) {
      W(xn + 1 + HS - 1 - i) = W(dg15 + P->aa_shift + i + XY);
      W(yn + 1 + HS - 1 - i) = W(dg15 + P->aa_shift + F + i + XY);
    }
    run_bits2num(c, xn, HS);
    run_bits2num(c, yn, HS);
    W(h + 1) = W(xn); W(h + 2) = W(yn);
    run_poseidon(c, h, 2);
    W(b) = W(h);
  } else if (P->aa) {
    size_t chunks[5];
    for (int j = 0; j < 4; j++) {
      chunks[j] = p; p += sz_bits2num(200);
      for (int i = 0; i < 200; i++) W(chunks[j] + 1 + 199 - i) = W(dg15 + P->aa_shift + j * 200 + i);
      run_bits2num(c, chunks[j], 200);
    }
    chunks[4] = p; p += sz_bits2num(224);
    for (int i = 0; i < 224; i++) W(chunks[4] + 1 + 223 - i) = W(dg15 + P->aa_shift + 800 + i);
    run_bits2num(c, chunks[4], 224);
    size_t h = p; p += sz_poseidon(5);
    for (int i = 0; i < 5; i++) W(h + 1 + i) = W(chunks[i]);
    run_poseidon(c, h, 5);
    W(b) = W(h);
  } else {
    W(b) = fr_zero();
  }
  size_t dg1Hasher = p; p += sz_poseidon(5);
  size_t chk[4];
  for (int i = 0; i < 4; i++) {
    chk[i] = p; p += sz_bits2num(ch);
    for (int j = 0; j < ch; j++) W(chk[i] + 1 + j) = W(dg1 + i * ch + j);
    run_bits2num(c, chk[i], ch);
    W(dg1Hasher + 1 + i) = W(chk[i]);
  }
  size_t skH = p; p += sz_poseidon(1);
  W(skH + 1) = W(sk);
  run_poseidon(c, skH, 1);
  W(dg1Hasher + 5) = W(skH);
  run_poseidon(c, dg1Hasher, 5);
  W(b + 1) = W(dg1Hasher);
  size_t bjj = p; p += sz_bjjmul();
  W(bjj + 2) = W(sk);
  run_bjjmul(c, bjj);
  size_t pkh = p;
  W(pkh + 1) = W(bjj); W(pkh + 2) = W(bjj + 1);
  run_poseidon(c, pkh, 2);
  W(b + 2) = W(pkh);
}

/* =================================================== RegisterIdentityBuilder */
static int orc_init_done = 0;
static void orc_init(void) {
  if (orc_init_done) return;
  init_pow2();
  INV2_64 = fr_inv(POW2[64]);
  orc_init_done = 1;
}

/* The flow reads encapsulatedContentHash[i] for i < DG_HASH_TYPE (passportVerificationFlow.circom:36-40), so DG <= EC_HASH_TYPE;
 * RegisterIdentity's dg15 (DG15_SIZE x DG_HASH_BLOCK_SIZE) is assigned from an input of DG15_BLOCK_NUMBER x
 * HASH_BLOCK_SIZE (registerIdentityBuilder.circom:151), so the block sizes agree or there is no dg15 */
static int params_ok(const orc_params *P) {
  const int HT = sig_hash(P->sig);
  return ((P->sig >= 1 && P->sig <= 4) || is_pss(P->sig) || (ec_index(P->sig) >= 0 && EC_GPOW_T[ec_index(P->sig)])) &&
         (P->dg_hash == 256 || P->dg_hash == 224 || P->dg_hash == 160 || P->dg_hash == 384) && P->dg_hash <= ec_hash(P->sig) &&
         (hblock(P->dg_hash) == hblock(HT) || P->dg15_blocks == 0) && (P->doc == 1 || P->doc == 3) && (P->aa >= 0 && P->aa <= 25) &&
         P->ec_blocks > 0 && P->ec_blocks <= 16 && P->dg15_blocks >= 0 && P->dg15_blocks <= 16;
}

size_t orc_register_n_inputs(const orc_params *P) {
  int K = sig_len(P->sig);
  const int bs = hblock(sig_hash(P->sig));
  return 1 + (size_t)P->ec_blocks * bs + 1024 + (size_t)P->dg15_blocks * bs + 1024 + 2 * K + 80 + 1;
}
size_t orc_register_witness_size(const orc_params *P) {
  if (!pos_loaded || !params_ok(P)) return 0;
  orc_init();
  if (P->sig >= 20) ec_select(ec_index(P->sig));
  return 1 + 4 + orc_register_n_inputs(P) + sz_pvb(P) + sz_regid(P);
}

/* inputs: nInputs x 32 B LE, witness order (slaveMerkleRoot first, then encapsulatedContent, dg1, dg15,
 * signedAttributes, signature, pubkey, slaveMerkleInclusionBranches, skIdentity). Returns check-site id. */
int orc_register_witness(const orc_params *P, const uint8_t *inputs, uint8_t *wit) {
  if (!pos_loaded || !params_ok(P)) return -1;
  orc_init();
  ctx_t cc = {(fr_t *)wit, 0}, *c = &cc;
  if (P->sig >= 20) ec_select(ec_index(P->sig));
  size_t nIn = orc_register_n_inputs(P), nW = orc_register_witness_size(P);
  memset(wit, 0, nW * 32);
  W(0) = ONE();
  memcpy(&W(5), inputs, nIn * 32);
  int K = sig_len(P->sig), ecLen = P->ec_blocks * hblock(sig_hash(P->sig)), dg15Len = P->dg15_blocks * hblock(sig_hash(P->sig));
  size_t root = 5, ec = 6, dg1 = ec + ecLen, dg15 = dg1 + 1024, sa = dg15 + dg15Len, sig = sa + 1024, pk = sig + K,
         br = pk + K, sk = br + 80;
  size_t pvb = 5 + nIn, rid = pvb + sz_pvb(P);
  /* passportVerifier inputs: encapsulatedContent, dg1, dg15, signedAttributes, signature, pubkey, branches, root */
  size_t q = pvb + 1;
  for (int i = 0; i < ecLen; i++) W(q++) = W(ec + i);
  for (int i = 0; i < 1024; i++) W(q++) = W(dg1 + i);
  for (int i = 0; i < dg15Len; i++) W(q++) = W(dg15 + i);
  for (int i = 0; i < 1024; i++) W(q++) = W(sa + i);
  for (int i = 0; i < K; i++) W(q++) = W(sig + i);
  for (int i = 0; i < K; i++) W(q++) = W(pk + i);
  for (int i = 0; i < 80; i++) W(q++) = W(br + i);
  W(q++) = W(root);
  run_pvb(c, pvb, P);
  W(2) = W(pvb);
  for (int i = 0; i < 1024; i++) W(rid + 3 + i) = W(dg1 + i);
  for (int i = 0; i < dg15Len; i++) W(rid + 3 + 1024 + i) = W(dg15 + i);
  W(rid + 3 + 1024 + dg15Len) = W(sk);
  run_regid(c, rid, P);
  W(1) = W(rid); W(3) = W(rid + 1); W(4) = W(rid + 2);
  return c->err;
}

#include "query.inc.c"

/* ----- standalone circuits for configs 1 and 2 ----- */
/* config 1: component main = PoseidonHash(n): [1, out, in[n], pEx...] */
size_t orc_poseidon_witness_size(int n) { if (!pos_loaded) return 0; orc_init(); return 1 + sz_poseidon(n); }
int orc_poseidon_witness(int n, const uint8_t *inputs, uint8_t *wit) {
  if (!pos_loaded) return -1;
  orc_init();
  ctx_t cc = {(fr_t *)wit, 0}, *c = &cc;
  memset(wit, 0, orc_poseidon_witness_size(n) * 32);
  W(0) = ONE();
  memcpy(&W(2), inputs, (size_t)n * 32);
  run_poseidon(c, 1, n);
  return c->err;
}
/* single Poseidon permutation output only (golden checks) */
int orc_poseidon_hash(int n, const uint8_t *inputs, uint8_t *out) {
  size_t sz = orc_poseidon_witness_size(n);
  uint8_t *w = malloc(sz * 32);
  int r = orc_poseidon_witness(n, inputs, w);
  memcpy(out, w + 32, 32);
  free(w);
  return r;
}
/* config 2: component main = Sha256HashChunks(B): [1, out[256], in[512B], ...] */
size_t orc_sha256_witness_size(int B) { orc_init(); return 1 + sz_sha256chunks(B); }
/* Sha1HashChunks(B) as main: [1, out[160], in[512B], ...] */
size_t orc_sha1_witness_size(int B) { orc_init(); return 1 + sz_sha1chunks(B); }
int orc_sha1_witness(int B, const uint8_t *inputs, uint8_t *wit) {
  orc_init();
  ctx_t cc = {(fr_t *)wit, 0}, *c = &cc;
  size_t nW = orc_sha1_witness_size(B);
  memset(wit, 0, nW * 32);
  W(0) = ONE();
  memcpy(&W(1 + 160), inputs, 512 * (size_t)B * 32);
  run_sha1chunks(c, 1, B);
  return c->err;
}
/* Sha384HashChunks(B) / Sha512HashChunks(B) as main (O = 384 / 512): [1, out[O], in[1024B], ...] */
size_t orc_sha512_witness_size(int B, int O) { orc_init(); return 1 + sz_sha5chunks(O, B); }
int orc_sha512_witness(int B, int O, const uint8_t *inputs, uint8_t *wit) {
  orc_init();
  if (O != 384 && O != 512) return -1;
  ctx_t cc = {(fr_t *)wit, 0}, *c = &cc;
  memset(wit, 0, orc_sha512_witness_size(B, O) * 32);
  W(0) = ONE();
  memcpy(&W(1 + (size_t)O), inputs, (size_t)B * 1024 * 32);
  run_sha5chunks(c, 1, B, O);
  return c->err;
}
int orc_sha256_witness(int B, const uint8_t *inputs, uint8_t *wit) {
  orc_init();
  ctx_t cc = {(fr_t *)wit, 0}, *c = &cc;
  memset(wit, 0, orc_sha256_witness_size(B) * 32);
  W(0) = ONE();
  memcpy(&W(1 + 256), inputs, (size_t)B * 512 * 32);
  run_sha256chunks(c, 1, B);
  return c->err;
}

/* get_a_coeff dontOpenPlease.circom:5-376 — only the entries reachable from RSA chunk counts are
 * needed (a = CHUNK_NUMBER_GREATER in {8..128}); values for the power-of-two sizes: */
static int get_a_coeff(int a) {
  if (a < 8) return -1;
  if (a > 128) return 0;
  switch (a) {
    case 8: return 70;
    case 16: return 211;
    case 32: return 640;
    case 64: return 1940;
    case 128: return 5881;
    default: return 1 << 30; /* non-power-of-two sizes never reach Karatsuba (bigIntOverflow.circom:43-50) */
  }
}
