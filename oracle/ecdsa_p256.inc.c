/* oracle/ecdsa_p256.inc.c — ECDSA secp256r1 (SIGNATURE_TYPE 20) part of the CPU restatement.
 *
 * TEST INFRASTRUCTURE ONLY (included by witness_oracle.c; see its header). Restates, template by
 * template and in the O0 layout of DESIGN.md §2:
 *   VerifySignature(20)            signatureVerification.circom:177-191
 *   verifyECDSABits(64,4,A,B,P,256) signatures/ecdsa.circom:18-87
 *   EllipicCurveGetOrder / EllipticCurveGetDummy  ec/get.circom:79-195
 *   EllipticCurveDouble / EllipticCurveAdd         ec/curve.circom:281-345
 *   PointOnCurve / PointOnTangent / PointOnLine    ec/curve.circom:110-245
 *   EllipticCurvePrecomputePipinger               ec/curve.circom:249-272
 *   EllipticCurveScalarMult(…,4)                   ec/curve.circom:356-494
 *   EllipicCurveScalarGeneratorMult                ec/curve.circom:672-906
 *   BigModInv                                      bigInt/bigInt.circom:344-368
 *   BigIntIsZeroModP                               bigInt/bigIntComparators.circom:158-212
 *   BigAddOverflow / BigSubModOverflow / ScalarMultOverflow  bigInt/bigIntOverflow.circom:22-111
 * and the witness-time functions they call (bigIntFunc.circom: prod_mod, long_add_mod,
 * long_sub_mod, mod_inv/mod_exp, long_div, reduce_overflow_signed).
 */

/* ------------------------------------------------------------ curve constants */
/* A, B, P: signatureVerification.circom:179-182 (20: secp256r1), :191-196 (21: brainpoolP256r1);
 * order: get.circom:155-156 / :158-159; dummyPoint: get.circom:91-93 / :87-89 */
typedef struct {
  uint64_t A[4], B[4], P[4], N[4], D[2][4];
} ec_curve_t;
static const ec_curve_t EC_CURVES[2] = {
    {{18446744073709551612ULL, 4294967295ULL, 0ULL, 18446744069414584321ULL},
     {4309448131093880907ULL, 7285987128567378166ULL, 12964664127075681980ULL, 6540974713487397863ULL},
     {18446744073709551615ULL, 4294967295ULL, 0ULL, 18446744069414584321ULL},
     {17562291160714782033ULL, 13611842547513532036ULL, 18446744073709551615ULL, 18446744069414584320ULL},
     {{4148137498610012746ULL, 51237685452122967ULL, 6555942389409504868ULL, 799804747332166731ULL},
      {13395177781894339167ULL, 1107697421929919296ULL, 6228258783500845564ULL, 11862546499924939746ULL}}},
    {{16810331318623712729ULL, 18122579188607900780ULL, 17219079075415130087ULL, 9032542404991529047ULL},
     {7767825457231955894ULL, 10773760575486288334ULL, 17523706096862592191ULL, 2800214691157789508ULL},
     {2311270323689771895ULL, 7943213001558335528ULL, 4496292894210231666ULL, 12248480212390422972ULL},
     {10384753744809580199ULL, 10104242082523752183ULL, 4496292894210231665ULL, 12248480212390422972ULL},
     {{5870538370169240658ULL, 13064052279558318326ULL, 1032222391323187885ULL, 10478252910764369874ULL},
      {9125809427693782222ULL, 4479624720887462683ULL, 4313457861005768495ULL, 11848267593595748038ULL}}}};
/* the curve of the witness being computed (ec_select) */
static const uint64_t *EC_A = EC_CURVES[0].A, *EC_B = EC_CURVES[0].B, *EC_P = EC_CURVES[0].P, *EC_N = EC_CURVES[0].N;
static const uint64_t (*EC_DUMMY)[4] = EC_CURVES[0].D;

/* get_g_pow_stride8_table_<curve> (ec/powers/p256pows.circom:3, brainpoolP256r1pows.circom:3): [32][256][2][4],
 * from data/<p256|bp256>_gpow8.bin (tools/extract_ec_table.py) */
static uint64_t *EC_GPOW_T[2] = {NULL, NULL};
static uint64_t *EC_GPOW = NULL;
int orc_load_ec_table(int curve, const char *path) {
  if (curve < 0 || curve > 1) return -3;
  FILE *f = fopen(path, "rb");
  if (!f) return -1;
  uint64_t *t = malloc(32 * 256 * 8 * sizeof(uint64_t));
  size_t got = fread(t, sizeof(uint64_t), 32 * 256 * 8, f);
  fclose(f);
  if (got != 32 * 256 * 8) { free(t); return -2; }
  free(EC_GPOW_T[curve]);
  EC_GPOW_T[curve] = t;
  return 0;
}
int orc_load_p256(const char *path) { return orc_load_ec_table(0, path); }
static void ec_select(int curve) {
  const ec_curve_t *C = &EC_CURVES[curve];
  EC_A = C->A; EC_B = C->B; EC_P = C->P; EC_N = C->N; EC_DUMMY = C->D;
  EC_GPOW = EC_GPOW_T[curve];
}
#define GPOW(i, j, a, k) EC_GPOW[((((size_t)(i) * 256 + (j)) * 2 + (a)) * 4) + (k)]

/* ------------------------------------------- witness-time big-int functions (k = 4) */
typedef struct { uint64_t l[4]; } u256;

static int u256_gt(const u256 *a, const u256 *b) { /* long_gt bigIntFunc.circom:126-140 */
  for (int i = 3; i >= 0; i--) {
    if (a->l[i] > b->l[i]) return 1;
    if (a->l[i] < b->l[i]) return 0;
  }
  return 0;
}
static u256 u256_sub(const u256 *a, const u256 *b) { /* long_sub :142-167 (mod 2^256) */
  u256 r; uint64_t br = 0;
  for (int i = 0; i < 4; i++) {
    u128 d = (u128)a->l[i] - b->l[i] - br;
    r.l[i] = (uint64_t)d; br = (uint64_t)(d >> 64) & 1;
  }
  return r;
}
static u256 u256_add(const u256 *a, const u256 *b, uint64_t *carry) { /* long_add :503-514 */
  u256 r; uint64_t c = 0;
  for (int i = 0; i < 4; i++) {
    u128 s = (u128)a->l[i] + b->l[i] + c;
    r.l[i] = (uint64_t)s; c = (uint64_t)(s >> 64);
  }
  *carry = c;
  return r;
}
static u256 u256_of(const uint64_t *x) { u256 r; memcpy(r.l, x, 32); return r; }
/* prod_mod :524-528 = remainder of the exact 512-bit product */
static u256 ec_prod_mod(const u256 *a, const u256 *b, const uint64_t *m) {
  uint64_t pr[8] = {0}, q[8], r[4];
  for (int i = 0; i < 4; i++) {
    uint64_t cy = 0;
    for (int j = 0; j < 4; j++) {
      u128 t = (u128)a->l[i] * b->l[j] + pr[i + j] + cy;
      pr[i + j] = (uint64_t)t; cy = (uint64_t)(t >> 64);
    }
    pr[i + 4] = cy;
  }
  mp_divmod(pr, 8, m, 4, q, r);
  return u256_of(r);
}
/* long_add_mod :497-501 (a, b < m: the sum's remainder) */
static u256 ec_add_mod(const u256 *a, const u256 *b, const uint64_t *m) {
  uint64_t cy; u256 s = u256_add(a, b, &cy);
  u256 mm = u256_of(m);
  if (cy || !u256_gt(&mm, &s)) s = u256_sub(&s, &mm);
  return s;
}
/* long_sub_mod :516-522: B > A ? A + (P - B) : A - B */
static u256 ec_sub_mod(const u256 *a, const u256 *b, const uint64_t *m) {
  if (u256_gt(b, a)) {
    u256 mm = u256_of(m), t = u256_sub(&mm, b);
    uint64_t cy;
    return u256_add(a, &t, &cy);
  }
  return u256_sub(a, b);
}
/* mod_inv :430-466 (0 -> 0, else a^(m-2) by mod_exp :385-420) */
static u256 ec_mod_inv(const u256 *a, const uint64_t *m) {
  if (!(a->l[0] | a->l[1] | a->l[2] | a->l[3])) return *a;
  u256 e = u256_of(m), two = {{2, 0, 0, 0}};
  e = u256_sub(&e, &two);
  u256 out = {{1, 0, 0, 0}};
  for (int i = 255; i >= 0; i--) {
    if ((e.l[i >> 6] >> (i & 63)) & 1) out = ec_prod_mod(&out, a, m);
    if (i > 0) out = ec_prod_mod(&out, &out, m);
  }
  return out;
}

typedef struct { u256 x, y; } ecpt;

/* EllipticCurveDouble witness values curve.circom:286-296 */
static ecpt ec_double_val(const ecpt *p) {
  u256 three = {{3, 0, 0, 0}}, A = u256_of(EC_A);
  u256 xx = ec_prod_mod(&p->x, &p->x, EC_P), t = ec_prod_mod(&three, &xx, EC_P);
  u256 num = ec_add_mod(&A, &t, EC_P), den = ec_add_mod(&p->y, &p->y, EC_P);
  u256 inv = ec_mod_inv(&den, EC_P), lam = ec_prod_mod(&num, &inv, EC_P);
  u256 l2 = ec_prod_mod(&lam, &lam, EC_P), x2 = ec_add_mod(&p->x, &p->x, EC_P);
  ecpt r;
  r.x = ec_sub_mod(&l2, &x2, EC_P);
  u256 d = ec_sub_mod(&p->x, &r.x, EC_P), ld = ec_prod_mod(&lam, &d, EC_P);
  r.y = ec_sub_mod(&ld, &p->y, EC_P);
  return r;
}
/* EllipticCurveAdd witness values curve.circom:324-330 */
static ecpt ec_add_val(const ecpt *p, const ecpt *q) {
  u256 dy = ec_sub_mod(&q->y, &p->y, EC_P), dx = ec_sub_mod(&q->x, &p->x, EC_P);
  u256 inv = ec_mod_inv(&dx, EC_P), lam = ec_prod_mod(&dy, &inv, EC_P), l2 = ec_prod_mod(&lam, &lam, EC_P);
  ecpt r;
  u256 t = ec_sub_mod(&l2, &p->x, EC_P);
  r.x = ec_sub_mod(&t, &q->x, EC_P);
  u256 d = ec_sub_mod(&p->x, &r.x, EC_P), ld = ec_prod_mod(&lam, &d, EC_P);
  r.y = ec_sub_mod(&ld, &p->y, EC_P);
  return r;
}

/* point <-> 8 consecutive witness limbs ([axis][chunk]) */
static ecpt ec_get(ctx_t *c, size_t at) {
  ecpt p;
  for (int i = 0; i < 4; i++) { p.x.l[i] = W(at + i).l[0]; p.y.l[i] = W(at + 4 + i).l[0]; }
  return p;
}
static void ec_put(ctx_t *c, size_t at, const ecpt *p) {
  for (int i = 0; i < 4; i++) { W(at + i) = fr_u64(p->x.l[i]); W(at + 4 + i) = fr_u64(p->y.l[i]); }
}
static void ec_copy(ctx_t *c, size_t dst, size_t src, int n) { for (int i = 0; i < n; i++) W(dst + i) = W(src + i); }
static void ec_consts(ctx_t *c, size_t at, const uint64_t *v, int n) { for (int i = 0; i < n; i++) W(at + i) = fr_u64(v[i]); }

/* ------------------------------------------------ overflow big-int templates */
/* ScalarMultOverflow(N) bigIntOverflow.circom:101-111: out[N] | in[N], scalar */
static size_t sz_smo(int N) { return 2 * (size_t)N + 1; }
static void run_smo(ctx_t *c, size_t b, int N) {
  for (int i = 0; i < N; i++) W(b + i) = mulg(W(b + 2 * N), W(b + N + i));
}
/* BigAddOverflow(n,G,L) bigIntOverflow.circom:22-35: out[G] | in1[G], in2[L] */
static size_t sz_bao(int G, int L) { return 2 * (size_t)G + L; }
static void run_bao(ctx_t *c, size_t b, int G, int L) {
  for (int i = 0; i < G; i++) W(b + i) = i < L ? fr_add(W(b + G + i), W(b + 2 * G + i)) : W(b + G + i);
}
/* BigSubModOverflow(n,N) bigIntOverflow.circom:78-98: out[N] | in1[N], in2[N], modulus[N] */
static size_t sz_bsmo(int N) { return 4 * (size_t)N; }
static void run_bsmo(ctx_t *c, size_t b, int N) {
  for (int i = 0; i < N; i++) {
    fr_t v = fr_sub(fr_add(W(b + 3 * N + i), W(b + N + i)), W(b + 2 * N + i));
    if (i != N - 1) v = fr_add(v, POW2[64]);
    if (i != 0) v = fr_sub(v, ONE());
    W(b + i) = v;
  }
}

/* BigIntIsZeroModP(n,MAX,CN,MCN,CNM) bigIntComparators.circom:158-212:
 * in[CN], modulus[CNM] | sign, k[DIV] | kRangeChecks[DIV], mult, isZero, swicher[CN] */
static size_t sz_bizmp(int n, int MAX, int CN, int MCN, int CNM) {
  int DIV = MCN - CNM + 1;
  size_t m = DIV >= CNM ? sz_bmo(DIV, CNM) : sz_bmo(CNM, DIV);
  return (size_t)CN + CNM + 1 + DIV + (size_t)DIV * sz_num2bits(n) + m + sz_bisz(n, MAX, MCN) + (size_t)CN * 6;
}
static void run_bizmp(ctx_t *c, size_t b, int n, int MAX, int CN, int MCN, int CNM) {
  int DIV = MCN - CNM + 1;
  size_t in = b, mod = in + CN, sign = mod + CNM, k = sign + 1, krc = k + DIV, per = sz_num2bits(n);
  size_t mult = krc + (size_t)DIV * per;
  size_t isz = mult + (DIV >= CNM ? sz_bmo(DIV, CNM) : sz_bmo(CNM, DIV));
  size_t sw = isz + sz_bisz(n, MAX, MCN);
  /* reduce_overflow_signed (bigIntFunc.circom:646-694): a chunk is negative iff its canonical
   * representative is >= 2^MAX (then it stands for v - p). Floor-carry normalisation of the
   * signed sum S = sum in[i] 2^(64 i); sign = 1 iff S >= 0, reduced = |S| in MCN limbs. */
  uint64_t acc[24] = {0};
  for (int i = 0; i < CN; i++) {
    fr_t v = W(in + i);
    int neg = 0;
    for (int w = 3; w >= 0; w--) {
      int lo = w * 64;
      if (MAX >= lo + 64) break;
      uint64_t mask = MAX <= lo ? ~0ULL : ~((1ULL << (MAX - lo)) - 1);
      if (v.l[w] & mask) { neg = 1; break; }
    }
    uint64_t mag[4];
    if (neg) { fr_t m = fr_neg(v); memcpy(mag, m.l, 32); } else memcpy(mag, v.l, 32);
    /* acc += / -= mag << (64 i), two's complement over 24 limbs */
    uint64_t cy = 0;
    for (int w = 0; w + i < 24; w++) {
      uint64_t t = w < 4 ? mag[w] : 0;
      if (!neg) {
        u128 s = (u128)acc[w + i] + t + cy;
        acc[w + i] = (uint64_t)s; cy = (uint64_t)(s >> 64);
      } else {
        u128 s = (u128)acc[w + i] - t - cy;
        acc[w + i] = (uint64_t)s; cy = (uint64_t)(s >> 64) & 1;
      }
    }
  }
  int positive = !(acc[23] >> 63);
  if (!positive) { /* negate */
    uint64_t cy = 1;
    for (int w = 0; w < 24; w++) { u128 s = (u128)(~acc[w]) + cy; acc[w] = (uint64_t)s; cy = (uint64_t)(s >> 64); }
  }
  W(sign) = fr_u64((uint64_t)positive);
  uint64_t modl[8], q[24], r[8];
  for (int i = 0; i < CNM; i++) modl[i] = W(mod + i).l[0];
  int nb = CNM;
  while (nb > 1 && modl[nb - 1] == 0) nb--;
  memset(q, 0, sizeof q);
  mp_divmod(acc, MCN, modl, nb, q, r); /* long_div(n, CNM, DIV-1, reduced, modulus) */
  for (int i = 0; i < DIV; i++) {
    W(k + i) = fr_u64(q[i]);
    size_t rc = krc + (size_t)i * per;
    W(rc + n) = W(k + i);
    run_num2bits(c, rc, n);
  }
  if (DIV >= CNM) {
    size_t a1 = mult + MCN;
    for (int i = 0; i < DIV; i++) W(a1 + i) = W(k + i);
    for (int i = 0; i < CNM; i++) W(a1 + DIV + i) = W(mod + i);
    run_bmo(c, mult, DIV, CNM);
  } else {
    size_t a1 = mult + MCN;
    for (int i = 0; i < CNM; i++) W(a1 + i) = W(mod + i);
    for (int i = 0; i < DIV; i++) W(a1 + CNM + i) = W(k + i);
    run_bmo(c, mult, CNM, DIV);
  }
  for (int i = 0; i < CN; i++) {
    size_t s = sw + 6 * (size_t)i;
    W(s + 2) = W(sign); W(s + 3) = W(in + i); W(s + 4) = fr_neg(W(in + i));
    run_switcher(c, s);
    W(isz + i) = fr_sub(W(mult + i), W(s + 1));
  }
  for (int i = CN; i < MCN; i++) W(isz + i) = W(mult + i);
  run_bisz(c, isz, n, MAX, MCN);
}

/* --------------------------------------------------------- point checks */
/* PointOnCurve curve.circom:110-138: in[2][4] | squareX, cubeX, squareY, coefMult, isZeroModP */
static size_t sz_poncurve(void) { return 8 + 3 * sz_bmo(4, 4) + sz_bmo(7, 4) + sz_bizmp(64, 200, 10, 12, 4); }
static void run_poncurve(ctx_t *c, size_t b) {
  size_t sx = b + 8, cx = sx + sz_bmo(4, 4), sy = cx + sz_bmo(7, 4), cm = sy + sz_bmo(4, 4), iz = cm + sz_bmo(4, 4);
  for (int i = 0; i < 4; i++) { W(sx + 7 + i) = W(b + i); W(sx + 11 + i) = W(b + i); }
  run_bmo(c, sx, 4, 4);
  for (int i = 0; i < 7; i++) W(cx + 10 + i) = W(sx + i);
  for (int i = 0; i < 4; i++) W(cx + 17 + i) = W(b + i);
  run_bmo(c, cx, 7, 4);
  for (int i = 0; i < 4; i++) { W(sy + 7 + i) = W(b + 4 + i); W(sy + 11 + i) = W(b + 4 + i); }
  run_bmo(c, sy, 4, 4);
  for (int i = 0; i < 4; i++) { W(cm + 7 + i) = W(b + i); W(cm + 11 + i) = fr_u64(EC_A[i]); }
  run_bmo(c, cm, 4, 4);
  for (int i = 0; i < 10; i++) {
    fr_t v = W(cx + i);
    if (i < 7) v = fr_sub(fr_add(v, W(cm + i)), W(sy + i));
    if (i < 4) v = fr_add(v, fr_u64(EC_B[i]));
    W(iz + i) = v;
  }
  ec_consts(c, iz + 10, EC_P, 4);
  run_bizmp(c, iz, 64, 200, 10, 12, 4);
}
/* PointOnTangent curve.circom:145-197: in1[2][4], in2[2][4] | squareX, scalarMult, bigAdd, bigSub,
 * rightMult, scalarMult2, bigAdd2, leftMult, isZeroModP */
static size_t sz_pontangent(void) {
  return 16 + sz_bmo(4, 4) + sz_smo(7) + sz_bao(7, 4) + sz_bsmo(4) + sz_bmo(7, 4) + sz_smo(4) + sz_bao(4, 4) +
         sz_bmo(4, 4) + sz_bizmp(64, 200, 10, 13, 4);
}
static void run_pontangent(ctx_t *c, size_t b) {
  size_t x1 = b, y1 = b + 4, x2 = b + 8, y2 = b + 12;
  size_t sx = b + 16, sm = sx + sz_bmo(4, 4), ba = sm + sz_smo(7), bs = ba + sz_bao(7, 4), rm = bs + sz_bsmo(4),
         sm2 = rm + sz_bmo(7, 4), ba2 = sm2 + sz_smo(4), lm = ba2 + sz_bao(4, 4), iz = lm + sz_bmo(4, 4);
  for (int i = 0; i < 4; i++) { W(sx + 7 + i) = W(x1 + i); W(sx + 11 + i) = W(x1 + i); }
  run_bmo(c, sx, 4, 4);
  for (int i = 0; i < 7; i++) W(sm + 7 + i) = W(sx + i);
  W(sm + 14) = fr_u64(3);
  run_smo(c, sm, 7);
  for (int i = 0; i < 7; i++) W(ba + 7 + i) = W(sm + i);
  ec_consts(c, ba + 14, EC_A, 4);
  run_bao(c, ba, 7, 4);
  for (int i = 0; i < 4; i++) { W(bs + 4 + i) = W(x1 + i); W(bs + 8 + i) = W(x2 + i); }
  ec_consts(c, bs + 12, EC_P, 4);
  run_bsmo(c, bs, 4);
  for (int i = 0; i < 7; i++) W(rm + 10 + i) = W(ba + i);
  for (int i = 0; i < 4; i++) W(rm + 17 + i) = W(bs + i);
  run_bmo(c, rm, 7, 4);
  for (int i = 0; i < 4; i++) W(sm2 + 4 + i) = W(y1 + i);
  W(sm2 + 8) = fr_u64(2);
  run_smo(c, sm2, 4);
  for (int i = 0; i < 4; i++) { W(ba2 + 4 + i) = W(y1 + i); W(ba2 + 8 + i) = W(y2 + i); }
  run_bao(c, ba2, 4, 4);
  for (int i = 0; i < 4; i++) { W(lm + 7 + i) = W(ba2 + i); W(lm + 11 + i) = W(sm2 + i); }
  run_bmo(c, lm, 4, 4);
  for (int i = 0; i < 10; i++) W(iz + i) = i < 7 ? fr_sub(W(rm + i), W(lm + i)) : W(rm + i);
  ec_consts(c, iz + 10, EC_P, 4);
  run_bizmp(c, iz, 64, 200, 10, 13, 4);
}
/* PointOnLine curve.circom:204-245: in1, in2, in3 | bigAdd, bigSub, bigSub2, bigSub3, leftMult,
 * rightMult, isZeroModP */
static size_t sz_ponline(void) { return 24 + sz_bao(4, 4) + 3 * sz_bsmo(4) + 2 * sz_bmo(4, 4) + sz_bizmp(64, 136, 7, 9, 4); }
static void run_ponline(ctx_t *c, size_t b) {
  size_t x1 = b, y1 = b + 4, x2 = b + 8, y2 = b + 12, x3 = b + 16, y3 = b + 20;
  size_t ba = b + 24, s1 = ba + sz_bao(4, 4), s2 = s1 + sz_bsmo(4), s3 = s2 + sz_bsmo(4), lm = s3 + sz_bsmo(4),
         rm = lm + sz_bmo(4, 4), iz = rm + sz_bmo(4, 4);
  for (int i = 0; i < 4; i++) { W(ba + 4 + i) = W(y1 + i); W(ba + 8 + i) = W(y3 + i); }
  run_bao(c, ba, 4, 4);
  size_t subs[3] = {s1, s2, s3}, a1[3] = {x2, y2, x1}, a2[3] = {x1, y1, x3};
  for (int s = 0; s < 3; s++) {
    for (int i = 0; i < 4; i++) { W(subs[s] + 4 + i) = W(a1[s] + i); W(subs[s] + 8 + i) = W(a2[s] + i); }
    ec_consts(c, subs[s] + 12, EC_P, 4);
    run_bsmo(c, subs[s], 4);
  }
  for (int i = 0; i < 4; i++) { W(lm + 7 + i) = W(ba + i); W(lm + 11 + i) = W(s1 + i); }
  run_bmo(c, lm, 4, 4);
  for (int i = 0; i < 4; i++) { W(rm + 7 + i) = W(s2 + i); W(rm + 11 + i) = W(s3 + i); }
  run_bmo(c, rm, 4, 4);
  for (int i = 0; i < 7; i++) W(iz + i) = fr_sub(W(lm + i), W(rm + i));
  ec_consts(c, iz + 7, EC_P, 4);
  run_bizmp(c, iz, 64, 136, 7, 9, 4);
}

/* ------------------------------------------------------------ point ops */
/* EllipticCurveDouble curve.circom:281-310: out[2][4] | in[2][4] | onTangentCheck, onCurveCheck */
static size_t sz_ecdbl(void) { return 16 + sz_pontangent() + sz_poncurve(); }
static void run_ecdbl(ctx_t *c, size_t b) {
  ecpt p = ec_get(c, b + 8), r = ec_double_val(&p);
  ec_put(c, b, &r);
  size_t t = b + 16, k = t + sz_pontangent();
  ec_copy(c, t, b + 8, 8); ec_copy(c, t + 8, b, 8);
  run_pontangent(c, t);
  ec_copy(c, k, b, 8);
  run_poncurve(c, k);
}
/* EllipticCurveAdd curve.circom:314-345: out[2][4] | in1[2][4], in2[2][4] | onCurveCheck, onLineCheck */
static size_t sz_ecadd(void) { return 24 + sz_poncurve() + sz_ponline(); }
static void run_ecadd(ctx_t *c, size_t b) {
  ecpt p = ec_get(c, b + 8), q = ec_get(c, b + 16), r = ec_add_val(&p, &q);
  ec_put(c, b, &r);
  size_t k = b + 24, l = k + sz_poncurve();
  ec_copy(c, k, b, 8);
  run_poncurve(c, k);
  ec_copy(c, l, b + 8, 16); ec_copy(c, l + 16, b, 8);
  run_ponline(c, l);
}

/* EllipticCurvePrecomputePipinger(…,4) curve.circom:249-272: out[16][2][4] | in[2][4] | getDummy,
 * then doublers[i/2-1] (even i) / adders[i/2-1] (odd i) in order i = 2..15 */
static size_t sz_precomp(void) { return 128 + 8 + 8 + 7 * sz_ecdbl() + 7 * sz_ecadd(); }
static void run_precomp(ctx_t *c, size_t b) {
  size_t in = b + 128, gd = in + 8, p = gd + 8;
  ec_consts(c, gd, &EC_DUMMY[0][0], 8);
  ec_copy(c, b, gd, 8);
  ec_copy(c, b + 8, in, 8);
  for (int i = 2; i < 16; i++) {
    if (i % 2 == 0) {
      ec_copy(c, p + 8, b + 8 * (i / 2), 8);
      run_ecdbl(c, p);
      ec_copy(c, b + 8 * i, p, 8);
      p += sz_ecdbl();
    } else {
      ec_copy(c, p + 8, b + 8, 8); ec_copy(c, p + 16, b + 8 * (i - 1), 8);
      run_ecadd(c, p);
      ec_copy(c, b + 8 * i, p, 8);
      p += sz_ecadd();
    }
  }
}

/* EllipticCurveScalarMult(64,4,A,B,P,4) curve.circom:356-494:
 * out[2][4] | in[2][4], scalar[4] | scalarBits[256], resultingPoints[65][2][4], additionPoints[64][2][4]
 * | precompute, getDummy, num2Bits[4], then per window w: bits2Num[w], isZeroResult[w],
 *   (w>0: doublers[4w-4], doubleSwitcher[w-1][8], doublers[4w-3..4w-1]), getSum[w][8],
 *   partsEqual[w][16], (w>0: adders[w-1], isZeroAddition[w], (resultSwitcherAddition,
 *   resultSwitcherDoubling)[w-1][8]) */
static size_t sz_win(int w) {
  size_t s = sz_bits2num(4) + 6 + 8 * (1 + 16 + 15) + 16 * 6;
  if (w > 0) s += 4 * sz_ecdbl() + 8 * 6 + sz_ecadd() + 6 + 16 * 6;
  return s;
}
static size_t sz_scalarmult(void) {
  size_t s = 8 + 8 + 4 + 256 + 65 * 8 + 64 * 8 + sz_precomp() + 8 + 4 * sz_num2bits(64);
  for (int w = 0; w < 64; w++) s += sz_win(w);
  return s;
}
static void run_scalarmult(ctx_t *c, size_t b) {
  size_t in = b + 8, sc = in + 8, bits = sc + 4, rp = bits + 256, ap = rp + 65 * 8, pre = ap + 64 * 8,
         gd = pre + sz_precomp(), n2b = gd + 8, p = n2b + 4 * sz_num2bits(64);
  ec_copy(c, pre + 128, in, 8);
  run_precomp(c, pre);
  ec_consts(c, gd, &EC_DUMMY[0][0], 8);
  for (int i = 0; i < 4; i++) {
    size_t nb = n2b + (size_t)i * sz_num2bits(64);
    W(nb + 64) = W(sc + i);
    run_num2bits(c, nb, 64);
    for (int j = 0; j < 64; j++) W(bits + 256 - 64 * (i + 1) + j) = W(nb + 63 - j);
  }
  ec_copy(c, rp, pre, 8);
  size_t prev_dbl = 0;
  for (int w = 0; w < 64; w++) {
    size_t b2n = p; p += sz_bits2num(4);
    for (int j = 0; j < 4; j++) W(b2n + 1 + j) = W(bits + 4 * w + 3 - j);
    run_bits2num(c, b2n, 4);
    size_t izr = p; p += 6;
    W(izr + 1) = W(rp + 8 * (size_t)w); W(izr + 2) = W(gd);
    run_isequal(c, izr);
    if (w > 0) {
      size_t d0 = p; p += sz_ecdbl();
      size_t dsw = p; p += 8 * 6;
      for (int q = 0; q < 8; q++) {
        size_t s = dsw + 6 * (size_t)q;
        W(s + 2) = W(izr); W(s + 3) = W(gd + q); W(s + 4) = W(rp + 8 * (size_t)w + q);
        run_switcher(c, s);
        W(d0 + 8 + q) = W(s + 1);
      }
      run_ecdbl(c, d0);
      prev_dbl = d0;
      for (int j = 1; j < 4; j++) {
        size_t d = p; p += sz_ecdbl();
        ec_copy(c, d + 8, prev_dbl, 8);
        run_ecdbl(c, d);
        prev_dbl = d;
      }
    }
    size_t gs = p; p += 8 * 32;
    size_t pe = p; p += 16 * 6;
    for (int k = 0; k < 16; k++) {
      size_t e = pe + 6 * (size_t)k;
      W(e + 1) = fr_u64((uint64_t)k); W(e + 2) = W(b2n);
      run_isequal(c, e);
      for (int q = 0; q < 8; q++) W(gs + 32 * (size_t)q + 1 + k) = mulg(W(e), W(pre + 8 * (size_t)k + q));
    }
    for (int q = 0; q < 8; q++) {
      run_getsum(c, gs + 32 * (size_t)q, 16);
      W(ap + 8 * (size_t)w + q) = W(gs + 32 * (size_t)q);
    }
    if (w == 0) {
      ec_copy(c, rp + 8, ap, 8);
    } else {
      size_t ad = p; p += sz_ecadd();
      ec_copy(c, ad + 8, prev_dbl, 8); ec_copy(c, ad + 16, ap + 8 * (size_t)w, 8);
      run_ecadd(c, ad);
      size_t iza = p; p += 6;
      W(iza + 1) = W(ap + 8 * (size_t)w); W(iza + 2) = W(gd);
      run_isequal(c, iza);
      size_t rs = p; p += 16 * 6;
      for (int q = 0; q < 8; q++) {
        size_t sa = rs + 12 * (size_t)q, sd = sa + 6;
        W(sa + 2) = W(iza); W(sa + 3) = W(ad + q); W(sa + 4) = W(prev_dbl + q);
        run_switcher(c, sa);
        W(sd + 2) = W(izr); W(sd + 3) = W(ap + 8 * (size_t)w + q); W(sd + 4) = W(sa);
        run_switcher(c, sd);
        W(rp + 8 * (size_t)(w + 1) + q) = W(sd + 1);
      }
    }
  }
  ec_copy(c, b, rp + 64 * 8, 8);
}

/* EllipicCurveScalarGeneratorMult(64,4,…) curve.circom:672-906:
 * out[2][4] | scalar[4] | resultCoordinateComputation[32][256][2][4], additionPoints[32][2][4],
 *   resultingPointsLeft, Left2, Right, Right2 (never assigned), resultingPoints [32][2][4]
 * | num2bits[4], bits2num[32], getDummy, getSecondDummy, equal[32][256], getSumOfNElements[32][2][4],
 *   per i < 31: adders[i], isFirstDummyLeft, isSecondDummyLeft, isFirstDummyRight, isSecondDummyRight,
 *   (switcherRight, switcherLeft)[axis][j] */
static size_t sz_genmult(void) {
  return 8 + 4 + 32 * 256 * 8 + 32 * 8 * 6 + 4 * sz_num2bits(64) + 32 * sz_bits2num(8) + 8 + sz_ecdbl() +
         32 * 256 * 6 + 32 * 8 * 512 + 31 * (sz_ecadd() + 4 * 6 + 16 * 6);
}
static void run_genmult(ctx_t *c, size_t b) {
  size_t sc = b + 8, rcc = sc + 4, ap = rcc + 32 * 256 * 8, rp = ap + 32 * 8 + 4 * 32 * 8,
         n2b = rp + 32 * 8, b2n = n2b + 4 * sz_num2bits(64), gd = b2n + 32 * sz_bits2num(8), sd = gd + 8,
         eq = sd + sz_ecdbl(), gs = eq + 32 * 256 * 6, p = gs + 32 * 8 * 512;
  for (int i = 0; i < 4; i++) {
    size_t nb = n2b + (size_t)i * sz_num2bits(64);
    W(nb + 64) = W(sc + i);
    run_num2bits(c, nb, 64);
  }
  for (int i = 0; i < 32; i++) {
    size_t bn = b2n + (size_t)i * sz_bits2num(8);
    for (int j = 0; j < 8; j++) W(bn + 1 + j) = W(n2b + (size_t)((i * 8 + j) / 64) * sz_num2bits(64) + (i * 8 + j) % 64);
    run_bits2num(c, bn, 8);
  }
  ec_consts(c, gd, &EC_DUMMY[0][0], 8);
  ec_copy(c, sd + 8, gd, 8);
  run_ecdbl(c, sd);
  for (int i = 0; i < 32; i++) {
    size_t bn = b2n + (size_t)i * sz_bits2num(8);
    for (int j = 0; j < 256; j++) {
      size_t e = eq + 6 * ((size_t)i * 256 + j);
      W(e + 1) = fr_u64((uint64_t)j); W(e + 2) = W(bn);
      run_isequal(c, e);
      for (int a = 0; a < 2; a++)
        for (int k = 0; k < 4; k++) {
          fr_t v;
          if (j == 0) v = (i % 2 == 0) ? W(gd + 4 * a + k) : W(sd + 4 * a + k);
          else v = fr_u64(GPOW(i, j, a, k));
          W(rcc + (((size_t)i * 256 + j) * 2 + a) * 4 + k) = mulg(W(e), v);
        }
    }
  }
  for (int i = 0; i < 32; i++)
    for (int a = 0; a < 2; a++)
      for (int k = 0; k < 4; k++) {
        size_t g = gs + 512 * (((size_t)i * 2 + a) * 4 + k);
        for (int s = 0; s < 256; s++) W(g + 1 + s) = W(rcc + (((size_t)i * 256 + s) * 2 + a) * 4 + k);
        run_getsum(c, g, 256);
        W(ap + 8 * (size_t)i + 4 * a + k) = W(g);
      }
  for (int i = 0; i < 31; i++) {
    size_t ad = p; p += sz_ecadd();
    size_t fl = p, sl = p + 6, fr_ = p + 12, sr = p + 18; p += 24;
    size_t sw = p; p += 16 * 6;
    size_t left = i == 0 ? ap : rp + 8 * (size_t)(i - 1), right = ap + 8 * (size_t)(i + 1);
    W(fl + 1) = W(gd); W(sl + 1) = W(sd); W(fr_ + 1) = W(gd); W(sr + 1) = W(sd);
    W(fl + 2) = W(left); W(sl + 2) = W(left); W(fr_ + 2) = W(right); W(sr + 2) = W(right);
    ec_copy(c, ad + 8, left, 8); ec_copy(c, ad + 16, right, 8);
    run_ecadd(c, ad);
    run_isequal(c, fl); run_isequal(c, sl); run_isequal(c, fr_); run_isequal(c, sr);
    for (int q = 0; q < 8; q++) {
      size_t swr = sw + 12 * (size_t)q, swl = swr + 6;
      W(swr + 2) = fr_add(W(sr), W(fr_)); W(swr + 3) = W(ad + q); W(swr + 4) = W(left + q);
      run_switcher(c, swr);
      W(swl + 2) = fr_add(W(sl), W(fl)); W(swl + 3) = W(right + q); W(swl + 4) = W(swr);
      run_switcher(c, swl);
      W(rp + 8 * (size_t)i + q) = W(swl + 1);
    }
  }
  ec_copy(c, b, rp + 30 * 8, 8);
}

/* BigModInv(64,4) bigInt.circom:344-368: out[4] | in[4], modulus[4] | mult */
static size_t sz_bigmodinv(void) { return 12 + sz_bmmp(64, 4, 4, 4); }
static void run_bigmodinv(ctx_t *c, size_t b) {
  u256 a, m;
  for (int i = 0; i < 4; i++) { a.l[i] = W(b + 4 + i).l[0]; m.l[i] = W(b + 8 + i).l[0]; }
  u256 inv = ec_mod_inv(&a, m.l);
  for (int i = 0; i < 4; i++) W(b + i) = fr_u64(inv.l[i]);
  size_t mm = b + 12, o = mm + 5 + 4;
  for (int i = 0; i < 4; i++) { W(o + i) = W(b + 4 + i); W(o + 4 + i) = W(b + i); W(o + 8 + i) = W(b + 8 + i); }
  run_bmmp(c, mm, 64, 4, 4, 4);
  int bad = !fr_eq(W(mm + 5), ONE());
  for (int i = 1; i < 4; i++) bad |= !fr_is_zero(W(mm + 5 + i));
  if (bad && !c->err) c->err = S_ECDSA_INV;
}

/* verifyECDSABits(64,4,A,B,P,256) ecdsa.circom:18-87:
 * pubkey[2][4], signature[2][4], hashed[256] | hashedChunked[4], one[4], order[4], sinv[4]
 * | bits2Num[4], getOrder, modInv, mult, mult2, scalarMult1, scalarMult2, add, modOrder */
static size_t sz_ecdsa(void) {
  return 16 + 256 + 16 + 4 * sz_bits2num(64) + 4 + sz_bigmodinv() + 3 * sz_bmmp(64, 4, 4, 4) + sz_genmult() +
         sz_scalarmult() + sz_ecadd();
}
static void run_ecdsa(ctx_t *c, size_t b) {
  size_t pk = b, sig = b + 8, hashed = b + 16, hc = hashed + 256, one = hc + 4, ord = one + 4, sinv = ord + 4;
  size_t p = sinv + 4, b2n = p; p += 4 * sz_bits2num(64);
  size_t go = p; p += 4;
  size_t mi = p; p += sz_bigmodinv();
  size_t m1 = p; p += sz_bmmp(64, 4, 4, 4);
  size_t m2 = p; p += sz_bmmp(64, 4, 4, 4);
  size_t s1 = p; p += sz_genmult();
  size_t s2 = p; p += sz_scalarmult();
  size_t ad = p; p += sz_ecadd();
  size_t mo = p;
  const size_t o_in1 = 9, o_in2 = 13, o_mod = 17, o_res = 5; /* BigMultModP(64,4,4,4) offsets */
  for (int i = 0; i < 4; i++) {
    size_t bn = b2n + (size_t)i * sz_bits2num(64);
    for (int j = 0; j < 64; j++) W(bn + 1 + 63 - j) = W(hashed + i * 64 + j);
    run_bits2num(c, bn, 64);
    W(hc + 3 - i) = W(bn);
  }
  W(one) = ONE();
  ec_consts(c, go, EC_N, 4);
  ec_copy(c, ord, go, 4);
  ec_copy(c, mi + 4, sig + 4, 4); ec_copy(c, mi + 8, ord, 4);
  run_bigmodinv(c, mi);
  ec_copy(c, sinv, mi, 4);
  ec_copy(c, m1 + o_in1, sinv, 4); ec_copy(c, m1 + o_in2, hc, 4); ec_copy(c, m1 + o_mod, ord, 4);
  run_bmmp(c, m1, 64, 4, 4, 4);
  ec_copy(c, m2 + o_in1, sinv, 4); ec_copy(c, m2 + o_in2, sig, 4); ec_copy(c, m2 + o_mod, ord, 4);
  run_bmmp(c, m2, 64, 4, 4, 4);
  ec_copy(c, s1 + 8, m1 + o_res, 4);
  run_genmult(c, s1);
  ec_copy(c, s2 + 16, m2 + o_res, 4); ec_copy(c, s2 + 8, pk, 8);
  run_scalarmult(c, s2);
  ec_copy(c, ad + 8, s1, 8); ec_copy(c, ad + 16, s2, 8);
  run_ecadd(c, ad);
  ec_copy(c, mo + o_in1, ad, 4); ec_copy(c, mo + o_in2, one, 4); ec_copy(c, mo + o_mod, ord, 4);
  run_bmmp(c, mo, 64, 4, 4, 4);
  int bad = 0;
  for (int i = 0; i < 4; i++) bad |= !fr_eq(W(mo + o_res + i), W(sig + i));
  if (bad && !c->err) c->err = S_ECDSA_R;
}

/* VerifySignature(20) signatureVerification.circom:177-191: pubkey[8], signature[8], hashed[256] | p256Verification */
static size_t sz_verifysig_ec(void) { return 8 + 8 + 256 + sz_ecdsa(); }
static void run_verifysig_ec(ctx_t *c, size_t b) {
  size_t e = b + 272;
  ec_copy(c, e, b, 8); ec_copy(c, e + 8, b + 8, 8); ec_copy(c, e + 16, b + 16, 256);
  run_ecdsa(c, e);
}
