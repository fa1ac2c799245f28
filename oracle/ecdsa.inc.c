/* oracle/ecdsa.inc.c — ECDSA (SIGNATURE_TYPE 20, 21, 24, 25) part of the CPU restatement.
 *
 * TEST INFRASTRUCTURE ONLY (included by witness_oracle.c; see its header). Restates, template by
 * template and in the O0 layout of DESIGN.md §2, for CHUNK_NUMBER N chunks of CHUNK_SIZE CS bits
 * (20 / 21: 4 x 64, 24: 7 x 32, 25: 6 x 64; signatureVerification.circom:77-116):
 *   VerifySignature(20..25)        signatureVerification.circom:177-263
 *   verifyECDSABits(CS,N,A,B,P,N*CS) signatures/ecdsa.circom:18-87
 *   EllipicCurveGetOrder / EllipticCurveGetDummy  ec/get.circom:79-195
 *   EllipticCurveDouble / EllipticCurveAdd         ec/curve.circom:281-345
 *   PointOnCurve / PointOnTangent / PointOnLine    ec/curve.circom:107-245
 *   EllipticCurvePrecomputePipinger               ec/curve.circom:249-272
 *   EllipticCurveScalarMult(…,4)                   ec/curve.circom:356-494
 *   EllipicCurveScalarGeneratorMult                ec/curve.circom:680-906
 *   BigModInv                                      bigInt/bigInt.circom:344-368
 *   BigIntIsZeroModP                               bigInt/bigIntComparators.circom:158-212
 *   BigAddOverflow / BigSubModOverflow / ScalarMultOverflow  bigInt/bigIntOverflow.circom:22-111
 * and the witness-time functions they call (bigIntFunc.circom: prod_mod, long_add_mod,
 * long_sub_mod, mod_inv/mod_exp, long_div, reduce_overflow_signed). Those functions work on chunk
 * arrays; every value they return here is canonical (< the modulus), so they are computed on 64-bit
 * words and converted to chunks at the signal boundary.
 *
 * SIGNATURE_TYPE 22 (brainpoolP320r1, 5 x 64) and 23 (secp192r1, 3 x 64) are not restated: their
 * verifyECDSABits reads hashed[i * CHUNK_SIZE + j] for N * CS = 320 / 192 bits of a 256 / 160-bit
 * hash (ecdsa.circom:31-37), an out-of-bounds access circom rejects — no circuit with them compiles.
 */

/* ------------------------------------------------------------ curve constants */
/* A, B, P as chunk arrays: signatureVerification.circom:179-182 (20: secp256r1), :193-196 (21: brainpoolP256r1),
 * :235-238 (24: secp224r1), :249-252 (25: brainpoolP384r1); order: get.circom:157 / :154 / :183 / :165;
 * dummyPoint: get.circom:92-93 / :88-89 / :124-125 / :102-103 */
#define EC_MAXN 7
typedef struct {
  int nl, cs; /* CHUNK_NUMBER, CHUNK_SIZE */
  uint64_t A[EC_MAXN], B[EC_MAXN], P[EC_MAXN], N[EC_MAXN], D[2][EC_MAXN];
} ec_curve_t;
static const ec_curve_t EC_CURVES[4] = {
    {4, 64,
     {18446744073709551612ULL, 4294967295ULL, 0ULL, 18446744069414584321ULL},
     {4309448131093880907ULL, 7285987128567378166ULL, 12964664127075681980ULL, 6540974713487397863ULL},
     {18446744073709551615ULL, 4294967295ULL, 0ULL, 18446744069414584321ULL},
     {17562291160714782033ULL, 13611842547513532036ULL, 18446744073709551615ULL, 18446744069414584320ULL},
     {{4148137498610012746ULL, 51237685452122967ULL, 6555942389409504868ULL, 799804747332166731ULL},
      {13395177781894339167ULL, 1107697421929919296ULL, 6228258783500845564ULL, 11862546499924939746ULL}}},
    {4, 64,
     {16810331318623712729ULL, 18122579188607900780ULL, 17219079075415130087ULL, 9032542404991529047ULL},
     {7767825457231955894ULL, 10773760575486288334ULL, 17523706096862592191ULL, 2800214691157789508ULL},
     {2311270323689771895ULL, 7943213001558335528ULL, 4496292894210231666ULL, 12248480212390422972ULL},
     {10384753744809580199ULL, 10104242082523752183ULL, 4496292894210231665ULL, 12248480212390422972ULL},
     {{5870538370169240658ULL, 13064052279558318326ULL, 1032222391323187885ULL, 10478252910764369874ULL},
      {9125809427693782222ULL, 4479624720887462683ULL, 4313457861005768495ULL, 11848267593595748038ULL}}},
    {7, 32,
     {4294967294ULL, 4294967295ULL, 4294967295ULL, 4294967294ULL, 4294967295ULL, 4294967295ULL, 4294967295ULL},
     {592838580ULL, 655046979ULL, 3619674298ULL, 1346678967ULL, 4114690646ULL, 201634731ULL, 3020229253ULL},
     {1ULL, 0ULL, 0ULL, 4294967295ULL, 4294967295ULL, 4294967295ULL, 4294967295ULL},
     {1549543997ULL, 333261125ULL, 3770216510ULL, 4294907554ULL, 4294967295ULL, 4294967295ULL, 4294967295ULL},
     {{2477436510ULL, 406882550ULL, 2884834286ULL, 2269163287ULL, 3636783260ULL, 3699382582ULL, 912817446ULL},
      {582933619ULL, 1778719645ULL, 3780674687ULL, 3008581200ULL, 3586474874ULL, 866709652ULL, 3566930607ULL}}},
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
       16161625210166602047ULL, 946254366129831718ULL}}}};
/* SIGNATURE_TYPE -> curve index (-1: not an ECDSA type this restatement covers) */
static int ec_index(int sig) { return sig == 20 ? 0 : sig == 21 ? 1 : sig == 24 ? 2 : sig == 25 ? 3 : -1; }

/* the curve of the witness being computed (ec_select): EN chunks of ECS bits, EFB = EN * ECS field bits */
static const ec_curve_t *EC = &EC_CURVES[0];
static int EN = 4, ECS = 64, EFB = 256;
static const uint64_t *EC_A = EC_CURVES[0].A, *EC_B = EC_CURVES[0].B, *EC_P = EC_CURVES[0].P, *EC_N = EC_CURVES[0].N;

/* get_g_pow_stride8_table_<curve> (ec/powers/<curve>pows.circom:3): [EFB / 8][256][2][EN] chunks, one u64 each,
 * from data/<p256|bp256|p224|bp384>_gpow8.bin (tools/gen_ec_tables.py) */
static uint64_t *EC_GPOW_T[4] = {NULL, NULL, NULL, NULL};
static uint64_t *EC_GPOW = NULL;
static size_t ec_table_words(int curve) {
  const ec_curve_t *C = &EC_CURVES[curve];
  return (size_t)(C->nl * C->cs / 8) * 256 * 2 * C->nl;
}
int orc_load_ec_table(int curve, const char *path) {
  if (curve < 0 || curve > 3) return -3;
  FILE *f = fopen(path, "rb");
  if (!f) return -1;
  size_t n = ec_table_words(curve);
  uint64_t *t = malloc(n * sizeof(uint64_t));
  size_t got = fread(t, sizeof(uint64_t), n, f);
  int extra = fgetc(f) != EOF;
  fclose(f);
  if (got != n || extra) { free(t); return -2; }
  free(EC_GPOW_T[curve]);
  EC_GPOW_T[curve] = t;
  return 0;
}
int orc_load_p256(const char *path) { return orc_load_ec_table(0, path); }
static void ec_select(int curve) {
  EC = &EC_CURVES[curve];
  EN = EC->nl; ECS = EC->cs; EFB = EN * ECS;
  EC_A = EC->A; EC_B = EC->B; EC_P = EC->P; EC_N = EC->N;
  EC_GPOW = EC_GPOW_T[curve];
}
#define GPOW(i, j, a, k) EC_GPOW[((((size_t)(i) * 256 + (j)) * 2 + (a)) * EN) + (k)]

/* ------------------------------------- witness-time big-int functions, on words */
#define ECW 6 /* 64-bit words of the largest field (384 bits) */
typedef struct { uint64_t l[ECW]; } ecb;

static uint64_t ec_chunk_mask(void) { return ECS == 64 ? ~0ULL : (1ULL << ECS) - 1; }
static ecb ecb_of_chunks(const uint64_t *ch) { /* sum ch[i] 2^(CS i) */
  ecb r; memset(&r, 0, sizeof r);
  for (int i = 0; i < EN; i++) {
    int off = ECS * i;
    r.l[off >> 6] |= ch[i] << (off & 63);
  }
  return r;
}
static void ecb_to_chunks(const ecb *a, uint64_t *ch) {
  for (int i = 0; i < EN; i++) {
    int off = ECS * i;
    ch[i] = (a->l[off >> 6] >> (off & 63)) & ec_chunk_mask();
  }
}
static int ecb_gt(const ecb *a, const ecb *b) { /* long_gt bigIntFunc.circom:126-140 */
  for (int i = ECW - 1; i >= 0; i--) {
    if (a->l[i] > b->l[i]) return 1;
    if (a->l[i] < b->l[i]) return 0;
  }
  return 0;
}
static int ecb_zero(const ecb *a) {
  uint64_t o = 0;
  for (int i = 0; i < ECW; i++) o |= a->l[i];
  return !o;
}
static ecb ecb_sub(const ecb *a, const ecb *b) { /* long_sub :142-167 */
  ecb r; uint64_t br = 0;
  for (int i = 0; i < ECW; i++) {
    u128 d = (u128)a->l[i] - b->l[i] - br;
    r.l[i] = (uint64_t)d; br = (uint64_t)(d >> 64) & 1;
  }
  return r;
}
static ecb ecb_add(const ecb *a, const ecb *b, uint64_t *carry) { /* long_add :503-514 */
  ecb r; uint64_t c = 0;
  for (int i = 0; i < ECW; i++) {
    u128 s = (u128)a->l[i] + b->l[i] + c;
    r.l[i] = (uint64_t)s; c = (uint64_t)(s >> 64);
  }
  *carry = c;
  return r;
}
static ecb ecb_small(uint64_t v) { ecb r; memset(&r, 0, sizeof r); r.l[0] = v; return r; }
static int ecb_words(const ecb *m) { int nb = ECW; while (nb > 1 && m->l[nb - 1] == 0) nb--; return nb; }
/* prod_mod :524-528 = remainder of the exact product */
static ecb ec_prod_mod(const ecb *a, const ecb *b, const ecb *m) {
  uint64_t pr[2 * ECW] = {0}, q[2 * ECW + 1], r[ECW];
  for (int i = 0; i < ECW; i++) {
    uint64_t cy = 0;
    for (int j = 0; j < ECW; j++) {
      u128 t = (u128)a->l[i] * b->l[j] + pr[i + j] + cy;
      pr[i + j] = (uint64_t)t; cy = (uint64_t)(t >> 64);
    }
    pr[i + ECW] = cy;
  }
  int nb = ecb_words(m);
  mp_divmod(pr, 2 * ECW, m->l, nb, q, r);
  ecb o; memset(&o, 0, sizeof o);
  for (int i = 0; i < nb; i++) o.l[i] = r[i];
  return o;
}
/* long_add_mod :497-501 (a, b < m: the sum's remainder) */
static ecb ec_add_mod(const ecb *a, const ecb *b, const ecb *m) {
  uint64_t cy;
  ecb s = ecb_add(a, b, &cy); /* a + b may carry out of 384 bits (brainpoolP384r1) */
  if (cy || !ecb_gt(m, &s)) s = ecb_sub(&s, m);
  return s;
}
/* long_sub_mod :516-522: B > A ? A + (P - B) : A - B */
static ecb ec_sub_mod(const ecb *a, const ecb *b, const ecb *m) {
  if (ecb_gt(b, a)) {
    uint64_t cy;
    ecb t = ecb_sub(m, b);
    return ecb_add(a, &t, &cy);
  }
  return ecb_sub(a, b);
}
/* mod_inv :430-466 (0 -> 0, else a^(m-2) by mod_exp :385-420) */
static ecb ec_mod_inv(const ecb *a, const ecb *m) {
  if (ecb_zero(a)) return *a;
  ecb two = ecb_small(2), e = ecb_sub(m, &two), out = ecb_small(1);
  int top = ECW * 64 - 1;
  while (top > 0 && !((e.l[top >> 6] >> (top & 63)) & 1)) top--;
  for (int i = top; i >= 0; i--) {
    if ((e.l[i >> 6] >> (i & 63)) & 1) out = ec_prod_mod(&out, a, m);
    if (i > 0) out = ec_prod_mod(&out, &out, m);
  }
  return out;
}

typedef struct { ecb x, y; } ecpt;

/* EllipticCurveDouble witness values curve.circom:286-292 */
static ecpt ec_double_val(const ecpt *p) {
  ecb Pm = ecb_of_chunks(EC_P), A = ecb_of_chunks(EC_A), three = ecb_small(3);
  ecb xx = ec_prod_mod(&p->x, &p->x, &Pm), t = ec_prod_mod(&three, &xx, &Pm);
  ecb num = ec_add_mod(&A, &t, &Pm), den = ec_add_mod(&p->y, &p->y, &Pm);
  ecb inv = ec_mod_inv(&den, &Pm), lam = ec_prod_mod(&num, &inv, &Pm);
  ecb l2 = ec_prod_mod(&lam, &lam, &Pm), x2 = ec_add_mod(&p->x, &p->x, &Pm);
  ecpt r;
  r.x = ec_sub_mod(&l2, &x2, &Pm);
  ecb d = ec_sub_mod(&p->x, &r.x, &Pm), ld = ec_prod_mod(&lam, &d, &Pm);
  r.y = ec_sub_mod(&ld, &p->y, &Pm);
  return r;
}
/* EllipticCurveAdd witness values curve.circom:319-325 */
static ecpt ec_add_val(const ecpt *p, const ecpt *q) {
  ecb Pm = ecb_of_chunks(EC_P);
  ecb dy = ec_sub_mod(&q->y, &p->y, &Pm), dx = ec_sub_mod(&q->x, &p->x, &Pm);
  ecb inv = ec_mod_inv(&dx, &Pm), lam = ec_prod_mod(&dy, &inv, &Pm), l2 = ec_prod_mod(&lam, &lam, &Pm);
  ecpt r;
  ecb t = ec_sub_mod(&l2, &p->x, &Pm);
  r.x = ec_sub_mod(&t, &q->x, &Pm);
  ecb d = ec_sub_mod(&p->x, &r.x, &Pm), ld = ec_prod_mod(&lam, &d, &Pm);
  r.y = ec_sub_mod(&ld, &p->y, &Pm);
  return r;
}

/* point <-> 2N consecutive witness chunks ([axis][chunk]) */
static ecpt ec_get(ctx_t *c, size_t at) {
  uint64_t x[EC_MAXN], y[EC_MAXN];
  for (int i = 0; i < EN; i++) { x[i] = W(at + i).l[0]; y[i] = W(at + EN + i).l[0]; }
  ecpt p = {ecb_of_chunks(x), ecb_of_chunks(y)};
  return p;
}
static void ec_put(ctx_t *c, size_t at, const ecpt *p) {
  uint64_t x[EC_MAXN], y[EC_MAXN];
  ecb_to_chunks(&p->x, x); ecb_to_chunks(&p->y, y);
  for (int i = 0; i < EN; i++) { W(at + i) = fr_u64(x[i]); W(at + EN + i) = fr_u64(y[i]); }
}
static void ec_copy(ctx_t *c, size_t dst, size_t src, int n) { for (int i = 0; i < n; i++) W(dst + i) = W(src + i); }
static void ec_consts(ctx_t *c, size_t at, const uint64_t *v, int n) { for (int i = 0; i < n; i++) W(at + i) = fr_u64(v[i]); }
static void ec_dummy(ctx_t *c, size_t at) { ec_consts(c, at, EC->D[0], EN); ec_consts(c, at + EN, EC->D[1], EN); }

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
    if (i != N - 1) v = fr_add(v, POW2[ECS]);
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
   * signed sum S = sum in[i] 2^(n i); sign = 1 iff S >= 0, reduced = |S| in MCN chunks. */
  enum { AW = 40 };
  uint64_t acc[AW] = {0};
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
    acc_shifted(acc, AW, mag, n * i, neg);
  }
  int positive = !(acc[AW - 1] >> 63);
  if (!positive) { /* negate */
    uint64_t cy = 1;
    for (int w = 0; w < AW; w++) { u128 s = (u128)(~acc[w]) + cy; acc[w] = (uint64_t)s; cy = (uint64_t)(s >> 64); }
  }
  W(sign) = fr_u64((uint64_t)positive);
  /* long_div(n, CNM, DIV-1, reduced, modulus) on words */
  uint64_t modc[16], modw[16] = {0}, q[AW + 1], r[16];
  for (int i = 0; i < CNM; i++) modc[i] = W(mod + i).l[0];
  for (int i = 0; i < CNM; i++) {
    int off = n * i;
    modw[off >> 6] |= modc[i] << (off & 63);
  }
  int nb = (n * CNM + 63) / 64;
  while (nb > 1 && modw[nb - 1] == 0) nb--;
  int na = (n * MCN + 63) / 64;
  if (na < nb) na = nb;
  memset(q, 0, sizeof q);
  mp_divmod(acc, na, modw, nb, q, r);
  for (int i = 0; i < DIV; i++) {
    W(k + i) = fr_u64(word_chunk(q, n, i));
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
/* PointOnCurve curve.circom:107-137: in[2][N] | squareX, cubeX, squareY, coefMult,
 * isZeroModP(CS, 3 CS + 2N, 3N - 2, 3N, N) */
static size_t sz_poncurve(void) {
  const int N = EN;
  return 2 * (size_t)N + 3 * sz_bmo(N, N) + sz_bmo(2 * N - 1, N) + sz_bizmp(ECS, 3 * ECS + 2 * N, 3 * N - 2, 3 * N, N);
}
static void run_poncurve(ctx_t *c, size_t b) {
  const int N = EN;
  size_t sx = b + 2 * N, cx = sx + sz_bmo(N, N), sy = cx + sz_bmo(2 * N - 1, N), cm = sy + sz_bmo(N, N),
         iz = cm + sz_bmo(N, N);
  for (int i = 0; i < N; i++) { W(sx + 2 * N - 1 + i) = W(b + i); W(sx + 3 * N - 1 + i) = W(b + i); }
  run_bmo(c, sx, N, N);
  for (int i = 0; i < 2 * N - 1; i++) W(cx + 3 * N - 2 + i) = W(sx + i);
  for (int i = 0; i < N; i++) W(cx + 5 * N - 3 + i) = W(b + i);
  run_bmo(c, cx, 2 * N - 1, N);
  for (int i = 0; i < N; i++) { W(sy + 2 * N - 1 + i) = W(b + N + i); W(sy + 3 * N - 1 + i) = W(b + N + i); }
  run_bmo(c, sy, N, N);
  for (int i = 0; i < N; i++) { W(cm + 2 * N - 1 + i) = W(b + i); W(cm + 3 * N - 1 + i) = fr_u64(EC_A[i]); }
  run_bmo(c, cm, N, N);
  for (int i = 0; i < 3 * N - 2; i++) {
    fr_t v = W(cx + i);
    if (i < 2 * N - 1) v = fr_sub(fr_add(v, W(cm + i)), W(sy + i));
    if (i < N) v = fr_add(v, fr_u64(EC_B[i]));
    W(iz + i) = v;
  }
  ec_consts(c, iz + 3 * N - 2, EC_P, N);
  run_bizmp(c, iz, ECS, 3 * ECS + 2 * N, 3 * N - 2, 3 * N, N);
}
/* PointOnTangent curve.circom:144-190: in1[2][N], in2[2][N] | squareX, scalarMult, bigAdd, bigSub,
 * rightMult, scalarMult2, bigAdd2, leftMult, isZeroModP(CS, 3 CS + 2N, 3N - 2, 3N + 1, N) */
static size_t sz_pontangent(void) {
  const int N = EN;
  return 4 * (size_t)N + sz_bmo(N, N) + sz_smo(2 * N - 1) + sz_bao(2 * N - 1, N) + sz_bsmo(N) + sz_bmo(2 * N - 1, N) +
         sz_smo(N) + sz_bao(N, N) + sz_bmo(N, N) + sz_bizmp(ECS, 3 * ECS + 2 * N, 3 * N - 2, 3 * N + 1, N);
}
static void run_pontangent(ctx_t *c, size_t b) {
  const int N = EN, M = 2 * N - 1;
  size_t x1 = b, y1 = b + N, x2 = b + 2 * N, y2 = b + 3 * N;
  size_t sx = b + 4 * N, sm = sx + sz_bmo(N, N), ba = sm + sz_smo(M), bs = ba + sz_bao(M, N), rm = bs + sz_bsmo(N),
         sm2 = rm + sz_bmo(M, N), ba2 = sm2 + sz_smo(N), lm = ba2 + sz_bao(N, N), iz = lm + sz_bmo(N, N);
  for (int i = 0; i < N; i++) { W(sx + M + i) = W(x1 + i); W(sx + M + N + i) = W(x1 + i); }
  run_bmo(c, sx, N, N);
  for (int i = 0; i < M; i++) W(sm + M + i) = W(sx + i);
  W(sm + 2 * M) = fr_u64(3);
  run_smo(c, sm, M);
  for (int i = 0; i < M; i++) W(ba + M + i) = W(sm + i);
  ec_consts(c, ba + 2 * M, EC_A, N);
  run_bao(c, ba, M, N);
  for (int i = 0; i < N; i++) { W(bs + N + i) = W(x1 + i); W(bs + 2 * N + i) = W(x2 + i); }
  ec_consts(c, bs + 3 * N, EC_P, N);
  run_bsmo(c, bs, N);
  for (int i = 0; i < M; i++) W(rm + M + N - 1 + i) = W(ba + i);
  for (int i = 0; i < N; i++) W(rm + 2 * M + N - 1 + i) = W(bs + i);
  run_bmo(c, rm, M, N);
  for (int i = 0; i < N; i++) W(sm2 + N + i) = W(y1 + i);
  W(sm2 + 2 * N) = fr_u64(2);
  run_smo(c, sm2, N);
  for (int i = 0; i < N; i++) { W(ba2 + N + i) = W(y1 + i); W(ba2 + 2 * N + i) = W(y2 + i); }
  run_bao(c, ba2, N, N);
  for (int i = 0; i < N; i++) { W(lm + M + i) = W(ba2 + i); W(lm + M + N + i) = W(sm2 + i); }
  run_bmo(c, lm, N, N);
  for (int i = 0; i < 3 * N - 2; i++) W(iz + i) = i < M ? fr_sub(W(rm + i), W(lm + i)) : W(rm + i);
  ec_consts(c, iz + 3 * N - 2, EC_P, N);
  run_bizmp(c, iz, ECS, 3 * ECS + 2 * N, 3 * N - 2, 3 * N + 1, N);
}
/* PointOnLine curve.circom:197-245: in1, in2, in3 | bigAdd, bigSub, bigSub2, bigSub3, leftMult,
 * rightMult, isZeroModP(CS, 2 CS + 2N, 2N - 1, 2N + 1, N) */
static size_t sz_ponline(void) {
  const int N = EN;
  return 6 * (size_t)N + sz_bao(N, N) + 3 * sz_bsmo(N) + 2 * sz_bmo(N, N) +
         sz_bizmp(ECS, 2 * ECS + 2 * N, 2 * N - 1, 2 * N + 1, N);
}
static void run_ponline(ctx_t *c, size_t b) {
  const int N = EN, M = 2 * N - 1;
  size_t x1 = b, y1 = b + N, x2 = b + 2 * N, y2 = b + 3 * N, x3 = b + 4 * N, y3 = b + 5 * N;
  size_t ba = b + 6 * N, s1 = ba + sz_bao(N, N), s2 = s1 + sz_bsmo(N), s3 = s2 + sz_bsmo(N), lm = s3 + sz_bsmo(N),
         rm = lm + sz_bmo(N, N), iz = rm + sz_bmo(N, N);
  for (int i = 0; i < N; i++) { W(ba + N + i) = W(y1 + i); W(ba + 2 * N + i) = W(y3 + i); }
  run_bao(c, ba, N, N);
  size_t subs[3] = {s1, s2, s3}, a1[3] = {x2, y2, x1}, a2[3] = {x1, y1, x3};
  for (int s = 0; s < 3; s++) {
    for (int i = 0; i < N; i++) { W(subs[s] + N + i) = W(a1[s] + i); W(subs[s] + 2 * N + i) = W(a2[s] + i); }
    ec_consts(c, subs[s] + 3 * N, EC_P, N);
    run_bsmo(c, subs[s], N);
  }
  for (int i = 0; i < N; i++) { W(lm + M + i) = W(ba + i); W(lm + M + N + i) = W(s1 + i); }
  run_bmo(c, lm, N, N);
  for (int i = 0; i < N; i++) { W(rm + M + i) = W(s2 + i); W(rm + M + N + i) = W(s3 + i); }
  run_bmo(c, rm, N, N);
  for (int i = 0; i < M; i++) W(iz + i) = fr_sub(W(lm + i), W(rm + i));
  ec_consts(c, iz + M, EC_P, N);
  run_bizmp(c, iz, ECS, 2 * ECS + 2 * N, M, 2 * N + 1, N);
}

/* ------------------------------------------------------------ point ops */
/* EllipticCurveDouble curve.circom:281-310: out[2][N] | in[2][N] | onTangentCheck, onCurveCheck */
static size_t sz_ecdbl(void) { return 4 * (size_t)EN + sz_pontangent() + sz_poncurve(); }
static void run_ecdbl(ctx_t *c, size_t b) {
  const int P2 = 2 * EN;
  ecpt p = ec_get(c, b + P2), r = ec_double_val(&p);
  ec_put(c, b, &r);
  size_t t = b + 2 * P2, k = t + sz_pontangent();
  ec_copy(c, t, b + P2, P2); ec_copy(c, t + P2, b, P2);
  run_pontangent(c, t);
  ec_copy(c, k, b, P2);
  run_poncurve(c, k);
}
/* EllipticCurveAdd curve.circom:314-345: out[2][N] | in1[2][N], in2[2][N] | onCurveCheck, onLineCheck */
static size_t sz_ecadd(void) { return 6 * (size_t)EN + sz_poncurve() + sz_ponline(); }
static void run_ecadd(ctx_t *c, size_t b) {
  const int P2 = 2 * EN;
  ecpt p = ec_get(c, b + P2), q = ec_get(c, b + 2 * P2), r = ec_add_val(&p, &q);
  ec_put(c, b, &r);
  size_t k = b + 3 * P2, l = k + sz_poncurve();
  ec_copy(c, k, b, P2);
  run_poncurve(c, k);
  ec_copy(c, l, b + P2, 2 * P2); ec_copy(c, l + 2 * P2, b, P2);
  run_ponline(c, l);
}

/* EllipticCurvePrecomputePipinger(…,4) curve.circom:249-272: out[16][2][N] | in[2][N] | getDummy,
 * then doublers[i/2-1] (even i) / adders[i/2-1] (odd i) in order i = 2..15 */
static size_t sz_precomp(void) { return 18 * 2 * (size_t)EN + 7 * sz_ecdbl() + 7 * sz_ecadd(); }
static void run_precomp(ctx_t *c, size_t b) {
  const int P2 = 2 * EN;
  size_t in = b + 16 * P2, gd = in + P2, p = gd + P2;
  ec_dummy(c, gd);
  ec_copy(c, b, gd, P2);
  ec_copy(c, b + P2, in, P2);
  for (int i = 2; i < 16; i++) {
    if (i % 2 == 0) {
      ec_copy(c, p + P2, b + (size_t)P2 * (i / 2), P2);
      run_ecdbl(c, p);
      ec_copy(c, b + (size_t)P2 * i, p, P2);
      p += sz_ecdbl();
    } else {
      ec_copy(c, p + P2, b + P2, P2); ec_copy(c, p + 2 * P2, b + (size_t)P2 * (i - 1), P2);
      run_ecadd(c, p);
      ec_copy(c, b + (size_t)P2 * i, p, P2);
      p += sz_ecadd();
    }
  }
}

/* EllipticCurveScalarMult(CS,N,A,B,P,4) curve.circom:356-494 (WINS = N CS / 4 windows):
 * out[2][N] | in[2][N], scalar[N] | scalarBits[N CS], resultingPoints[WINS+1][2][N], additionPoints[WINS][2][N]
 * | precompute, getDummy, num2Bits[N], then per window w: bits2Num[w], isZeroResult[w],
 *   (w>0: doublers[4w-4], doubleSwitcher[w-1][2N], doublers[4w-3..4w-1]), getSum[w][2N],
 *   partsEqual[w][16], (w>0: adders[w-1], isZeroAddition[w], (resultSwitcherAddition,
 *   resultSwitcherDoubling)[w-1][2N]) */
static size_t sz_win(int w) {
  const size_t P2 = 2 * (size_t)EN;
  size_t s = sz_bits2num(4) + 6 + P2 * (1 + 16 + 15) + 16 * 6;
  if (w > 0) s += 4 * sz_ecdbl() + P2 * 6 + sz_ecadd() + 6 + 2 * P2 * 6;
  return s;
}
static size_t sz_scalarmult(void) {
  const size_t P2 = 2 * (size_t)EN;
  const int WINS = EFB / 4;
  size_t s = 2 * P2 + EN + EFB + (WINS + 1) * P2 + WINS * P2 + sz_precomp() + P2 + (size_t)EN * sz_num2bits(ECS);
  for (int w = 0; w < WINS; w++) s += sz_win(w);
  return s;
}
static void run_scalarmult(ctx_t *c, size_t b) {
  const int P2 = 2 * EN, WINS = EFB / 4;
  size_t in = b + P2, sc = in + P2, bits = sc + EN, rp = bits + EFB, ap = rp + (size_t)(WINS + 1) * P2,
         pre = ap + (size_t)WINS * P2, gd = pre + sz_precomp(), n2b = gd + P2, p = n2b + (size_t)EN * sz_num2bits(ECS);
  ec_copy(c, pre + 16 * (size_t)P2, in, P2);
  run_precomp(c, pre);
  ec_dummy(c, gd);
  for (int i = 0; i < EN; i++) {
    size_t nb = n2b + (size_t)i * sz_num2bits(ECS);
    W(nb + ECS) = W(sc + i);
    run_num2bits(c, nb, ECS);
    for (int j = 0; j < ECS; j++) W(bits + EFB - ECS * (i + 1) + j) = W(nb + ECS - 1 - j);
  }
  ec_copy(c, rp, pre, P2);
  size_t prev_dbl = 0;
  for (int w = 0; w < WINS; w++) {
    size_t b2n = p; p += sz_bits2num(4);
    for (int j = 0; j < 4; j++) W(b2n + 1 + j) = W(bits + 4 * w + 3 - j);
    run_bits2num(c, b2n, 4);
    size_t izr = p; p += 6;
    W(izr + 1) = W(rp + (size_t)P2 * w); W(izr + 2) = W(gd);
    run_isequal(c, izr);
    if (w > 0) {
      size_t d0 = p; p += sz_ecdbl();
      size_t dsw = p; p += (size_t)P2 * 6;
      for (int q = 0; q < P2; q++) {
        size_t s = dsw + 6 * (size_t)q;
        W(s + 2) = W(izr); W(s + 3) = W(gd + q); W(s + 4) = W(rp + (size_t)P2 * w + q);
        run_switcher(c, s);
        W(d0 + P2 + q) = W(s + 1);
      }
      run_ecdbl(c, d0);
      prev_dbl = d0;
      for (int j = 1; j < 4; j++) {
        size_t d = p; p += sz_ecdbl();
        ec_copy(c, d + P2, prev_dbl, P2);
        run_ecdbl(c, d);
        prev_dbl = d;
      }
    }
    size_t gs = p; p += (size_t)P2 * 32;
    size_t pe = p; p += 16 * 6;
    for (int k = 0; k < 16; k++) {
      size_t e = pe + 6 * (size_t)k;
      W(e + 1) = fr_u64((uint64_t)k); W(e + 2) = W(b2n);
      run_isequal(c, e);
      for (int q = 0; q < P2; q++) W(gs + 32 * (size_t)q + 1 + k) = mulg(W(e), W(pre + (size_t)P2 * k + q));
    }
    for (int q = 0; q < P2; q++) {
      run_getsum(c, gs + 32 * (size_t)q, 16);
      W(ap + (size_t)P2 * w + q) = W(gs + 32 * (size_t)q);
    }
    if (w == 0) {
      ec_copy(c, rp + P2, ap, P2);
    } else {
      size_t ad = p; p += sz_ecadd();
      ec_copy(c, ad + P2, prev_dbl, P2); ec_copy(c, ad + 2 * P2, ap + (size_t)P2 * w, P2);
      run_ecadd(c, ad);
      size_t iza = p; p += 6;
      W(iza + 1) = W(ap + (size_t)P2 * w); W(iza + 2) = W(gd);
      run_isequal(c, iza);
      size_t rs = p; p += 2 * (size_t)P2 * 6;
      for (int q = 0; q < P2; q++) {
        size_t sa = rs + 12 * (size_t)q, sd = sa + 6;
        W(sa + 2) = W(iza); W(sa + 3) = W(ad + q); W(sa + 4) = W(prev_dbl + q);
        run_switcher(c, sa);
        W(sd + 2) = W(izr); W(sd + 3) = W(ap + (size_t)P2 * w + q); W(sd + 4) = W(sa);
        run_switcher(c, sd);
        W(rp + (size_t)P2 * (w + 1) + q) = W(sd + 1);
      }
    }
  }
  ec_copy(c, b, rp + (size_t)WINS * P2, P2);
}

/* EllipicCurveScalarGeneratorMult(CS,N,…) curve.circom:680-906 (PARTS = N CS / 8):
 * out[2][N] | scalar[N] | resultCoordinateComputation[PARTS][256][2][N], additionPoints[PARTS][2][N],
 *   resultingPointsLeft, Left2, Right, Right2 (never assigned), resultingPoints [PARTS][2][N]
 * | num2bits[N], bits2num[PARTS], getDummy, getSecondDummy, equal[PARTS][256], getSumOfNElements[PARTS][2][N],
 *   per i < PARTS-1: adders[i], isFirstDummyLeft, isSecondDummyLeft, isFirstDummyRight, isSecondDummyRight,
 *   (switcherRight, switcherLeft)[axis][j] */
static size_t sz_genmult(void) {
  const size_t P2 = 2 * (size_t)EN;
  const int PARTS = EFB / 8;
  return P2 + EN + (size_t)PARTS * 256 * P2 + 5 * (size_t)PARTS * P2 + (size_t)PARTS * P2 + (size_t)EN * sz_num2bits(ECS) +
         (size_t)PARTS * sz_bits2num(8) + P2 + sz_ecdbl() + (size_t)PARTS * 256 * 6 + (size_t)PARTS * P2 * 512 +
         (size_t)(PARTS - 1) * (sz_ecadd() + 4 * 6 + 2 * P2 * 6);
}
static void run_genmult(ctx_t *c, size_t b) {
  const int P2 = 2 * EN, PARTS = EFB / 8;
  size_t sc = b + P2, rcc = sc + EN, ap = rcc + (size_t)PARTS * 256 * P2, rp = ap + 5 * (size_t)PARTS * P2,
         n2b = rp + (size_t)PARTS * P2, b2n = n2b + (size_t)EN * sz_num2bits(ECS), gd = b2n + (size_t)PARTS * sz_bits2num(8),
         sd = gd + P2, eq = sd + sz_ecdbl(), gs = eq + (size_t)PARTS * 256 * 6, p = gs + (size_t)PARTS * P2 * 512;
  for (int i = 0; i < EN; i++) {
    size_t nb = n2b + (size_t)i * sz_num2bits(ECS);
    W(nb + ECS) = W(sc + i);
    run_num2bits(c, nb, ECS);
  }
  for (int i = 0; i < PARTS; i++) {
    size_t bn = b2n + (size_t)i * sz_bits2num(8);
    for (int j = 0; j < 8; j++)
      W(bn + 1 + j) = W(n2b + (size_t)((i * 8 + j) / ECS) * sz_num2bits(ECS) + (i * 8 + j) % ECS);
    run_bits2num(c, bn, 8);
  }
  ec_dummy(c, gd);
  ec_copy(c, sd + P2, gd, P2);
  run_ecdbl(c, sd);
  for (int i = 0; i < PARTS; i++) {
    size_t bn = b2n + (size_t)i * sz_bits2num(8);
    for (int j = 0; j < 256; j++) {
      size_t e = eq + 6 * ((size_t)i * 256 + j);
      W(e + 1) = fr_u64((uint64_t)j); W(e + 2) = W(bn);
      run_isequal(c, e);
      for (int a = 0; a < 2; a++)
        for (int k = 0; k < EN; k++) {
          fr_t v;
          if (j == 0) v = (i % 2 == 0) ? W(gd + EN * a + k) : W(sd + EN * a + k);
          else v = fr_u64(GPOW(i, j, a, k));
          W(rcc + (((size_t)i * 256 + j) * 2 + a) * EN + k) = mulg(W(e), v);
        }
    }
  }
  for (int i = 0; i < PARTS; i++)
    for (int a = 0; a < 2; a++)
      for (int k = 0; k < EN; k++) {
        size_t g = gs + 512 * (((size_t)i * 2 + a) * EN + k);
        for (int s = 0; s < 256; s++) W(g + 1 + s) = W(rcc + (((size_t)i * 256 + s) * 2 + a) * EN + k);
        run_getsum(c, g, 256);
        W(ap + (size_t)P2 * i + EN * a + k) = W(g);
      }
  for (int i = 0; i < PARTS - 1; i++) {
    size_t ad = p; p += sz_ecadd();
    size_t fl = p, sl = p + 6, fr_ = p + 12, sr = p + 18; p += 24;
    size_t sw = p; p += 2 * (size_t)P2 * 6;
    size_t left = i == 0 ? ap : rp + (size_t)P2 * (i - 1), right = ap + (size_t)P2 * (i + 1);
    W(fl + 1) = W(gd); W(sl + 1) = W(sd); W(fr_ + 1) = W(gd); W(sr + 1) = W(sd);
    W(fl + 2) = W(left); W(sl + 2) = W(left); W(fr_ + 2) = W(right); W(sr + 2) = W(right);
    ec_copy(c, ad + P2, left, P2); ec_copy(c, ad + 2 * P2, right, P2);
    run_ecadd(c, ad);
    run_isequal(c, fl); run_isequal(c, sl); run_isequal(c, fr_); run_isequal(c, sr);
    for (int q = 0; q < P2; q++) {
      size_t swr = sw + 12 * (size_t)q, swl = swr + 6;
      W(swr + 2) = fr_add(W(sr), W(fr_)); W(swr + 3) = W(ad + q); W(swr + 4) = W(left + q);
      run_switcher(c, swr);
      W(swl + 2) = fr_add(W(sl), W(fl)); W(swl + 3) = W(right + q); W(swl + 4) = W(swr);
      run_switcher(c, swl);
      W(rp + (size_t)P2 * i + q) = W(swl + 1);
    }
  }
  ec_copy(c, b, rp + (size_t)(PARTS - 2) * P2, P2);
}

/* BigMultModP(CS,N,N,N) signal offsets: div[N+1] | mod[N] | in1[N], in2[N], modulus[N] */
#define BM_RES(N) ((size_t)(N) + 1)
#define BM_IN1(N) (2 * (size_t)(N) + 1)
#define BM_IN2(N) (3 * (size_t)(N) + 1)
#define BM_MOD(N) (4 * (size_t)(N) + 1)

/* BigModInv(CS,N) bigInt.circom:344-368: out[N] | in[N], modulus[N] | mult */
static size_t sz_bigmodinv(void) { return 3 * (size_t)EN + sz_bmmp(ECS, EN, EN, EN); }
static void run_bigmodinv(ctx_t *c, size_t b) {
  const int N = EN;
  uint64_t ac[EC_MAXN], mc[EC_MAXN], oc[EC_MAXN];
  for (int i = 0; i < N; i++) { ac[i] = W(b + N + i).l[0]; mc[i] = W(b + 2 * N + i).l[0]; }
  ecb a = ecb_of_chunks(ac), m = ecb_of_chunks(mc), inv = ec_mod_inv(&a, &m);
  ecb_to_chunks(&inv, oc);
  for (int i = 0; i < N; i++) W(b + i) = fr_u64(oc[i]);
  size_t mm = b + 3 * N;
  for (int i = 0; i < N; i++) {
    W(mm + BM_IN1(N) + i) = W(b + N + i); W(mm + BM_IN2(N) + i) = W(b + i); W(mm + BM_MOD(N) + i) = W(b + 2 * N + i);
  }
  run_bmmp(c, mm, ECS, N, N, N);
  int bad = !fr_eq(W(mm + BM_RES(N)), ONE());
  for (int i = 1; i < N; i++) bad |= !fr_is_zero(W(mm + BM_RES(N) + i));
  if (bad && !c->err) c->err = S_ECDSA_INV;
}

/* verifyECDSABits(CS,N,A,B,P,N CS) ecdsa.circom:18-87:
 * pubkey[2][N], signature[2][N], hashed[N CS] | hashedChunked[N], one[N], order[N], sinv[N]
 * | bits2Num[N], getOrder, modInv, mult, mult2, scalarMult1, scalarMult2, add, modOrder */
static size_t sz_ecdsa(void) {
  const int N = EN;
  return 4 * (size_t)N + EFB + 4 * (size_t)N + (size_t)N * sz_bits2num(ECS) + N + sz_bigmodinv() +
         3 * sz_bmmp(ECS, N, N, N) + sz_genmult() + sz_scalarmult() + sz_ecadd();
}
static void run_ecdsa(ctx_t *c, size_t b) {
  const int N = EN;
  size_t pk = b, sig = b + 2 * N, hashed = b + 4 * N, hc = hashed + EFB, one = hc + N, ord = one + N, sinv = ord + N;
  size_t p = sinv + N, b2n = p; p += (size_t)N * sz_bits2num(ECS);
  size_t go = p; p += N;
  size_t mi = p; p += sz_bigmodinv();
  size_t m1 = p; p += sz_bmmp(ECS, N, N, N);
  size_t m2 = p; p += sz_bmmp(ECS, N, N, N);
  size_t s1 = p; p += sz_genmult();
  size_t s2 = p; p += sz_scalarmult();
  size_t ad = p; p += sz_ecadd();
  size_t mo = p;
  for (int i = 0; i < N; i++) {
    size_t bn = b2n + (size_t)i * sz_bits2num(ECS);
    for (int j = 0; j < ECS; j++) W(bn + 1 + ECS - 1 - j) = W(hashed + i * ECS + j);
    run_bits2num(c, bn, ECS);
    W(hc + N - 1 - i) = W(bn);
  }
  W(one) = ONE();
  ec_consts(c, go, EC_N, N);
  ec_copy(c, ord, go, N);
  ec_copy(c, mi + N, sig + N, N); ec_copy(c, mi + 2 * N, ord, N);
  run_bigmodinv(c, mi);
  ec_copy(c, sinv, mi, N);
  ec_copy(c, m1 + BM_IN1(N), sinv, N); ec_copy(c, m1 + BM_IN2(N), hc, N); ec_copy(c, m1 + BM_MOD(N), ord, N);
  run_bmmp(c, m1, ECS, N, N, N);
  ec_copy(c, m2 + BM_IN1(N), sinv, N); ec_copy(c, m2 + BM_IN2(N), sig, N); ec_copy(c, m2 + BM_MOD(N), ord, N);
  run_bmmp(c, m2, ECS, N, N, N);
  ec_copy(c, s1 + 2 * N, m1 + BM_RES(N), N);
  run_genmult(c, s1);
  ec_copy(c, s2 + 4 * N, m2 + BM_RES(N), N); ec_copy(c, s2 + 2 * N, pk, 2 * N);
  run_scalarmult(c, s2);
  ec_copy(c, ad + 2 * N, s1, 2 * N); ec_copy(c, ad + 4 * N, s2, 2 * N);
  run_ecadd(c, ad);
  ec_copy(c, mo + BM_IN1(N), ad, N); ec_copy(c, mo + BM_IN2(N), one, N); ec_copy(c, mo + BM_MOD(N), ord, N);
  run_bmmp(c, mo, ECS, N, N, N);
  int bad = 0;
  for (int i = 0; i < N; i++) bad |= !fr_eq(W(mo + BM_RES(N) + i), W(sig + i));
  if (bad && !c->err) c->err = S_ECDSA_R;
}

/* VerifySignature(20 / 21 / 24 / 25) signatureVerification.circom:177-263:
 * pubkey[2N], signature[2N], hashed[N CS] | verification */
static size_t sz_verifysig_ec(void) { return 4 * (size_t)EN + EFB + sz_ecdsa(); }
static void run_verifysig_ec(ctx_t *c, size_t b) {
  size_t e = b + 4 * (size_t)EN + EFB;
  ec_copy(c, e, b, 4 * EN + EFB);
  run_ecdsa(c, e);
}
