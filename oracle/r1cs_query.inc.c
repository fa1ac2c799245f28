/* oracle/r1cs_query.inc.c — QueryIdentity(80) constraints; included by r1cs_check.c.
 *
 * TEST INFRASTRUCTURE ONLY. Each `<==` / `===` of the query templates as the relation it compiles to, walked in
 * the O0 allocation of DESIGN.md §2 from the templates themselves (not from oracle/query.inc.c):
 *   queryIdentity.circom:37-229, dg1DataExtractor.circom:5-97, identityStateVerifier.circom:8-46,
 *   citizenshipCheck.circom:6-275, dateEncoder.circom:4-32, dateDecoder.circom:6-23, dateComparison.circom:5-55,
 *   dateComparisonEncoded.circom:6-28, dateComparisonEncodedNormalized.circom:13-49, comparators.circom:36-91.
 * IdentityStateVerifier's BabyPbk (undefined in the snapshot) is checked as the reference's
 * BabyjubjubBase8Multiplication, with BabyPbk's port names: in = scalar, Ax/Ay = out[0]/out[1].
 */

static int CKQ_TD1 = 0;  /* 0: QueryIdentity (queryIdentity.circom), 1: QueryIdentityTD1 (queryIdentityTD1.circom) */

static const uint32_t CKQ_COUNTRY[240] = {
#include "../passport-zk-circuits_amd/data/citizenship_codes.inc"
};

/* GreaterThan(L) comparators.circom:72-80: out | in[2] | LessThan(L) */
static size_t ck_greaterthan(ck_t *c, size_t b, int L) {
  const char *T = "GreaterThan comparators.circom";
  size_t lt = b + 3, sz = 3 + ck_lessthan(c, lt, L);
  EQ(S(c, lt + 1), S(c, b + 2), T, 77);
  EQ(S(c, lt + 2), S(c, b + 1), T, 78);
  EQ(S(c, b), S(c, lt), T, 79);
  return sz;
}
/* GreaterEqThan(L) comparators.circom:83-91: out | in[2] | LessThan(L) */
static size_t ck_greatereq(ck_t *c, size_t b, int L) {
  const char *T = "GreaterEqThan comparators.circom";
  size_t lt = b + 3, sz = 3 + ck_lessthan(c, lt, L);
  EQ(S(c, lt + 1), S(c, b + 2), T, 89);
  EQ(S(c, lt + 2), ADD(S(c, b + 1), KC(1)), T, 90);
  EQ(S(c, b), S(c, lt), T, 91);
  return sz;
}
/* ForceEqualIfEnabled comparators.circom:36-43: enabled, in[2] | IsEqual */
static size_t ck_feie(ck_t *c, size_t b) {
  const char *T = "ForceEqualIfEnabled comparators.circom";
  size_t ie = b + 3;
  ck_isequal(c, ie);
  EQ(S(c, ie + 1), S(c, b + 1), T, 40);
  EQ(S(c, ie + 2), S(c, b + 2), T, 40);
  EQ(MUL(SUB(KC(1), S(c, ie)), S(c, b)), fr_zero(), T, 42);
  return 9;
}
/* DateEncoder dateEncoder.circom:4-32: encoded | day month year | dayDecimals dayRest monthDecimals monthRest
 * yearDecimals yearRest dayEncoded monthEncoded yearEncoded */
static size_t ck_dateencoder(ck_t *c, size_t b) {
  const char *T = "DateEncoder dateUtilities/dateEncoder.circom";
  const int lines[3] = {13, 18, 23};
  for (int k = 0; k < 3; k++) {
    size_t dec = b + 4 + 2 * (size_t)k, rest = dec + 1, enc = b + 10 + (size_t)k;
    EQ(ADD(MUL(S(c, dec), KC(10)), S(c, rest)), S(c, b + 1 + k), T, lines[k]);
    EQ(S(c, enc), ADD(ADD(MUL(S(c, dec), KC(256)), S(c, rest)), KC(12336)), T, 26 + k);
  }
  EQ(S(c, b), ADD(ADD(MUL(S(c, b + 12), P2[32]), MUL(S(c, b + 11), P2[16])), S(c, b + 10)), T, 29);
  return 13;
}
/* DateDecoder dateDecoder.circom:6-23: day month year | dateEncoded | DateEncoder */
static size_t ck_datedecoder(ck_t *c, size_t b) {
  const char *T = "DateDecoder dateUtilities/dateDecoder.circom";
  size_t de = b + 4;
  ck_dateencoder(c, de);
  for (int k = 0; k < 3; k++) EQ(S(c, de + 1 + k), S(c, b + k), T, 18 + k);
  EQ(S(c, de), S(c, b + 3), T, 22);
  return 17;
}
/* DateIsLess dateComparison.circom:5-55: out | firstDay secondDay firstMonth secondMonth firstYear secondYear |
 * isYearLess isMonthLess isDayLess isYearEqual isMonthEqual isLess1 isLess2 temp isLess3 | yearLess monthLess
 * dayLess yearEqual monthEqual greaterThen */
static size_t ck_dateisless(ck_t *c, size_t b) {
  const char *T = "DateIsLess dateUtilities/dateComparison.circom";
  size_t o = b + 16, lt[3], eq[2];
  for (int k = 0; k < 3; k++) { lt[k] = o; o += ck_lessthan(c, o, 8); }
  for (int k = 0; k < 2; k++) { eq[k] = o; o += ck_isequal(c, o); }
  size_t gt = o;
  o += ck_greaterthan(c, gt, 3);
  const size_t fy = b + 5, fm = b + 3, fd = b + 1;  /* second = first + 1 */
  EQ(S(c, lt[0] + 1), S(c, fy), T, 18); EQ(S(c, lt[0] + 2), S(c, fy + 1), T, 19); EQ(S(c, b + 7), S(c, lt[0]), T, 20);
  EQ(S(c, lt[1] + 1), S(c, fm), T, 23); EQ(S(c, lt[1] + 2), S(c, fm + 1), T, 24); EQ(S(c, b + 8), S(c, lt[1]), T, 25);
  EQ(S(c, lt[2] + 1), S(c, fd), T, 28); EQ(S(c, lt[2] + 2), S(c, fd + 1), T, 29); EQ(S(c, b + 9), S(c, lt[2]), T, 30);
  EQ(S(c, eq[0] + 1), S(c, fy), T, 35); EQ(S(c, eq[0] + 2), S(c, fy + 1), T, 36); EQ(S(c, b + 10), S(c, eq[0]), T, 37);
  EQ(S(c, eq[1] + 1), S(c, fm), T, 40); EQ(S(c, eq[1] + 2), S(c, fm + 1), T, 41); EQ(S(c, b + 11), S(c, eq[1]), T, 42);
  EQ(S(c, b + 12), S(c, b + 7), T, 45);
  EQ(S(c, b + 13), MUL(S(c, b + 10), S(c, b + 8)), T, 46);
  EQ(S(c, b + 14), MUL(S(c, b + 10), S(c, b + 11)), T, 47);
  EQ(S(c, b + 15), MUL(S(c, b + 14), S(c, b + 9)), T, 48);
  EQ(S(c, gt + 1), ADD(ADD(S(c, b + 12), S(c, b + 13)), S(c, b + 15)), T, 51);
  EQ(S(c, gt + 2), fr_zero(), T, 52);
  EQ(S(c, b), S(c, gt), T, 54);
  return o - b;
}
/* EncodedDateIsLess dateComparisonEncoded.circom:6-28: out | first second | firstDateDecoder secondDateDecoder
 * dateIsLess */
static size_t ck_edil(ck_t *c, size_t b) {
  const char *T = "EncodedDateIsLess dateUtilities/dateComparisonEncoded.circom";
  size_t d1 = b + 3, d2 = d1 + ck_datedecoder(c, d1), dl = d2 + ck_datedecoder(c, d2);
  size_t sz = dl + ck_dateisless(c, dl) - b;
  EQ(S(c, d1 + 3), S(c, b + 1), T, 13);
  EQ(S(c, d2 + 3), S(c, b + 2), T, 16);
  for (int k = 0; k < 3; k++) {  /* day, month, year */
    EQ(S(c, dl + 1 + 2 * k), S(c, d1 + k), T, 20 + 2 * k);
    EQ(S(c, dl + 2 + 2 * k), S(c, d2 + k), T, 21 + 2 * k);
  }
  EQ(S(c, b), S(c, dl), T, 27);
  return sz;
}
/* EncodedDateIsLessNormalized dateComparisonEncodedNormalized.circom:13-49: out | first second currentDate |
 * CENTURY | firstDateDecoder secondDateDecoder firstDateNormalization secondDateNormalization dateIsLess */
static size_t ck_ediln(ck_t *c, size_t b) {
  const char *T = "EncodedDateIsLessNormalized dateUtilities/dateComparisonEncodedNormalized.circom";
  size_t d1 = b + 5, d2 = d1 + ck_datedecoder(c, d1), n1 = d2 + ck_datedecoder(c, d2), n2 = n1 + ck_edil(c, n1),
         dl = n2 + ck_edil(c, n2);
  size_t sz = dl + ck_dateisless(c, dl) - b;
  EQ(S(c, d1 + 3), S(c, b + 1), T, 22);
  EQ(S(c, d2 + 3), S(c, b + 2), T, 25);
  EQ(S(c, n1 + 1), S(c, b + 1), T, 29); EQ(S(c, n1 + 2), S(c, b + 3), T, 30);
  EQ(S(c, n2 + 1), S(c, b + 2), T, 34); EQ(S(c, n2 + 2), S(c, b + 3), T, 35);
  EQ(S(c, b + 4), KC(100), T, 39);
  for (int k = 0; k < 2; k++) {  /* day, month */
    EQ(S(c, dl + 1 + 2 * k), S(c, d1 + k), T, 41 + 2 * k);
    EQ(S(c, dl + 2 + 2 * k), S(c, d2 + k), T, 42 + 2 * k);
  }
  EQ(S(c, dl + 5), ADD(S(c, d1 + 2), MUL(S(c, b + 4), S(c, n1))), T, 45);
  EQ(S(c, dl + 6), ADD(S(c, d2 + 2), MUL(S(c, b + 4), S(c, n2))), T, 46);
  EQ(S(c, b), S(c, dl), T, 48);
  return sz;
}
/* DG1DataExtractor dg1DataExtractor.circom:5-97: 8 outputs | dg1[744] | Bits2Num encoders;
 * DG1TD1DataExtractor dg1TD1DataExtractor.circom:5-107: 9 outputs | dg1[760] | Bits2Num encoders */
static size_t ck_dgx(ck_t *c, size_t b) {
  const char *T = CKQ_TD1 ? "DG1TD1DataExtractor identityManagement/dg1TD1DataExtractor.circom"
                          : "DG1DataExtractor identityManagement/dg1DataExtractor.circom";
  static const int L3[8] = {48, 48, 248, 64, 24, 24, 8, 72}, SH3[8] = {496, 560, 80, 328, 472, 56, 552, 392},
                   IN3[8] = {27, 36, 49, 53, 64, 74, 84, 94}, OUT3[8] = {29, 39, 55, 56, 66, 76, 86, 97};
  static const int L1[9] = {48, 48, 240, 24, 24, 8, 72, 88, 16}, SH1[9] = {280, 344, 520, 400, 56, 336, 80, 160, 40},
                   IN1[9] = {26, 35, 45, 55, 65, 75, 85, 95, 105}, OUT1[9] = {28, 37, 47, 57, 67, 77, 87, 97, 107};
  const int NF = CKQ_TD1 ? 9 : 8, DG = CKQ_TD1 ? 760 : 744;
  const int *L = CKQ_TD1 ? L1 : L3, *SH = CKQ_TD1 ? SH1 : SH3, *IN_LINE = CKQ_TD1 ? IN1 : IN3, *OUT_LINE = CKQ_TD1 ? OUT1 : OUT3;
  size_t o = b + NF + DG;
  for (int k = 0; k < NF; k++) {
    size_t e = o;
    o += ck_bits2num(c, e, L[k]);
    for (int i = 0; i < L[k]; i++) EQ(S(c, e + 1 + L[k] - 1 - i), S(c, b + NF + SH[k] + i), T, IN_LINE[k]);
    EQ(S(c, b + k), S(c, e), T, OUT_LINE[k]);
  }
  return o - b;
}
/* CitizenshipCheck citizenshipCheck.circom:6-275: citizenship blacklist | validCheck[241] bitmask[240] | num2bits
 * (isEqual[i] isEqual2[i]) */
static size_t ck_citizenship(ck_t *c, size_t b) {
  const char *T = "CitizenshipCheck identityManagement/citizenshipCheck.circom";
  size_t vc = b + 2, bm = vc + 241, nb = bm + 240, o = nb + ck_num2bits(c, nb, 240);
  EQ(S(c, vc), fr_zero(), T, 258);
  EQ(S(c, nb + 240), S(c, b + 1), T, 260);
  for (int i = 0; i < 240; i++) {
    size_t e1 = o, e2 = e1 + ck_isequal(c, e1);
    o = e2 + ck_isequal(c, e2);
    EQ(S(c, bm + i), S(c, nb + 239 - i), T, 264);
    EQ(S(c, e1 + 1), KC(CKQ_COUNTRY[i]), T, 266);
    EQ(S(c, e1 + 2), S(c, b), T, 267);
    EQ(S(c, e2 + 1), KC(1), T, 269);
    EQ(S(c, e2 + 2), S(c, bm + i), T, 270);
    EQ(MUL(S(c, e1), S(c, e2)), fr_zero(), T, 271);
    EQ(S(c, vc + i + 1), ADD(S(c, e1), S(c, vc + i)), T, 272);
  }
  EQ(S(c, vc + 240), KC(1), T, 274);
  return o - b;
}
/* IdentityStateVerifier(80) identityStateVerifier.circom:8-46: skIdentity pkPassHash dgCommit identityCounter timestamp
 * idStateRoot idStateSiblings[80] | treePosition | babyPbk pkIdentityHasher positionHasher valueHasher smtVerifier */
static size_t ck_isv(ck_t *c, size_t b) {
  const char *T = "IdentityStateVerifier identityManagement/identityStateVerifier.circom";
  size_t tp = b + 86, bjj = b + 87, pkh = bjj + ck_bjjmul(c, bjj), posh = pkh + ck_poseidon(c, pkh, 2),
         valh = posh + ck_poseidon(c, posh, 2), smt = valh + ck_poseidon(c, valh, 3);
  size_t sz = smt + ck_smt(c, smt, 80) - b;
  EQ(S(c, bjj + 2), S(c, b), T, 20);
  EQ(S(c, pkh + 1), S(c, bjj), T, 24);
  EQ(S(c, pkh + 2), S(c, bjj + 1), T, 25);
  EQ(S(c, posh + 1), S(c, b + 1), T, 29);
  EQ(S(c, posh + 2), S(c, pkh), T, 30);
  EQ(S(c, tp), S(c, posh), T, 31);
  for (int k = 0; k < 3; k++) EQ(S(c, valh + 1 + k), S(c, b + 2 + k), T, 35 + k);
  EQ(S(c, smt + 3), S(c, tp), T, 41);
  EQ(S(c, smt + 1), S(c, b + 5), T, 42);
  EQ(S(c, smt + 2), S(c, valh), T, 43);
  for (int i = 0; i < 80; i++) EQ(S(c, smt + 4 + i), S(c, b + 6 + i), T, 44);
  EQ(S(c, smt), KC(1), T, 46);
  return sz;
}
/* QueryIdentity(80) queryIdentity.circom:37-229 as main: [1] nullifier birthDate expirationDate name nameResidual
 * nationality citizenship sex documentNumber | 842 inputs (declaration order) | eventDataSquare | subcomponents */
static size_t ck_queryid(ck_t *c, size_t b) {
  const char *T = CKQ_TD1 ? "QueryIdentity identityManagement/queryIdentityTD1.circom"
                          : "QueryIdentity identityManagement/queryIdentity.circom";
  enum { EVID, EVDATA, ROOT, SEL, CUR, TSLO, TSHI, ICLO, ICHI, BDLO, BDHI, EDLO, EDHI, CMASK, SK, PKPASS, DG1 };
  const int DGL = CKQ_TD1 ? 760 : 744, SIB = DG1 + DGL, TS = SIB + 80, IC = TS + 1, NIN = IC + 1, NOUT = CKQ_TD1 ? 10 : 9;
  const int NF = CKQ_TD1 ? 9 : 8;
  const size_t in = b + (size_t)NOUT;
#define QIN(k) (in + (size_t)(k))
  size_t o = in + (size_t)NIN + 1;
  EQ(S(c, in + NIN), MUL(S(c, QIN(EVDATA)), S(c, QIN(EVDATA))), T, 209);
  size_t selb = o;
  o += ck_num2bits(c, selb, 18);
  EQ(S(c, selb + 18), S(c, QIN(SEL)), T, 81);
  size_t dgx = o;
  o += ck_dgx(c, dgx);
  for (int i = 0; i < DGL; i++) EQ(S(c, dgx + NF + i), S(c, QIN(DG1 + i)), T, 86);
  if (!CKQ_TD1) {
    static const int OSEL[8] = {1, 2, 3, 3, 4, 5, 6, 7};
    for (int k = 0; k < 8; k++) EQ(S(c, b + 1 + k), MUL(S(c, dgx + k), S(c, selb + OSEL[k])), T, 88 + k);
  } else {  /* documentNumberHasher, personalNumberHasher (:89-95), outputs (:97-105) */
    size_t dnh = o;
    o += ck_poseidon(c, dnh, 1);
    EQ(S(c, dnh + 1), S(c, dgx + 6), T, 91);
    size_t pnh = o;
    o += ck_poseidon(c, pnh, 1);
    EQ(S(c, pnh + 1), S(c, dgx + 7), T, 95);
    for (int k = 0; k < 6; k++) EQ(S(c, b + 1 + k), MUL(S(c, dgx + k), S(c, selb + 1 + k)), T, 97 + k);
    EQ(S(c, b + 7), MUL(S(c, dnh), S(c, selb + 7)), T, 103);
    EQ(S(c, b + 8), MUL(S(c, pnh), S(c, selb + 16)), T, 104);
    EQ(S(c, b + 9), MUL(S(c, dgx + 8), S(c, selb + 17)), T, 105);
  }
  size_t skh = o;
  o += ck_poseidon(c, skh, 1);
  EQ(S(c, skh + 1), S(c, QIN(SK)), T, 100);
  size_t nul = o;
  o += ck_poseidon(c, nul, 3);
  EQ(S(c, nul + 1), S(c, QIN(SK)), T, 103);
  EQ(S(c, nul + 2), S(c, skh), T, 104);
  EQ(S(c, nul + 3), S(c, QIN(EVID)), T, 105);
  EQ(S(c, b), MUL(S(c, nul), S(c, selb)), T, 107);
  const int CX[4] = {TS, TS, IC, IC}, CY[4] = {TSLO, TSHI, ICLO, ICHI}, CL[4] = {112, 122, 133, 143};
  for (int k = 0; k < 4; k++) {
    size_t cb = o;
    o += (k & 1) ? ck_lessthan(c, cb, 64) : ck_greatereq(c, cb, 64);
    EQ(S(c, cb + 1), S(c, QIN(CX[k])), T, CL[k]);
    EQ(S(c, cb + 2), S(c, QIN(CY[k])), T, CL[k] + 1);
    size_t fe = o;
    o += ck_feie(c, fe);
    EQ(S(c, fe + 1), S(c, cb), T, CL[k] + 4);
    EQ(S(c, fe + 2), KC(1), T, CL[k] + 5);
    EQ(S(c, fe), S(c, selb + 8 + k), T, CL[k] + 6);
  }
  for (int k = 0; k < 2; k++) {  /* expiration date bounds: first/second (:153-169) */
    size_t eb = o;
    o += ck_edil(c, eb);
    EQ(S(c, eb + 1), k ? S(c, dgx + 1) : S(c, QIN(EDLO)), T, 153 + 10 * k);
    EQ(S(c, eb + 2), k ? S(c, QIN(EDHI)) : S(c, dgx + 1), T, 154 + 10 * k);
    size_t fe = o;
    o += ck_feie(c, fe);
    EQ(S(c, fe + 1), S(c, eb), T, 157 + 10 * k);
    EQ(S(c, fe + 2), KC(1), T, 158 + 10 * k);
    EQ(S(c, fe), S(c, selb + 12 + k), T, 159 + 10 * k);
  }
  for (int k = 0; k < 2; k++) {  /* birth date bounds (:173-191) */
    size_t eb = o;
    o += ck_ediln(c, eb);
    EQ(S(c, eb + 1), k ? S(c, dgx) : S(c, QIN(BDLO)), T, 173 + 11 * k);
    EQ(S(c, eb + 2), k ? S(c, QIN(BDHI)) : S(c, dgx), T, 174 + 11 * k);
    EQ(S(c, eb + 3), S(c, QIN(CUR)), T, 175 + 11 * k);
    size_t fe = o;
    o += ck_feie(c, fe);
    EQ(S(c, fe + 1), S(c, eb), T, 178 + 11 * k);
    EQ(S(c, fe + 2), KC(1), T, 179 + 11 * k);
    EQ(S(c, fe), S(c, selb + 14 + k), T, 180 + 11 * k);
  }
  size_t dgh = o;  /* created before dg1Chunking[i] */
  o += ck_poseidon(c, dgh, 5);
  const int CH = CKQ_TD1 ? 190 : 186;
  for (int i = 0; i < 4; i++) {
    size_t ch = o;
    o += ck_bits2num(c, ch, CH);
    for (int j = 0; j < CH; j++) EQ(S(c, ch + 1 + j), S(c, QIN(DG1 + i * CH + j)), T, 199);
    EQ(S(c, dgh + 1 + i), S(c, ch), T, 201);
  }
  size_t skh2 = o;
  o += ck_poseidon(c, skh2, 1);
  EQ(S(c, skh2 + 1), S(c, QIN(SK)), T, 205);
  EQ(S(c, dgh + 5), S(c, skh2), T, 206);
  size_t isv = o;
  o += ck_isv(c, isv);
  EQ(S(c, isv), S(c, QIN(SK)), T, 213);
  EQ(S(c, isv + 1), S(c, QIN(PKPASS)), T, 214);
  EQ(S(c, isv + 2), S(c, dgh), T, 215);
  EQ(S(c, isv + 3), S(c, QIN(IC)), T, 216);
  EQ(S(c, isv + 4), S(c, QIN(TS)), T, 217);
  EQ(S(c, isv + 5), S(c, QIN(ROOT)), T, 219);
  for (int i = 0; i < 80; i++) EQ(S(c, isv + 6 + i), S(c, QIN(SIB + i)), T, 220);
  size_t cit = o;
  o += ck_citizenship(c, cit);
  EQ(S(c, cit), S(c, dgx + (CKQ_TD1 ? 4 : 5)), T, 226);
  EQ(S(c, cit + 1), S(c, QIN(CMASK)), T, 227);
  /* main's inputs are read by the wiring above; the 14 public inputs each feed some constraint */
#undef QIN
  return o - b;
}
