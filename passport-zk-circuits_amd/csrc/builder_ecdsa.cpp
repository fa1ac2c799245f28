// ECDSA secp256r1 layout (SIGNATURE_TYPE 20): the VerifySignature(20) subtree
// (signatureVerification.circom:177-191 -> signatures/ecdsa.circom:18-87) as regions, and the
// descriptor programs of the table blocks (EllipticCurveDouble / EllipticCurveAdd /
// BigMultModP(64,4,4,4)), produced by running the shared walkers (ec_walk.hpp) symbolically.
#include "builder_impl.hpp"
#include "ec_walk.hpp"

namespace pzk {

namespace {

struct EcSym { int idx = -1; };

// Symbolic walker context: put() allocates the next table entry; signals get descriptors.
struct EcProgCtx {
  using V = EcSym;
  uint32_t* d;
  uint32_t size;
  uint32_t n = 0;
  bool bad = false;
  uint32_t& at(uint32_t off) {
    static uint32_t sink;
    if (off >= size) { bad = true; return sink; }
    return d[off];
  }
  V put(uint32_t off, const V&) { at(off) = ecd(ECD_COPY, n); return V{(int)n++}; }
  V put_hidden(const V&) { return V{(int)n++}; }
  void cp(uint32_t off, const V& v) {
    if (v.idx < 0) bad = true;
    else at(off) = ecd(ECD_COPY, (uint32_t)v.idx);
  }
  void bits(uint32_t off, const V& v, int L) {
    if (v.idx < 0) bad = true;
    for (int i = 0; i < L; i++) at(off + i) = ecd(ECD_BIT, (uint32_t)v.idx, (uint32_t)i);
  }
  void masks(uint32_t off, const V& v, int L) {  // sum[i] = v mod 2^(i+1)
    if (v.idx < 0) bad = true;
    for (int i = 0; i < L; i++) at(off + i) = ecd(ECD_MASK, (uint32_t)v.idx, (uint32_t)i);
  }
  V rec(int) const { return {}; }
  V u64(uint64_t) const { return {}; }
  V pow2(int) const { return {}; }
  V add(const V&, const V&) const { return {}; }
  V sub(const V&, const V&) const { return {}; }
  V mul(const V&, const V&) const { return {}; }
  V neg(const V&) const { return {}; }
  V sel(const V&, const V&, const V&) const { return {}; }
  V is_zero(const V&) const { return {}; }
  V bit(const V&, int) const { return {}; }
  V shr64_exact(const V&) const { return {}; }
  V inv_fr(const V&) const { return {}; }
  void check_zero(const V&) const {}
  void check_one(const V&) const {}
  void div_signed(const V*, int, int MCN, V& sign, V* k) const {
    sign = {};
    for (int i = 0; i < MCN - 3; i++) k[i] = {};
  }
  void divmod_n(const V*, V* q, V* r) const {
    for (int i = 0; i < 5; i++) q[i] = {};
    for (int i = 0; i < 4; i++) r[i] = {};
  }
};

uint32_t sz_n2b(int L) { return 2 * L + 1; }

}  // namespace

bool ec_programs(Layout& L, std::string& why) {
  L.ec_prog.clear();
  for (int t = 0; t < ECT_N; t++) {
    const uint32_t size = ec_type_size(t);
    std::vector<uint32_t> P(size, ecd(ECD_ZERO, 0));
    EcProgCtx c{P.data(), size};
    EcWalk<EcProgCtx> walk(c);
    walk.run(t);
    if (c.bad || c.n > EC_TABLE_MAX) {
      why = "internal: ECDSA table program " + std::to_string(t) + (c.bad ? " addresses a signal outside its block" : " too large");
      return false;
    }
    L.ec_prog_off[t] = (uint32_t)L.ec_prog.size();
    L.ec_tab_n[t] = c.n;
    L.ec_prog.insert(L.ec_prog.end(), P.begin(), P.end());
  }
  L.ec_tab_off.clear();
  for (int i = 0; i < ECT_N; i++) L.ec_ops[i].clear();
  uint32_t off = 0;
  for (int t = 0; t < EC_N_OPS + EC_N_MM; t++) {
    const int type = t >= EC_N_OPS ? ECT_MM : ec_op_is_dbl(t) ? ECT_DBL : ECT_ADD;
    L.ec_tab_off.push_back(off);
    L.ec_ops[type].push_back(t);
    off += L.ec_tab_n[type];
  }
  L.ec_tab_entries = off;
  return true;
}

// VerifySignature(20): pubkey[8], signature[8], hashed[256] | verifyECDSABits(64,4,A,B,P,256)
void ec_verify_regions(Builder& b, int IN_PK, int IN_SIG, int J_SA) {
  auto ect = [&](int t, int type) { b.region(RK_ECT, ec_type_size(type), {t, type}); };
  auto ecop = [&](int op) { ect(op, ec_op_is_dbl(op) ? ECT_DBL : ECT_ADD); };
  b.region(RK_INCOPY, 8, {IN_PK});
  b.region(RK_INCOPY, 8, {IN_SIG});
  b.region(RK_DIGEST, 256, {J_SA});
  // verifyECDSABits own: pubkey[2][4], signature[2][4], hashed[256] | hashedChunked[4], one[4], order[4], sinv[4]
  b.region(RK_INCOPY, 8, {IN_PK});
  b.region(RK_INCOPY, 8, {IN_SIG});
  b.region(RK_DIGEST, 256, {J_SA});
  b.region(RK_HCHUNK, 4, {J_SA});
  b.region(RK_EC_CONST, 4, {EC_K_ONE});
  b.region(RK_EC_CONST, 4, {EC_K_ORDER});
  b.region(RK_EC_U64, 4, {ECC_SINV});
  // bits2Num[i].in[63-j] = hashed[64 i + j] (ecdsa.circom:31-37)
  for (int i = 0; i < 4; i++) b.region(RK_BITS2NUM, sz_n2b(64), {64, 1, i * 64 + 63, -1, J_SA});
  b.region(RK_EC_CONST, 4, {EC_K_ORDER});  // getOrder
  // modInv (BigModInv): out[4] | in[4], modulus[4] | mult
  b.region(RK_EC_U64, 4, {ECC_SINV});
  b.region(RK_INCOPY, 4, {IN_SIG + 4});
  b.region(RK_EC_CONST, 4, {EC_K_ORDER});
  ect(EC_N_OPS + EC_MM_INV, ECT_MM);
  ect(EC_N_OPS + EC_MM_U1, ECT_MM);
  ect(EC_N_OPS + EC_MM_U2, ECT_MM);
  // scalarMult1 = EllipicCurveScalarGeneratorMult (curve.circom:672-906)
  b.region(RK_EC_U64, 8, {ECC_GM_RP + 8 * 30});  // out = resultingPoints[30]
  b.region(RK_EC_U64, 4, {ECC_U1});
  b.region(RK_EC_GM_RCC, 32 * 256 * 8);
  b.region(RK_EC_U64, 256, {ECC_GM_AP});
  b.region(RK_VALUE, 4 * 256, {-2});  // resultingPointsLeft/Left2/Right/Right2: declared, never assigned
  b.region(RK_EC_U64, 248, {ECC_GM_RP});
  b.region(RK_VALUE, 8, {-2});        // resultingPoints[31]
  for (int i = 0; i < 4; i++) b.region(RK_EC_N2B, sz_n2b(64), {0, ECC_U1 + i});
  b.region(RK_EC_B2N8, 32 * 17, {ECC_U1});
  b.region(RK_EC_CONST, 8, {EC_K_DUMMY});
  ecop(EC_OP_SD);
  b.region(RK_EC_GM_EQ, 32 * 256 * 6);
  b.region(RK_EC_GM_SUM, 32 * 8 * 512);
  for (int i = 0; i < 31; i++) {
    ecop(ec_op_gm_add(i));
    b.region(RK_EC_GM_STEP, 4 * 6 + 16 * 6, {i});
  }
  // scalarMult2 = EllipticCurveScalarMult(…,4) (curve.circom:356-494)
  b.region(RK_EC_U64, 8, {ECC_SM_RP + 8 * 64});
  b.region(RK_INCOPY, 8, {IN_PK});
  b.region(RK_EC_U64, 4, {ECC_U2});
  b.region(RK_EC_SBITS, 256, {ECC_U2});
  b.region(RK_EC_U64, 65 * 8, {ECC_SM_RP});
  b.region(RK_EC_U64, 64 * 8, {ECC_SM_AP});
  //   precompute (EllipticCurvePrecomputePipinger): out[16][2][4] | in[2][4] | getDummy, ops i = 2..15
  b.region(RK_EC_U64, 128, {ECC_PRE});
  b.region(RK_INCOPY, 8, {IN_PK});
  b.region(RK_EC_CONST, 8, {EC_K_DUMMY});
  for (int i = 2; i < 16; i++) ecop(ec_op_pre(i));
  b.region(RK_EC_CONST, 8, {EC_K_DUMMY});  // getDummy
  for (int i = 0; i < 4; i++) b.region(RK_EC_N2B, sz_n2b(64), {0, ECC_U2 + i});
  for (int w = 0; w < 64; w++) {
    b.region(RK_EC_SM_W0, sz_n2b(4) + 6, {w});
    if (w > 0) {
      ecop(ec_op_sm_dbl(4 * w - 4));
      b.region(RK_EC_SM_DSW, 8 * 6, {w});
      for (int j = 1; j < 4; j++) ecop(ec_op_sm_dbl(4 * w - 4 + j));
    }
    b.region(RK_EC_SM_SEL, 8 * 32 + 16 * 6, {w});
    if (w > 0) {
      ecop(ec_op_sm_add(w - 1));
      b.region(RK_EC_SM_RSW, 6 + 16 * 6, {w});
    }
  }
  ecop(EC_OP_FINAL);
  ect(EC_N_OPS + EC_MM_XN, ECT_MM);
}

}  // namespace pzk
