// ECDSA layout (SIGNATURE_TYPE 20, 21, 24, 25): the VerifySignature(SIG) subtree
// (signatureVerification.circom:177-263 -> signatures/ecdsa.circom:18-87) as regions, and the
// descriptor programs of the table blocks (EllipticCurveDouble / EllipticCurveAdd /
// BigMultModP(CS,N,N,N)), produced by running the shared walkers (ec_walk.hpp) symbolically.
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
  V shr_exact(const V&, int) const { return {}; }
  V inv_fr(const V&) const { return {}; }
  void check_zero(const V&) const {}
  void check_one(const V&) const {}
  int nl = 4;
  void div_signed(const V*, int, int MCN, V& sign, V* k) const {
    sign = {};
    for (int i = 0; i < MCN - nl + 1; i++) k[i] = {};
  }
  void divmod_n(const V*, V* q, V* r) const {
    for (int i = 0; i < nl + 1; i++) q[i] = {};
    for (int i = 0; i < nl; i++) r[i] = {};
  }
};

template <int CV>
bool ec_program(int t, std::vector<uint32_t>& P, uint32_t& n) {
  const uint32_t size = ec_type_size(EC_GEO[CV], t);
  P.assign(size, ecd(ECD_ZERO, 0));
  EcProgCtx c{P.data(), size};
  c.nl = EC_GEO[CV].nl;
  EcWalk<EcProgCtx, CV> walk(c);
  walk.run(t);
  n = c.n;
  return !c.bad;
}

uint32_t sz_n2b(int L) { return 2 * L + 1; }

}  // namespace

bool ec_programs(Layout& L, std::string& why) {
  const int cv = L.reg.ec_curve;
  const EcGeo& G = EC_GEO[cv];
  L.ec_prog.clear();
  for (int t = 0; t < ECT_N; t++) {
    std::vector<uint32_t> P;
    uint32_t n = 0;
    const bool ok = cv == 0 ? ec_program<0>(t, P, n) : cv == 1 ? ec_program<1>(t, P, n) : cv == 2 ? ec_program<2>(t, P, n)
                                                                                         : ec_program<3>(t, P, n);
    if (!ok || n > EC_TABLE_MAX[cv]) {
      why = "internal: ECDSA table program " + std::to_string(t) +
            (!ok ? " addresses a signal outside its block" : " too large (" + std::to_string(n) + " entries)");
      return false;
    }
    L.ec_prog_off[t] = (uint32_t)L.ec_prog.size();
    L.ec_tab_n[t] = n;
    L.ec_prog.insert(L.ec_prog.end(), P.begin(), P.end());
  }
  L.ec_tab_off.clear();
  for (int i = 0; i < ECT_N; i++) L.ec_ops[i].clear();
  uint32_t off = 0;
  for (int t = 0; t < G.n_ops + EC_N_MM; t++) {
    const int type = t >= G.n_ops ? ECT_MM : ec_op_is_dbl(G, t) ? ECT_DBL : ECT_ADD;
    L.ec_tab_off.push_back(off);
    L.ec_ops[type].push_back(t);
    off += L.ec_tab_n[type];
  }
  L.ec_tab_entries = off;
  return true;
}

// VerifySignature(SIG): pubkey[2N], signature[2N], hashed[N CS] | verifyECDSABits(CS,N,A,B,P,N CS)
void ec_verify_regions(Builder& b, int cv, int IN_PK, int IN_SIG, int J_SA) {
  const EcGeo& G = EC_GEO[cv];
  const int N = G.nl, CS = G.cs, F = G.fb, P2 = 2 * N;
  auto ect = [&](int t, int type) { b.region(RK_ECT, ec_type_size(G, type), {t, type}); };
  auto ecop = [&](int op) { ect(op, ec_op_is_dbl(G, op) ? ECT_DBL : ECT_ADD); };
  b.region(RK_INCOPY, P2, {IN_PK});
  b.region(RK_INCOPY, P2, {IN_SIG});
  b.region(RK_DIGEST, F, {J_SA});
  // verifyECDSABits own: pubkey[2][N], signature[2][N], hashed[F] | hashedChunked[N], one[N], order[N], sinv[N]
  b.region(RK_INCOPY, P2, {IN_PK});
  b.region(RK_INCOPY, P2, {IN_SIG});
  b.region(RK_DIGEST, F, {J_SA});
  b.region(RK_HCHUNK, N, {J_SA, N, CS});
  b.region(RK_EC_CONST, N, {EC_K_ONE});
  b.region(RK_EC_CONST, N, {EC_K_ORDER});
  b.region(RK_EC_U64, N, {G.c_sinv});
  // bits2Num[i].in[CS-1-j] = hashed[CS i + j] (ecdsa.circom:31-37)
  for (int i = 0; i < N; i++) b.region(RK_BITS2NUM, sz_n2b(CS), {CS, 1, i * CS + CS - 1, -1, J_SA});
  b.region(RK_EC_CONST, N, {EC_K_ORDER});  // getOrder
  // modInv (BigModInv): out[N] | in[N], modulus[N] | mult
  b.region(RK_EC_U64, N, {G.c_sinv});
  b.region(RK_INCOPY, N, {IN_SIG + N});
  b.region(RK_EC_CONST, N, {EC_K_ORDER});
  ect(G.n_ops + EC_MM_INV, ECT_MM);
  ect(G.n_ops + EC_MM_U1, ECT_MM);
  ect(G.n_ops + EC_MM_U2, ECT_MM);
  // scalarMult1 = EllipicCurveScalarGeneratorMult (curve.circom:680-906)
  b.region(RK_EC_U64, P2, {G.c_gm_rp + P2 * (G.parts - 2)});  // out = resultingPoints[PARTS-2]
  b.region(RK_EC_U64, N, {G.c_u1});
  b.region(RK_EC_GM_RCC, (uint64_t)G.parts * 256 * P2);
  b.region(RK_EC_U64, G.parts * P2, {G.c_gm_ap});
  b.region(RK_VALUE, 4 * G.parts * P2, {-2});  // resultingPointsLeft/Left2/Right/Right2: declared, never assigned
  b.region(RK_EC_U64, (G.parts - 1) * P2, {G.c_gm_rp});
  b.region(RK_VALUE, P2, {-2});                 // resultingPoints[PARTS-1]
  for (int i = 0; i < N; i++) b.region(RK_EC_N2B, sz_n2b(CS), {0, G.c_u1 + i, CS});
  b.region(RK_EC_B2N8, G.parts * 17, {G.c_u1});
  b.region(RK_EC_CONST, P2, {EC_K_DUMMY});
  ecop(EC_OP_SD);
  b.region(RK_EC_GM_EQ, (uint64_t)G.parts * 256 * 6);
  b.region(RK_EC_GM_SUM, (uint64_t)G.parts * P2 * 512);
  for (int i = 0; i < G.parts - 1; i++) {
    ecop(ec_op_gm_add(i));
    b.region(RK_EC_GM_STEP, 4 * 6 + 2 * P2 * 6, {i});
  }
  // scalarMult2 = EllipticCurveScalarMult(…,4) (curve.circom:356-494)
  b.region(RK_EC_U64, P2, {G.c_sm_rp + P2 * G.wins});
  b.region(RK_INCOPY, P2, {IN_PK});
  b.region(RK_EC_U64, N, {G.c_u2});
  b.region(RK_EC_SBITS, F, {G.c_u2});
  b.region(RK_EC_U64, (G.wins + 1) * P2, {G.c_sm_rp});
  b.region(RK_EC_U64, G.wins * P2, {G.c_sm_ap});
  //   precompute (EllipticCurvePrecomputePipinger): out[16][2][N] | in[2][N] | getDummy, ops i = 2..15
  b.region(RK_EC_U64, 16 * P2, {G.c_pre});
  b.region(RK_INCOPY, P2, {IN_PK});
  b.region(RK_EC_CONST, P2, {EC_K_DUMMY});
  for (int i = 2; i < 16; i++) ecop(ec_op_pre(G, i));
  b.region(RK_EC_CONST, P2, {EC_K_DUMMY});  // getDummy
  for (int i = 0; i < N; i++) b.region(RK_EC_N2B, sz_n2b(CS), {0, G.c_u2 + i, CS});
  for (int w = 0; w < G.wins; w++) {
    b.region(RK_EC_SM_W0, sz_n2b(4) + 6, {w});
    if (w > 0) {
      ecop(ec_op_sm_dbl(G, 4 * w - 4));
      b.region(RK_EC_SM_DSW, P2 * 6, {w});
      for (int j = 1; j < 4; j++) ecop(ec_op_sm_dbl(G, 4 * w - 4 + j));
    }
    b.region(RK_EC_SM_SEL, P2 * 32 + 16 * 6, {w});
    if (w > 0) {
      ecop(ec_op_sm_add(G, w - 1));
      b.region(RK_EC_SM_RSW, 6 + 2 * P2 * 6, {w});
    }
  }
  ecop(G.op_final);
  ect(G.n_ops + EC_MM_XN, ECT_MM);
}

}  // namespace pzk
