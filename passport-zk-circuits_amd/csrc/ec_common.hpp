// ECDSA path (SIGNATURE_TYPE 20, 21, 24, 25): curve constants, per-curve geometry (chunking, EC-op
// numbering, per-witness core layout, template sizes) shared by the host layout builder and the kernels.
//
// verifyECDSABits(CHUNK_SIZE, CHUNK_NUMBER, ...) (signatures/ecdsa.circom:18-87) evaluates
// 1 + (PARTS - 1) + 14 + 5 (WINS - 1) + 1 elliptic-curve point operations per witness (P-256: 362,
// P-224: 318, brainpoolP384r1: 538; PARTS = N CS / 8 generator-table parts, WINS = N CS / 4 windows), every
// one a full template instance (EllipticCurveDouble / EllipticCurveAdd, ec/curve.circom:281-345) whose
// PointOnCurve / PointOnTangent / PointOnLine sub-blocks hold ~7-30 k signals. The path is split into
//   * k_ec_scalars / k_ec_chain / k_ec_final — the scalars (s^-1, u1, u2 mod n) and the two point
//                   chains (lane per (witness, chain)) in Jacobian coordinates;
//   * k_ec_affine / k_ec_link / k_ec_inv — lane-parallel: affine points (one inversion per 8 ops),
//                   an op RECORD (in1, in2, out) per point operation, the IsEqual inverses;
//   * k_ec_table  — lane per (witness, op): the op's template walker (ec_walk.hpp) expands the
//                   record into a VALUE TABLE (every distinct non-bit signal value, Fr normal form);
//   * k_emit_ect  — workgroup per (witness, op): table -> LDS, then one u32 descriptor per signal
//                   (COPY / BIT / MASK of a table entry), built once per op type on the host by the
//                   same walker run symbolically.
// Values of CHUNK_SIZE-bit chunks are kept one per u64 word everywhere (core, records, tables' inputs).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pzk {

// ---- curves: 0 = secp256r1 (SIG 20), 1 = brainpoolP256r1 (21), 2 = secp224r1 (24), 3 = brainpoolP384r1 (25).
// SIG 22 / 23 read hashed[] past its end in verifyECDSABits (ecdsa.circom:31-37: 5 x 64 / 3 x 64 chunks of a
// 256 / 160-bit hash), so no circuit with them compiles.
constexpr int EC_N_CURVES = 4;
constexpr int EC_MAXN = 7;  // largest CHUNK_NUMBER
__host__ __device__ constexpr int ec_curve_of_sig(int sig) {
  return sig == 20 ? 0 : sig == 21 ? 1 : sig == 24 ? 2 : sig == 25 ? 3 : -1;
}
// CHUNK_NUMBER, CHUNK_SIZE (signatureVerification.circom:77-116)
constexpr int EC_NL[EC_N_CURVES] = {4, 4, 7, 6};
constexpr int EC_CS[EC_N_CURVES] = {64, 64, 32, 64};

// curve constants as CHUNK_SIZE-bit chunks, little-endian: [curve][A, B, P, order, dummy (x then y)][chunk]
// A, B, P: signatureVerification.circom:179-182, :193-196, :235-238, :249-252; order: ec/get.circom:157, :154,
// :183, :165; dummy: get.circom:92-93, :88-89, :124-125, :102-103
constexpr uint64_t EC_CURVE_K[EC_N_CURVES][5][2 * EC_MAXN] = {
    {{18446744073709551612ull, 4294967295ull, 0ull, 18446744069414584321ull},
     {4309448131093880907ull, 7285987128567378166ull, 12964664127075681980ull, 6540974713487397863ull},
     {18446744073709551615ull, 4294967295ull, 0ull, 18446744069414584321ull},
     {17562291160714782033ull, 13611842547513532036ull, 18446744073709551615ull, 18446744069414584320ull},
     {4148137498610012746ull, 51237685452122967ull, 6555942389409504868ull, 799804747332166731ull,
      13395177781894339167ull, 1107697421929919296ull, 6228258783500845564ull, 11862546499924939746ull}},
    {{16810331318623712729ull, 18122579188607900780ull, 17219079075415130087ull, 9032542404991529047ull},
     {7767825457231955894ull, 10773760575486288334ull, 17523706096862592191ull, 2800214691157789508ull},
     {2311270323689771895ull, 7943213001558335528ull, 4496292894210231666ull, 12248480212390422972ull},
     {10384753744809580199ull, 10104242082523752183ull, 4496292894210231665ull, 12248480212390422972ull},
     {5870538370169240658ull, 13064052279558318326ull, 1032222391323187885ull, 10478252910764369874ull,
      9125809427693782222ull, 4479624720887462683ull, 4313457861005768495ull, 11848267593595748038ull}},
    {{4294967294ull, 4294967295ull, 4294967295ull, 4294967294ull, 4294967295ull, 4294967295ull, 4294967295ull},
     {592838580ull, 655046979ull, 3619674298ull, 1346678967ull, 4114690646ull, 201634731ull, 3020229253ull},
     {1ull, 0ull, 0ull, 4294967295ull, 4294967295ull, 4294967295ull, 4294967295ull},
     {1549543997ull, 333261125ull, 3770216510ull, 4294907554ull, 4294967295ull, 4294967295ull, 4294967295ull},
     {2477436510ull, 406882550ull, 2884834286ull, 2269163287ull, 3636783260ull, 3699382582ull, 912817446ull,
      582933619ull, 1778719645ull, 3780674687ull, 3008581200ull, 3586474874ull, 866709652ull, 3566930607ull}},
    {{335737924824737830ull, 9990533504564909291ull, 1410020238645393679ull, 14032832221039175559ull,
      4355552632119865248ull, 8918115475071440140ull},
     {4230998357940653073ull, 8985869839777909140ull, 3352946025465340629ull, 3438355245973688998ull,
      10032249017711215740ull, 335737924824737830ull},
     {9747760000893709395ull, 12453481191562877553ull, 1347097566612230435ull, 1526563086152259252ull,
      1107163671716839903ull, 10140169582434348328ull},
     {4289733633151100261ull, 14932448379039367952ull, 2240099277684876711ull, 1526563086152259251ull,
      1107163671716839903ull, 10140169582434348328ull},
     {522720248942821492ull, 13227018843434759032ull, 17067096815187998133ull, 8957183796380674257ull,
      7544165743263758981ull, 6159107397665645433ull, 9174881270872499347ull, 7148726877058227897ull,
      1584493337432922624ull, 1438582915076653591ull, 16161625210166602047ull, 946254366129831718ull}}};
// constant chunk i of curve constant id (RK_EC_CONST regions)
enum { EC_K_A = 0, EC_K_B = 1, EC_K_P = 2, EC_K_ORDER = 3, EC_K_DUMMY = 4, EC_K_ONE = 5 };
__host__ __device__ inline uint64_t ec_k(int curve, int id, int i) {
  return id == EC_K_ONE ? (i == 0 ? 1 : 0) : EC_CURVE_K[curve][id][i];
}

// ---- template sizes (ec/curve.circom, bigInt/*.circom; oracle/ecdsa.inc.c derives them independently). Every
// BigMultOverflow of these templates is the schoolbook BigMultNonEqualOverflow (no power-of-two G >= 8 with a
// Karatsuba-optimal L, bigIntOverflow.circom:43-53).
__host__ __device__ constexpr uint32_t ec_n2b(int L) { return 2 * L + 1; }
__host__ __device__ constexpr uint32_t ec_bmneq(int G, int L) { return (G + L - 1) + G + L + G * L + (G + L - 1) * L; }
__host__ __device__ constexpr uint32_t ec_bmo(int G, int L) { return (G + L - 1) + G + L + ec_bmneq(G, L); }
__host__ __device__ constexpr uint32_t ec_bisz(int cs, int MAX, int K) { return K + (K - 1) + (K - 1) * ec_n2b(MAX + 3 - cs); }
// BigIntIsZeroModP(cs, MAX, CN, MCN, N): in[CN], modulus[N] | sign, k[DIV] | kRangeChecks[DIV], mult, isZero, swicher[CN]
__host__ __device__ constexpr uint32_t ec_bizmp(int cs, int N, int MAX, int CN, int MCN) {
  return CN + N + 1 + (MCN - N + 1) + (MCN - N + 1) * ec_n2b(cs) +
         (MCN - N + 1 >= N ? ec_bmo(MCN - N + 1, N) : ec_bmo(N, MCN - N + 1)) + ec_bisz(cs, MAX, MCN) + CN * 6;
}
__host__ __device__ constexpr int ec_log_ceil(int n) { return n == 0 ? 0 : 1 + ec_log_ceil(n >> 1); }

struct EcGeo {
  int nl, cs, fb, parts, wins, n_ops;      // CHUNK_NUMBER, CHUNK_SIZE, field bits, generator parts, scalar-mult windows
  int op_sm0, op_final;                    // first scalar-mult op, verifyECDSABits.add
  // per-witness EC core (u64 words, one chunk each)
  int c_sinv, c_u1, c_u2, c_h, c_mm, c_gm_ap, c_gm_rp, c_pre, c_sm_ap, c_sm_rp, c_rec, rec_words, core_words;
  // IsEqual inverses (Fr): genmult 4 per step, scalarMult isZeroResult[WINS], isZeroAddition[1..WINS-1]
  int i_sm_zr, i_sm_za, n_inv;
  // k_ec_chain scratch (u64): per op X, Y, Z (jw words each, Montgomery) + handles; then the forwarded points' handles
  int n_pts, jw, j_op, j_pts, jac_words;
  // block sizes
  uint32_t sz_poncurve, sz_pontangent, sz_ponline, sz_dbl, sz_add, sz_blet, sz_mm;
};
__host__ __device__ constexpr EcGeo ec_geo_make(int N, int cs) {
  EcGeo g{};
  g.nl = N; g.cs = cs; g.fb = N * cs; g.parts = g.fb / 8; g.wins = g.fb / 4;
  g.op_sm0 = g.parts + 14;
  g.n_ops = g.op_sm0 + 5 * (g.wins - 1) + 1;
  g.op_final = g.n_ops - 1;
  const int P2 = 2 * N;
  g.c_sinv = 0; g.c_u1 = N; g.c_u2 = 2 * N; g.c_h = 3 * N;
  g.c_mm = 4 * N;                                   // [4] x (in1[N], in2[N])
  g.c_gm_ap = g.c_mm + 4 * P2;                      // genmult additionPoints[PARTS][2][N]
  g.c_gm_rp = g.c_gm_ap + g.parts * P2;             // genmult resultingPoints[PARTS-1][2][N]
  g.c_pre = g.c_gm_rp + (g.parts - 1) * P2;         // precompute out[16][2][N]
  g.c_sm_ap = g.c_pre + 16 * P2;                    // scalarMult additionPoints[WINS][2][N]
  g.c_sm_rp = g.c_sm_ap + g.wins * P2;              // scalarMult resultingPoints[WINS+1][2][N]
  g.c_rec = g.c_sm_rp + (g.wins + 1) * P2;          // op records: (in1, in2, out) x [2][N]
  g.rec_words = 3 * P2;
  g.core_words = g.c_rec + g.n_ops * g.rec_words;
  g.i_sm_zr = 4 * (g.parts - 1);
  g.i_sm_za = g.i_sm_zr + g.wins;
  g.n_inv = g.i_sm_za + g.wins - 1;
  g.n_pts = g.parts + (g.parts - 1) + 16 + g.wins + (g.wins + 1);
  g.jw = (g.fb + 63) / 64;
  g.j_op = (3 * g.jw + 2) & ~1;
  g.j_pts = g.n_ops * g.j_op;
  g.jac_words = g.j_pts + (g.n_pts + 1) / 2;
  g.sz_poncurve = P2 + 3 * ec_bmo(N, N) + ec_bmo(2 * N - 1, N) + ec_bizmp(cs, N, 3 * cs + 2 * N, 3 * N - 2, 3 * N);
  g.sz_pontangent = 4 * N + ec_bmo(N, N) + (2 * (2 * N - 1) + 1) + (2 * (2 * N - 1) + N) + 4 * N + ec_bmo(2 * N - 1, N) +
                    (2 * N + 1) + 3 * N + ec_bmo(N, N) + ec_bizmp(cs, N, 3 * cs + 2 * N, 3 * N - 2, 3 * N + 1);
  g.sz_ponline = 6 * N + 3 * N + 3 * 4 * N + 2 * ec_bmo(N, N) + ec_bizmp(cs, N, 2 * cs + 2 * N, 2 * N - 1, 2 * N + 1);
  g.sz_dbl = 4 * N + g.sz_pontangent + g.sz_poncurve;
  g.sz_add = 6 * N + g.sz_poncurve + g.sz_ponline;
  // BigLessEqThan(cs, N): out | in[2][N] | result[N] | (LessThan(cs) = out | in[2] | Num2Bits(cs + 1), IsEqual)[N]
  g.sz_blet = 1 + 2 * N + N + N * ((3 + ec_n2b(cs + 1)) + 6);
  // BigMultModP(cs,N,N,N): div[N+1], mod[N] | in1, in2, modulus | mult, modChecks[N], greaterThan, mult2, isZero
  g.sz_mm = (N + 1) + N + 3 * N + ec_bmo(N, N) + N * ec_n2b(cs) + (1 + 2 * N + g.sz_blet) + ec_bmneq(N + 1, N) +
            ec_bisz(cs, 2 * cs + ec_log_ceil(2 * N), 2 * N - 1);
  return g;
}
constexpr EcGeo EC_GEO[EC_N_CURVES] = {ec_geo_make(4, 64), ec_geo_make(4, 64), ec_geo_make(7, 32), ec_geo_make(6, 64)};
static_assert(EC_GEO[0].n_ops == 362 && EC_GEO[2].n_ops == 318 && EC_GEO[3].n_ops == 538, "EC op counts");

// ---- EC point operations of one witness (fixed numbering, execution order of k_ec_chain)
constexpr int EC_OP_SD = 0;                                                        // genmult getSecondDummy = 2 D (DBL)
__host__ __device__ constexpr int ec_op_gm_add(int i) { return 1 + i; }            // genmult adders[i], i < PARTS-1
__host__ __device__ constexpr int ec_op_pre(const EcGeo& G, int i) { return G.parts + (i - 2); }  // precompute out[i], i = 2..15
__host__ __device__ constexpr int ec_op_sm_dbl(const EcGeo& G, int d) { return G.op_sm0 + (d / 4) * 5 + (d % 4); }  // doublers[d]
__host__ __device__ constexpr int ec_op_sm_add(const EcGeo& G, int a) { return G.op_sm0 + a * 5 + 4; }  // scalarMult adders[a]
__host__ __device__ constexpr bool ec_op_is_dbl(const EcGeo& G, int op) {
  return op == EC_OP_SD || (op >= G.parts && op < G.op_sm0 && (op - G.parts) % 2 == 0) ||
         (op >= G.op_sm0 && op < G.op_final && (op - G.op_sm0) % 5 != 4);
}
// BigMultModP(cs,N,N,N) instances (bigInt.circom:206-272): modInv.mult, mult, mult2, modOrder
enum { EC_MM_INV = 0, EC_MM_U1 = 1, EC_MM_U2 = 2, EC_MM_XN = 3, EC_N_MM = 4 };

// ---- table-block descriptor: op (3) | bit (9) | entry (20)
enum : uint32_t { ECD_ZERO = 0, ECD_COPY = 1, ECD_BIT = 2, ECD_MASK = 3 };
__host__ __device__ constexpr uint32_t ecd(uint32_t op, uint32_t idx, uint32_t bit = 0) {
  return (op << 29) | (bit << 20) | idx;
}
enum EcType { ECT_DBL = 0, ECT_ADD = 1, ECT_MM = 2, ECT_N = 3 };
__host__ __device__ constexpr uint32_t ec_type_size(const EcGeo& G, int t) {
  return t == ECT_DBL ? G.sz_dbl : t == ECT_ADD ? G.sz_add : G.sz_mm;
}
// table entries per op, upper bound per curve (checked by the host walker; the DBL table is the largest: 597, 597,
// 1596, 1211 entries); k_emit_ect stages the table in LDS (32 B per entry)
constexpr uint32_t EC_TABLE_MAX[EC_N_CURVES] = {640, 640, 1600, 1216};

// ---- the curve of an EC translation unit (kernels_ec*.hip compile ec_core.hpp once per curve, PZK_EC_CURVE 0..3):
// device code lives in an inline namespace per curve, so the instantiations link side by side and the curve's
// constants and geometry are compile-time immediates in each.
#ifndef PZK_EC_CURVE
#define PZK_EC_CURVE 0
#endif
#if PZK_EC_CURVE == 0
#define PZK_EC_NS ec_c0
#elif PZK_EC_CURVE == 1
#define PZK_EC_NS ec_c1
#elif PZK_EC_CURVE == 2
#define PZK_EC_NS ec_c2
#else
#define PZK_EC_NS ec_c3
#endif
inline namespace PZK_EC_NS {
static constexpr int EC_CV = PZK_EC_CURVE;
static constexpr EcGeo ECG = EC_GEO[EC_CV];
static constexpr const uint64_t (&EC_A)[2 * EC_MAXN] = EC_CURVE_K[EC_CV][EC_K_A];
static constexpr const uint64_t (&EC_B)[2 * EC_MAXN] = EC_CURVE_K[EC_CV][EC_K_B];
static constexpr const uint64_t (&EC_P)[2 * EC_MAXN] = EC_CURVE_K[EC_CV][EC_K_P];
static constexpr const uint64_t (&EC_N)[2 * EC_MAXN] = EC_CURVE_K[EC_CV][EC_K_ORDER];
static constexpr const uint64_t (&EC_D)[2 * EC_MAXN] = EC_CURVE_K[EC_CV][EC_K_DUMMY];
}  // namespace PZK_EC_NS

}  // namespace pzk
