// ECDSA secp256r1 (SIGNATURE_TYPE 20) path: constants, EC-op numbering and the per-witness
// core layout shared by the host layout builder and the device kernels.
//
// verifyECDSABits (signatures/ecdsa.circom:18-87) evaluates 362 elliptic-curve point operations
// per witness, every one a full template instance (EllipticCurveDouble / EllipticCurveAdd,
// ec/curve.circom:281-345) whose PointOnCurve / PointOnTangent / PointOnLine sub-blocks hold
// ~7-10 k signals. The path is split into
//   * k_ec_scalars / k_ec_chain / k_ec_final — the scalars (s^-1, u1, u2 mod n) and the two point
//                   chains (lane per (witness, chain)) in Jacobian coordinates;
//   * k_ec_affine / k_ec_link / k_ec_inv — lane-parallel: affine points (one inversion per 8 ops),
//                   an op RECORD (in1, in2, out) per point operation, the IsEqual inverses;
//   * k_ec_table  — lane per (witness, op): the op's template walker (ec_walk.hpp) expands the
//                   record into a VALUE TABLE (every distinct non-bit signal value, Fr normal form);
//   * k_emit_ect  — workgroup per (witness, op): table -> LDS, then one u32 descriptor per signal
//                   (COPY / BIT / MASK of a table entry), built once per op type on the host by the
//                   same walker run symbolically.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pzk {

// ---- curve constants, 64-bit limbs little-endian: [curve][A, B, P, order, dummy][limb]
// curve 0 = secp256r1 (SIGNATURE_TYPE 20), 1 = brainpoolP256r1 (21). A, B, P: signatureVerification.circom:179-182,
// :191-196; order: ec/get.circom:155-159; dummy: get.circom:87-93
constexpr int EC_N_CURVES = 2;
constexpr uint64_t EC_CURVE_K[EC_N_CURVES][5][8] = {
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
      9125809427693782222ull, 4479624720887462683ull, 4313457861005768495ull, 11848267593595748038ull}}};
// constant limb i of curve constant id (RK_EC_CONST regions)
enum { EC_K_A = 0, EC_K_B = 1, EC_K_P = 2, EC_K_ORDER = 3, EC_K_DUMMY = 4, EC_K_ONE = 5 };
__host__ __device__ inline uint64_t ec_k(int curve, int id, int i) {
  return id == EC_K_ONE ? (i == 0 ? 1 : 0) : EC_CURVE_K[curve][id][i];
}

// The EC kernels are compiled once per curve (kernels_ec.hip: PZK_EC_CURVE 0, kernels_ec_bp.hip: 1); their
// device code lives in an inline namespace per curve, so the two instantiations link side by side and
// the constants below are compile-time immediates in each.
#ifndef PZK_EC_CURVE
#define PZK_EC_CURVE 0
#endif
#if PZK_EC_CURVE == 0
#define PZK_EC_NS ec_c0
#else
#define PZK_EC_NS ec_c1
#endif
inline namespace PZK_EC_NS {
static constexpr int EC_CV = PZK_EC_CURVE;
static constexpr const uint64_t (&EC_A)[8] = EC_CURVE_K[EC_CV][EC_K_A];
static constexpr const uint64_t (&EC_B)[8] = EC_CURVE_K[EC_CV][EC_K_B];
static constexpr const uint64_t (&EC_P)[8] = EC_CURVE_K[EC_CV][EC_K_P];
static constexpr const uint64_t (&EC_N)[8] = EC_CURVE_K[EC_CV][EC_K_ORDER];
static constexpr const uint64_t (&EC_D)[8] = EC_CURVE_K[EC_CV][EC_K_DUMMY];
}  // namespace PZK_EC_NS

// ---- EC point operations of one witness (fixed numbering, execution order of k_ec_core)
constexpr int EC_OP_SD = 0;                                          // genmult getSecondDummy = 2 D (DBL)
__host__ __device__ constexpr int ec_op_gm_add(int i) { return 1 + i; }            // genmult adders[i], i < 31
__host__ __device__ constexpr int ec_op_pre(int i) { return 32 + (i - 2); }        // precompute out[i], i = 2..15
__host__ __device__ constexpr int ec_op_sm_dbl(int d) { return 46 + (d / 4) * 5 + (d % 4); }  // doublers[d], d < 252
__host__ __device__ constexpr int ec_op_sm_add(int a) { return 46 + a * 5 + 4; }   // scalarMult adders[a], a < 63
constexpr int EC_OP_FINAL = 361;                                     // verifyECDSABits.add
constexpr int EC_N_OPS = 362;
__host__ __device__ constexpr bool ec_op_is_dbl(int op) {
  return op == EC_OP_SD || (op >= 32 && op < 46 && (op - 32) % 2 == 0) || (op >= 46 && op < 361 && (op - 46) % 5 != 4);
}
// BigMultModP(64,4,4,4) instances (bigInt.circom:206-272): modInv.mult, mult, mult2, modOrder
enum { EC_MM_INV = 0, EC_MM_U1 = 1, EC_MM_U2 = 2, EC_MM_XN = 3, EC_N_MM = 4 };

// ---- per-witness EC core (u64 words)
constexpr int ECC_SINV = 0, ECC_U1 = 4, ECC_U2 = 8, ECC_H = 12;
constexpr int ECC_MM = 32;                      // [4] x (in1[4], in2[4])
constexpr int ECC_GM_AP = 64;                   // genmult additionPoints[32][2][4]
constexpr int ECC_GM_RP = ECC_GM_AP + 256;      // genmult resultingPoints[31][2][4]
constexpr int ECC_PRE = ECC_GM_RP + 248;        // precompute out[16][2][4]
constexpr int ECC_SM_AP = ECC_PRE + 128;        // scalarMult additionPoints[64][2][4]
constexpr int ECC_SM_RP = ECC_SM_AP + 512;      // scalarMult resultingPoints[65][2][4]
constexpr int ECC_REC = ECC_SM_RP + 520;        // op records: [362] x (in1[8], in2[8], out[8])
constexpr int ECC_REC_WORDS = 24;
constexpr int EC_CORE_WORDS = ECC_REC + EC_N_OPS * ECC_REC_WORDS;
// IsEqual inverses (Fr normal form): genmult steps 4 per step (isFirst/SecondDummyLeft/Right),
// scalarMult isZeroResult[64], isZeroAddition[1..63]
constexpr int ECI_GM = 0, ECI_SM_ZR = 124, ECI_SM_ZA = 188, EC_N_INV = 251;
// Jacobian scratch of k_ec_core per witness (u64): X, Y, Z per op + prefix products
constexpr int EC_JAC_WORDS = EC_N_OPS * 16 + 112;

// ---- table-block descriptor: op (3) | bit (9) | entry (20)
enum : uint32_t { ECD_ZERO = 0, ECD_COPY = 1, ECD_BIT = 2, ECD_MASK = 3 };
__host__ __device__ constexpr uint32_t ecd(uint32_t op, uint32_t idx, uint32_t bit = 0) {
  return (op << 29) | (bit << 20) | idx;
}
enum EcType { ECT_DBL = 0, ECT_ADD = 1, ECT_MM = 2, ECT_N = 3 };



// template sizes (ec/curve.circom; oracle/ecdsa_p256.inc.c derives them independently)
__host__ __device__ constexpr uint32_t ec_n2b(int L) { return 2 * L + 1; }
__host__ __device__ constexpr uint32_t ec_bmneq(int G, int L) { return (G + L - 1) + G + L + G * L + (G + L - 1) * L; }
__host__ __device__ constexpr uint32_t ec_bmo(int G, int L) { return (G + L - 1) + G + L + ec_bmneq(G, L); }
__host__ __device__ constexpr uint32_t ec_bisz(int MAX, int K) { return K + (K - 1) + (K - 1) * ec_n2b(MAX + 3 - 64); }
__host__ __device__ constexpr uint32_t ec_bizmp(int MAX, int CN, int MCN) {
  return CN + 4 + 1 + (MCN - 3) + (MCN - 3) * ec_n2b(64) + ec_bmo(MCN - 3, 4) + ec_bisz(MAX, MCN) + CN * 6;
}
constexpr uint32_t EC_SZ_PONCURVE = 8 + 3 * ec_bmo(4, 4) + ec_bmo(7, 4) + ec_bizmp(200, 10, 12);
constexpr uint32_t EC_SZ_PONTANGENT = 16 + ec_bmo(4, 4) + 15 + 18 + 16 + ec_bmo(7, 4) + 9 + 12 + ec_bmo(4, 4) + ec_bizmp(200, 10, 13);
constexpr uint32_t EC_SZ_PONLINE = 24 + 12 + 3 * 16 + 2 * ec_bmo(4, 4) + ec_bizmp(136, 7, 9);
constexpr uint32_t EC_SZ_DBL = 16 + EC_SZ_PONTANGENT + EC_SZ_PONCURVE;
constexpr uint32_t EC_SZ_ADD = 24 + EC_SZ_PONCURVE + EC_SZ_PONLINE;
// BigMultModP(64,4,4,4): div[5], mod[4] | in1, in2, modulus | mult, modChecks[4], greaterThan, mult2, isZero
constexpr uint32_t EC_SZ_BLET = 1 + 8 + 4 + 4 * ((3 + ec_n2b(65)) + 6);
constexpr uint32_t EC_SZ_MM = 5 + 4 + 12 + ec_bmo(4, 4) + 4 * ec_n2b(64) + (1 + 8 + EC_SZ_BLET) + ec_bmneq(5, 4) + ec_bisz(132, 7);
__host__ __device__ constexpr uint32_t ec_type_size(int t) { return t == ECT_DBL ? EC_SZ_DBL : t == ECT_ADD ? EC_SZ_ADD : EC_SZ_MM; }
constexpr uint32_t EC_TABLE_MAX = 1024;   // table entries per op (checked by the host walker)

}  // namespace pzk
