// Instance layout: where every template instance's signals live in the witness, and the
// work lists the kernels run over. Built once per instance on the host (layout.cpp),
// uploaded to the device, shared by every batch.
//
// Witness numbering: witness[0] = 1, then the main component; each
// component instance is one contiguous block = its own signals (outputs, inputs,
// intermediates, each in declaration order) followed by its subcomponents' blocks in
// creation order. The layout is data-driven: a region table, not hard-coded offsets.
#pragma once
#include <stdint.h>

namespace pzk {

// lane status codes (mirror include/pzkwit.h PZK_ST_*)
constexpr int32_t ST_NUM2BITS = 1, ST_ALIAS = 2, ST_ISZERO = 3, ST_FLOW = 7, ST_RSA_HASH = 8,
                  ST_RSA_PREFIX = 9, ST_RSA_PAD = 10, ST_BIGMOD_GT = 11, ST_BIGISZERO = 12,
                  ST_SMT_LAST = 13, ST_ECDSA_INV = 15, ST_ECDSA_R = 16, ST_PSS_TRAILER = 17,
                  ST_PSS_HASH = 18, ST_QUERY = 19, ST_DATE = 20, ST_CIT_BLACKLIST = 21, ST_CIT_LIST = 22,
                  ST_ISV_ROOT = 23, ST_INPUT_RANGE = 64;

// ---- emit regions: a contiguous run of witness signals with one closed-form generator
enum RegionKind : uint32_t {
  RK_ONE = 0,        // witness[0] = 1
  RK_INCOPY = 1,     // a0 = input element offset: w[off+i] = in[a0+i]
  RK_SHA_OWN = 2,    // ShaHashChunks wrapper (a3) + Sha256HashChunks own signals + iv;
                     //   a0 = sha slot, a1 = blocks, a2 = input element offset of the bits, a3 = wrapper
  RK_SHA_BLOCK = 3,  // Sha2_224_256Shedule + Sha2_224_256Rounds(64) of one block; a0 = sha slot, a1 = block
  RK_POSEIDON = 4,   // PoseidonHash(n) block; a0 = poseidon task, a1 = n
  RK_MODMUL = 5,     // BigMultModP(64,K,K,K); a0 = modmul index
  RK_VALUE = 6,      // w[off+i] = value-store slot a0+i (normal-form conversion)
  RK_BITS2NUM = 7,   // Bits2Num(L) over bits taken from a bit source; a0 = L, a1 = bit source id,
                     //   a2 = first bit, a3 = stride(+1/-1), a4 = alias-check flag
  RK_NUM2BITS = 8,   // Num2Bits(L) of a value-store slot; a0 = L, a1 = slot
  RK_DIGEST = 9,     // 256 digest bits (MSB first) of SHA job a0
  RK_TEMPMOD = 10,   // tempModulus[5] = pk[3i]*2^128 + pk[3i+1]*2^64; a0 = pubkey input offset
  RK_FLOW = 11,      // PassportVerificationFlow (passportVerificationFlow.circom:6-109), whole block
  RK_HCHUNK = 12,    // hashed_chunks[N] (RsaVerifyPkcs1v15 4 x 64, verifyECDSABits N x CS); a0 = SHA job, a1 = N, a2 = CS
  RK_RSA_OUT = 13,   // PowerMod.out[K] = EM limbs (RSA core)
  RK_SMT_OWN = 14,   // SMTVerifier own signals
  RK_SMTHASH = 15,   // SMTHash1/2 own (out, key/L, value/R); a0 = level (-1 = hash1New)
  RK_LEVINS = 16,    // SMTLevIns(80) block
  RK_SM = 17,        // sm[80] SMTVerifierSM blocks
  RK_SMT_LEVEL = 18, // SMTVerifierLevel own signals; a0 = level
  RK_SWITCHER = 19,  // Switcher of SMT level a0
  RK_ISEQ_ROOT = 20, // SMTVerifier.isEqual block
  RK_BJJ_OWN = 21,   // BabyjubjubBase8Multiplication own (out[2], scalar) + GetBabyjubjubBase8
  RK_BJJ_STEPS = 22, // adders[0], (adders[i], doublers[i-1]) i = 1..253
  RK_SIG_OWN = 23,   // VerifySignature / RsaVerifyPkcs1v15 / PowerMod input copies (a0 = sub-kind)
  // ---- ECDSA (ec_common.hpp, ec_emit.hpp); chunked values have CHUNK_SIZE bits, points 2 x CHUNK_NUMBER chunks
  RK_ECT = 24,        // table block: a0 = table op (EC op, or EC_N_OPS + BigMultModP index), a1 = EcType
  RK_EC_U64 = 25,     // w[off+i] = EC core word a0 + i
  RK_EC_CONST = 26,   // curve constant a0 (ec_k ids)
  RK_EC_GM_RCC = 27,  // generator mult resultCoordinateComputation[PARTS][256][2][N]
  RK_EC_GM_EQ = 28,   // generator mult equal[PARTS][256] (IsEqual)
  RK_EC_GM_SUM = 29,  // generator mult getSumOfNElements[PARTS][2][N] (GetSum(256))
  RK_EC_GM_STEP = 30, // generator mult step a0: 4 IsEqual dummy tests + 16 switchers
  RK_EC_N2B = 31,     // Num2Bits(a2 = CS): a0 = 0 EC core word a1 / 1 input element a1
  RK_EC_B2N8 = 32,    // generator mult bits2num[PARTS] (Bits2Num(8)) of the scalar at core word a0
  RK_EC_SBITS = 33,   // scalarMult scalarBits[N CS] of the scalar at core word a0
  RK_EC_SM_W0 = 34,   // scalarMult window a0: bits2Num(4) + isZeroResult
  RK_EC_SM_DSW = 35,  // scalarMult window a0: doubleSwitcher[2N]
  RK_EC_SM_SEL = 36,  // scalarMult window a0: getSum[2N] (GetSum(16)) + partsEqual[16]
  RK_EC_SM_RSW = 37,  // scalarMult window a0: isZeroAddition + (resultSwitcherAddition, resultSwitcherDoubling)[2N]
  RK_EC_PKBITS = 38,  // PassportVerificationBuilder ecBitsX[F], ecBitsY[F] of pubkey input a0 (a1 = N, a2 = CS)
  RK_EC_B2N248 = 39,  // Bits2Num(a3 = min(F, 248)) of the N-chunk input at a0 (xToNum / yToNum; a1 = N, a2 = CS)
  // ---- RSA-PSS (SIGNATURE_TYPE 10-12, rsaPss.circom:18-204; pss.hpp)
  RK_PSS_OWN = 40,    // VerifyRsaPssSig eM .. mDash (after its pubkey/signature/hashed inputs); a0 = salt bits
  RK_PSS_B2N8 = 41,   // bits2Num[8K] (Bits2Num(8)) of the EM bytes
  RK_PSS_MGF = 42,    // Mgf1Sha256 own: out[DB8] | seed[256] | hashed[256 IT]
  RK_PSS_CTR = 43,    // Mgf1Sha256 num2Bits[a0] = Num2Bits(32)(a0)
  RK_PSS_XOR = 44,    // Xor2(DB8): out | in1 | in2
  // ---- SHA-1 (hasher/sha1/*.circom; sha1.hpp)
  RK_SHA1_OWN = 45,   // Sha1HashChunks out[160] | in[512B] | H(0..4); a0 = sha slot, a1 = blocks, a2 = input offset
  RK_SHA1_BLOCK = 46, // Sha1compression of one block; a0 = sha slot, a1 = block
  // ---- SHA-384 / SHA-512 (hasher/sha2/sha384, sha512; sha512.hpp)
  RK_SHA5_OWN = 47,   // [ShaHashChunks out[O] | in[1024B] (a4 = 1)] Sha384/512HashChunks out[O] | in[1024B] | states | iv;
                      // a0 = sha slot, a1 = blocks, a2 = input offset, a3 = O
  RK_SHA5_BLOCK = 48, // Sha2_384_512Schedule + Sha2_384_512Rounds(80) of one block; a0 = sha slot, a1 = block
  // ---- QueryIdentity(80) (identityManagement/queryIdentity.circom; query.hpp), all from the input row + value store
  RK_Q_OUT = 49,      // main outputs: nullifier, birthDate .. documentNumber (selector-masked)
  RK_Q_SQ = 50,       // eventDataSquare
  RK_Q_CMP = 51,      // GreaterEqThan(64) / LessThan(64) block a0 = 0..3 (timestamp / identity counter bounds)
  RK_Q_FEIE = 52,     // ForceEqualIfEnabled block a0 = 0..7 (condition a0, enabled = selector bit 8 + a0)
  RK_Q_EDIL = 53,     // EncodedDateIsLess block a0 = 0 (expirationDateLowerbound, exp) / 1 (exp, expirationDateUpperbound)
  RK_Q_EDILN = 54,    // EncodedDateIsLessNormalized block a0 = 0 (birthDateLowerbound, birth) / 1 (birth, birthDateUpperbound)
  RK_Q_CIT = 55,      // CitizenshipCheck own: citizenship, blacklist | validCheck[241], bitmask[240]
  RK_Q_CITEQ = 56,    // CitizenshipCheck (isEqual[i], isEqual2[i]) i < 240
  RK_COUNT
};

// emit kernels (one work list each)
// E_GENR = generic regions that read the RSA core (they run after it, off the main chain)
// E_ECT = ECDSA table blocks (k_emit_ect); E_ECR = the generator multiplication's selection tables (k_emit_ecr:
// resultCoordinateComputation, equal[][], getSumOfNElements, ec_core.hpp)
// E_SHAD = SHA regions of hashers fed by derived messages (RSA-PSS MGF1 / M'), emitted after the PSS chain
// E_SHA1 = SHA-1 hasher regions (k_emit_sha1); E_SHA5 = SHA-384/512 hasher regions (k_emit_sha512); E_SHA5D = the
// SHA-384 hashers of derived messages (RSA-PSS SHA-384 MGF1 / M'), emitted after the PSS chain like E_SHAD
// E_QRY = QueryIdentity's small regions (k_emit_qry, query.hpp)
enum Emitter { E_GEN = 0, E_SHA, E_POS, E_BITS, E_FLOW, E_MM, E_BJJ, E_GENR, E_ECT, E_SHAD, E_SHA1, E_SHA5, E_SHA5D, E_ECR, E_QRY, E_COUNT };
__host__ __device__ inline int emitter_of(uint32_t kind) {
  switch (kind) {
    case RK_SHA_OWN: case RK_SHA_BLOCK: return E_SHA;
    case RK_SHA1_OWN: case RK_SHA1_BLOCK: return E_SHA1;
    case RK_SHA5_OWN: case RK_SHA5_BLOCK: return E_SHA5;
    case RK_POSEIDON: return E_POS;
    case RK_BITS2NUM: case RK_NUM2BITS: return E_BITS;
    case RK_FLOW: return E_FLOW;
    case RK_MODMUL: return E_MM;
    case RK_BJJ_STEPS: return E_BJJ;
    case RK_RSA_OUT: return E_GENR;
    case RK_ECT: return E_ECT;
    case RK_EC_GM_RCC: case RK_EC_GM_EQ: case RK_EC_GM_SUM: return E_ECR;
    case RK_Q_OUT: case RK_Q_SQ: case RK_Q_CMP: case RK_Q_FEIE: case RK_Q_EDIL: case RK_Q_EDILN: case RK_Q_CIT:
    case RK_Q_CITEQ: return E_QRY;
    default: return kind >= RK_EC_U64 && kind <= RK_PSS_XOR ? E_GENR : E_GEN;
  }
}
// regions whose emit workgroup needs the whole region (LDS pre-pass over all of it)
__host__ __device__ inline bool emitter_whole(int e) { return e == E_POS || e == E_BITS || e == E_FLOW; }
// emitters whose work items pack many small regions (Work.region = first GenPiece, Work.pad = pieces)
__host__ __device__ inline bool emitter_packed(int e) { return e == E_GEN || e == E_GENR || e == E_QRY; }

constexpr int REGION_ARGS = 10;
struct Region {
  uint64_t off;   // witness element offset
  uint32_t len;   // number of signals
  uint32_t kind;  // RegionKind
  int32_t a[REGION_ARGS];
};

// one workgroup's slice of a region
struct Work {
  uint32_t region;
  uint32_t start;
  uint32_t count;
  uint32_t pad;
};
// packed work: a run of region slices emitted by one workgroup; cum = signals before this piece
struct GenPiece {
  uint32_t region;
  uint32_t start;
  uint32_t cum;
  uint32_t pad;
};
constexpr uint32_t GEN_PACK = 512;         // signals per packed work item (2 per k_emit_gen lane, in registers)
constexpr uint32_t GEN_MAX_PIECES = 256;   // pieces per packed work item

// SHA hasher job: one (witness, hasher) lane of the SHA core kernel
struct ShaJob {
  int32_t in_off;   // input element offset of the first message bit
  int32_t blocks;   // number of 512-bit blocks
  int32_t core_off; // u32 offset of this hasher's core inside the per-witness SHA core
  int32_t digest_slot; // value-store slot receiving the 256 digest bits (packed) or -1
  int32_t src;      // 0: message bits are input elements; 1: derived elements (RSA-PSS, pss.hpp)
  int32_t algo;     // 0: SHA-256 (sha.hpp), 1: SHA-1 (sha1.hpp), 2: SHA-224 (SHA-256 blocks, own IV, 224-bit out),
                    // 3 / 4: SHA-384 / SHA-512 (sha512.hpp, 1024-bit blocks)
  int32_t hout;     // u32 offset of the digest words (Hout[8] / Hout[5]) inside the per-witness SHA core
};

// per block core: Hin[8] W[64] A[1..64] E[1..64]; per hasher: blocks*200 + Hout[8]
constexpr int SHA_BLOCK_CORE = 200;
// SHA-1: per block Hin[5] W[80] A[1..80]; per hasher blocks*165 + Hout[5] (+3 pad)
constexpr int SHA1_BLOCK_CORE = 165;
constexpr uint32_t SHA1_BLOCK_SIGS = 198034;  // Sha1compression (sha1.hpp)
constexpr uint32_t SHA1_CONST_SIGS = 97;      // H(x): out[32] | Num2Bits(32)
// SHA-384/512: per block Hin[8] W[80] A[1..80] E[1..80] as 64-bit words; per hasher blocks*496 + Hout[16]
constexpr int SHA5_BLOCK_CORE = 496;
constexpr uint32_t SHA5_BLOCK_SIGS = 378362;  // Sha2_384_512Schedule (94,480) + Sha2_384_512Rounds(80) (283,882)

// Poseidon task: one permutation PoseidonHash(n) per (witness, task) lane
struct PosTask {
  int32_t n;          // inputs (t = n + 1)
  int32_t in_slot[5]; // value-store slots (Montgomery) of the inputs
  int32_t out_slot;   // value-store slot for the hash
  int32_t core_off;   // Fr offset of this task's round states inside the per-witness Poseidon core
  int32_t level;      // dependency level (launch wave)
  int32_t smt_level;  // >= 0: SMTVerifierLevel hash of that level (skipped where it depends on the chain)
};

// RegisterIdentityBuilder instance facts the kernels need (value-store slots, input offsets)
struct RegInfo {
  int32_t K;                       // RSA limbs (32 or 64)
  int32_t in_pk, in_sig, in_br, in_root;
  int32_t j_dg1, j_dg15, j_ec, j_sa; // SHA jobs
  int32_t v_one, v_sk, v_pk, v_aa, v_dg1, v_sanum, v_bjj, v_smt_lr;  // slots (v_pk/v_aa/v_dg1: first of 5/5/4)
  int32_t v_pkhash, v_leaf, v_smt_h;  // Poseidon outputs (v_smt_h: first of 80 level hashes)
  int32_t dg1_chunk, aa_shift, in_dg1, in_dg15, aa;
  int32_t n_modmul;
  // PowerMod schedule (bigInt.circom:280-340, exp_to_bits bigIntFunc.circom:590-616): operands of BigMultModP k
  // are the remainders of multiplications mm_x[k], mm_y[k] (-1: the signature)
  int8_t mm_x[32], mm_y[32];
  uint32_t modmul_size;
  int32_t ecdsa;                   // SIGNATURE_TYPE >= 20 (ECDSA)
  int32_t ec_curve;                // 0..3: SIG 20, 21, 24, 25 (ec_common.hpp)
  int32_t ec_nl, ec_cs;            // its CHUNK_NUMBER, CHUNK_SIZE
  int32_t v_pkx, v_pky;            // ECDSA pubkey hash inputs (x, y mod 2^min(N CS, 248))
  int32_t aa_ec, aa_f, aa_hs;      // EC active-authentication key: field bits, hashed bits (identity.circom:51-84)
  int32_t pss_s8;                  // RSA-PSS salt bits (0: not PSS)
  int32_t pss_h;                   // RSA-PSS hash bits (256 or 384)
  int32_t j_mgf, n_mgf, j_hd;      // RSA-PSS SHA jobs: MGF1 blocks [j_mgf, j_mgf + n_mgf), M' hasher
  // SMTVerifier key / value slots (RegisterIdentityBuilder: both the pubkey hash; QueryIdentity: treePosition and
  // the identity-state value hash); smt_check: isVerified === 1 is a constraint (identityStateVerifier.circom:46)
  int32_t v_smt_key, v_smt_val, smt_check;
  // QueryIdentity: first of the 8 DG1DataExtractor outputs, first of the 240 CitizenshipCheck IsEqual inverses
  // (Montgomery), the citizenship's index in COUNTRY_ARR (raw u32 in limb 0; 240 = absent), the nullifier hash
  int32_t q_dgf, q_cinv, q_cidx, q_nul;
  // QueryIdentityTD1 (document_type 1): 9 DG1 fields, dg1[760]; PoseidonHash(1) of documentNumber / personalNumber
  int32_t q_td1, q_doch, q_persh;
};

// per-witness core sizes of the register-circuit kernels
constexpr int MM_CORE_WORDS(int K) { return 12 * K - 3; }  // x[K] y[K] q[K+1] r[K] inv[K](4 words) carry[2K-2](2 words)
constexpr int BJJ_STEPS = 254;
constexpr int BJJ_EMIT_STEPS = 32;                           // ladder steps per k_emit_bjj work item
constexpr int BJJ_SCRATCH_STEPS = 256;                       // k_bjj_core: SEGS lanes per witness x 256 / SEGS steps
constexpr int BJJ_SEGS_DEFAULT = 32;                        // k_bjj_core lanes per witness; A/B 8 / 16 / 32: 2.00 / 1.47 / 1.22 ms per 2048 witnesses
constexpr int BJJ_RC_SEGS_DEFAULT = 64;                     // k_bjj_core_rc (recompute, no scratch): lanes per witness
constexpr int BJJ_TABLE_WINDOWS = 32;                        // fixed-base table: 32 windows x 256 x (x, y, t2d)
constexpr int BJJ_SCRATCH_FR = 9 * BJJ_SCRATCH_STEPS;        // per witness, for any segment count
constexpr int BJJ_CORE_FR = 5 * BJJ_STEPS;                  // per step: Dx, Dy, Ax, Ay, inv(Dx)   (Montgomery)
constexpr int SMT_LEVELS = 80;
constexpr int SMT_CHAIN_LANES = 4;                          // k_smt_chain: lanes per witness (one PoseidonHash(2) group)
constexpr int SMT_PREP_LANES = 8;                           // k_smt_prep: lanes per witness (10 levels each)
constexpr int SMT_CORE_FR = 3 * SMT_LEVELS + 2;             // inv(sibling), root, flags per level; j; inv(root-root0)
// the quad SMT chain's constant table (smt_chain4.hpp k_qc_build; Montgomery-form Fr entries, width 3)
constexpr int QC_RP = 57;                    // partial rounds of width 3 (pos_rp(3))
constexpr int QC_INIT = 0;                   // [C0, C1, C2, 0]: per quad, the initial Ark constants
constexpr int QC_FULL = 4;                   // 8 records of 16: full rounds 0..6, then the hash; per quad 4 entries
constexpr int QC_PART = QC_FULL + 8 * 16;    // 57 records of 10 (QC_P_*)
constexpr int QC_R2 = QC_PART + QC_RP * 10;  // R^2 mod p (normal form -> Montgomery)
constexpr int QC_SIZE = QC_R2 + 1;
// a partial-round record: the step-2 multipliers (quad 0 S0, quad 1 S'1, quad 2 S'2), the step-3 row constants S1,
// S2, the constant terms K0, K1, K2, the Montgomery one and a zero
enum { QC_P_S0 = 0, QC_P_SP1, QC_P_SP2, QC_P_S1, QC_P_S2, QC_P_K0, QC_P_K1, QC_P_K2, QC_P_ONE, QC_P_ZERO };

constexpr int POS_MAX_T = 6;
__host__ __device__ inline int pos_nrp(int t) {
  return t == 2 ? 56 : t == 3 ? 57 : t == 4 ? 56 : t == 5 ? 60 : 60;
}
// round states kept per permutation: X0..X3, Y0..Y_RP, Z1..Z3 (t each)
__host__ __device__ inline int pos_core_len(int t) { return (pos_nrp(t) + 8) * t; }
// signals of PoseidonEx(n,1)
__host__ __device__ inline uint32_t pos_ex_size(int n) {
  int t = n + 1, RP = pos_nrp(t);
  return (uint32_t)((2 + n) + 8 * (2 * t) + 8 * t * 4 + 7 * (2 * t + 2 * t * t) + RP * (4 + 4 * t) + (3 * t + 1));
}
__host__ __device__ inline uint32_t pos_hash_size(int n) { return 1 + n + pos_ex_size(n); }
__host__ __device__ constexpr uint32_t pos_hash_size_c(int n) {
  return 1 + n + (uint32_t)((2 + n) + 8 * (2 * (n + 1)) + 8 * (n + 1) * 4 + 7 * (2 * (n + 1) + 2 * (n + 1) * (n + 1)) +
                            (n + 1 == 2 ? 56 : n + 1 == 3 ? 57 : n + 1 == 4 ? 56 : 60) * (4 + 4 * (n + 1)) +
                            (3 * (n + 1) + 1));
}

// Poseidon parameters on device: per t, offsets (in Fr) into one constant array, Montgomery form
struct PosParamIndex {
  int32_t nrp[POS_MAX_T + 1];
  int32_t c_off[POS_MAX_T + 1];
  int32_t m_off[POS_MAX_T + 1];
  int32_t p_off[POS_MAX_T + 1];
  int32_t s_off[POS_MAX_T + 1];
};

// .sym-mapped output (mapsink.hpp): keep bitmap over the O0 signal indices and the number of kept
// signals below every 64-signal boundary; bits == nullptr: the O0 layout
struct KeepMap {
  const uint64_t* bits;
  const uint32_t* rank;
};

// everything the kernels need about an instance (device copy lives in Instance)
struct DevLayout {
  uint64_t wit_size;      // elements per witness
  uint64_t n_inputs;      // elements per input row
  uint64_t n_derived;     // derived message elements per witness (RSA-PSS MGF1 / M' hasher inputs)
  uint32_t n_regions, n_work;
  uint32_t n_sha, sha_core_words;   // SHA jobs; u32 words of SHA core per witness
  uint32_t n_pos, pos_core_elems;   // Poseidon tasks; Fr per witness of Poseidon core
  uint32_t n_values;                // value-store slots per witness (Fr, Montgomery)
  uint32_t n_pos_levels;
  const Region* regions;
  const Work* work;
  const GenPiece* gen_pieces;
  const uint32_t* sha_prog;         // SHA block program (sha_prog.hpp)
  const uint16_t* pos_prog;         // Poseidon block programs (pos_prog.hpp), at pos_prog_off[t]
  uint32_t pos_prog_off[POS_MAX_T + 1];
  const ShaJob* sha;
  const PosTask* pos;
  const uint32_t* pos_level_start;  // tasks sorted by level: [start_l, start_{l+1})
  RegInfo reg;
  uint32_t rsa_core_words;          // u64 per witness
  uint32_t bjj_core_fr, smt_core_fr;
  // ECDSA (ec_common.hpp)
  const uint64_t* ec_gpow;          // fixed-base table [PARTS][256][2][N] chunks (ec_common.hpp)
  const uint32_t* ec_prog;          // table-block descriptor programs, at ec_prog_off[type]
  uint32_t ec_prog_off[3], ec_tab_n[3];
  const uint32_t* ec_tab_off;       // entry offset of table op t inside a witness's tables
  uint32_t ec_tab_entries;          // table entries per witness
  KeepMap keep;                     // direct emission into a .sym-mapped witness (mapsink.hpp)
  const uint32_t* mprog;            // mapped: kept descriptors of the SHA / Poseidon / EC table work items, at Work.pad
  uint32_t pos_nomix;               // mapped: bit t set when no width-t block keeps a GetSum signal (k_emit_pos LDS size)
};

}  // namespace pzk
