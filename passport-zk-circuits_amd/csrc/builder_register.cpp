// RegisterIdentityBuilder layout (registerIdentityBuilder.circom:41-196).
//
// Walks the component tree in creation order and emits one region per contiguous run of
// signals that shares a closed-form generator. Sizes are re-derived here from the
// templates (cited inline); the CPU oracle derives them independently and the parity tests
// compare every element.
#include "builder_impl.hpp"
#include "ec_common.hpp"
#include "mm_prog.hpp"

namespace pzk {

namespace {

// sizes of small templates (own signals + subcomponents)
constexpr uint32_t SZ_ISEQUAL = 6;        // IsEqual: out | in[2] | IsZero(out, in, inv)
constexpr uint32_t SZ_SWITCHER = 6;       // Switcher: out[2] | bool, in[2] | aux
uint32_t sz_num2bits(int L) { return 2 * L + 1 + (L == 254 ? 254 + 383 + 271 : 0); }  // + AliasCheck
uint32_t sz_bits2num(int L) { return 2 * L + 1 + (L == 254 ? 254 + 383 + 271 : 0); }

int log_ceil(int n) { int i = 0; while (n) { n >>= 1; i++; } return i; }
int get_a_coeff(int a) { return a == 8 ? 70 : a == 16 ? 211 : a == 32 ? 640 : a == 64 ? 1940 : a == 128 ? 5881 : 1 << 30; }
uint32_t sz_karatsuba(int N) { return N == 1 ? 4 : 4 * N + 3 * sz_karatsuba(N / 2); }
uint32_t sz_bmneq(int G, int L) { return (G + L - 1) + G + L + G * L + (G + L - 1) * L; }

}  // namespace

bool ec_programs(Layout& L, std::string& why);
void ec_verify_regions(Builder& b, int cv, int IN_PK, int IN_SIG, int J_SA);

// BigMultModP(64,K,K,K) block size (bigInt.circom:206-272)
uint32_t modmul_size(int K) {
  int BASE = 2 * K, DIV = K + 1, MAX = 128 + log_ceil(K + DIV - 1);
  bool kara = (K & (K - 1)) == 0 && K >= 8 && get_a_coeff(K) <= K * K;
  uint32_t bmo = (BASE - 1) + 2 * K + (kara ? sz_karatsuba(K) : sz_bmneq(K, K));
  uint32_t bgt = 1 + 2 * K + (1 + 2 * K + K + K * ((3 + sz_num2bits(65)) + SZ_ISEQUAL));
  uint32_t bisz = (BASE - 1) + (BASE - 2) + (BASE - 2) * sz_num2bits(MAX + 3 - 64);
  return DIV + K + 3 * K + bmo + K * sz_num2bits(64) + bgt + sz_bmneq(DIV, K) + bisz;
}

bool build_register(const pzk_params& p, Layout& L, std::string& why) {
  // RSA-PSS: 10-12 RSA-2048 SHA-256 (e = 3 for 10, salt 64 for 12), 13 RSA-2048 SHA-384 salt 48, 14 RSA-3072 SHA-256
  // (signatureVerification.circom:46-75)
  const bool pss = p.signature_type >= 10 && p.signature_type <= 14;
  // RSA exponent (signatureVerification.circom:14-75): 3 for SIG 10, 37187 for SIG 4, else 65537
  const long EXP = p.signature_type == 10 ? 3 : p.signature_type == 4 ? 37187 : 65537;
  const int cv = ec_curve_of_sig(p.signature_type);
  if (p.signature_type == 22 || p.signature_type == 23) {
    why = "SIGNATURE_TYPE " + std::to_string(p.signature_type) +
          ": verifyECDSABits reads hashed[] past its end (ecdsa.circom:31-37, 5 x 64 / 3 x 64 chunks of a 256 / 160-bit "
          "hash), so the reference circuit does not compile";
    return false;
  }
  if ((p.signature_type < 1 || p.signature_type > 4) && !pss && cv < 0) {
    why = "SIGNATURE_TYPE " + std::to_string(p.signature_type) +
          " not supported (RSA PKCS#1 v1.5 types 1-4, RSA-PSS types 10-14, ECDSA 20, 21, 24, 25 are)";
    return false;
  }
  const bool ecdsa = cv >= 0;
  // DG_HASH_TYPE 160, 224, 256 or 384. HASH_TYPE (SA hasher, passportVerificationBuilder.circom:16-59): 160 for
  // SIG 3 / 4, 384 for SIG 13 / 25, 224 for SIG 24, else 256; EC_HASH_TYPE (EC hasher, :53) is the HASH_TYPE before
  // SIG 24 sets 224, so 256 there. The flow's `encapsulatedContentHash[i], i < HASH_SIZE` loop
  // (passportVerificationFlow.circom:36-40) runs over the DG hash bits, so DG <= EC_HASH_TYPE or the reference cannot
  // compile.
  if (p.dg_hash_type != 256 && p.dg_hash_type != 224 && p.dg_hash_type != 160 && p.dg_hash_type != 384) {
    why = "DG_HASH_TYPE must be 160, 224, 256 or 384";
    return false;
  }
  const bool sha1_sig = p.signature_type == 3 || p.signature_type == 4;
  const int DG = p.dg_hash_type,
            HT = sha1_sig ? 160 : (p.signature_type == 13 || p.signature_type == 25) ? 384 : p.signature_type == 24 ? 224 : 256;
  const int EHT = p.signature_type == 24 ? 256 : HT;
  if (DG > EHT) {
    why = "DG_HASH_TYPE " + std::to_string(DG) + " is wider than this SIGNATURE_TYPE's encapsulated-content hash (" +
          std::to_string(EHT) + "): passportVerificationFlow.circom:36-40 would read encapsulatedContentHash past its end";
    return false;
  }
  // HASH_BLOCK_SIZE / DG_HASH_BLOCK_SIZE (registerIdentityBuilder.circom:95-102): 1024-bit blocks above 256-bit hashes
  const int HBS = HT > 256 ? 1024 : 512, DBS = DG > 256 ? 1024 : 512;
  if (p.document_type != 1 && p.document_type != 3) { why = "DOCUMENT_TYPE must be 1 or 3"; return false; }
  // AA_SIGNATURE_ALGO: 0 none, 1..19 RSA-1024 key (identity.circom:25-49), >= 20 EC key (:51-84); the raw value
  // also scales the DG15 IsEqual inputs of the flow (passportVerificationFlow.circom:45-46,73-74)
  if (p.aa_signature_algo < 0 || p.aa_signature_algo > 25) { why = "AA_SIGNATURE_ALGO must be 0..25"; return false; }
  const bool aa_ec = p.aa_signature_algo >= 20;
  const int aa_f = p.aa_signature_algo == 22 ? 320 : p.aa_signature_algo == 23 ? 192 : 256;
  const int aa_hs = p.aa_signature_algo == 23 ? 192 : 248;
  // signature / pubkey input length: 2 x CHUNK_NUMBER for ECDSA (registerIdentityBuilder.circom:124-135)
  const int K = ecdsa ? 2 * EC_GEO[cv].nl : p.signature_type == 2 ? 64 : (p.signature_type == 14 || p.signature_type == 4) ? 48 : 32;
  const int ecB = p.ec_block_number, d15B = p.dg15_block_number;
  const bool aa = p.aa_signature_algo != 0;
  if (ecB < 1 || ecB > 16 || d15B < 0 || d15B > 16 || (aa && d15B < 1)) { why = "block numbers out of range"; return false; }
  const int ecLen = HBS * ecB, d15Len = HBS * d15B;
  if (HBS != DBS && d15B) {
    why = "dg15 block sizes differ: registerIdentityBuilder.circom:151 assigns dg15[DG15_BLOCK_NUMBER * HASH_BLOCK_SIZE] to "
          "RegisterIdentity's dg15[DG15_SIZE * DG_HASH_BLOCK_SIZE] (identity.circom:22)";
    return false;
  }
  // (64-bit sums: the shifts are caller-supplied int32)
  const int64_t dg15shift = aa ? p.dg15_shift : DG;
  if (p.dg1_shift < 0 || (int64_t)p.dg1_shift + DG > ecLen || dg15shift < 24 || dg15shift + DG > ecLen ||
      p.ec_shift < 0 || (int64_t)p.ec_shift + HT > 1024 ||
      (aa && (p.aa_shift < 0 || (int64_t)p.aa_shift + (aa_ec ? 2 * aa_f : 1024) > d15Len))) {
    why = "shift parameters address bits outside the inputs";
    return false;
  }
  const int chunk = p.document_type == 1 ? 190 : 186;

  Builder b(L);
  // flat inputs in witness order (public first): root, ec, dg1, dg15, sa, signature, pubkey, branches, sk
  const int IN_ROOT = 0, IN_EC = 1, IN_DG1 = IN_EC + ecLen, IN_DG15 = IN_DG1 + 1024, IN_SA = IN_DG15 + d15Len,
            IN_SIG = IN_SA + 1024, IN_PK = IN_SIG + K, IN_BR = IN_PK + K, IN_SK = IN_BR + 80;
  L.n_inputs = IN_SK + 1;
  L.n_outputs = 4;
  L.n_public = 1;
  L.inputs = {{"slaveMerkleRoot", (uint64_t)IN_ROOT, 1},   {"encapsulatedContent", (uint64_t)IN_EC, (uint64_t)ecLen},
              {"dg1", (uint64_t)IN_DG1, 1024},             {"dg15", (uint64_t)IN_DG15, (uint64_t)d15Len},
              {"signedAttributes", (uint64_t)IN_SA, 1024},  {"signature", (uint64_t)IN_SIG, (uint64_t)K},
              {"pubkey", (uint64_t)IN_PK, (uint64_t)K},     {"slaveMerkleInclusionBranches", (uint64_t)IN_BR, 80},
              {"skIdentity", (uint64_t)IN_SK, 1}};
  L.is_register = true;
  L.params = p;
  L.reg.K = K;
  L.reg.in_pk = IN_PK;
  L.reg.in_sig = IN_SIG;
  L.reg.in_br = IN_BR;
  L.reg.in_root = IN_ROOT;
  L.reg.in_dg1 = IN_DG1;
  L.reg.in_dg15 = IN_DG15;
  L.reg.aa = aa ? 1 : 0;
  L.reg.aa_shift = p.aa_shift;
  L.reg.aa_ec = aa_ec ? 1 : 0;
  L.reg.aa_f = aa_f;
  L.reg.aa_hs = aa_hs;
  L.reg.ecdsa = ecdsa ? 1 : 0;
  L.reg.ec_curve = ecdsa ? cv : 0;
  L.reg.ec_nl = ecdsa ? EC_GEO[cv].nl : 0;
  L.reg.ec_cs = ecdsa ? EC_GEO[cv].cs : 0;
  L.is_ecdsa = ecdsa;
  if (ecdsa && !ec_programs(L, why)) return false;

  // ---- value-store slots that feed Poseidon tasks (filled by k_prep / core kernels)
  const int V_ONE = b.value();        // Montgomery 1 (SMTHash1 in[2])
  const int V_SK = b.value();
  int V_PK[5], V_AA[5], V_DG1[4];
  for (int i = 0; i < 5; i++) V_PK[i] = b.value();
  for (int i = 0; i < 5; i++) V_AA[i] = b.value();
  for (int i = 0; i < 4; i++) V_DG1[i] = b.value();
  const int V_SANUM = b.value();
  const int V_BJJ_X = b.value(), V_BJJ_Y = b.value();
  int V_L[80], V_R[80];
  for (int i = 0; i < 80; i++) { V_L[i] = b.value(); V_R[i] = b.value(); }
  L.loads.push_back(ValueLoad{V_SK, IN_SK});
  const int V_PKX = b.value(), V_PKY = b.value();
  L.reg.v_pkx = V_PKX; L.reg.v_pky = V_PKY;
  L.reg.v_one = V_ONE; L.reg.v_sk = V_SK; L.reg.v_pk = V_PK[0]; L.reg.v_aa = V_AA[0]; L.reg.v_dg1 = V_DG1[0];
  L.reg.v_sanum = V_SANUM; L.reg.v_bjj = V_BJJ_X; L.reg.v_smt_lr = V_L[0];
  L.reg.dg1_chunk = chunk;

  // Poseidon tasks are created where their components are created (creation order = layout
  // order); region() records the block. Levels encode the data dependencies:
  //   0: pk hash, sk hash, AA hash, passportHash, pkIdentity hash (after BJJ core)
  //   1: SMT leaf (needs pk hash), dg1Commitment (needs sk hash)
  //   2: SMT level hashes (need the leaf / key bits)

  // =========================== main: [1 | outputs(4) | inputs] =========================
  b.region(RK_ONE, 1);
  const uint32_t r_out = b.region(RK_VALUE, 4, {-1});  // outputs patched below (4 slots, non-contiguous)
  b.region(RK_INCOPY, L.n_inputs, {0});

  // =========================== PassportVerificationBuilder ============================
  // own: passportHash | inputs (ec, dg1, dg15, sa, sig, pk, branches, root) | dg1Hash, dg15Hash, ecHash, saHash,
  //      pubkeyHash, tempModulus[5]
  const uint32_t r_pvb_out = b.region(RK_VALUE, 1, {-1});
  b.region(RK_INCOPY, IN_SK - IN_EC, {IN_EC});
  b.region(RK_INCOPY, 1, {IN_ROOT});
  // SHA jobs are created when the hashers are created; their digests are referenced earlier,
  // so reserve the job ids first (creation order dg1, dg15, ec, sa).
  const int J_DG1 = b.hash_job(DG, IN_DG1, 1024 / DBS);
  const int J_DG15 = aa ? b.hash_job(DG, IN_DG15, d15B) : -1;  // the first d15B x DG_HASH_BLOCK_SIZE bits (:117-120)
  const int J_EC = b.hash_job(EHT, IN_EC, ecB);
  const int J_SA = b.hash_job(HT, IN_SA, 1024 / HBS);
  L.reg.j_dg1 = J_DG1; L.reg.j_dg15 = J_DG15; L.reg.j_ec = J_EC; L.reg.j_sa = J_SA;
  b.region(RK_DIGEST, DG, {J_DG1});
  if (aa) b.region(RK_DIGEST, DG, {J_DG15});
  else b.region(RK_VALUE, DG, {-2});  // dg15Hash <== 0 (zeros)
  b.region(RK_DIGEST, EHT, {J_EC});
  b.region(RK_DIGEST, HT, {J_SA});
  const uint32_t r_pkhash = b.region(RK_VALUE, 1, {-1});
  if (ecdsa) b.region(RK_EC_PKBITS, 2 * EC_GEO[cv].fb, {IN_PK, EC_GEO[cv].nl, EC_GEO[cv].cs});  // ecBitsX[F], ecBitsY[F]
  else b.region(RK_TEMPMOD, 5, {IN_PK});
  auto sha_blocks = [&](int job, int in_off, int blocks) {
    if (L.sha[job].algo == 1) { b.sha1_regions(job, in_off, blocks, true); return; }  // ShaHashChunks(B, 160)
    if (L.sha[job].algo >= 3) { b.sha512_regions(job, in_off, blocks, true); return; }  // ShaHashChunks(B, 384 | 512)
    const int O = L.sha[job].algo == 2 ? 224 : 256;  // ShaHashChunks(B, 224 | 256)
    uint64_t own = O + 512ull * blocks + O + 512ull * blocks + 256ull * (blocks + 1) + 256;
    b.region(RK_SHA_OWN, own, {job, blocks, in_off, 1, O});
    for (int m = 0; m < blocks; m++) b.region(RK_SHA_BLOCK, 150762, {job, m});
  };
  sha_blocks(J_DG1, IN_DG1, 1024 / DBS);
  if (aa) sha_blocks(J_DG15, IN_DG15, d15B);
  sha_blocks(J_EC, IN_EC, ecB);
  sha_blocks(J_SA, IN_SA, 1024 / HBS);
  // PassportVerificationFlow(ecLen, DG, EHT, DG1_SHIFT, DG15_ACTUAL_SHIFT, EC_SHIFT, AA): 3 DG + 8 IsEqual
  b.region(RK_FLOW, 1 + 2 * DG + ecLen + EHT + 1024 + (3 * DG + 8) * (1 + SZ_ISEQUAL),
           {J_DG1, J_DG15, J_EC, J_SA, IN_EC, IN_SA, p.dg1_shift, (int32_t)dg15shift, p.ec_shift, p.aa_signature_algo});
  L.bjj_core_fr = BJJ_CORE_FR;
  L.smt_core_fr = SMT_CORE_FR;
  if (ecdsa) {
    ec_verify_regions(b, cv, IN_PK, IN_SIG, J_SA);
  } else {
    // PowerMod(64,K,EXP): out[K] | base[K], modulus[K] | muls[], resultMuls[] (bigInt.circom:280-340).
    // exp_to_bits(65537) = [16, 2, 0, 16], exp_to_bits(3) = [1, 2, 0, 1]: muls[i] = muls[i-1]^2
    // (muls[0] = base^2), then resultMuls[0] = base * muls[last]
    // exp_to_bits(EXP): bit-length - 1 squarings muls[i] = muls[i-1]^2 (muls[0] = base^2), then one
    // resultMuls per further set bit: resultMuls[0] = (bit 0 ? base : muls[b0-1]) * muls[b1-1],
    // resultMuls[i] = resultMuls[i-1] * muls[b_{i+1}-1]
    int ones[64], n_ones = 0, nbits = 0;
    for (long v = EXP; v > 0; v >>= 1, nbits++)
      if (v & 1) ones[n_ones++] = nbits;
    const int nsq = nbits - 1, n_modmul = nsq + n_ones - 1;
    if (n_modmul > 32 || n_ones < 2) { why = "internal: PowerMod schedule"; return false; }
    for (int i = 0; i < nsq; i++) L.reg.mm_x[i] = L.reg.mm_y[i] = (int8_t)(i == 0 ? -1 : i - 1);
    for (int i = 0; i + 1 < n_ones; i++) {
      const int k = nsq + i;
      L.reg.mm_x[k] = (int8_t)(i == 0 ? (ones[0] == 0 ? -1 : ones[0] - 1) : k - 1);
      L.reg.mm_y[k] = (int8_t)(ones[i + 1] - 1);
    }
    auto power_mod = [&]() -> bool {
      b.region(RK_RSA_OUT, K);
      b.region(RK_INCOPY, K, {IN_SIG});
      b.region(RK_INCOPY, K, {IN_PK});
      const uint32_t mm = modmul_size(K);
      L.reg.modmul_size = mm;
      if (mm_section_start(K, MM_SECTIONS) != mm) { why = "internal: BigMultModP section sizes"; return false; }
      L.reg.n_modmul = n_modmul;
      L.rsa_core_words = n_modmul * MM_CORE_WORDS(K);
      for (int i = 0; i < n_modmul; i++) b.region(RK_MODMUL, mm, {i, IN_PK});
      return true;
    };
    // VerifySignature(SIG): pubkey[K], signature[K], hashed[256] | RsaVerifyPkcs1v15 or VerifyRsaPssSig
    b.region(RK_INCOPY, K, {IN_PK});
    b.region(RK_INCOPY, K, {IN_SIG});
    b.region(RK_DIGEST, HT, {J_SA});
    if (HT == 160) {
      //   RsaVerifyPkcs1v15(64,K,65537,160) (rsa.circom:73-109): signature, pubkey, hashed[160] | hashed_chunks[2]
      //   (never assigned) | pm, bits2num[0..1], getBits = Num2Bits(64)(EM limb 2), getDiv = Bits2Num(32)(its top bits)
      b.region(RK_INCOPY, K, {IN_SIG});
      b.region(RK_INCOPY, K, {IN_PK});
      b.region(RK_DIGEST, 160, {J_SA});
      b.region(RK_VALUE, 2, {-2});
      if (!power_mod()) return false;
      for (int i = 0; i < 2; i++) b.region(RK_BITS2NUM, sz_bits2num(64), {64, 1, 159 - 64 * i, -1, J_SA});
      b.region(RK_NUM2BITS, sz_num2bits(64), {64, 1, 2});
      b.region(RK_BITS2NUM, sz_bits2num(32), {32, 2, 32, 1, 2});
    } else if (!pss) {
      //   RsaVerifyPkcs1v15(64,K,65537,256): signature, pubkey, hashed | hashed_chunks[4] | pm, bits2num[3..0], num2bits_6
      b.region(RK_INCOPY, K, {IN_SIG});
      b.region(RK_INCOPY, K, {IN_PK});
      b.region(RK_DIGEST, 256, {J_SA});
      b.region(RK_HCHUNK, 4, {J_SA, 4, 64});
      if (!power_mod()) return false;
      for (int i = 0; i < 4; i++) b.region(RK_BITS2NUM, sz_bits2num(64), {64, 1, i * 64 + 63, -1, J_SA});
      b.region(RK_NUM2BITS, sz_num2bits(64), {64, 1, 6});  // Num2Bits(64)(EM limb 6)
    } else {
      //   VerifyRsaPssSig(64,K,SALT,EXP,H) (rsaPss.circom:18-254): pubkey, signature, hashed | eM .. mDash
      //   | powerMod, num2Bits[K], bits2Num[8K], MGF1_H, xor, hDash (pss.hpp); H = 384, salt 48 for SIG 13
      const int H = HT, S8 = p.signature_type == 12 ? 512 : p.signature_type == 13 ? 384 : 256, EML = 8 * K,
                DBL = EML - H / 8 - 1, DB8 = 8 * DBL, IT = DBL / (H / 8) + 1, BS = H > 256 ? 1024 : 512;
      b.region(RK_INCOPY, K, {IN_PK});
      b.region(RK_INCOPY, K, {IN_SIG});
      b.region(RK_DIGEST, H, {J_SA});
      b.region(RK_PSS_OWN, EML + 64 * K + K + 3 * DB8 + S8 + H + 1024, {S8});
      if (!power_mod()) return false;
      for (int i = 0; i < K; i++) b.region(RK_NUM2BITS, sz_num2bits(64), {64, 1, K - 1 - i});  // EM limb K-1-i
      b.region(RK_PSS_B2N8, 17 * EML);
      //   Mgf1ShaH(H/8, DB) (mgf1.circom:5-133): out | seed | hashed, then (ShaHashChunks(1,H), Num2Bits(32))
      //   per block; the hashers read derived messages (ShaJob.src = 1)
      b.region(RK_PSS_MGF, DB8 + H + H * IT);
      L.reg.j_mgf = (int)L.sha.size();
      L.reg.n_mgf = IT;
      for (int c = 0; c < IT; c++) {
        if (H > 256) b.sha512(BS * c, 1, H, 1, true);
        else b.sha256(BS * c, 1, true, 1);
        b.region(RK_PSS_CTR, sz_num2bits(32), {c});
      }
      b.region(RK_PSS_XOR, 3 * DB8);
      // hDash: ShaHashChunks(2, 256) or ShaHashChunks(1, 384) over the 1024-bit M'
      L.reg.j_hd = H > 256 ? b.sha512(BS * IT, 1, H, 1, true) : b.sha256(BS * IT, 2, true, 1);
      L.reg.pss_s8 = S8;
      L.reg.pss_h = H;
      L.n_derived = (uint64_t)BS * IT + 1024;
    }
  }
  // signedAttributesNum = Bits2Num(252)(saHash[0..251]), or of 252 - HT zeros | saHash[0..HT-1] for HT < 252
  b.region(RK_BITS2NUM, sz_bits2num(252), {252, 1, HT < 252 ? HT - 252 : 0, 1, J_SA});
  int S_PKH;
  if (ecdsa) {
    // num2bitsX[i], num2bitsY[i] (Num2Bits(CS)), xToNum, yToNum (Bits2Num(F - DIFF), F - DIFF = min(F, 248)),
    // PoseidonHash(2) (passportVerificationBuilder.circom:193-230)
    const int N = EC_GEO[cv].nl, CS = EC_GEO[cv].cs, F = EC_GEO[cv].fb, FD = F > 248 ? 248 : F;
    for (int i = 0; i < N; i++) {
      b.region(RK_EC_N2B, sz_num2bits(CS), {1, IN_PK + i, CS});
      b.region(RK_EC_N2B, sz_num2bits(CS), {1, IN_PK + N + i, CS});
    }
    b.region(RK_EC_B2N248, sz_bits2num(FD), {IN_PK, N, CS, FD});
    b.region(RK_EC_B2N248, sz_bits2num(FD), {IN_PK + N, N, CS, FD});
    S_PKH = b.poseidon(2, {V_PKX, V_PKY}, 0);
  } else {
    // pubkeyHasherRsa = PoseidonHash(5)
    S_PKH = b.poseidon(5, {V_PK[0], V_PK[1], V_PK[2], V_PK[3], V_PK[4]}, 0);
  }
  // ---- SMTVerifier(80): isVerified | root, leaf, key, siblings[80] | value
  //      | hash1New, n2bNew, smtLevIns, sm[80], levels[79..0], isEqual
  b.region(RK_SMT_OWN, 1 + 3 + 80 + 1, {IN_ROOT, IN_BR});
  b.region(RK_SMTHASH, 3, {-1});
  const int S_LEAF = b.poseidon(3, {S_PKH, S_PKH, V_ONE}, 1);
  b.region(RK_NUM2BITS, sz_num2bits(254), {254, 0, S_PKH});
  b.region(RK_LEVINS, 80 + 80 + 79 + 80 * 3, {IN_BR});
  b.region(RK_SM, 80 * 4);
  int S_H[80];
  for (int i = 0; i < 80; i++) S_H[i] = b.value();  // level hashes: contiguous slots
  for (int i = 79; i >= 0; i--) {
    b.region(RK_SMT_LEVEL, 8, {i, IN_BR});
    b.region(RK_SMTHASH, 3, {i});
    b.poseidon(2, {V_L[i], V_R[i]}, 2, S_H[i]);
    L.pos.back().smt_level = i;
    b.region(RK_SWITCHER, SZ_SWITCHER, {i, IN_BR});
  }
  b.region(RK_ISEQ_ROOT, SZ_ISEQUAL, {IN_ROOT});
  L.reg.v_pkhash = S_PKH; L.reg.v_leaf = S_LEAF; L.reg.v_smt_h = S_H[0];
  L.reg.v_smt_key = L.reg.v_smt_val = S_PKH;  // SMTVerifier key = leaf = the pubkey hash (passportVerificationBuilder.circom:232-239)
  for (int i = 1; i < 80; i++)
    if (S_H[i] != S_H[0] + i) { why = "internal: SMT hash slots not contiguous"; return false; }
  // signedAttributesHashHasher = PoseidonHash(1)(signedAttributesNum)
  const int S_PASS = b.poseidon(1, {V_SANUM}, 0);

  // =========================== RegisterIdentity ============================
  // own: dg15PubKeyHash, dg1Commitment, pkIdentityHash | dg1[1024], dg15[d15Len], skIdentity
  const uint32_t r_rid_out = b.region(RK_VALUE, 3, {-1});
  b.region(RK_INCOPY, 1024, {IN_DG1});
  if (d15Len) b.region(RK_INCOPY, d15Len, {IN_DG15});
  b.region(RK_INCOPY, 1, {IN_SK});
  int S_AA = -1;
  if (aa && aa_ec) {
    // xToNum, yToNum = Bits2Num(HASH_SIZE) of the key's low bits, in[HS-1-i] = dg15[AA_SHIFT + XY + i] (+ EC_FIELD_SIZE for y)
    const int xy = aa_f - aa_hs;
    b.region(RK_BITS2NUM, sz_bits2num(aa_hs), {aa_hs, 0, IN_DG15 + p.aa_shift + xy + aa_hs - 1, -1});
    b.region(RK_BITS2NUM, sz_bits2num(aa_hs), {aa_hs, 0, IN_DG15 + p.aa_shift + aa_f + xy + aa_hs - 1, -1});
    S_AA = b.poseidon(2, {V_AA[0], V_AA[1]}, 0);
  } else if (aa) {
    for (int j = 0; j < 4; j++) b.region(RK_BITS2NUM, sz_bits2num(200), {200, 0, IN_DG15 + p.aa_shift + j * 200 + 199, -1});
    b.region(RK_BITS2NUM, sz_bits2num(224), {224, 0, IN_DG15 + p.aa_shift + 800 + 223, -1});
    S_AA = b.poseidon(5, {V_AA[0], V_AA[1], V_AA[2], V_AA[3], V_AA[4]}, 0);
  }
  // dg1Hasher is created before dg1Chunking[i] (identity.circom:89-92); its 5th input is P1(sk)
  const size_t dg1_task = L.pos.size();
  const int S_DG1C = b.poseidon(5, {V_DG1[0], V_DG1[1], V_DG1[2], V_DG1[3], -1}, 1);
  for (int i = 0; i < 4; i++) b.region(RK_BITS2NUM, sz_bits2num(chunk), {chunk, 0, IN_DG1 + i * chunk, 1});
  const int S_SKH = b.poseidon(1, {V_SK}, 0);
  L.pos[dg1_task].in_slot[4] = S_SKH;
  // BabyjubjubBase8Multiplication: out[2] | scalar | getBase8, num2Bits(254), adders/doublers
  b.region(RK_BJJ_OWN, 3 + 2);
  b.region(RK_NUM2BITS, sz_num2bits(254), {254, 0, V_SK});
  b.region(RK_BJJ_STEPS, 46 + 253 * 60);
  const int S_PKID = b.poseidon(2, {V_BJJ_X, V_BJJ_Y}, 3);  // level 3: after the BJJ core joins

  // outputs: main [dg15PubKeyHash, passportHash, dg1Commitment, pkIdentityHash]
  L.out_slots = {aa ? S_AA : -2, S_PASS, S_DG1C, S_PKID};
  auto set_value = [&](uint32_t r, std::vector<int> slots) {
    L.regions[r].a[0] = -3;  // explicit list
    for (size_t i = 0; i < slots.size(); i++) L.regions[r].a[1 + i] = slots[i];
  };
  set_value(r_out, {aa ? S_AA : -2, S_PASS, S_DG1C, S_PKID});
  set_value(r_pvb_out, {S_PASS});
  set_value(r_pkhash, {S_PKH});
  set_value(r_rid_out, {aa ? S_AA : -2, S_DG1C, S_PKID});
  b.finalize();
  return true;
}

}  // namespace pzk
