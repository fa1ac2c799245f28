// RSA-PSS signature check (SIGNATURE_TYPE 10-14): VerifyRsaPssSig(64, K, SALT, EXP, H)
// (rsaPss.circom:18-254) with Mgf1Sha256(32, DB_LEN) / Mgf1Sha384(48, DB_LEN) (mgf1.circom:5-133); H = 384 for SIG 13.
//
// EM = PowerMod.out comes from the RSA core (rsa_coop.hpp). The MGF1 and M' hashers are plain
// ShaHashChunks instances whose message bits are not circuit inputs but functions of EM and of
// other digests. They are materialised once per witness as "derived" 32-byte elements in the
// input-row encoding, which the SHA core and the SHA emitter read in place of the input row
// (ShaJob.src = 1):
//   k_pss_mgf   : EM -> MGF1 messages  seed | counter | padding        (one BS-bit block each, BS = 512 / 1024)
//   k_sha_core over the MGF1 jobs
//   k_pss_mdash : EM, MGF1 digests, SA digest -> M' = 0^64 | mHash | salt | padding (1024 bits: two SHA-256
//                 blocks or one SHA-384 block)
//   k_sha_core over the M' job
// The checks (assert eM[0] == 188, hDash256.out === hash) run in k_rsa_check; every other PSS
// signal is a closed-form function of EM and the digests (pss_small, emitted by k_emit_gen).
#pragma once
#include "fr.hpp"
#include "layout.hpp"
#include "sha.hpp"

namespace pzk {

struct PssView {
  const uint64_t* em;   // EM limbs, K x 64 bits, least significant first
  const uint32_t* sha;  // this witness's SHA core
  const ShaJob* jobs;
  int K, s8, h, j_mgf, j_hd, j_sa;

  __device__ __forceinline__ int emb() const { return 64 * K; }
  __device__ __forceinline__ int db8() const { return 8 * (8 * K - h / 8 - 1); }
  __device__ __forceinline__ int bs() const { return h > 256 ? 1024 : 512; }
  // eMsgInBits[t] (rsaPss.circom:45-53): EM bit t counted from the most significant
  __device__ __forceinline__ uint32_t em_bit(int t) const {
    const int i = emb() - 1 - t;
    return (uint32_t)(em[i >> 6] >> (i & 63)) & 1u;
  }
  // byte k of EM, least significant first = eM[k] (:55-61)
  __device__ __forceinline__ uint32_t em_byte(int k) const { return (uint32_t)(em[k >> 3] >> (8 * (k & 7))) & 0xFFu; }
  __device__ __forceinline__ uint32_t dig(int job, int i) const {  // digest bit i (MSB first) of a SHA job
    const ShaJob& J = jobs[job];
    const uint32_t* H = sha + J.hout;  // big-endian 32-bit words for every algorithm
    return (H[i >> 5] >> (31 - (i & 31))) & 1u;
  }
  __device__ __forceinline__ uint32_t hash_bit(int i) const { return em_bit(emb() - h - 8 + i); }   // hash (:86-89)
  __device__ __forceinline__ uint32_t mgf_bit(int i) const { return dig(j_mgf + i / h, i % h); }     // dbMask
  __device__ __forceinline__ uint32_t xor_bit(int i) const { return em_bit(i) ^ mgf_bit(i); }        // xor.out
  __device__ __forceinline__ uint32_t db_bit(int i) const { return i == 0 ? 0u : xor_bit(i); }       // db (:131-138)
  __device__ __forceinline__ uint32_t salt_bit(int k) const { return db_bit(db8() - s8 + k); }      // salt (:141-143)
  // mDash[i] = 0^64 | hashed | salt | padding of a (64 + h + s8)-bit message to 1024 bits (:146-226)
  __device__ __forceinline__ uint32_t mdash_bit(int i) const {
    const int lm = 64 + h + s8;
    if (i < 64) return 0u;
    if (i < 64 + h) return dig(j_sa, i - 64);
    if (i < lm) return salt_bit(i - 64 - h);
    if (i == lm) return 1u;
    if (i >= 1013) return (uint32_t)(lm >> (1023 - i)) & 1u;
    return 0u;
  }
  // concated bit j of MGF1 block c: seed | counter c (MSB first) | padding of an (h + 32)-bit message
  // (mgf1.circom:30-58, 95-121)
  __device__ __forceinline__ uint32_t mgf_msg_bit(int c, int j) const {
    const int lm = h + 32, n = bs();
    if (j < h) return hash_bit(j);
    if (j < lm) return (uint32_t)(c >> (lm - 1 - j)) & 1u;
    if (j == lm) return 1u;
    if (j >= n - 11) return (uint32_t)(lm >> (n - 1 - j)) & 1u;
    return 0u;
  }
};

__device__ __forceinline__ PssView pss_view(const DevLayout& L, const uint64_t* rsa_core, const uint32_t* sha_core,
                                            uint32_t w) {
  PssView v;
  v.K = L.reg.K;
  v.em = rsa_core + (size_t)w * L.rsa_core_words + (size_t)(L.reg.n_modmul - 1) * MM_CORE_WORDS(v.K) + 3 * v.K + 1;
  v.sha = sha_core + (size_t)w * L.sha_core_words;
  v.jobs = L.sha;
  v.s8 = L.reg.pss_s8;
  v.h = L.reg.pss_h;
  v.j_mgf = L.reg.j_mgf;
  v.j_hd = L.reg.j_hd;
  v.j_sa = L.reg.j_sa;
  return v;
}

// derived row of a witness: MGF1 block c at elements [BS c, BS c + BS), M' at [BS n_mgf, + 1024)
#ifndef PZK_TEMPLATE_KERNELS_ONLY  // defined once, in kernels.hip
__global__ void __launch_bounds__(256) k_pss_mgf(DevLayout L, const uint64_t* rsa_core, const uint32_t* sha_core,
                                                 uint8_t* derived) {
  const uint32_t w = blockIdx.y;
  const PssView P = pss_view(L, rsa_core, sha_core, w);
  uint8_t* row = derived + 32ull * w * L.n_derived;
  const int bs = P.bs(), n = bs * L.reg.n_mgf;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x)
    store_u64(row + 32ull * e, P.mgf_msg_bit(e / bs, e % bs));
}
#endif

#ifndef PZK_TEMPLATE_KERNELS_ONLY  // defined once, in kernels.hip
__global__ void __launch_bounds__(256) k_pss_mdash(DevLayout L, const uint64_t* rsa_core, const uint32_t* sha_core,
                                                   uint8_t* derived) {
  const uint32_t w = blockIdx.y;
  const PssView P = pss_view(L, rsa_core, sha_core, w);
  uint8_t* row = derived + 32ull * (w * L.n_derived + (uint64_t)P.bs() * L.reg.n_mgf);
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < 1024; e += gridDim.x * blockDim.x)
    store_u64(row + 32ull * e, P.mdash_bit(e));
}
#endif

// lane checks of VerifyRsaPssSig (called from k_rsa_check)
__device__ __forceinline__ void pss_check(const PssView& P, int32_t* status) {
  if (P.em_byte(0) != 188u) lane_status(status, ST_PSS_TRAILER);  // rsaPss.circom:73
  bool bad = false;
  for (int i = 0; i < P.h; i++) bad |= P.dig(P.j_hd, i) != P.hash_bit(i);
  if (bad) lane_status(status, ST_PSS_HASH);  // rsaPss.circom:182,201,225
}

// signals of the PSS regions (emit_small)
__device__ __forceinline__ El pss_small(const PssView& P, const Region& R, uint32_t s) {
  const int K = P.K, EML = 8 * K, EMB = 64 * K, DB8 = P.db8();
  int i = (int)s;
  switch (R.kind) {
    case RK_PSS_OWN: {  // eM | eMsgInBits | encoded | dbMask | db | salt | maskedDB | hash | mDash
      if (i < EML) return el_u64(P.em_byte(i));
      i -= EML;
      if (i < EMB) return el_u64(P.em_bit(i));
      i -= EMB;
      if (i < K) return el_u64(P.em[i]);
      i -= K;
      if (i < DB8) return el_u64(P.mgf_bit(i));
      i -= DB8;
      if (i < DB8) return el_u64(P.db_bit(i));
      i -= DB8;
      if (i < P.s8) return el_u64(P.salt_bit(i));
      i -= P.s8;
      if (i < DB8) return el_u64(P.em_bit(i));
      i -= DB8;
      if (i < P.h) return el_u64(P.hash_bit(i));
      return el_u64(P.mdash_bit(i - P.h));
    }
    case RK_PSS_B2N8: {  // bits2Num[b] = Bits2Num(8): out | in[8] | sum[8]; in[k] = eMsgInBits[8b + 7 - k]
      const int b = i / 17, j = i - 17 * b;
      const uint32_t v = P.em_byte(EML - 1 - b);
      return el_u64(j == 0 ? v : j <= 8 ? (v >> (j - 1)) & 1u : v & ((1u << (j - 8)) - 1u));
    }
    case RK_PSS_MGF: {  // out[DB8] | seed[h] | hashed[h IT]
      if (i < DB8) return el_u64(P.mgf_bit(i));
      i -= DB8;
      if (i < P.h) return el_u64(P.hash_bit(i));
      return el_u64(P.mgf_bit(i - P.h));
    }
    case RK_PSS_CTR: {  // Num2Bits(32)(c): out[32] | in | sum[32]
      const uint32_t c = (uint32_t)R.a[0];
      return el_u64(i < 32 ? (c >> i) & 1u : i == 32 ? c : c & (uint32_t)mask_lo(i - 32));
    }
    default: {  // RK_PSS_XOR, Xor2 (bitGates.circom:232-240): out | in1 | in2
      if (i < DB8) return el_u64(P.xor_bit(i));
      i -= DB8;
      if (i < DB8) return el_u64(P.em_bit(i));
      return el_u64(P.mgf_bit(i - DB8));
    }
  }
}

}  // namespace pzk
