/* pzkpassport.h — host-side bulk SOD preprocessor.
 *
 * Replaces the per-passport input step of the reference, test/process_passport.js:674-816
 * (processPassport: decode EF.SOD with test/asn1.js, pull out the encapsulated content, the signed
 * attributes, the signature and the document-signer key, find the DG1 / DG15 / EC hash positions,
 * classify the signature, pad every hashed message and chunk the key and signature), and its
 * writeToJson (:659-672) / writeToCircom (:573-588) outputs: one call parses a whole batch on host
 * threads and writes the flat input rows pzk_witness_batch takes (pzkwit.h).
 *
 * The decisions are the reference's own, including its quirks: the ASN.1 walks of
 * getFirstOctetString / getZero / findParentOfLastOctetString / get_*_key_location, string-search
 * shifts (a hash found at an odd hex digit gives a shift in half bytes), ceil((len + 8) / 64) block
 * counts, the AA shift that writeToCircom passes in bytes (reported in ref_aa_shift; params.aa_shift
 * holds it in bits, as the circuit reads it, identity.circom:12).
 * Conventions as pzkwit.h: plain pointers and sizes, 0 or a negative PZK_E_* code (pzk_last_error()).
 * Parsing never touches a GPU.
 */
#ifndef PZKPASSPORT_H
#define PZKPASSPORT_H
#include "pzkwit.h"

#ifdef __cplusplus
extern "C" {
#endif

/* one passport as processPassport reads it: the JSON's dg1 / dg15 / sod fields, decoded to bytes */
typedef struct pzk_passport_src {
  const uint8_t* dg1;  size_t dg1_len;
  const uint8_t* dg15; size_t dg15_len;  /* 0 = no DG15 (no active authentication) */
  const uint8_t* sod;  size_t sod_len;   /* EF.SOD, DER */
} pzk_passport_src;

typedef struct pzk_passport_info {
  pzk_params params;       /* RegisterIdentityBuilder(...) the passport needs; shifts in bits */
  int32_t ref_aa_shift;    /* AA_SHIFT as writeToCircom writes it (extractFromDg15's byte offset, :795) */
  int32_t dg_hash_bytes;   /* dg_hash_type: digest length in the LDS object (:690) */
  int32_t hash_bytes;      /* hash_type: digest length in the signed attributes (:693) */
  int32_t dg1_len, dg15_len, ec_len, sa_len;  /* bytes */
  int32_t chunk_number;    /* getChunkedParams chunk_number (:590-626): limbs per coordinate */
  int32_t chunk_bits;      /* 64 (66 for fields wider than 512 bits) */
  int32_t salt;            /* RSA-PSS salt length from the signature algorithm; 0 = PKCS#1 v1.5 / ECDSA */
  int32_t reserved;
  char name[128];          /* old_naming_convention (:772), the generated circuit's name */
} pzk_passport_info;

/* per-passport status of pzk_passport_inputs */
enum {
  PZK_PP_OK = 0,
  PZK_PP_PARSE = 1,     /* the reference would throw: DER / structure / hash-length error */
  PZK_PP_UNKNOWN = 2,   /* getSigType returns 0 ("UNKNOWN TECHONOLY"), or an unknown AA curve */
  PZK_PP_PARAMS = 3,    /* the passport needs other RegisterIdentityBuilder parameters than the instance's */
  PZK_PP_SIZE = 4,      /* a padded message does not have the length the circuit's input has */
  PZK_PP_LIMBS = 5      /* chunks the instance cannot take (66-bit limbs, other limb counts) */
};

/* Parse one passport. Returns 0 (info filled), or PZK_E_ARG with the reason in pzk_last_error(). */
int pzk_passport_parse(const pzk_passport_src* src, pzk_passport_info* info);

/* Parse n passports on `threads` host threads (<= 0: all hardware threads) and write each one's input
 * row for an instance of `params`: rows = n x n_inputs x 32 B (pzk_instance_info; the pzk_witness_batch
 * input layout: slaveMerkleRoot, encapsulatedContent, dg1, dg15, signedAttributes, signature, pubkey,
 * slaveMerkleInclusionBranches, skIdentity). identity = n x 82 x 32 B field elements per passport
 * (slaveMerkleRoot, skIdentity, 80 inclusion branches; NULL = zeros): processPassport's
 * getFakeIdenData (:628-657) is test scaffolding, the identity is the caller's. status = n x PZK_PP_*;
 * a row whose status is not OK is zero-filled. Returns 0, or a negative PZK_E_* for bad arguments. */
int pzk_passport_inputs(const pzk_params* params, const pzk_passport_src* srcs, size_t n, const uint8_t* identity,
                        uint8_t* rows, int32_t* status, int threads);

#ifdef __cplusplus
}
#endif
#endif
