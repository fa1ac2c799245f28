/* pzkwit.h — C-ABI of the MI355X batched witness generator (libpzkwit.so).
 *
 * Drop-in boundary for the witness-calculation surface of the reference:
 *   - circom's generated witness calculator, used by circom_tester
 *     (test/automatisationTest.js:37-51: wasm_tester -> circuit.calculateWitness(input, true))
 *     and by generate_witness.js (circuits/scripts/gen-witness.sh:25 -> calculateWTNSBin);
 *   - the per-input serial loop of test/automatisationTest.js:24, replaced by one batched call.
 * The JS binding (passport-zk-circuits_amd/js, Node N-API) and the Python binding
 * (passport-zk-circuits_amd/pzkwit) sit on top of these entry points; INTEGRATION.md shows
 * the bindings a maintainer adds.
 *
 * Conventions: plain pointers and sizes; every function returns 0 on success or a negative
 * PZK_E_* code, with a message in pzk_last_error() (thread-local). Caller owns all input and
 * output buffers; the instance owns its device scratch. Calls on one instance are serialised by an
 * internal mutex (concurrent callers wait); every call runs on the instance's device, whatever the
 * calling thread's current device (which is restored on return).
 * Field elements are 32 bytes, little-endian, NORMAL form (< p), as in a .wtns file.
 */
#ifndef PZKWIT_H
#define PZKWIT_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* circuit families (the `component main` the instance evaluates) */
enum {
  PZK_CIRCUIT_REGISTER = 0, /* RegisterIdentityBuilder(...)  registerIdentityBuilder.circom:41 */
  PZK_CIRCUIT_POSEIDON = 1, /* PoseidonHash(n)               poseidon.circom:214 (config 1) */
  PZK_CIRCUIT_SHA256 = 2,   /* Sha256HashChunks(blocks)      sha256HashChunks.circom:8 (config 2) */
  PZK_CIRCUIT_SHA1 = 3,     /* Sha1HashChunks(blocks)        hasher/sha1/sha1.circom:7 */
  PZK_CIRCUIT_SHA384 = 4,   /* Sha384HashChunks(blocks)      hasher/sha2/sha384/sha384HashChunks.circom:8 */
  PZK_CIRCUIT_SHA512 = 5,   /* Sha512HashChunks(blocks)      hasher/sha2/sha512/sha512HashChunks.circom */
  PZK_CIRCUIT_QUERY = 6     /* QueryIdentity(idTreeDepth = size_arg, 80)  identityManagement/queryIdentity.circom:37;
                               BabyPbk (undefined in the snapshot) is the reference's BabyjubjubBase8Multiplication,
                               DESIGN.md §11 */
};

/* Template parameters of RegisterIdentityBuilder (registerIdentityBuilder.circom:41-52),
 * verbatim, plus the circuit family and its size argument for the standalone circuits. */
typedef struct pzk_params {
  int32_t circuit;            /* PZK_CIRCUIT_* */
  int32_t size_arg;           /* n for POSEIDON, blocks for SHA256 / SHA1 / SHA384 / SHA512, idTreeDepth (80) for
                                 QUERY; ignored for REGISTER */
  int32_t signature_type;     /* SIGNATURE_TYPE (signatureVerification.circom:9-127): 1 = RSA-2048 PKCS#1 v1.5
                                 SHA-256 e = 65537, 2 = RSA-4096, 3 = RSA-2048 SHA-1, 4 = RSA-3072 SHA-1
                                 e = 37187; 10-12 = RSA-2048 PSS SHA-256 (10: e = 3; 12: salt 64), 13 = RSA-2048
                                 PSS SHA-384 (salt 48), 14 = RSA-3072 PSS SHA-256; 20 = ECDSA secp256r1,
                                 21 = ECDSA brainpoolP256r1 (SHA-256), 24 = ECDSA secp224r1 (7 x 32-bit chunks;
                                 SHA-224 signed attributes, SHA-256 encapsulated content), 25 = ECDSA
                                 brainpoolP384r1 (6 x 64-bit chunks, SHA-384). 22 / 23 do not compile in the
                                 reference (ecdsa.circom:31-37 reads past hashed[]). Others: PZK_E_PARAMS */
  int32_t dg_hash_type;       /* DG_HASH_TYPE (160, 224, 256, 384) */
  int32_t document_type;      /* DOCUMENT_TYPE (1 = TD1, 3 = TD3) */
  int32_t ec_block_number;    /* EC_BLOCK_NUMBER */
  int32_t ec_shift;           /* EC_SHIFT (bits) */
  int32_t dg1_shift;          /* DG1_SHIFT (bits) */
  int32_t aa_signature_algo;  /* AA_SIGNATURE_ALGO (0 = none, 1..19 = RSA-1024 key, 20..25 = EC key) */
  int32_t dg15_shift;         /* DG15_SHIFT (bits) */
  int32_t dg15_block_number;  /* DG15_BLOCK_NUMBER */
  int32_t aa_shift;           /* AA_SHIFT (bits) */
} pzk_params;

typedef struct pzk_info {
  uint64_t witness_size;   /* number of field elements per witness (wtns section 2 / 32) */
  uint64_t n_inputs;       /* number of input signals (flat input buffer length / 32) */
  uint32_t n_outputs;      /* main outputs (witness[1 .. n_outputs]) */
  uint32_t n_public_inputs;/* public inputs, right after the outputs */
  uint32_t n_input_groups; /* named input signals (see pzk_instance_input) */
  uint32_t pipeline_depth; /* calls in flight with a NULL stream: call k + pipeline_depth starts after call k
                              has completed (pzk_witness_batch) */
} pzk_info;

typedef struct pzk_exec {
  int32_t device;   /* HIP device ordinal: must be the instance's device, or < 0 for "the instance's" */
  int32_t flags;    /* PZK_EXEC_* */
  void* stream;     /* hipStream_t the call is ordered after and joined into at exit (serialises calls);
                       NULL = the instance's own streams, pipelined across calls: complete after
                       pzk_instance_sync() (or PZK_EXEC_SYNC / a device-wide synchronise) */
} pzk_exec;

enum {
  PZK_EXEC_SYNC = 1,   /* synchronise the stream before returning */
  PZK_EXEC_TIMING = 2  /* bracket every kernel phase with HIP events on the launch stream */
};

/* lane status codes: 0 = OK, else the first failing `===` site (reference file:line) */
enum {
  PZK_ST_OK = 0,
  PZK_ST_NUM2BITS = 1,    /* bitify.circom:26 */
  PZK_ST_ALIAS = 2,       /* aliascheck.circom:14 */
  PZK_ST_ISZERO = 3,      /* comparators.circom:20 */
  PZK_ST_LASTBIT = 4,     /* int/arithmetic.circom:169-170 */
  PZK_ST_LASTNBITS = 5,   /* int/arithmetic.circom:203 */
  PZK_ST_BITS2 = 6,       /* sha2Common.circom:65-68 */
  PZK_ST_FLOW = 7,        /* passportVerificationBuilder.circom:155 */
  PZK_ST_RSA_HASH = 8,    /* rsa.circom:48 */
  PZK_ST_RSA_PREFIX = 9,  /* rsa.circom:53-54 */
  PZK_ST_RSA_PAD = 10,    /* rsa.circom:57-71 */
  PZK_ST_BIGMOD_GT = 11,  /* bigInt.circom:245 */
  PZK_ST_BIGISZERO = 12,  /* bigIntComparators.circom:128 */
  PZK_ST_SMT_LAST = 13,   /* SMTVerifier.circom:54 */
  PZK_ST_BJJ_ADD = 14,    /* babyjubjub/curve.circom:98,102 */
  PZK_ST_ECDSA_INV = 15,  /* bigInt.circom:364-368 (in * inv mod n === 1) */
  PZK_ST_ECDSA_R = 16,    /* ecdsa.circom:81-83 (x1 mod n === r) */
  PZK_ST_PSS_TRAILER = 17,/* rsaPss.circom:73 (assert eM[0] == 188) */
  PZK_ST_PSS_HASH = 18,   /* rsaPss.circom:182,201 (hDash256.out === hash) */
  PZK_ST_QUERY = 19,      /* comparators.circom:42 ((1 - isEqual.out) * enabled === 0: a selected query bound fails) */
  PZK_ST_DATE = 20,       /* dateDecoder.circom:22 (encoded === dateEncoded: not a "YYMMDD" digit string) */
  PZK_ST_CIT_BLACKLIST = 21, /* citizenshipCheck.circom:271 (the citizenship is in the mask) */
  PZK_ST_CIT_LIST = 22,   /* citizenshipCheck.circom:274 (the citizenship is not in COUNTRY_ARR) */
  PZK_ST_ISV_ROOT = 23,   /* identityStateVerifier.circom:46 (smtVerifier.isVerified === 1) */
  PZK_ST_INPUT_RANGE = 64 /* an input outside the domain the GPU path evaluates (e.g. a non-bit
                             SHA input, a limb >= 2^64); see DESIGN.md §5 */
};

enum {
  PZK_E_ARG = -1,       /* invalid argument */
  PZK_E_PARAMS = -2,    /* unsupported template parameters */
  PZK_E_HIP = -3,       /* HIP runtime error */
  PZK_E_NOMEM = -4,     /* device allocation failed */
  PZK_E_DATA = -5,      /* Poseidon parameter file missing/corrupt */
  PZK_E_NODEVICE = -6   /* no HIP device: the library never falls back to a CPU path */
};

typedef struct pzk_instance pzk_instance;

/* Replaces: circom compile + WitnessCalculator builder(wasm) — witness_calculator.js builder(). */
int pzk_instance_create(const pzk_params* params, pzk_instance** out);
void pzk_instance_destroy(pzk_instance* inst);

/* Same, with a signal -> witness map in circom's .sym format (circom --sym: one line per signal,
 * "signal_idx,witness_idx,component_idx,name", witness_idx = -1 for a signal the compiler eliminated;
 * signal indices in the --O0 numbering of DESIGN.md §2). The instance's witness is then the mapped
 * one: witness_size = number of kept signals + 1, element k = the O0 signal whose witness_idx is k,
 * and the .wtns header reports that size. sym = NULL is pzk_instance_create (the identity map).
 * Replaces: the witness layout circom --O1/--O2 bakes into the WASM (circuits/scripts/compile-circuit.sh:34). */
int pzk_instance_create_mapped(const pzk_params* params, const char* sym, size_t sym_len, pzk_instance** out);
/* Host-only: validate a .sym against an instance's O0 numbering; *witness_size = mapped size. */
int pzk_sym_check(const pzk_params* params, const char* sym, size_t sym_len, uint64_t* witness_size);

/* Host-only layout queries (no device needed): witness/input sizes of an instance and its
 * emit-region table (offset, length, kind). Used by the CPU test suite. */
int pzk_layout_query(const pzk_params* params, pzk_info* info, uint32_t* n_regions);
int pzk_layout_region(const pzk_params* params, uint32_t i, uint64_t* off, uint32_t* len, uint32_t* kind);

/* Replaces: wc.witnessSize / wc.n32 / wc.prime fields and getInputSignalSize(fnv(name)). */
int pzk_instance_info(const pzk_instance* inst, pzk_info* info);
/* i-th named input signal, in flat-input order: name, element offset and length. */
int pzk_instance_input(const pzk_instance* inst, uint32_t i, const char** name, uint64_t* offset,
                       uint64_t* length);

/* The 76-byte .wtns header (wtns v2, 2 sections, n8 = 32, prime, witnessSize) that
 * calculateWTNSBin prepends. */
int pzk_wtns_header(const pzk_instance* inst, uint8_t header[76]);

/* Batched witness calculation on device buffers (inputs resident in HBM).
 *   d_inputs : batch x n_inputs x 32 B (normal form), device pointer
 *   d_wtns   : batch x witness_size x 32 B elements, row stride wtns_stride bytes (>= 32*witness_size,
 *              multiple of 16), device pointer
 *   d_status : batch x int32 lane status (PZK_ST_*), device pointer (may be NULL)
 * The buffers must stay untouched until the call has completed (see pzk_exec.stream). With a NULL
 * stream consecutive calls overlap: the instance keeps pzk_info.pipeline_depth (3) scratch sets, call
 * k uses set k mod 3, so calls k, k + 1 and k + 2 may run at the same time (call k + 1's cores beside
 * call k's emitters) and call k + 3 starts after call k has completed. A caller that reuses call k's
 * d_inputs / d_wtns / d_status for a later call must therefore either give the later call an index
 * >= k + 3 or synchronise first (pzk_instance_sync, PZK_EXEC_SYNC, or a stream).
 * Replaces: for (input of inputs) await wc.calculateWitness(input) (automatisationTest.js:24-50). */
int pzk_witness_batch(pzk_instance* inst, const uint8_t* d_inputs, size_t batch, uint8_t* d_wtns,
                      size_t wtns_stride, int32_t* d_status, const pzk_exec* exec);

/* Wait until every call issued on the instance so far has completed (all instance streams). */
int pzk_instance_sync(pzk_instance* inst);

/* Host-buffer convenience (copies in/out; used by the single-input calculateWitness path). */
int pzk_witness_batch_host(pzk_instance* inst, const uint8_t* h_inputs, size_t batch, uint8_t* h_wtns,
                           int32_t* h_status, const pzk_exec* exec);

/* Streamed delivery to host memory (replaces gen-witness.sh's one generate_witness.js + .wtns write per
 * input, circuits/scripts/gen-witness.sh:25, for a whole batch): h_inputs = batch x n_inputs x 32 B (host);
 * the batch runs in chunks of `chunk` witnesses (0: ~4 GiB of rows per chunk), and as each chunk's rows
 * arrive in pinned host memory the calling thread passes them to
 *   sink(user, first, n, rows, row_stride, status): rows[i * row_stride ..] is witness first + i (32 B
 *   elements, witness_size of them; the .wtns section 2 payload), status[i] its lane status.
 * The rows are valid only during the call (the buffer is reused two chunks later); a non-zero return stops
 * the stream (PZK_E_ARG). Chunk c + 1 computes and chunk c copies down while the sink runs on chunk c - 1,
 * so a sink that keeps up leaves the host link (PCIe) as the bound. */
typedef int (*pzk_sink_fn)(void* user, size_t first, size_t n, const uint8_t* rows, size_t row_stride,
                           const int32_t* status);
int pzk_witness_stream(pzk_instance* inst, const uint8_t* h_inputs, size_t batch, size_t chunk, pzk_sink_fn sink,
                       void* user, const pzk_exec* exec);

/* Per-phase kernel time accumulated (ms) by calls made with PZK_EXEC_TIMING, and the number of
 * launches of each phase. On input *count is the capacity of the arrays; on output the number of
 * phases. Synchronises on the recorded events. reset != 0 clears the accumulators afterwards. */
int pzk_timing(pzk_instance* inst, const char** names, double* ms, uint64_t* launches, uint32_t* count, int reset);

/* Static description of a kernel phase: name, kernel symbol, and its ALGORITHMIC HBM bytes per
 * witness (each element written once + the unique bytes it must read). Used for roofline math. */
int pzk_phase_info(const pzk_instance* inst, uint32_t phase, const char** name, const char** kernel,
                   uint64_t* bytes_per_witness);

/* Reason for the last failure on this thread. */
const char* pzk_last_error(void);

/* Library version string. */
const char* pzk_version(void);

#ifdef __cplusplus
}
#endif
#endif
