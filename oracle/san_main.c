/* oracle/san_main.c — host AddressSanitizer / UndefinedBehaviorSanitizer driver for the CPU restatement.
 *
 * TEST INFRASTRUCTURE ONLY: `make -C oracle san` links witness_oracle.c and r1cs_check.c with
 * -fsanitize=address,undefined into build/san_main; tests/test_sanitize.py feeds it input rows and runs
 * every witness through the oracle and then the constraint checker, so an out-of-bounds access, a
 * use of uninitialised shift counts, a signed overflow or a misaligned load anywhere on those paths
 * aborts the run with the sanitizer's report (host ASan/UBSan build of the CPU restatement).
 *
 * usage: san_main DATA_DIR CASES_FILE
 * CASES_FILE: records of int32 kind, int32 params[10], int32 n_in, then n_in x 32 bytes of input elements
 *   kind 0 register (params = the 10 template parameters), 1 Sha256HashChunks(params[0]), 2 Sha1HashChunks(params[0]),
 *   3 Sha384/512HashChunks(params[0], out bits params[1]), 4 PoseidonHash(params[0])
 * prints one line per case: "case k kind K rc R check C failed F uncovered_nonzero U" */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct { int p[10]; } params10;  /* orc_params / ck_params: ten ints in the template's order */
typedef struct {
  uint64_t n_constraints, n_failed, n_uncovered, size_walked;
  int64_t first_failed;
  int32_t first_line, oob;
  char first_template[96];
  uint64_t first_component;
  int64_t first_uncovered;
  uint64_t n_uncovered_nonzero;
} ck_report;

int orc_load_poseidon(const char *path);
int orc_load_ec_table(int curve, const char *path);
size_t orc_register_n_inputs(const params10 *P);
size_t orc_register_witness_size(const params10 *P);
int orc_register_witness(const params10 *P, const uint8_t *inputs, uint8_t *wit);
size_t orc_sha256_witness_size(int B);
int orc_sha256_witness(int B, const uint8_t *inputs, uint8_t *wit);
size_t orc_sha1_witness_size(int B);
int orc_sha1_witness(int B, const uint8_t *inputs, uint8_t *wit);
size_t orc_sha512_witness_size(int B, int O);
int orc_sha512_witness(int B, int O, const uint8_t *inputs, uint8_t *wit);
size_t orc_poseidon_witness_size(int n);
int orc_poseidon_witness(int n, const uint8_t *inputs, uint8_t *wit);
int ck_load_poseidon(const char *path);
int ck_load_ec_table(int curve, const char *path);
int ck_register(const params10 *P, const uint8_t *wit, size_t nw, ck_report *r);
int ck_sha256(int B, const uint8_t *wit, size_t n, ck_report *r);
int ck_sha1(int B, const uint8_t *wit, size_t n, ck_report *r);
int ck_sha512(int B, int O, const uint8_t *wit, size_t n, ck_report *r);
int ck_poseidon_circuit(int n, const uint8_t *wit, size_t nw, ck_report *r);

static int load_all(const char *dir) {
  char path[4096];
  static const char *ec[4] = {"p256_gpow8.bin", "bp256_gpow8.bin", "p224_gpow8.bin", "bp384_gpow8.bin"};
  snprintf(path, sizeof path, "%s/poseidon_t2_6.bin", dir);
  if (orc_load_poseidon(path) || ck_load_poseidon(path)) return 1;
  for (int c = 0; c < 4; c++) {
    snprintf(path, sizeof path, "%s/%s", dir, ec[c]);
    if (orc_load_ec_table(c, path) || ck_load_ec_table(c, path)) return 2;
  }
  return 0;
}

int main(int argc, char **argv) {
  if (argc != 3) { fprintf(stderr, "usage: %s DATA_DIR CASES_FILE\n", argv[0]); return 2; }
  if (load_all(argv[1])) { fprintf(stderr, "cannot load the tables in %s\n", argv[1]); return 2; }
  FILE *fp = fopen(argv[2], "rb");
  if (!fp) { perror(argv[2]); return 2; }
  for (int k = 0;; k++) {
    int32_t kind, n_in;
    params10 P;
    if (fread(&kind, 4, 1, fp) != 1) break;
    if (fread(P.p, 4, 10, fp) != 10 || fread(&n_in, 4, 1, fp) != 1 || n_in < 0) { fprintf(stderr, "bad record\n"); return 2; }
    uint8_t *in = malloc((size_t)n_in * 32 + 1);
    if (fread(in, 32, (size_t)n_in, fp) != (size_t)n_in) { fprintf(stderr, "short record\n"); return 2; }
    size_t nw = 0, need = 0;
    switch (kind) {
      case 0: nw = orc_register_witness_size(&P); need = orc_register_n_inputs(&P); break;
      case 1: nw = orc_sha256_witness_size(P.p[0]); need = 512 * (size_t)P.p[0]; break;
      case 2: nw = orc_sha1_witness_size(P.p[0]); need = 512 * (size_t)P.p[0]; break;
      case 3: nw = orc_sha512_witness_size(P.p[0], P.p[1]); need = 1024 * (size_t)P.p[0]; break;
      case 4: nw = orc_poseidon_witness_size(P.p[0]); need = (size_t)P.p[0]; break;
      default: fprintf(stderr, "unknown kind %d\n", kind); return 2;
    }
    if (!nw || need != (size_t)n_in) { fprintf(stderr, "case %d: size mismatch (%zu inputs expected)\n", k, need); return 2; }
    uint8_t *w = malloc(nw * 32);
    int rc = 0, cr = 0;
    ck_report r;
    memset(&r, 0, sizeof r);
    switch (kind) {
      case 0: rc = orc_register_witness(&P, in, w); cr = ck_register(&P, w, nw, &r); break;
      case 1: rc = orc_sha256_witness(P.p[0], in, w); cr = ck_sha256(P.p[0], w, nw, &r); break;
      case 2: rc = orc_sha1_witness(P.p[0], in, w); cr = ck_sha1(P.p[0], w, nw, &r); break;
      case 3: rc = orc_sha512_witness(P.p[0], P.p[1], in, w); cr = ck_sha512(P.p[0], P.p[1], w, nw, &r); break;
      case 4: rc = orc_poseidon_witness(P.p[0], in, w); cr = ck_poseidon_circuit(P.p[0], w, nw, &r); break;
    }
    printf("case %d kind %d rc %d check %d failed %llu uncovered_nonzero %llu\n", k, kind, rc, cr,
           (unsigned long long)r.n_failed, (unsigned long long)r.n_uncovered_nonzero);
    fflush(stdout);
    free(w);
    free(in);
  }
  fclose(fp);
  return 0;
}
