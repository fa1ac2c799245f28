/* oracle/fr.h — BN254 scalar field Fr for the CPU oracle.
 *
 * TEST INFRASTRUCTURE ONLY: this header belongs to the CPU restatement under
 * oracle/, used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg as the checker. The shipped path (passport-zk-circuits_amd/csrc) never
 * includes it.
 *
 * p = 21888242871839275222246405745257275088548364400416034343698204186575808495617
 * (test/automatisationTest.js:9). Elements are stored in NORMAL form
 * (canonical representative in [0,p), 4 x u64 little-endian) — exactly the
 * 32-byte LE layout of a .wtns element. Multiplication goes through
 * Montgomery form internally (two CIOS products per normal-form product).
 */
#ifndef PZK_ORACLE_FR_H
#define PZK_ORACLE_FR_H
#include <stdint.h>
#include <string.h>

typedef struct { uint64_t l[4]; } fr_t;
typedef unsigned __int128 u128;

static const fr_t FR_P = {{0x43e1f593f0000001ULL, 0x2833e84879b97091ULL,
                           0xb85045b68181585dULL, 0x30644e72e131a029ULL}};
static const fr_t FR_R2 = {{0x1bb8e645ae216da7ULL, 0x53fe3ab1e35c59e3ULL,
                            0x8c49833d53bb8085ULL, 0x0216d0b17f4e44a5ULL}};
static const uint64_t FR_INV = 0xc2e1f593efffffffULL; /* -p^-1 mod 2^64 */

static inline fr_t fr_zero(void) { fr_t r = {{0, 0, 0, 0}}; return r; }
static inline fr_t fr_u64(uint64_t x) { fr_t r = {{x, 0, 0, 0}}; return r; }
static inline int fr_is_zero(fr_t a) { return (a.l[0] | a.l[1] | a.l[2] | a.l[3]) == 0; }
static inline int fr_eq(fr_t a, fr_t b) { return memcmp(&a, &b, sizeof a) == 0; }

/* compare canonical representatives: -1, 0, 1 */
static inline int fr_cmp(fr_t a, fr_t b) {
  for (int i = 3; i >= 0; i--) {
    if (a.l[i] < b.l[i]) return -1;
    if (a.l[i] > b.l[i]) return 1;
  }
  return 0;
}

static inline fr_t fr_sub_raw(fr_t a, fr_t b, uint64_t *borrow_out) {
  fr_t r; uint64_t br = 0;
  for (int i = 0; i < 4; i++) {
    u128 d = (u128)a.l[i] - b.l[i] - br;
    r.l[i] = (uint64_t)d;
    br = (uint64_t)(d >> 64) & 1;
  }
  *borrow_out = br;
  return r;
}

static inline fr_t fr_add(fr_t a, fr_t b) {
  fr_t r; uint64_t c = 0;
  for (int i = 0; i < 4; i++) {
    u128 s = (u128)a.l[i] + b.l[i] + c;
    r.l[i] = (uint64_t)s; c = (uint64_t)(s >> 64);
  }
  uint64_t br; fr_t t = fr_sub_raw(r, FR_P, &br);
  return (c || !br) ? t : r;
}

static inline fr_t fr_sub(fr_t a, fr_t b) {
  uint64_t br; fr_t r = fr_sub_raw(a, b, &br);
  if (br) {
    uint64_t c = 0;
    for (int i = 0; i < 4; i++) {
      u128 s = (u128)r.l[i] + FR_P.l[i] + c;
      r.l[i] = (uint64_t)s; c = (uint64_t)(s >> 64);
    }
  }
  return r;
}

static inline fr_t fr_neg(fr_t a) { return fr_sub(fr_zero(), a); }

/* Montgomery product a*b*2^-256 mod p (CIOS) */
static inline fr_t fr_mont(fr_t a, fr_t b) {
  uint64_t t[6] = {0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 4; i++) {
    uint64_t c = 0;
    for (int j = 0; j < 4; j++) {
      u128 s = (u128)a.l[j] * b.l[i] + t[j] + c;
      t[j] = (uint64_t)s; c = (uint64_t)(s >> 64);
    }
    u128 s = (u128)t[4] + c; t[4] = (uint64_t)s; t[5] = (uint64_t)(s >> 64);
    uint64_t m = t[0] * FR_INV;
    s = (u128)m * FR_P.l[0] + t[0]; c = (uint64_t)(s >> 64);
    for (int j = 1; j < 4; j++) {
      s = (u128)m * FR_P.l[j] + t[j] + c;
      t[j - 1] = (uint64_t)s; c = (uint64_t)(s >> 64);
    }
    s = (u128)t[4] + c; t[3] = (uint64_t)s; t[4] = t[5] + (uint64_t)(s >> 64);
  }
  fr_t r = {{t[0], t[1], t[2], t[3]}};
  uint64_t br; fr_t q = fr_sub_raw(r, FR_P, &br);
  return (t[4] || !br) ? q : r;
}

static inline fr_t fr_mul(fr_t a, fr_t b) { return fr_mont(fr_mont(a, b), FR_R2); }
static inline fr_t fr_sqr(fr_t a) { return fr_mul(a, a); }

static inline fr_t fr_pow(fr_t a, fr_t e) {
  fr_t r = fr_u64(1);
  for (int i = 255; i >= 0; i--) {
    r = fr_mul(r, r);
    if ((e.l[i >> 6] >> (i & 63)) & 1) r = fr_mul(r, a);
  }
  return r;
}

/* field inverse (Fermat); inverse of 0 is 0 (IsZero's `in != 0 ? 1/in : 0`) */
static inline fr_t fr_inv(fr_t a) {
  if (fr_is_zero(a)) return a;
  fr_t e = FR_P; e.l[0] -= 2;
  return fr_pow(a, e);
}

static inline fr_t fr_div(fr_t a, fr_t b) { return fr_mul(a, fr_inv(b)); }

/* signed 64-bit integer -> field (negative x maps to p - |x|) */
static inline fr_t fr_i64(int64_t x) {
  return x >= 0 ? fr_u64((uint64_t)x) : fr_neg(fr_u64((uint64_t)(-(x + 1)) + 1));
}

/* 2^k for k < 254 */
static inline fr_t fr_pow2(int k) { fr_t r = fr_zero(); r.l[k >> 6] = 1ULL << (k & 63); return r; }

static inline int fr_bit(fr_t a, int i) { return (int)((a.l[i >> 6] >> (i & 63)) & 1); }

/* canonical representative shifted right by k (circom `>>` on a field value) */
static inline fr_t fr_shr(fr_t a, int k) {
  fr_t r = fr_zero();
  int w = k >> 6, b = k & 63;
  for (int i = 0; i + w < 4; i++) {
    uint64_t lo = a.l[i + w] >> b;
    uint64_t hi = (b && i + w + 1 < 4) ? a.l[i + w + 1] << (64 - b) : 0;
    r.l[i] = lo | hi;
  }
  return r;
}

/* does the canonical representative fit in `bits` bits */
static inline int fr_fits(fr_t a, int bits) {
  for (int i = bits; i < 256; i++) if (fr_bit(a, i)) return 0;
  return 1;
}

#endif
