// ECDSA kernels (SIGNATURE_TYPE 20, 21, 24, 25): k_ec_scalars / k_ec_chain / k_ec_final / k_ec_affine /
// k_ec_link / k_ec_inv (the EC core), k_ec_table, k_emit_ect. Compiled once per curve (PZK_EC_CURVE, see
// ec_common.hpp for the split, the per-curve geometry ECG and the per-witness layouts).
#pragma once
#include "ec_common.hpp"
#include "ec_walk.hpp"
#include "fr.hpp"
#include "layout.hpp"
#include "core_util.hpp"
#include "mapsink.hpp"
#include "bufs.hpp"
#include "ec_emit.hpp"

namespace pzk {
inline namespace PZK_EC_NS {

// this curve's chunking: NL chunks of CS bits; field elements as NW 32-bit words, JW 64-bit words
static constexpr int NL = ECG.nl, CS = ECG.cs, P2 = 2 * ECG.nl;
static constexpr int NW = (ECG.fb + 31) / 32, JW = ECG.jw;
static constexpr uint64_t CS_MASK = CS == 64 ? ~0ull : (1ull << CS) - 1;

// ============================================================ signed 256-bit integers
struct I256 { uint32_t w[8]; };
__device__ __forceinline__ I256 i_u64(uint64_t x) {
  I256 r; r.w[0] = (uint32_t)x; r.w[1] = (uint32_t)(x >> 32);
#pragma unroll
  for (int i = 2; i < 8; i++) r.w[i] = 0;
  return r;
}
__device__ __forceinline__ I256 i_pow2(int k) {
  I256 r = i_u64(0);
#pragma unroll
  for (int i = 0; i < 8; i++) r.w[i] = (k >> 5) == i ? (1u << (k & 31)) : 0u;
  return r;
}
__device__ __forceinline__ I256 i_add(const I256& a, const I256& b) {
  I256 r; uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) { uint64_t s = (uint64_t)a.w[i] + b.w[i] + c; r.w[i] = (uint32_t)s; c = s >> 32; }
  return r;
}
__device__ __forceinline__ I256 i_sub(const I256& a, const I256& b) {
  I256 r; uint64_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) { uint64_t d = (uint64_t)a.w[i] - b.w[i] - br; r.w[i] = (uint32_t)d; br = (d >> 32) & 1; }
  return r;
}
__device__ __forceinline__ I256 i_neg(const I256& a) { return i_sub(i_u64(0), a); }
__device__ __forceinline__ I256 i_mul(const I256& a, const I256& b) {  // low 256 bits (two's complement ring)
  uint32_t t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; i + j < 8; j++) {
      uint64_t s = (uint64_t)a.w[i] * b.w[j] + t[i + j] + c;
      t[i + j] = (uint32_t)s; c = (uint32_t)(s >> 32);
    }
  }
  I256 r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.w[i] = t[i];
  return r;
}
__device__ __forceinline__ bool i_is_neg(const I256& a) { return a.w[7] >> 31; }
__device__ __forceinline__ bool i_is_zero(const I256& a) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) o |= a.w[i];
  return o == 0;
}
__device__ __forceinline__ I256 i_shr64(const I256& a) {  // arithmetic
  I256 r; uint32_t s = i_is_neg(a) ? ~0u : 0u;
#pragma unroll
  for (int i = 0; i < 8; i++) r.w[i] = i + 2 < 8 ? a.w[i + 2] : s;
  return r;
}
__device__ __forceinline__ uint32_t i_bit(const I256& a, int b) { return (a.w[b >> 5] >> (b & 31)) & 1u; }
// v >= 0 and v < 2^L
__device__ __forceinline__ bool i_fits(const I256& a, int L) {
  if (i_is_neg(a)) return false;
  bool ok = true;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    int lo = 32 * i;
    uint32_t m = L <= lo ? ~0u : L >= lo + 32 ? 0u : ~((1u << (L - lo)) - 1u);
    ok &= (a.w[i] & m) == 0;
  }
  return ok;
}
// normal-form Fr of a signed integer |v| < p (negative v -> p + v)
__device__ __forceinline__ I256 i_to_fr(const I256& a) {
  if (!i_is_neg(a)) return a;
  I256 p;
#pragma unroll
  for (int i = 0; i < 8; i++) p.w[i] = P_[i];
  return i_add(a, p);
}
__device__ __forceinline__ fr i_as_fr(const I256& a) { fr r; for (int i = 0; i < 8; i++) r.v[i] = a.w[i]; return r; }

// ============================================================ multiprecision division (64-bit words)
// floor(a / b), b = NB words with b[NB-1] != 0 (this curve's p or n); q[na-NB+1], r[NB]. Knuth D with the
// 128/64 step of core_util.hpp (divlu). Same unique quotient/remainder long_div (bigIntFunc.circom:190-232)
// produces.
template <int NB>
__device__ __forceinline__ void mp_divmod(const uint64_t* a, int na, const uint64_t* b, uint64_t* q, uint64_t* r) {
  const int s = __clzll((long long)b[NB - 1]);
  uint64_t v[NB], u[32];
#pragma unroll
  for (int i = NB - 1; i > 0; i--) v[i] = (b[i] << s) | (s ? b[i - 1] >> (64 - s) : 0);
  v[0] = b[0] << s;
  u[na] = s ? a[na - 1] >> (64 - s) : 0;
  for (int i = na - 1; i > 0; i--) u[i] = (a[i] << s) | (s ? a[i - 1] >> (64 - s) : 0);
  u[0] = a[0] << s;
  for (int j = na - NB; j >= 0; j--) {
    uint64_t qhat, rhat;
    bool big = false;
    if (u[j + NB] >= v[NB - 1]) {
      qhat = ~0ull;
      rhat = u[j + NB - 1] + v[NB - 1];
      big = rhat < v[NB - 1];
    } else {
      qhat = divlu(u[j + NB], u[j + NB - 1], v[NB - 1], &rhat);
    }
    while (!big) {
      uint64_t ph = __umul64hi(qhat, v[NB - 2]), pl = qhat * v[NB - 2];
      if (ph > rhat || (ph == rhat && pl > u[j + NB - 2])) {
        qhat--; rhat += v[NB - 1]; big = rhat < v[NB - 1];
      } else break;
    }
    uint64_t carry = 0, borrow = 0;
#pragma unroll
    for (int i = 0; i < NB; i++) {
      uint64_t pl = qhat * v[i], ph = __umul64hi(qhat, v[i]);
      pl += carry; ph += pl < carry;
      uint64_t t = u[i + j] - pl;
      uint64_t b1 = u[i + j] < pl;
      uint64_t t2 = t - borrow;
      b1 += t < borrow;
      u[i + j] = t2; borrow = b1; carry = ph;
    }
    uint64_t t = u[j + NB] - carry, b1 = u[j + NB] < carry;
    uint64_t t2 = t - borrow; b1 += t < borrow;
    u[j + NB] = t2;
    if (b1) {  // add back
      qhat--;
      uint64_t c = 0;
#pragma unroll
      for (int i = 0; i < NB; i++) {
        uint64_t s1 = u[i + j] + v[i], c1 = s1 < v[i];
        uint64_t s2 = s1 + c; c1 += s2 < c;
        u[i + j] = s2; c = c1;
      }
      u[j + NB] += c;
    }
    q[j] = qhat;
  }
#pragma unroll
  for (int i = 0; i < NB; i++) r[i] = (u[i] >> s) | (s ? u[i + 1] << (64 - s) : 0);
}
// chunks (one per u64, CS bits) <-> 64-bit words of the integer they spell
__device__ __forceinline__ void chunks_to_words(const uint64_t* ch, int n, uint64_t* w, int nw) {
  for (int i = 0; i < nw; i++) w[i] = 0;
  for (int i = 0; i < n; i++) w[(CS * i) >> 6] |= ch[i] << ((CS * i) & 63);
}
__device__ __forceinline__ uint64_t word_chunk(const uint64_t* w, int i) {
  return (w[(CS * i) >> 6] >> ((CS * i) & 63)) & CS_MASK;
}
// words (32-bit) of p and n for the divisions
static constexpr int PWORDS = (ECG.fb + 63) / 64;
__device__ __forceinline__ void const_words(const uint64_t* ch, uint64_t* w) { chunks_to_words(ch, NL, w, PWORDS); }

// two's-complement accumulation of signed I256 values shifted by CS i bits (32-bit words)
template <int AW32>
__device__ __forceinline__ void acc_signed(uint32_t* acc, const I256& v, int i) {
  const int off = (CS / 32) * i;
  const uint32_t ext = i_is_neg(v) ? ~0u : 0u;
  uint64_t c = 0;
  for (int j = 0; off + j < AW32; j++) {
    const uint64_t s = (uint64_t)acc[off + j] + (j < 8 ? v.w[j] : ext) + c;
    acc[off + j] = (uint32_t)s; c = s >> 32;
  }
}

// ============================================================ table context (device walker)
struct EcTabCtx {
  using V = I256;
  uint4* tab;            // this op's table: 2 x uint4 per entry
  uint32_t n;
  const uint64_t* rp;    // op record
  int32_t err;
  __device__ void fail(int32_t code) { if (!err || code < err) err = code; }
  __device__ void store(const V& v) {
    I256 f = i_to_fr(v);
    tab[2 * n] = make_uint4(f.w[0], f.w[1], f.w[2], f.w[3]);
    tab[2 * n + 1] = make_uint4(f.w[4], f.w[5], f.w[6], f.w[7]);
    n++;
  }
  __device__ V put(uint32_t, const V& v) { store(v); return v; }
  __device__ V put_hidden(const V& v) { store(v); return v; }
  __device__ void cp(uint32_t, const V&) {}
  __device__ void bits(uint32_t, const V& v, int L) { if (!i_fits(v, L)) fail(ST_NUM2BITS); }  // bitify.circom:26
  __device__ void masks(uint32_t, const V&, int) {}
  __device__ V u64(uint64_t x) const { return i_u64(x); }
  __device__ V pow2(int k) const { return i_pow2(k); }
  __device__ V add(const V& a, const V& b) const { return i_add(a, b); }
  __device__ V sub(const V& a, const V& b) const { return i_sub(a, b); }
  __device__ V mul(const V& a, const V& b) const { return i_mul(a, b); }
  __device__ V neg(const V& a) const { return i_neg(a); }
  __device__ V sel(const V& c, const V& a, const V& b) const { return c.w[0] ? a : b; }
  __device__ V is_zero(const V& a) const { return i_u64(i_is_zero(a) ? 1 : 0); }
  __device__ V bit(const V& a, int b) const { return i_u64(i_bit(a, b)); }
  // carry = (in + carry') / 2^CS, field division (bigIntComparators.circom:119-122): exact for a passing witness
  __device__ V shr_exact(const V& t, int) {
    I256 r; const uint32_t s = i_is_neg(t) ? ~0u : 0u;
    if (CS == 64) {
      if (t.w[0] | t.w[1]) fail(ST_BIGISZERO);
      return i_shr64(t);
    }
    if (t.w[0]) fail(ST_BIGISZERO);
#pragma unroll
    for (int i = 0; i < 8; i++) r.w[i] = i + 1 < 8 ? t.w[i + 1] : s;
    return r;
  }
  __device__ V inv_fr(const V& d) const {  // FIPS products: 64 independent lanes per wave, one op each
    fr x = fr_mul_fast(i_as_fr(i_to_fr(d)), fr_const(R2_));
    fr y = fr_from_mont_fast(fr_inv<true>(x));
    I256 r;
    for (int i = 0; i < 8; i++) r.w[i] = y.v[i];
    return r;
  }
  __device__ void check_zero(const V& v) { if (!i_is_zero(v)) fail(ST_BIGISZERO); }  // bigIntComparators.circom:128
  __device__ void check_one(const V& v) {                                              // bigInt.circom:245
    if (!i_is_zero(i_sub(v, i_u64(1)))) fail(ST_BIGMOD_GT);
  }
  // reduce_overflow_signed (bigIntFunc.circom:646-694) + long_div by P (:190-232): the signed sum
  // S = sum in[i] 2^(CS i); sign = S >= 0; k = |S| / p (MCN - NL + 1 chunks)
  __device__ void div_signed(const V* in, int CN, int MCN, V& sign, V* k) {
    constexpr int AW = ((3 * NL + 1) * CS + 63) / 64 + 2, AW32 = 2 * AW;
    uint32_t acc[AW32];
    for (int i = 0; i < AW32; i++) acc[i] = 0;
    for (int i = 0; i < CN; i++) acc_signed<AW32>(acc, in[i], i);
    const bool pos = !(acc[AW32 - 1] >> 31);
    if (!pos) {
      uint64_t c = 1;
      for (int i = 0; i < AW32; i++) { const uint64_t x = (uint64_t)(uint32_t)~acc[i] + c; acc[i] = (uint32_t)x; c = x >> 32; }
    }
    uint64_t a[AW], pw[PWORDS], q[AW], r[PWORDS];
    for (int i = 0; i < AW; i++) { a[i] = (uint64_t)acc[2 * i + 1] << 32 | acc[2 * i]; q[i] = 0; }
    const_words(EC_P, pw);
    const int na = (MCN * CS + 63) / 64;
    mp_divmod<PWORDS>(a, na < PWORDS ? PWORDS : na, pw, q, r);
    sign = i_u64(pos ? 1 : 0);
    for (int i = 0; i < MCN - NL + 1; i++) k[i] = i_u64(word_chunk(q, i));
  }
  // reduce_overflow(CS, 2N-1, 2N) (bigIntFunc.circom:570-588) + long_div by n
  __device__ void divmod_n(const V* mo, V* q, V* r) {
    constexpr int AW = (2 * NL * CS + 63) / 64 + 2, AW32 = 2 * AW;
    uint32_t acc[AW32];
    for (int i = 0; i < AW32; i++) acc[i] = 0;
    for (int i = 0; i < 2 * NL - 1; i++) acc_signed<AW32>(acc, mo[i], i);
    uint64_t a[AW], nw[PWORDS], qq[AW], rr[PWORDS + 1];
    for (int i = 0; i < AW; i++) { a[i] = (uint64_t)acc[2 * i + 1] << 32 | acc[2 * i]; qq[i] = 0; }
    rr[PWORDS] = 0;
    const_words(EC_N, nw);
    mp_divmod<PWORDS>(a, AW - 1, nw, qq, rr);
    for (int i = 0; i < NL + 1; i++) q[i] = i_u64(word_chunk(qq, i));
    for (int i = 0; i < NL; i++) r[i] = i_u64(word_chunk(rr, i));
  }
  __device__ V rec(int k) const { return i_u64(rp[k]); }
};

// ============================================================ Montgomery fields (p and n of this curve)
// NW 32-bit words; m, R^2 mod m, R mod m, m - 2 (Fermat exponent), -m^-1 mod 2^32, R = 2^(32 NW); aR = A R mod p
struct eW { uint32_t v[NW]; };
#if PZK_EC_CURVE == 0
static constexpr bool EC_A_M3 = true;  // A = p - 3
struct ModP {
  static constexpr uint32_t m[NW] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0x00000000u,
                                     0x00000000u, 0x00000000u, 0x00000001u, 0xffffffffu};
  static constexpr uint32_t r2[NW] = {0x00000003u, 0x00000000u, 0xffffffffu, 0xfffffffbu,
                                      0xfffffffeu, 0xffffffffu, 0xfffffffdu, 0x00000004u};
  static constexpr uint32_t r1[NW] = {0x00000001u, 0x00000000u, 0x00000000u, 0xffffffffu,
                                      0xffffffffu, 0xffffffffu, 0xfffffffeu, 0x00000000u};
  static constexpr uint32_t e[NW] = {0xfffffffdu, 0xffffffffu, 0xffffffffu, 0x00000000u,
                                     0x00000000u, 0x00000000u, 0x00000001u, 0xffffffffu};
  static constexpr uint32_t minv = 1u;
  static constexpr bool is_p = true;
};
struct ModN {
  static constexpr uint32_t m[NW] = {0xfc632551u, 0xf3b9cac2u, 0xa7179e84u, 0xbce6faadu,
                                     0xffffffffu, 0xffffffffu, 0x00000000u, 0xffffffffu};
  static constexpr uint32_t r2[NW] = {0xbe79eea2u, 0x83244c95u, 0x49bd6fa6u, 0x4699799cu,
                                      0x2b6bec59u, 0x2845b239u, 0xf3d95620u, 0x66e12d94u};
  static constexpr uint32_t r1[NW] = {0x039cdaafu, 0x0c46353du, 0x58e8617bu, 0x43190552u,
                                      0x00000000u, 0x00000000u, 0xffffffffu, 0x00000000u};
  static constexpr uint32_t e[NW] = {0xfc63254fu, 0xf3b9cac2u, 0xa7179e84u, 0xbce6faadu,
                                     0xffffffffu, 0xffffffffu, 0x00000000u, 0xffffffffu};
  static constexpr uint32_t minv = 0xee00bc4fu;
  static constexpr bool is_p = false;
};
#elif PZK_EC_CURVE == 1
// brainpoolP256r1 (RFC 5639 3.4)
static constexpr bool EC_A_M3 = false;
struct ModP {
  static constexpr uint32_t m[NW] = {0x1f6e5377u, 0x2013481du, 0xd5262028u, 0x6e3bf623u,
                                     0x9d838d72u, 0x3e660a90u, 0xa1eea9bcu, 0xa9fb57dbu};
  static constexpr uint32_t r2[NW] = {0xa6465b6cu, 0x8cfedf7bu, 0x614d4f4du, 0x5cce4c26u,
                                      0x6b1ac807u, 0xa1ecdacdu, 0xe5957fa8u, 0x4717aa21u};
  static constexpr uint32_t r1[NW] = {0xe091ac89u, 0xdfecb7e2u, 0x2ad9dfd7u, 0x91c409dcu,
                                      0x627c728du, 0xc199f56fu, 0x5e115643u, 0x5604a824u};
  static constexpr uint32_t e[NW] = {0x1f6e5375u, 0x2013481du, 0xd5262028u, 0x6e3bf623u,
                                     0x9d838d72u, 0x3e660a90u, 0xa1eea9bcu, 0xa9fb57dbu};
  static constexpr uint32_t minv = 0xcefd89b9u;
  static constexpr bool is_p = true;
  static constexpr uint32_t aR[NW] = {0x69696261u, 0xd5d18edfu, 0xc1d20c64u, 0xa68123f1u,
                                      0x6398556eu, 0x95ec1e5eu, 0xd666bc17u, 0x1e4676abu};
};
struct ModN {
  static constexpr uint32_t m[NW] = {0x974856a7u, 0x901e0e82u, 0xb561a6f7u, 0x8c397aa3u,
                                     0x9d838d71u, 0x3e660a90u, 0xa1eea9bcu, 0xa9fb57dbu};
  static constexpr uint32_t r2[NW] = {0x3312fca6u, 0xe1d8d8deu, 0x1134e4a0u, 0xf35d176au,
                                      0x6c815cb0u, 0x9b7f25e7u, 0xc3236762u, 0x0b25f1b9u};
  static constexpr uint32_t r1[NW] = {0x68b7a959u, 0x6fe1f17du, 0x4a9e5908u, 0x73c6855cu,
                                      0x627c728eu, 0xc199f56fu, 0x5e115643u, 0x5604a824u};
  static constexpr uint32_t e[NW] = {0x974856a5u, 0x901e0e82u, 0xb561a6f7u, 0x8c397aa3u,
                                     0x9d838d71u, 0x3e660a90u, 0xa1eea9bcu, 0xa9fb57dbu};
  static constexpr uint32_t minv = 0xcbb40ee9u;
  static constexpr bool is_p = false;
};
#elif PZK_EC_CURVE == 2
// secp224r1 (FIPS 186-4 D.1.2.2), 7 words
static constexpr bool EC_A_M3 = true;
struct ModP {
  static constexpr uint32_t m[NW] = {0x00000001u, 0x00000000u, 0x00000000u, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu};
  static constexpr uint32_t r2[NW] = {0x00000001u, 0x00000000u, 0x00000000u, 0xfffffffeu, 0xffffffffu, 0xffffffffu, 0x00000000u};
  static constexpr uint32_t r1[NW] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u};
  static constexpr uint32_t e[NW] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0xfffffffeu, 0xffffffffu, 0xffffffffu, 0xffffffffu};
  static constexpr uint32_t minv = 0xffffffffu;
  static constexpr bool is_p = true;
};
struct ModN {
  static constexpr uint32_t m[NW] = {0x5c5c2a3du, 0x13dd2945u, 0xe0b8f03eu, 0xffff16a2u, 0xffffffffu, 0xffffffffu, 0xffffffffu};
  static constexpr uint32_t r2[NW] = {0x3ad01289u, 0x6bdaae6cu, 0x97a54552u, 0x6ad09d91u, 0xb1e97961u, 0x1822bc47u, 0xd4baa4cfu};
  static constexpr uint32_t r1[NW] = {0xa3a3d5c3u, 0xec22d6bau, 0x1f470fc1u, 0x0000e95du, 0x00000000u, 0x00000000u, 0x00000000u};
  static constexpr uint32_t e[NW] = {0x5c5c2a3bu, 0x13dd2945u, 0xe0b8f03eu, 0xffff16a2u, 0xffffffffu, 0xffffffffu, 0xffffffffu};
  static constexpr uint32_t minv = 0x6a1fc2ebu;
  static constexpr bool is_p = false;
};
#else
// brainpoolP384r1 (RFC 5639 3.6), 12 words
static constexpr bool EC_A_M3 = false;
struct ModP {
  static constexpr uint32_t m[NW] = {0x3107ec53u, 0x87470013u, 0x901d1a71u, 0xacd3a729u, 0x7fb71123u, 0x12b1da19u,
                                     0xed5456b4u, 0x152f7109u, 0x50e641dfu, 0x0f5d6f7eu, 0xa3386d28u, 0x8cb91e82u};
  static constexpr uint32_t r2[NW] = {0x40b64bdeu, 0x087cefffu, 0x3d7fd965u, 0x53528334u, 0xc9940899u, 0x8e28f99cu,
                                      0x9918d5afu, 0x62140191u, 0xa57e052cu, 0xd5c6ef3bu, 0x178df842u, 0x36bf6883u};
  static constexpr uint32_t r1[NW] = {0xcef813adu, 0x78b8ffecu, 0x6fe2e58eu, 0x532c58d6u, 0x8048eedcu, 0xed4e25e6u,
                                      0x12aba94bu, 0xead08ef6u, 0xaf19be20u, 0xf0a29081u, 0x5cc792d7u, 0x7346e17du};
  static constexpr uint32_t e[NW] = {0x3107ec51u, 0x87470013u, 0x901d1a71u, 0xacd3a729u, 0x7fb71123u, 0x12b1da19u,
                                     0xed5456b4u, 0x152f7109u, 0x50e641dfu, 0x0f5d6f7eu, 0xa3386d28u, 0x8cb91e82u};
  static constexpr uint32_t minv = 0xea9ec825u;
  static constexpr bool is_p = true;
  static constexpr uint32_t aR[NW] = {0x466c3c99u, 0xdb26b895u, 0xf157b07bu, 0x75d7f3feu, 0xd7f10db4u, 0x936771b9u,
                                      0x35529374u, 0xe7ffe9e5u, 0x42b00c60u, 0x400a8fdfu, 0xa2e8c0d1u, 0x7c338021u};
};
struct ModN {
  static constexpr uint32_t m[NW] = {0xe9046565u, 0x3b883202u, 0x6b7fc310u, 0xcf3ab6afu, 0xac0425a7u, 0x1f166e6cu,
                                     0xed5456b3u, 0x152f7109u, 0x50e641dfu, 0x0f5d6f7eu, 0xa3386d28u, 0x8cb91e82u};
  static constexpr uint32_t r2[NW] = {0xde771c8eu, 0xac4ed3a2u, 0x2f2b6b6eu, 0x37264e20u, 0x9802688au, 0x2a927e3bu,
                                      0x52d748ffu, 0x574a74cbu, 0x65165fdbu, 0x8f886dc9u, 0x614e97c2u, 0x0ce8941au};
  static constexpr uint32_t r1[NW] = {0x16fb9a9bu, 0xc477cdfdu, 0x94803cefu, 0x30c54950u, 0x53fbda58u, 0xe0e99193u,
                                      0x12aba94cu, 0xead08ef6u, 0xaf19be20u, 0xf0a29081u, 0x5cc792d7u, 0x7346e17du};
  static constexpr uint32_t e[NW] = {0xe9046563u, 0x3b883202u, 0x6b7fc310u, 0xcf3ab6afu, 0xac0425a7u, 0x1f166e6cu,
                                     0xed5456b3u, 0x152f7109u, 0x50e641dfu, 0x0f5d6f7eu, 0xa3386d28u, 0x8cb91e82u};
  static constexpr uint32_t minv = 0x5cb5bb93u;
  static constexpr bool is_p = false;
};
#endif
using ModPFwd = ModP;
using ModNFwd = ModN;

template <class M> __device__ __forceinline__ eW m_const(const uint32_t (&c)[NW]) { eW r; for (int i = 0; i < NW; i++) r.v[i] = c[i]; return r; }
// r = t - m if t >= m (t < 2m, t given with a carry word)
template <class M> __device__ __forceinline__ eW m_reduce(const uint32_t* t, uint32_t top) {
  eW d; uint64_t br = 0;
#pragma unroll
  for (int i = 0; i < NW; i++) { uint64_t x = (uint64_t)t[i] - M::m[i] - br; d.v[i] = (uint32_t)x; br = (x >> 32) & 1; }
  if (top || !br) return d;
  eW r;
#pragma unroll
  for (int i = 0; i < NW; i++) r.v[i] = t[i];
  return r;
}
template <class M> __device__ __forceinline__ eW m_mul_inl(const eW& a, const eW& b) {
  uint32_t t[NW + 2];
#pragma unroll
  for (int j = 0; j < NW + 2; j++) t[j] = 0;
#pragma unroll
  for (int i = 0; i < NW; i++) {
    uint64_t C = 0;
#pragma unroll
    for (int j = 0; j < NW; j++) { uint64_t s = (uint64_t)a.v[j] * b.v[i] + t[j] + C; t[j] = (uint32_t)s; C = s >> 32; }
    uint64_t s = (uint64_t)t[NW] + C; t[NW] = (uint32_t)s; t[NW + 1] = (uint32_t)(s >> 32);
    const uint32_t m = t[0] * M::minv;
    s = (uint64_t)m * M::m[0] + t[0]; C = s >> 32;
#pragma unroll
    for (int j = 1; j < NW; j++) { s = (uint64_t)m * M::m[j] + t[j] + C; t[j - 1] = (uint32_t)s; C = s >> 32; }
    s = (uint64_t)t[NW] + C; t[NW - 1] = (uint32_t)s; t[NW] = t[NW + 1] + (uint32_t)(s >> 32);
  }
  return m_reduce<M>(t, t[NW]);
}
// Out of line: the point chains are long straight-line sequences of products; inlining every
// product makes k_ec_chain ~40 k instructions and instruction-fetch bound.
__device__ __noinline__ eW m_mul_p(eW a, eW b) { return m_mul_inl<ModPFwd>(a, b); }
__device__ __noinline__ eW m_mul_n(eW a, eW b) { return m_mul_inl<ModNFwd>(a, b); }
template <class M> __device__ __forceinline__ eW m_mul(const eW& a, const eW& b) {
  if constexpr (M::is_p) return m_mul_p(a, b); else return m_mul_n(a, b);
}
template <class M> __device__ __forceinline__ eW m_add(const eW& a, const eW& b) {
  uint32_t t[NW]; uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < NW; i++) { uint64_t s = (uint64_t)a.v[i] + b.v[i] + c; t[i] = (uint32_t)s; c = s >> 32; }
  return m_reduce<M>(t, (uint32_t)c);
}
template <class M> __device__ __forceinline__ eW m_sub(const eW& a, const eW& b) {
  eW r; uint64_t br = 0;
#pragma unroll
  for (int i = 0; i < NW; i++) { uint64_t d = (uint64_t)a.v[i] - b.v[i] - br; r.v[i] = (uint32_t)d; br = (d >> 32) & 1; }
  if (br) {
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < NW; i++) { uint64_t s = (uint64_t)r.v[i] + M::m[i] + c; r.v[i] = (uint32_t)s; c = s >> 32; }
  }
  return r;
}
template <class M> __device__ __forceinline__ eW m_to(const eW& a) { return m_mul<M>(a, m_const<M>(M::r2)); }
template <class M> __device__ __forceinline__ eW m_from(const eW& a) { eW one{}; for (int i = 0; i < NW; i++) one.v[i] = i == 0; return m_mul<M>(a, one); }
template <class M> __device__ __forceinline__ bool m_is_zero(const eW& a) { uint32_t o = 0; for (int i = 0; i < NW; i++) o |= a.v[i]; return o == 0; }
// a^(m-2) (Montgomery in/out), 4-bit fixed window; 0 -> 0 (mod_inv, bigIntFunc.circom:430-466)
template <class M> __device__ eW m_inv(const eW& a) {
  eW tbl[16];
  tbl[0] = m_const<M>(M::r1);
  tbl[1] = a;
  for (int i = 2; i < 16; i++) tbl[i] = m_mul<M>(tbl[i - 1], a);
  eW r = tbl[0];
  for (int w = 8 * NW - 1; w >= 0; w--) {
    if (w != 8 * NW - 1) for (int k = 0; k < 4; k++) r = m_mul<M>(r, r);
    const uint32_t nib = (M::e[w >> 3] >> ((w & 7) * 4)) & 15u;
    eW s = tbl[0];
#pragma unroll
    for (int q = 1; q < 16; q++) if ((uint32_t)q == nib) s = tbl[q];
    if (nib) r = m_mul<M>(r, s);
  }
  return r;
}
// chunks (NL x CS bits, one per u64) / 64-bit scratch words <-> field words
__device__ __forceinline__ eW ew_from_chunks(const uint64_t* x) {
  eW r;
  if (CS == 64) {
#pragma unroll
    for (int i = 0; i < NW / 2; i++) { r.v[2 * i] = (uint32_t)x[i]; r.v[2 * i + 1] = (uint32_t)(x[i] >> 32); }
  } else {
#pragma unroll
    for (int i = 0; i < NW; i++) r.v[i] = (uint32_t)x[i];
  }
  return r;
}
__device__ __forceinline__ void ew_to_chunks(const eW& a, uint64_t* x) {
  if (CS == 64) {
#pragma unroll
    for (int i = 0; i < NW / 2; i++) x[i] = (uint64_t)a.v[2 * i + 1] << 32 | a.v[2 * i];
  } else {
#pragma unroll
    for (int i = 0; i < NW; i++) x[i] = a.v[i];
  }
}
__device__ __forceinline__ eW ew_from_words(const uint64_t* x) {
  eW r;
#pragma unroll
  for (int i = 0; i < NW; i++) r.v[i] = (uint32_t)(x[i >> 1] >> (32 * (i & 1)));
  return r;
}
__device__ __forceinline__ void ew_to_words(const eW& a, uint64_t* x) {
#pragma unroll
  for (int i = 0; i < JW; i++) x[i] = (2 * i + 1 < NW ? (uint64_t)a.v[2 * i + 1] << 32 : 0ull) | a.v[2 * i];
}

// Jacobian points (Montgomery mod p)
struct Jac { eW x, y, z; };
template <class M = ModP>  // a template so the general-a branch (M::aR) is discarded for a = -3 curves
__device__ Jac jac_dbl(const Jac& P) {
  if constexpr (EC_A_M3) {  // dbl-2001-b, a = -3 (P-256, P-224: A = p - 3)
    eW delta = m_mul<M>(P.z, P.z), gamma = m_mul<M>(P.y, P.y), beta = m_mul<M>(P.x, gamma);
    eW t = m_mul<M>(m_sub<M>(P.x, delta), m_add<M>(P.x, delta));
    eW alpha = m_add<M>(m_add<M>(t, t), t);
    eW b4 = m_add<M>(beta, beta); b4 = m_add<M>(b4, b4);
    Jac R;
    R.x = m_sub<M>(m_mul<M>(alpha, alpha), m_add<M>(b4, b4));
    eW yz = m_add<M>(P.y, P.z);
    R.z = m_sub<M>(m_sub<M>(m_mul<M>(yz, yz), gamma), delta);
    eW g2 = m_mul<M>(gamma, gamma);
    eW g8 = m_add<M>(g2, g2); g8 = m_add<M>(g8, g8); g8 = m_add<M>(g8, g8);
    R.y = m_sub<M>(m_mul<M>(alpha, m_sub<M>(b4, R.x)), g8);
    return R;
  } else {  // dbl-2007-bl, general a (brainpool)
    eW xx = m_mul<M>(P.x, P.x), yy = m_mul<M>(P.y, P.y), zz = m_mul<M>(P.z, P.z), yyyy = m_mul<M>(yy, yy);
    eW xyy = m_add<M>(P.x, yy);
    eW s = m_sub<M>(m_sub<M>(m_mul<M>(xyy, xyy), xx), yyyy);
    s = m_add<M>(s, s);
    eW mm = m_add<M>(m_add<M>(xx, xx), xx);
    mm = m_add<M>(mm, m_mul<M>(m_const<M>(M::aR), m_mul<M>(zz, zz)));
    Jac R;
    R.x = m_sub<M>(m_mul<M>(mm, mm), m_add<M>(s, s));
    eW y8 = m_add<M>(yyyy, yyyy); y8 = m_add<M>(y8, y8); y8 = m_add<M>(y8, y8);
    R.y = m_sub<M>(m_mul<M>(mm, m_sub<M>(s, R.x)), y8);
    eW yz = m_add<M>(P.y, P.z);
    R.z = m_sub<M>(m_sub<M>(m_mul<M>(yz, yz), yy), zz);
    return R;
  }
}
// add-2007-bl (P != +-Q; H = 0 gives Z3 = 0, flagged by the caller)
__device__ Jac jac_add(const Jac& P, const Jac& Q) {
  using M = ModP;
  eW z1z1 = m_mul<M>(P.z, P.z), z2z2 = m_mul<M>(Q.z, Q.z);
  eW u1 = m_mul<M>(P.x, z2z2), u2 = m_mul<M>(Q.x, z1z1);
  eW s1 = m_mul<M>(m_mul<M>(P.y, Q.z), z2z2), s2 = m_mul<M>(m_mul<M>(Q.y, P.z), z1z1);
  eW h = m_sub<M>(u2, u1), h2 = m_add<M>(h, h);
  eW i = m_mul<M>(h2, h2), j = m_mul<M>(h, i);
  eW r = m_sub<M>(s2, s1); r = m_add<M>(r, r);
  eW v = m_mul<M>(u1, i);
  Jac R;
  R.x = m_sub<M>(m_sub<M>(m_mul<M>(r, r), j), m_add<M>(v, v));
  eW s1j = m_mul<M>(s1, j);
  R.y = m_sub<M>(m_mul<M>(r, m_sub<M>(v, R.x)), m_add<M>(s1j, s1j));
  eW zz = m_add<M>(P.z, Q.z);
  R.z = m_mul<M>(m_sub<M>(m_sub<M>(m_mul<M>(zz, zz), z1z1), z2z2), h);
  return R;
}

// madd-2007-bl: Q affine (Z2 = 1), 7M + 4S
__device__ Jac jac_add_aff(const Jac& P, const eW& x2, const eW& y2) {
  using M = ModP;
  eW z1z1 = m_mul<M>(P.z, P.z);
  eW u2 = m_mul<M>(x2, z1z1), s2 = m_mul<M>(m_mul<M>(y2, P.z), z1z1);
  eW h = m_sub<M>(u2, P.x), hh = m_mul<M>(h, h);
  eW i = m_add<M>(hh, hh); i = m_add<M>(i, i);
  eW j = m_mul<M>(h, i);
  eW r = m_sub<M>(s2, P.y); r = m_add<M>(r, r);
  eW v = m_mul<M>(P.x, i);
  Jac R;
  R.x = m_sub<M>(m_sub<M>(m_mul<M>(r, r), j), m_add<M>(v, v));
  eW yj = m_mul<M>(P.y, j);
  R.y = m_sub<M>(m_mul<M>(r, m_sub<M>(v, R.x)), m_add<M>(yj, yj));
  eW zh = m_add<M>(P.z, h);
  R.z = m_sub<M>(m_sub<M>(m_mul<M>(zh, zh), z1z1), hh);
  return R;
}

// ============================================================ the EC core
// handles of points: >= 0 op output; H_D dummy point; H_Q public key; <= -1000 fixed-base table entry
constexpr int H_D = -1, H_Q = -2;
__host__ __device__ constexpr int h_tab(int i, int j) { return -(1000 + i * 256 + j); }
enum { PT_GM_AP, PT_GM_RP, PT_PRE, PT_SM_AP, PT_SM_RP };

// Fr (BN254) of a - b for 64-bit a, b
__device__ __forceinline__ fr fr_diff_u64(uint64_t a, uint64_t b) {
  return a >= b ? fr_u64(a - b) : fr_sub(fr_zero(), fr_u64(b - a));
}

// forwarded points (additionPoints / resultingPoints / precompute) of the two scalar multiplications:
// index into the chain's handle list, and the EC core word of the affine point
__host__ __device__ constexpr int ec_pt_index(int kind, int i) {
  return kind == PT_GM_AP ? i : kind == PT_GM_RP ? ECG.parts + i : kind == PT_PRE ? 2 * ECG.parts - 1 + i
       : kind == PT_SM_AP ? 2 * ECG.parts + 15 + i : 2 * ECG.parts + 15 + ECG.wins + i;
}
__host__ __device__ constexpr int ec_pt_base(int idx) {
  return idx < ECG.parts ? ECG.c_gm_ap + P2 * idx
       : idx < 2 * ECG.parts - 1 ? ECG.c_gm_rp + P2 * (idx - ECG.parts)
       : idx < 2 * ECG.parts + 15 ? ECG.c_pre + P2 * (idx - (2 * ECG.parts - 1))
       : idx < 2 * ECG.parts + 15 + ECG.wins ? ECG.c_sm_ap + P2 * (idx - (2 * ECG.parts + 15))
       : ECG.c_sm_rp + P2 * (idx - (2 * ECG.parts + 15 + ECG.wins));
}
static_assert(ec_pt_index(PT_SM_RP, ECG.wins) + 1 == ECG.n_pts, "EC forwarded points");

// byte i / nibble at bit b of a chunked scalar
__device__ __forceinline__ int sc_byte(const uint64_t* s, int i) { return (int)((s[(8 * i) / CS] >> ((8 * i) % CS)) & 255); }
__device__ __forceinline__ int sc_nib(const uint64_t* s, int b) { return (int)((s[b / CS] >> (b % CS)) & 15); }

__device__ __forceinline__ void ec_aff_const(const DevLayout& L, const uint8_t* row, int hd, uint64_t* xy) {
  if (hd == H_D) { for (int i = 0; i < P2; i++) xy[i] = EC_D[i]; }
  else if (hd == H_Q) { for (int i = 0; i < P2; i++) xy[i] = *reinterpret_cast<const uint64_t*>(row + 32ull * (L.reg.in_pk + i)); }
  else {
    const uint64_t* T = L.ec_gpow + (size_t)(-hd - 1000) * P2;
    for (int i = 0; i < P2; i++) xy[i] = T[i];
  }
}
// an input chunk: < 2^CS
__device__ __forceinline__ bool in_is_chunk(const uint8_t* e) { return in_is_u64(e) && (in_u64(e) & ~CS_MASK) == 0; }

// Phase 0, lane = witness: the scalars mod n and the BigMultModP records
__global__ void __launch_bounds__(64) k_ec_scalars(DevLayout L, const uint8_t* inputs, const uint32_t* sha_core,
                                                   uint64_t* ec_core, int32_t* status, uint32_t batch) {
  core_priority();
  const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= batch) return;
  const RegInfo& G = L.reg;
  const uint8_t* row = inputs + 32ull * (uint64_t)w * L.n_inputs;
  uint64_t* C = ec_core + (size_t)w * ECG.core_words;
  int32_t* st = status ? status + w : nullptr;
  bool bad = false;
  uint64_t r[NL], s[NL], h[NL];
  for (int i = 0; i < NL; i++) {
    const uint8_t* a = row + 32ull * (G.in_sig + i);
    const uint8_t* b = row + 32ull * (G.in_sig + NL + i);
    bad |= !in_is_chunk(a) || !in_is_chunk(b);
    r[i] = in_u64(a); s[i] = in_u64(b);
  }
  for (int i = 0; i < P2; i++) bad |= !in_is_chunk(row + 32ull * (G.in_pk + i));
  if (bad) set_status(st, ST_INPUT_RANGE);
  {  // hashedChunked[N-1-i] = digest bits [CS i, CS i + CS) (ecdsa.circom:30-38); the digest as big-endian u32 words
    const ShaJob job = L.sha[G.j_sa];
    const uint32_t* H = sha_core + (size_t)w * L.sha_core_words + job.hout;
    for (int j = 0; j < NL; j++) {
      const int i = NL - 1 - j;
      h[j] = CS == 64 ? ((uint64_t)H[2 * i] << 32) | H[2 * i + 1] : H[i];
    }
  }
  // sinv = s^-1 (BigModInv, bigInt.circom:344-368), u1 = sinv h, u2 = sinv r (mod n)
  using N = ModN;
  auto red_n = [&](const uint64_t* x) { eW a = ew_from_chunks(x); return m_reduce<N>(a.v, 0); };
  const eW sm = m_to<N>(red_n(s)), sinv_m = m_inv<N>(sm);
  const eW u1 = m_from<N>(m_mul<N>(sinv_m, m_to<N>(red_n(h))));
  const eW u2 = m_from<N>(m_mul<N>(sinv_m, m_to<N>(red_n(r))));
  const eW one_chk = m_from<N>(m_mul<N>(sm, sinv_m));
  {
    uint32_t o = one_chk.v[0] ^ 1u;
    for (int i = 1; i < NW; i++) o |= one_chk.v[i];
    if (o) set_status(st, ST_ECDSA_INV);  // bigInt.circom:364-368
  }
  uint64_t sinv[NL], U1[NL], U2[NL];
  ew_to_chunks(m_from<N>(sinv_m), sinv);
  ew_to_chunks(u1, U1);
  ew_to_chunks(u2, U2);
  for (int i = 0; i < NL; i++) {
    C[ECG.c_sinv + i] = sinv[i]; C[ECG.c_u1 + i] = U1[i]; C[ECG.c_u2 + i] = U2[i]; C[ECG.c_h + i] = h[i];
    C[ECG.c_mm + P2 * EC_MM_INV + i] = s[i];    C[ECG.c_mm + P2 * EC_MM_INV + NL + i] = sinv[i];
    C[ECG.c_mm + P2 * EC_MM_U1 + i] = sinv[i];  C[ECG.c_mm + P2 * EC_MM_U1 + NL + i] = h[i];
    C[ECG.c_mm + P2 * EC_MM_U2 + i] = sinv[i];  C[ECG.c_mm + P2 * EC_MM_U2 + NL + i] = r[i];
  }
}

__device__ __forceinline__ void jac_store(uint64_t* d, const Jac& R, int h1, int h2) {
  ew_to_words(R.x, d); ew_to_words(R.y, d + JW); ew_to_words(R.z, d + 2 * JW);
  d[3 * JW] = (uint64_t)(uint32_t)h1 | ((uint64_t)(uint32_t)h2 << 32);
}
__device__ __forceinline__ Jac jac_load(const uint64_t* s0) {
  Jac P; P.x = ew_from_words(s0); P.y = ew_from_words(s0 + JW); P.z = ew_from_words(s0 + 2 * JW); return P;
}
__device__ __forceinline__ Jac jac_of_aff(const uint64_t* xy) {
  Jac P; P.x = m_to<ModP>(ew_from_chunks(xy)); P.y = m_to<ModP>(ew_from_chunks(xy + NL)); P.z = m_const<ModP>(ModP::r1); return P;
}

// Phase 1, lane = (witness, chain): chain 0 = the generator multiplication (ops 0 .. PARTS-1,
// curve.circom:680-906), chain 1 = precompute + the window-4 scalar multiplication of the public
// key (curve.circom:249-494). Jacobian coordinates, the running point in registers, mixed additions
// for affine operands; every op's result and input handles go to the scratch. The isZero / isDummy
// decisions compare handles: a forwarded dummy is the dummy itself, and a curve point equal in x[0]
// to a dummy by chance has probability ~2^-CS.
__global__ void __launch_bounds__(64) k_ec_chain(DevLayout L, const uint8_t* inputs, const uint64_t* ec_core,
                                                 uint64_t* ec_jac, uint32_t batch) {
  core_priority();
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t w = gid >> 1, chain = gid & 1;
  if (w >= batch) return;
  const uint8_t* row = inputs + 32ull * (uint64_t)w * L.n_inputs;
  const uint64_t* C = ec_core + (size_t)w * ECG.core_words;
  uint64_t* J = ec_jac + (size_t)w * ECG.jac_words;
  int32_t* pts = reinterpret_cast<int32_t*>(J + ECG.j_pts);
  using M = ModP;
  if (chain == 0) {
    uint64_t u1[NL];
    for (int i = 0; i < NL; i++) u1[i] = C[ECG.c_u1 + i];
    auto gm_ap = [&](int i) {
      int b = sc_byte(u1, i);
      return b ? h_tab(i, b) : (i % 2 == 0 ? H_D : EC_OP_SD);
    };
    uint64_t dxy[P2];
    for (int i = 0; i < P2; i++) dxy[i] = EC_D[i];
    const Jac D = jac_of_aff(dxy);
    const Jac SD = jac_dbl(D);
    jac_store(J + ECG.j_op * EC_OP_SD, SD, H_D, 0);
    for (int i = 0; i < ECG.parts; i++) pts[ec_pt_index(PT_GM_AP, i)] = gm_ap(i);
    auto point = [&](int hd) -> Jac {  // D, 2D or a table entry
      if (hd == H_D) return D;
      if (hd == EC_OP_SD) return SD;
      return jac_of_aff(L.ec_gpow + (size_t)(-hd - 1000) * P2);
    };
    int left = gm_ap(0);
    Jac acc = point(left);
    for (int i = 0; i < ECG.parts - 1; i++) {
      const int right = gm_ap(i + 1);
      Jac R;
      if (right <= -1000) {
        const uint64_t* T = L.ec_gpow + (size_t)(-right - 1000) * P2;
        R = jac_add_aff(acc, m_to<M>(ew_from_chunks(T)), m_to<M>(ew_from_chunks(T + NL)));
      } else {
        R = jac_add(acc, right == H_D ? D : SD);
      }
      jac_store(J + ECG.j_op * ec_op_gm_add(i), R, left, right);
      const bool ld = left == H_D || left == EC_OP_SD, rd = right == H_D || right == EC_OP_SD;
      const int rp = ld ? right : rd ? left : ec_op_gm_add(i);
      if (ld) acc = point(right);
      else if (!rd) acc = R;
      pts[ec_pt_index(PT_GM_RP, i)] = rp;
      left = rp;
    }
  } else {
    uint64_t u2[NL], qxy[P2], dxy[P2];
    for (int i = 0; i < NL; i++) u2[i] = C[ECG.c_u2 + i];
    ec_aff_const(L, row, H_Q, qxy);
    for (int i = 0; i < P2; i++) dxy[i] = EC_D[i];
    const Jac Q = jac_of_aff(qxy), D = jac_of_aff(dxy);
    const eW qx = Q.x, qy = Q.y;
    auto pre = [](int i) { return i == 0 ? H_D : i == 1 ? H_Q : ec_op_pre(ECG, i); };
    auto pre_jac = [&](int i) -> Jac { return i == 0 ? D : i == 1 ? Q : jac_load(J + ECG.j_op * ec_op_pre(ECG, i)); };
    pts[ec_pt_index(PT_PRE, 0)] = H_D;
    pts[ec_pt_index(PT_PRE, 1)] = H_Q;
    for (int i = 2; i < 16; i++) {
      Jac R;
      if (i % 2 == 0) { R = jac_dbl(pre_jac(i / 2)); jac_store(J + ECG.j_op * ec_op_pre(ECG, i), R, pre(i / 2), 0); }
      else { R = jac_add_aff(pre_jac(i - 1), qx, qy); jac_store(J + ECG.j_op * ec_op_pre(ECG, i), R, H_Q, pre(i - 1)); }
      pts[ec_pt_index(PT_PRE, i)] = ec_op_pre(ECG, i);
    }
    auto nib = [&](int w4) { return sc_nib(u2, ECG.fb - 4 - 4 * w4); };
    pts[ec_pt_index(PT_SM_RP, 0)] = H_D;
    int rp = pre(nib(0));
    Jac rpv = pre_jac(nib(0));
    pts[ec_pt_index(PT_SM_AP, 0)] = rp;
    pts[ec_pt_index(PT_SM_RP, 1)] = rp;
    for (int w4 = 1; w4 < ECG.wins; w4++) {
      const int n = nib(w4), ap = pre(n);
      pts[ec_pt_index(PT_SM_AP, w4)] = ap;
      const bool izr = rp == H_D, iza = ap == H_D;
      Jac d = izr ? D : rpv;
      int hin = izr ? H_D : rp;
      for (int j = 0; j < 4; j++) {
        const int op = ec_op_sm_dbl(ECG, 4 * w4 - 4 + j);
        d = jac_dbl(d);
        jac_store(J + ECG.j_op * op, d, hin, 0);
        hin = op;
      }
      const int dl = ec_op_sm_dbl(ECG, 4 * w4 - 1), ad = ec_op_sm_add(ECG, w4 - 1);
      Jac R = n == 1 ? jac_add_aff(d, qx, qy) : jac_add(d, pre_jac(n));
      jac_store(J + ECG.j_op * ad, R, dl, ap);
      if (izr) { rp = ap; rpv = pre_jac(n); }
      else if (iza) { rp = dl; rpv = d; }
      else { rp = ad; rpv = R; }
      pts[ec_pt_index(PT_SM_RP, w4 + 1)] = rp;
    }
  }
}

// Phase 1b, lane = witness: verifyECDSABits.add (the last op) of the two chains' results
__global__ void __launch_bounds__(64) k_ec_final(uint64_t* ec_jac, uint32_t batch) {
  const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= batch) return;
  uint64_t* J = ec_jac + (size_t)w * ECG.jac_words;
  const int32_t* pts = reinterpret_cast<const int32_t*>(J + ECG.j_pts);
  const int h1 = pts[ec_pt_index(PT_GM_RP, ECG.parts - 2)], h2 = pts[ec_pt_index(PT_SM_RP, ECG.wins)];
  // both are op outputs (a forwarded dummy would need an all-zero scalar, which fails BigModInv /
  // the final check anyway): fall back to zero points otherwise
  Jac P = h1 >= 0 ? jac_load(J + ECG.j_op * h1) : Jac{}, Q = h2 >= 0 ? jac_load(J + ECG.j_op * h2) : Jac{};
  jac_store(J + ECG.j_op * ECG.op_final, jac_add(P, Q), h1, h2);
}

// Phase 2, lane = (witness, group of 8 ops): affine out = (X / Z^2, Y / Z^3), one inversion per group
constexpr int EC_AFF_GROUP = 8, EC_AFF_GROUPS = (ECG.n_ops + EC_AFF_GROUP - 1) / EC_AFF_GROUP;
__global__ void __launch_bounds__(64) k_ec_affine(uint64_t* ec_core, const uint64_t* ec_jac, int32_t* status, uint32_t batch) {
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t w = gid / EC_AFF_GROUPS, g = gid % EC_AFF_GROUPS;
  if (w >= batch) return;
  using M = ModP;
  const uint64_t* J = ec_jac + (size_t)w * ECG.jac_words;
  uint64_t* C = ec_core + (size_t)w * ECG.core_words;
  const int op0 = g * EC_AFF_GROUP, n = min(EC_AFF_GROUP, ECG.n_ops - op0);
  eW pre[EC_AFF_GROUP];
  eW acc = m_const<M>(M::r1);
  bool degenerate = false;
  for (int k = 0; k < n; k++) {
    pre[k] = acc;
    eW z = ew_from_words(J + ECG.j_op * (op0 + k) + 2 * JW);
    if (m_is_zero<M>(z)) degenerate = true;
    else acc = m_mul<M>(acc, z);
  }
  if (degenerate && status) lane_status(status + w, ST_BIGISZERO);  // dx = 0 or y = 0: the affine formulas divide by 0
  eW inv = m_inv<M>(acc);
  for (int k = n - 1; k >= 0; k--) {
    const uint64_t* d = J + ECG.j_op * (op0 + k);
    uint64_t* o = C + ECG.c_rec + ECG.rec_words * (op0 + k) + 2 * P2;
    eW z = ew_from_words(d + 2 * JW);
    if (m_is_zero<M>(z)) { for (int i = 0; i < P2; i++) o[i] = 0; continue; }
    eW zi = m_mul<M>(inv, pre[k]);
    inv = m_mul<M>(inv, z);
    eW zi2 = m_mul<M>(zi, zi), zi3 = m_mul<M>(zi2, zi);
    ew_to_chunks(m_from<M>(m_mul<M>(ew_from_words(d), zi2)), o);
    ew_to_chunks(m_from<M>(m_mul<M>(ew_from_words(d + JW), zi3)), o + NL);
  }
}

// Phase 3, lane = (witness, item): op records' inputs (items < n_ops), forwarded points (next n_pts),
// and the final x1 mod n === r check + modOrder record (last item)
constexpr int EC_LINK_ITEMS = ECG.n_ops + ECG.n_pts + 1;
__global__ void __launch_bounds__(64) k_ec_link(DevLayout L, const uint8_t* inputs, uint64_t* ec_core, const uint64_t* ec_jac,
                                                int32_t* status, uint32_t batch) {
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t w = gid / EC_LINK_ITEMS;
  const int it = (int)(gid % EC_LINK_ITEMS);
  if (w >= batch) return;
  const uint8_t* row = inputs + 32ull * (uint64_t)w * L.n_inputs;
  const uint64_t* J = ec_jac + (size_t)w * ECG.jac_words;
  uint64_t* C = ec_core + (size_t)w * ECG.core_words;
  auto aff = [&](int hd, uint64_t* xy) {
    if (hd >= 0) { const uint64_t* o = C + ECG.c_rec + ECG.rec_words * hd + 2 * P2; for (int i = 0; i < P2; i++) xy[i] = o[i]; }
    else ec_aff_const(L, row, hd, xy);
  };
  if (it < ECG.n_ops) {
    const uint64_t hh = J[ECG.j_op * it + 3 * JW];
    uint64_t* rc = C + ECG.c_rec + ECG.rec_words * it;
    aff((int32_t)(uint32_t)hh, rc);
    if (ec_op_is_dbl(ECG, it)) { for (int i = 0; i < P2; i++) rc[P2 + i] = 0; }
    else aff((int32_t)(uint32_t)(hh >> 32), rc + P2);
  } else if (it < ECG.n_ops + ECG.n_pts) {
    const int idx = it - ECG.n_ops;
    aff(reinterpret_cast<const int32_t*>(J + ECG.j_pts)[idx], C + ec_pt_base(idx));
  } else {  // x1 mod n === r (ecdsa.circom:81-83); modOrder record
    const uint64_t* x1 = C + ECG.c_rec + ECG.rec_words * ECG.op_final + 2 * P2;
    eW xm = m_reduce<ModN>(ew_from_chunks(x1).v, 0);
    uint64_t xr[NL];
    ew_to_chunks(xm, xr);
    bool ok = true;
    for (int i = 0; i < NL; i++) {
      ok &= xr[i] == *reinterpret_cast<const uint64_t*>(row + 32ull * (L.reg.in_sig + i));
      C[ECG.c_mm + P2 * EC_MM_XN + i] = x1[i];
      C[ECG.c_mm + P2 * EC_MM_XN + NL + i] = i == 0 ? 1 : 0;
    }
    if (!ok && status) lane_status(status + w, ST_ECDSA_R);
  }
}

// the difference k_ec_inv inverts for (witness w, inverse j), normal form
__device__ __forceinline__ fr ec_inv_diff(const uint64_t* ec_core, uint32_t w, int j) {
  const uint64_t* C = ec_core + (size_t)w * ECG.core_words;
  const uint64_t dx = EC_D[0];
  fr d;
  if (j < ECG.i_sm_zr) {
    const int i = j >> 2, k = j & 3;
    const uint64_t lx = i == 0 ? C[ECG.c_gm_ap] : C[ECG.c_gm_rp + P2 * (i - 1)], rx = C[ECG.c_gm_ap + P2 * (i + 1)];
    const uint64_t sdx = C[ECG.c_rec + ECG.rec_words * EC_OP_SD + 2 * P2];
    d = fr_diff_u64(k < 2 ? lx : rx, (k & 1) ? sdx : dx);
  } else if (j < ECG.i_sm_za) {
    d = fr_diff_u64(dx, C[ECG.c_sm_rp + P2 * (j - ECG.i_sm_zr)]);
  } else {
    d = fr_diff_u64(dx, C[ECG.c_sm_ap + P2 * (j - ECG.i_sm_za + 1)]);
  }
  return d;
}

// Phase 4, lane = (witness, j): IsEqual inverses (genmult dummy tests, scalarMult isZeroResult /
// isZeroAddition) of the differences in[1] - in[0]; 0 -> 0 (comparators.circom:17). One batched inversion per wave
// (the wave's non-zero differences multiplied across it with shuffles, one Fr inversion shared by the 64 lanes;
// a Fr inversion per lane was 131k VALU per wave, pmc_r4e2).
__global__ void __launch_bounds__(64) k_ec_inv(const uint64_t* ec_core, fr* ec_inv, uint32_t batch) {
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t w = gid / ECG.n_inv;
  const int j = (int)(gid % ECG.n_inv);
  const bool live = w < batch;  // a lane past the batch multiplies 1 into the wave's product and stores nothing
  fr d = fr_zero();
  if (live) d = ec_inv_diff(ec_core, w, j);
  const fr a = fr_is_zero(d) ? fr_mont_one() : fr_mul_fast(d, fr_const(R2_));
  fr others, total;
  fr_group_others<64>(a, others, total);
  const fr r = fr_mul_fast(fr_inv<true>(total), others);  // = 1 / a
  if (live) ec_inv[(size_t)w * ECG.n_inv + j] = fr_is_zero(d) ? d : fr_from_mont_fast(r);
}


// ============================================================ k_ec_table: lane per (witness, op)
template <int TYPE>
__global__ void __launch_bounds__(64) k_ec_table(DevLayout L, const int32_t* ops, const uint64_t* ec_core, uint8_t* ec_tab,
                                                 int32_t* status, uint32_t batch) {
  const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= batch) return;
  const int t = ops[blockIdx.y];
  const uint64_t* C = ec_core + (size_t)w * ECG.core_words;
  const uint64_t* rec = t < ECG.n_ops ? C + ECG.c_rec + ECG.rec_words * t : C + ECG.c_mm + P2 * (t - ECG.n_ops);
  uint4* tab = reinterpret_cast<uint4*>(ec_tab + 32ull * ((size_t)w * L.ec_tab_entries + L.ec_tab_off[t]));
  EcTabCtx c{tab, 0, rec, 0};
  EcWalk<EcTabCtx, EC_CV> walk(c);
  walk.run(TYPE);
  if (c.err && status) lane_status(status + w, c.err);
}

// ============================================================ k_emit_ect: table -> signals
__device__ __forceinline__ uint4 ect_value(const uint4* tab, uint32_t d, uint32_t half) {
  const uint32_t op = d >> 29, bit = (d >> 20) & 511u, idx = d & 0xfffffu;
  if (op == ECD_ZERO) return make_uint4(0u, 0u, 0u, 0u);
  if (op == ECD_COPY) return tab[2 * idx + half];
  if (op == ECD_BIT) {
    if (half) return make_uint4(0u, 0u, 0u, 0u);
    const uint4 q = tab[2 * idx + (bit >> 7)];
    const uint32_t k = (bit >> 5) & 3u, wv = k == 0 ? q.x : k == 1 ? q.y : k == 2 ? q.z : q.w;
    return make_uint4((wv >> (bit & 31u)) & 1u, 0u, 0u, 0u);
  }
  // MASK: v & (2^(bit+1) - 1)
  const uint4 q = tab[2 * idx + half];
  const int nb = (int)bit + 1, lo = 128 * (int)half;
  auto mw = [&](uint32_t x, int k) -> uint32_t {
    const int b0 = lo + 32 * k;
    return nb >= b0 + 32 ? x : nb <= b0 ? 0u : (x & ((1u << (nb - b0)) - 1u));
  };
  return make_uint4(mw(q.x, 0), mw(q.y, 1), mw(q.z, 2), mw(q.w, 3));
}

// workgroup size: a big table (P-224 51 KB, brainpoolP384r1 39 KB of LDS) caps the workgroups per CU at 3-4, so
// those curves run 8 waves per workgroup to keep ~24-32 waves per CU in flight
constexpr int ECT_NT = EC_TABLE_MAX[EC_CV] > 1024 ? 512 : 256;
// Work item x a run of WPB witnesses (PZK_ECT_WPB): the next witness's table is loaded into registers while this
// one's elements are stored, so a workgroup waits out one table load (an HBM round trip, 13 % of the kernel as one
// load per workgroup: profiles/r4_ectab) per WPB witnesses. The descriptor program is the same for all of them.
template <int MM, int ECT_U>  // store mode (mapsink.hpp), descriptors per batch
__global__ void __launch_bounds__(ECT_NT) k_emit_ect(DevLayout L, const Work* work, const uint8_t* ec_tab, uint8_t* wtns,
                                                  size_t stride, int prefetch, uint32_t wpb, uint32_t batch) {
  __shared__ uint4 tab[2 * EC_TABLE_MAX[EC_CV]];
  constexpr int TL = (2 * EC_TABLE_MAX[EC_CV] + ECT_NT - 1) / ECT_NT;  // table uint4 per thread
  const Work wk = work[blockIdx.x];
  const uint32_t wb = blockIdx.y * wpb, we = wb + wpb < batch ? wb + wpb : batch;
  const Region R = L.regions[wk.region];
  const int t = R.a[0], type = R.a[1];
  const uint32_t n2 = 2 * L.ec_tab_n[type];
  // native 4-vectors: a uint4 (HIP_vector_type) copy lowers to memcpy, which keeps tv[] in scratch
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const u32x4* tab0 = reinterpret_cast<const u32x4*>(ec_tab + 32ull * L.ec_tab_off[t]);
  u32x4* tabv = reinterpret_cast<u32x4*>(tab);
  const size_t tab_stride = 2ull * L.ec_tab_entries;  // uint4 per witness
  uint32_t ti[TL];  // this thread's table elements (clamped: every load is issued, before any use)
#pragma unroll
  for (int k = 0; k < TL; k++) ti[k] = threadIdx.x + k * ECT_NT < n2 ? threadIdx.x + k * ECT_NT : 0u;
  u32x4 tv[TL];
  // mapped: the kept elements' descriptors, stored consecutively from their mapped index (desc_run)
  const uint64_t g = R.off + wk.start;
  const uint32_t* o0_prog = L.ec_prog + L.ec_prog_off[type] + wk.start;
  const DescRun dr0 = desc_run<MM>(L, wtns, stride, wb, wk, g, o0_prog);
  const uint32_t* prog = dr0.prog;
  // ECT_U descriptors per batch, loaded before the batch's stores (a global load issued after a store waits for it:
  // gfx9 vmcnt counts both, in order); with prefetch the next batch's descriptors (the next witness's first batch
  // at the end of a witness) are loaded ahead of this batch's stores (PZK_ECT_PREFETCH, PZK_ECT_U: tuning knobs).
  // Two lanes per element, 1 KiB per wave store.
  const uint32_t tot = 2 * dr0.count, step = ECT_U * blockDim.x;
  uint32_t d[ECT_U], dn[ECT_U];
  auto load = [&](uint32_t base, uint32_t* dd) {
#pragma unroll
    for (int k = 0; k < ECT_U; k++) {
      const uint32_t h = base + k * blockDim.x;
      dd[k] = h < tot ? prog[h >> 1] : 0u;
    }
  };
  load(threadIdx.x, dn);  // in flight with the first table's loads
#pragma unroll
  for (int k = 0; k < TL; k++) tv[k] = tab0[wb * tab_stride + ti[k]];
  for (uint32_t w = wb; w < we; w++) {
    if (w > wb) __syncthreads();  // the previous witness's lookups are done
#pragma unroll
    for (int k = 0; k < TL; k++) tabv[ti[k]] = tv[k];  // clamped elements rewrite element 0 with its own value
    __syncthreads();
    const bool more_w = w + 1 < we;
    const size_t nt = (more_w ? w + 1 : w) * tab_stride;  // the next witness's table behind this one's stores
#pragma unroll
    for (int k = 0; k < TL; k++) tv[k] = tab0[nt + ti[k]];
    const OutRow out = desc_run<MM>(L, wtns, stride, w, wk, g, o0_prog).out;
    for (uint32_t base = threadIdx.x; base < tot; base += step) {
#pragma unroll
      for (int k = 0; k < ECT_U; k++) d[k] = dn[k];
      const bool more = base + step < tot || more_w;
      const uint32_t nbase = base + step < tot ? base + step : threadIdx.x;
      if (prefetch && more) load(nbase, dn);
#pragma unroll
      for (int k = 0; k < ECT_U; k++) {
        const uint32_t h = base + k * blockDim.x;
        store_half<MAP_O0>(out, h, h < tot ? ect_value(tab, d[k], h & 1) : make_uint4(0u, 0u, 0u, 0u), h < tot);
      }
      if (!prefetch && more) load(nbase, dn);
    }
  }
}

// ============================================================ k_emit_ecr: the generator multiplication's selection tables
// EllipicCurveScalarGeneratorMult (curve.circom:750-797): resultCoordinateComputation[PARTS][256][2][N],
// equal[PARTS][256] (IsEqual) and getSumOfNElements[PARTS][2][N] (GetSum(256)) — 245 k signals per P-256 witness,
// every one a function of a part's scalar byte b_i and its additionPoints row. Work item = a chunk of one region;
// the chunk's parts (<= 4), their bytes and the 1/(b - j) table go to LDS first, so the store loop issues no
// global load (a load behind the wave's stores would wait for them: gfx9 vmcnt counts both).
template <int MM>
__global__ void __launch_bounds__(256) k_emit_ecr(DevLayout L, const Work* work, Bufs B) {
  constexpr int MAXP = 4;
  __shared__ uint64_t ap[MAXP][P2];
  __shared__ uint32_t bt[MAXP];
  __shared__ fr inv[256];
  __shared__ uint4 stage[2 * 256];
  const Work wk = work[blockIdx.x];
  const uint32_t w = blockIdx.y;
  const Region R = L.regions[wk.region];
  const uint64_t* C = B.ec_core + (size_t)w * ECG.core_words;
  const uint32_t per = R.kind == RK_EC_GM_RCC ? 256u * P2 : R.kind == RK_EC_GM_EQ ? 256u * 6 : 512u * P2;
  const uint32_t i0 = wk.start / per;
  for (uint32_t t = threadIdx.x; t < MAXP * P2; t += blockDim.x) {
    const uint32_t k = t / P2, q = t % P2, i = i0 + k;
    if (i < (uint32_t)ECG.parts) ap[k][q] = C[ECG.c_gm_ap + P2 * i + q];
  }
  if (threadIdx.x < MAXP && i0 + threadIdx.x < (uint32_t)ECG.parts) {
    uint64_t u1[NL];
    for (int k = 0; k < NL; k++) u1[k] = C[ECG.c_u1 + k];
    bt[threadIdx.x] = (uint32_t)sc_byte(u1, (int)(i0 + threadIdx.x));
  }
  if (R.kind == RK_EC_GM_EQ) inv[threadIdx.x] = B.inv_small[threadIdx.x];
  __syncthreads();
  const OutRow out = out_row(L, B.wtns, B.stride, w, R.off + wk.start);
  if (R.kind == RK_EC_GM_RCC) {  // = equal[i][j] * (point j of part i): the part's additionPoints row where j == b_i
    emit_run<MM>(out, wk.count, stage, [&](uint32_t q0) -> El {
      const uint32_t s = wk.start + q0, k = s / (256u * P2) - i0, j = (s / P2) % 256u, q = s % P2;
      return el_u64(bt[k] == j ? ap[k][q] : 0ull);
    });
  } else if (R.kind == RK_EC_GM_EQ) {  // IsEqual(j, b_i): out | in[2] | IsZero(out, b_i - j, 1 / (b_i - j))
    emit_run<MM>(out, wk.count, stage, [&](uint32_t q0) -> El {
      const uint32_t s = wk.start + q0, blk = s / 6, e = s % 6, k = (blk >> 8) - i0, j = blk & 255u, b = bt[k];
      const int d = (int)b - (int)j;
      return iseq_sig((int)e, j, b, d == 0 ? fr_zero() : d > 0 ? inv[d] : fr_sub(fr_zero(), inv[-d]));
    });
  } else {  // GetSumOfNElements(256) of column (i, a, k): out | in[256] | sum[255]
    emit_run<MM>(out, wk.count, stage, [&](uint32_t q0) -> El {
      const uint32_t s = wk.start + q0, blk = s >> 9, m = s & 511u, k = blk / P2 - i0, q = blk % P2, b = bt[k];
      const uint64_t v = ap[k][q];
      return el_u64(m == 0 ? v : m <= 256 ? (b == m - 1 ? v : 0ull) : (b <= m - 256 ? v : 0ull));
    });
  }
}

}  // namespace PZK_EC_NS
}  // namespace pzk
