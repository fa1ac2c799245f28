// SHA-384 / SHA-512 hashers (hasher/sha2/sha384/sha384HashChunks.circom:8-48,
// sha512/sha512HashChunks.circom, sha512Schedule.circom, sha512Rounds.circom, sha512Compress.circom):
// the SHA-256 templates at 64-bit words and 80 rounds. A block = Sha2_384_512Schedule (94,480
// signals) + Sha2_384_512Rounds(80) (283,882 signals).
//
// Two phases, as for SHA-256 (sha.hpp):
//  * core — lane per (witness, hasher): the word-level state machine, storing per block
//           Hin[8], W[80], A[1..80], E[1..80] (64-bit words, SHA5_BLOCK_CORE u32);
//  * emit — signal-parallel: every signal of a block is a closed-form function of those words
//           (staged in LDS), values up to 67 bits (the round sums before GetLastNBits(64)).
#pragma once
#include "fr.hpp"
#include "layout.hpp"
#include "sha.hpp"

namespace pzk {

__device__ __constant__ uint64_t SHA512_IV_[8] = {0x6a09e667f3bcc908ull, 0xbb67ae8584caa73bull, 0x3c6ef372fe94f82bull,
                                                  0xa54ff53a5f1d36f1ull, 0x510e527fade682d1ull, 0x9b05688c2b3e6c1full,
                                                  0x1f83d9abfb41bd6bull, 0x5be0cd19137e2179ull};
__device__ __constant__ uint64_t SHA384_IV_[8] = {0xcbbb9d5dc1059ed8ull, 0x629a292a367cd507ull, 0x9159015a3070dd17ull,
                                                  0x152fecd8f70e5939ull, 0x67332667ffc00b31ull, 0x8eb44a8768581511ull,
                                                  0xdb0c2e0d64f98fa7ull, 0x47b5481dbefa4fa4ull};
__device__ __constant__ uint64_t SHA512_K_[80] = {
    0x428a2f98d728ae22ull, 0x7137449123ef65cdull, 0xb5c0fbcfec4d3b2full, 0xe9b5dba58189dbbcull, 0x3956c25bf348b538ull,
    0x59f111f1b605d019ull, 0x923f82a4af194f9bull, 0xab1c5ed5da6d8118ull, 0xd807aa98a3030242ull, 0x12835b0145706fbeull,
    0x243185be4ee4b28cull, 0x550c7dc3d5ffb4e2ull, 0x72be5d74f27b896full, 0x80deb1fe3b1696b1ull, 0x9bdc06a725c71235ull,
    0xc19bf174cf692694ull, 0xe49b69c19ef14ad2ull, 0xefbe4786384f25e3ull, 0x0fc19dc68b8cd5b5ull, 0x240ca1cc77ac9c65ull,
    0x2de92c6f592b0275ull, 0x4a7484aa6ea6e483ull, 0x5cb0a9dcbd41fbd4ull, 0x76f988da831153b5ull, 0x983e5152ee66dfabull,
    0xa831c66d2db43210ull, 0xb00327c898fb213full, 0xbf597fc7beef0ee4ull, 0xc6e00bf33da88fc2ull, 0xd5a79147930aa725ull,
    0x06ca6351e003826full, 0x142929670a0e6e70ull, 0x27b70a8546d22ffcull, 0x2e1b21385c26c926ull, 0x4d2c6dfc5ac42aedull,
    0x53380d139d95b3dfull, 0x650a73548baf63deull, 0x766a0abb3c77b2a8ull, 0x81c2c92e47edaee6ull, 0x92722c851482353bull,
    0xa2bfe8a14cf10364ull, 0xa81a664bbc423001ull, 0xc24b8b70d0f89791ull, 0xc76c51a30654be30ull, 0xd192e819d6ef5218ull,
    0xd69906245565a910ull, 0xf40e35855771202aull, 0x106aa07032bbd1b8ull, 0x19a4c116b8d2d0c8ull, 0x1e376c085141ab53ull,
    0x2748774cdf8eeb99ull, 0x34b0bcb5e19b48a8ull, 0x391c0cb3c5c95a63ull, 0x4ed8aa4ae3418acbull, 0x5b9cca4f7763e373ull,
    0x682e6ff3d6b2b8a3ull, 0x748f82ee5defb2fcull, 0x78a5636f43172f60ull, 0x84c87814a1f0ab72ull, 0x8cc702081a6439ecull,
    0x90befffa23631e28ull, 0xa4506cebde82bde9ull, 0xbef9a3f7b2c67915ull, 0xc67178f2e372532bull, 0xca273eceea26619cull,
    0xd186b8c721c0c207ull, 0xeada7dd6cde0eb1eull, 0xf57d4f7fee6ed178ull, 0x06f067aa72176fbaull, 0x0a637dc5a2c898a6ull,
    0x113f9804bef90daeull, 0x1b710b35131c471bull, 0x28db77f523047d84ull, 0x32caab7b40c72493ull, 0x3c9ebe0a15c9bebcull,
    0x431d67c49c100d4cull, 0x4cc5d4becb3e42b6ull, 0x597f299cfc657e2aull, 0x5fcb6fab3ad6faecull, 0x6c44198c4a475817ull};

__device__ __forceinline__ uint64_t rotr64(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }
__device__ __forceinline__ uint64_t s5_big0(uint64_t a) { return rotr64(a, 28) ^ rotr64(a, 34) ^ rotr64(a, 39); }
__device__ __forceinline__ uint64_t s5_big1(uint64_t e) { return rotr64(e, 14) ^ rotr64(e, 18) ^ rotr64(e, 41); }
__device__ __forceinline__ uint64_t s5_small0(uint64_t w) { return rotr64(w, 1) ^ rotr64(w, 8) ^ (w >> 7); }
__device__ __forceinline__ uint64_t s5_small1(uint64_t w) { return rotr64(w, 19) ^ rotr64(w, 61) ^ (w >> 6); }
__device__ __forceinline__ uint64_t s5_ch(uint64_t e, uint64_t f, uint64_t g) { return (e & f) ^ (~e & g); }
__device__ __forceinline__ uint64_t s5_maj(uint64_t a, uint64_t b, uint64_t c) { return (a & b) ^ (a & c) ^ (b & c); }

// core lane: in_row holds the message bits as 32-byte elements (MSB first per 64-bit word)
__device__ __forceinline__ void sha512_core_lane(const uint8_t* in_row, const ShaJob& job, uint32_t* core,
                                                 int32_t* status) {
  uint64_t H[8];
#pragma unroll
  for (int j = 0; j < 8; j++) H[j] = job.algo == 3 ? SHA384_IV_[j] : SHA512_IV_[j];
  bool bad = false;
  for (int m = 0; m < job.blocks; m++) {
    uint64_t* bc = reinterpret_cast<uint64_t*>(core + job.core_off + m * SHA5_BLOCK_CORE);
    uint64_t W[80];
    for (int k = 0; k < 16; k++) {
      uint64_t w = 0;
      const uint4* e = reinterpret_cast<const uint4*>(in_row + 32ull * (job.in_off + m * 1024 + k * 64));
      for (int q = 0; q < 64; q++) {
        uint4 lo = e[2 * q], hi = e[2 * q + 1];
        bad |= (lo.x > 1u) | ((lo.y | lo.z | lo.w | hi.x | hi.y | hi.z | hi.w) != 0u);
        w = (w << 1) | (lo.x & 1u);
      }
      W[k] = w;
    }
    for (int t = 16; t < 80; t++) W[t] = s5_small1(W[t - 2]) + W[t - 7] + s5_small0(W[t - 15]) + W[t - 16];
    for (int j = 0; j < 8; j++) bc[j] = H[j];
    for (int t = 0; t < 80; t++) bc[8 + t] = W[t];
    uint64_t a = H[0], b = H[1], c = H[2], d = H[3], e = H[4], f = H[5], g = H[6], h = H[7];
    for (int t = 0; t < 80; t++) {
      const uint64_t t1 = h + s5_big1(e) + s5_ch(e, f, g) + SHA512_K_[t] + W[t], t2 = s5_big0(a) + s5_maj(a, b, c);
      h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
      bc[88 + t] = a;
      bc[168 + t] = e;
    }
    H[0] += a; H[1] += b; H[2] += c; H[3] += d; H[4] += e; H[5] += f; H[6] += g; H[7] += h;
  }
  uint64_t* hout = reinterpret_cast<uint64_t*>(core + job.core_off + job.blocks * SHA5_BLOCK_CORE);
  for (int j = 0; j < 8; j++) hout[j] = H[j];
  // the digest again as big-endian 32-bit words (job.hout): the form the digest consumers read (regemit.hpp digest_bit)
  uint32_t* hbe = core + job.hout;
  for (int j = 0; j < 8; j++) { hbe[2 * j] = (uint32_t)(H[j] >> 32); hbe[2 * j + 1] = (uint32_t)H[j]; }
  if (bad) lane_status(status, ST_INPUT_RANGE);
}

// ------------------------------------------------------------ closed-form signals of one block
// LDS view of a block core: h = Hin[8], w = W[80], a[t + 3] = A[t] for t = -3..80 and e[t + 3] = E[t]
// (A[0..-3] = Hin[0..3], E[0..-3] = Hin[4..7]), so the round-t registers are B = A[t-1], C = A[t-2],
// D = A[t-3], F = E[t-1], G = E[t-2], H = E[t-3].
struct Sha5Blk {
  const uint64_t *h, *w, *a, *e;
  __device__ __forceinline__ uint64_t A(int t) const { return a[t + 3]; }
  __device__ __forceinline__ uint64_t E(int t) const { return e[t + 3]; }
};
struct U128 { uint64_t lo, hi; };
__device__ __forceinline__ U128 u128(uint64_t lo, uint64_t hi = 0) { return U128{lo, hi}; }
__device__ __forceinline__ U128 u128_add(U128 x, uint64_t y) { U128 r{x.lo + y, x.hi}; r.hi += r.lo < y; return r; }
__device__ __forceinline__ uint64_t s5_bit(uint64_t x, uint32_t i) { return (x >> i) & 1u; }
__device__ __forceinline__ uint64_t s5_low(uint64_t x, uint32_t n) { return n >= 64 ? x : x & ((1ull << n) - 1); }
__device__ __forceinline__ U128 u128_shr(U128 x, uint32_t n) {  // n < 128
  if (n == 0) return x;
  if (n >= 64) return U128{x.hi >> (n - 64), 0};
  return U128{(x.lo >> n) | (x.hi << (64 - n)), x.hi >> n};
}
// GetSumOfNElements(64) fed with (1 << i) * bit_i(v): out | in[64] | sum[63]
__device__ __forceinline__ uint64_t s5_wordsum(uint64_t v, uint32_t u) {
  if (u == 0) return v;
  if (u <= 64) return v & (1ull << (u - 1));
  return s5_low(v, u - 65 + 2);
}
// GetLastNBits(64) of x (arithmetic.circom:178-204): div, out[64] | in | check[64] | GetLastBitUnsecure[64] (bit, div, in)
__device__ __forceinline__ U128 s5_lastnbits(U128 x, uint32_t u) {
  if (u == 0) return u128(x.hi);
  if (u <= 64) return u128(s5_bit(x.lo, u - 1));
  if (u == 65) return x;
  if (u < 130) return u128(s5_low(x.lo, u - 66 + 1));
  const uint32_t i = (u - 130) / 3, q = u - 130 - 3 * i;
  return q == 0 ? u128(s5_bit(x.lo, i)) : u128_shr(x, q == 1 ? i + 1 : i);
}

constexpr uint32_t S5_SCH_OWN = 80 + 1024 + 5120, S5_SCH_PER_M = 128 + 128 + 640 + 322 + 129;
constexpr uint32_t S5_SCH = S5_SCH_OWN + 16 * 128 + 64 * S5_SCH_PER_M;
constexpr uint32_t S5_RD_OWN = 512 + 80 + 512 + 6 * 81 * 64 + 2 * 81 + 80 + 8;
constexpr uint32_t S5_CI_OWN = 840, S5_CI = S5_CI_OWN + 6 * 128 + 64 * 13 + 2 * 322;
constexpr uint32_t S5_RD = S5_RD_OWN + 80 + 2 * 128 + 8 * 128 + 80 * S5_CI + 8 * 322 + 6 * 128;
static_assert(S5_SCH + S5_RD == SHA5_BLOCK_SIGS, "Sha2_384_512 block size");

// Sha2_384_512Schedule sha512Schedule.circom, local signal s
__device__ __forceinline__ U128 sha5_sched_sig(const Sha5Blk& X, uint32_t s) {
  if (s < 80) return u128(X.w[s]);                                                      // outWords
  if (s < 1104) { s -= 80; return u128(s5_bit(X.w[s >> 6], s & 63)); }                // chunkBits
  if (s < S5_SCH_OWN) { s -= 1104; return u128(s5_bit(X.w[s >> 6], s & 63)); }         // outBits
  s -= S5_SCH_OWN;
  if (s < 16 * 128) return u128(s5_wordsum(X.w[s >> 7], s & 127));                     // sumN[16]
  s -= 16 * 128;
  const uint32_t r = s / S5_SCH_PER_M, m = r + 16;
  uint32_t u = s - S5_SCH_PER_M * r;
  const uint64_t wk = X.w[m - 15], wl = X.w[m - 2], sg0 = s5_small0(wk), sg1 = s5_small1(wl);
  if (u < 128) return u128(s5_wordsum(sg0, u));                                        // s0Sum
  u -= 128;
  if (u < 128) return u128(s5_wordsum(sg1, u));                                        // s1Sum
  u -= 128;
  if (u < 640) {  // (s0Xor[i], s1Xor[i]): out x y z tmp
    const uint32_t i = u / 10, q = u - 10 * i;
    const bool one = q >= 5;
    const uint32_t k = one ? q - 5 : q;
    const uint64_t v = one ? wl : wk;
    const uint32_t ix = one ? (i + 19) & 63 : (i + 1) & 63, iy = one ? (i + 61) & 63 : (i + 8) & 63;
    const uint32_t lim = one ? 58 : 57, iz = one ? i + 6 : i + 7;
    const uint64_t x = s5_bit(v, ix), y = s5_bit(v, iy), z = i < lim ? s5_bit(v, iz) : 0;
    if (k == 0) return u128(s5_bit(one ? sg1 : sg0, i));
    return u128(k == 1 ? x : k == 2 ? y : k == 3 ? z : y & z);
  }
  u -= 640;
  if (u < 322) return s5_lastnbits(u128_add(u128_add(u128_add(u128(sg1), X.w[m - 7]), sg0), X.w[m - 16]), u);  // modulo
  u -= 322;  // bits2Num(64): out | in[64] | sum[64]
  const uint64_t wm = X.w[m];
  return u128(u == 0 ? wm : u <= 64 ? s5_bit(wm, u - 1) : s5_low(wm, u - 64));
}

// Sha2_384_512CompressInner sha512Compress.circom, round k, local signal u
__device__ __forceinline__ U128 sha5_compress_sig(const Sha5Blk& X, int k, uint32_t u) {
  const uint64_t a = X.A(k), b = X.A(k - 1), c = X.A(k - 2), dd = X.A(k - 3), e = X.E(k), f = X.E(k - 1),
                 g = X.E(k - 2), hh = X.E(k - 3), inp = X.w[k], key = SHA512_K_[k];
  const uint64_t S0 = s5_big0(a), S1 = s5_big1(e), ch = s5_ch(e, f, g), mj = s5_maj(a, b, c);
  if (u < 386) {  // outA outB outC outDD outE outF outG outHH
    if (u < 64) return u128(s5_bit(X.A(k + 1), u));
    if (u < 128) return u128(s5_bit(a, u - 64));
    if (u < 192) return u128(s5_bit(b, u - 128));
    if (u == 192) return u128(c);
    if (u < 257) return u128(s5_bit(X.E(k + 1), u - 193));
    if (u < 321) return u128(s5_bit(e, u - 257));
    if (u < 385) return u128(s5_bit(f, u - 321));
    return u128(g);
  }
  u -= 386;
  if (u < 388) {  // inp key a b c dd e f g hh
    if (u == 0) return u128(inp);
    if (u == 1) return u128(key);
    if (u < 66) return u128(s5_bit(a, u - 2));
    if (u < 130) return u128(s5_bit(b, u - 66));
    if (u < 194) return u128(s5_bit(c, u - 130));
    if (u == 194) return u128(dd);
    if (u < 259) return u128(s5_bit(e, u - 195));
    if (u < 323) return u128(s5_bit(f, u - 259));
    if (u < 387) return u128(s5_bit(g, u - 323));
    return u128(hh);
  }
  u -= 388;
  const U128 t1 = u128_add(u128_add(u128_add(u128_add(u128(hh), S1), ch), key), inp);
  if (u < 66) {  // chb[64] overflowE overflowA
    if (u < 64) return u128(s5_bit(ch, u));
    if (u == 64) return u128_add(t1, dd);
    return u128_add(u128_add(t1, S0), mj);
  }
  u -= 66;
  if (u < 6 * 128) {  // dSum hSum s0Sum s1Sum mjSum chSum
    const uint32_t q = u >> 7;
    const uint64_t v = q == 0 ? c : q == 1 ? g : q == 2 ? S0 : q == 3 ? S1 : q == 4 ? mj : ch;
    return u128(s5_wordsum(v, u & 127));
  }
  u -= 6 * 128;
  if (u < 64 * 13) {  // (major = Bits2: lo hi | xy, s0Xor, s1Xor)[64]
    const uint32_t i = u / 13, q = u - 13 * i;
    if (q < 3) {
      const uint64_t xy = s5_bit(a, i) + s5_bit(b, i) + s5_bit(c, i);
      return u128(q == 0 ? xy & 1 : q == 1 ? xy >> 1 : xy);
    }
    const bool one = q >= 8;
    const uint32_t kk = one ? q - 8 : q - 3;
    const uint64_t v = one ? e : a;
    const uint64_t x = s5_bit(v, (i + (one ? 14 : 28)) & 63), y = s5_bit(v, (i + (one ? 18 : 34)) & 63),
                   z = s5_bit(v, (i + (one ? 41 : 39)) & 63);
    if (kk == 0) return u128(s5_bit(one ? S1 : S0, i));
    return u128(kk == 1 ? x : kk == 2 ? y : kk == 3 ? z : y & z);
  }
  u -= 64 * 13;
  if (u < 322) return s5_lastnbits(u128_add(t1, dd), u);  // decomposeE
  return s5_lastnbits(u128_add(u128_add(t1, S0), mj), u - 322);  // decomposeA
}

// Sha2_384_512Rounds(80) sha512Rounds.circom, local signal s
__device__ __forceinline__ U128 sha5_rounds_sig(const Sha5Blk& X, uint32_t s) {
  constexpr uint32_t N1 = 81;
  if (s < S5_RD_OWN) {
    if (s < 512) { const uint32_t j = s >> 6; return u128(s5_bit(X.h[j] + (j < 4 ? X.A(80 - (int)j) : X.E(80 - (int)(j - 4))), s & 63)); }
    s -= 512;
    if (s < 80) return u128(X.w[s]);                                              // words
    s -= 80;
    if (s < 512) return u128(s5_bit(X.h[s >> 6], s & 63));                        // inpHash
    s -= 512;
    // a b c [81][64] dd[81] e f g [81][64] hh[81] ROUND_KEYS[80] hashWords[8]
    if (s < 3 * N1 * 64) { const uint32_t q = s / (N1 * 64), r = s - q * N1 * 64, k = r >> 6; return u128(s5_bit(X.A((int)k - (int)q), r & 63)); }
    s -= 3 * N1 * 64;
    if (s < N1) return u128(X.A((int)s - 3));
    s -= N1;
    if (s < 3 * N1 * 64) { const uint32_t q = s / (N1 * 64), r = s - q * N1 * 64, k = r >> 6; return u128(s5_bit(X.E((int)k - (int)q), r & 63)); }
    s -= 3 * N1 * 64;
    if (s < N1) return u128(X.E((int)s - 3));
    s -= N1;
    if (s < 80) return u128(SHA512_K_[s]);
    return u128(X.h[s - 80]);
  }
  s -= S5_RD_OWN;
  if (s < 80) return u128(SHA512_K_[s]);                                           // roundKeys.out
  s -= 80;
  if (s < 2 * 128) return u128(s5_wordsum(X.h[s < 128 ? 3 : 7], s & 127));         // sumDd sumHh
  s -= 2 * 128;
  if (s < 8 * 128) return u128(s5_wordsum(X.h[s >> 7], s & 127));                 // sum[8]
  s -= 8 * 128;
  if (s < 80 * S5_CI) { const uint32_t k = s / S5_CI; return sha5_compress_sig(X, (int)k, s - S5_CI * k); }
  s -= 80 * S5_CI;
  if (s < 8 * 322) {  // modulo[8]: Hin[j] + final register j
    const uint32_t j = s / 322;
    const uint64_t fin = j < 4 ? X.A(80 - (int)j) : X.E(80 - (int)(j - 4));
    return s5_lastnbits(u128_add(u128(X.h[j]), fin), s - 322 * j);
  }
  s -= 8 * 322;
  const uint32_t q = s >> 7;  // sumA sumB sumC sumE sumF sumG
  const uint64_t v = q < 3 ? X.A(80 - (int)q) : X.E(80 - (int)(q - 3));
  return u128(s5_wordsum(v, s & 127));
}

__device__ __forceinline__ U128 sha5_block_sig(const Sha5Blk& X, uint32_t s) {
  return s < S5_SCH ? sha5_sched_sig(X, s) : sha5_rounds_sig(X, s - S5_SCH);
}

// Sha384HashChunks / Sha512HashChunks(B) own signals: out[O] (MSB-first digest) | in[1024B] (copies) |
// states[B+1][8][64] | iv.out[8][64], after the ShaHashChunks(B, O) wrapper's out[O] | in[1024B] when wrap.
// hin(m, j) = H_m[j] (H_B = Hout).
template <typename HF>
__device__ __forceinline__ uint64_t sha5_own_sig(HF hin, int B, int O, const uint64_t* iv, uint32_t s, bool& is_copy,
                                                 bool wrap = false) {
  is_copy = false;
  if (wrap) {
    if (s < (uint32_t)O) return s5_bit(hin(B, s >> 6), 63 - (s & 63));
    s -= O;
    if (s < 1024u * B) { is_copy = true; return s; }
    s -= 1024u * B;
  }
  if (s < (uint32_t)O) return s5_bit(hin(B, s >> 6), 63 - (s & 63));
  s -= O;
  if (s < 1024u * B) { is_copy = true; return s; }
  s -= 1024u * B;
  if (s < 512u * (B + 1)) { const uint32_t m = s >> 9, r = s & 511; return s5_bit(hin((int)m, r >> 6), r & 63); }
  s -= 512u * (B + 1);
  return s5_bit(iv[s >> 6], s & 63);
}

}  // namespace pzk
