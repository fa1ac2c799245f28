// SHA-1 hasher (hasher/sha1/*.circom): Sha1HashChunks(B) = out[160] | in[512B] | H(0..4) | B x
// Sha1compression, each a 198,034-signal block of bit-level templates (RotL, Xor4, K, T = RotL5 +
// fT (Maj, Parity/XOR3_v3, Ch) + BinSum(5,32) + Bits2Num(35) + GetLastNBits(32), BinSum(2,32)).
//
// Two phases, as for SHA-256 (sha.hpp):
//  * core — lane per (witness, hasher): the word-level state machine, storing per block Hin[5],
//           W[0..79], A[1..80] (165 words); B..E of round t are A[t-1], rotl30(A[t-2..t-4]).
//  * emit — signal-parallel: every signal of a block is a closed-form function of those words
//           (the block's words staged in LDS), so consecutive lanes write consecutive elements.
#pragma once
#include "fr.hpp"
#include "layout.hpp"
#include "sha.hpp"

namespace pzk {

__device__ __constant__ uint32_t SHA1_IV[5] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u, 0xc3d2e1f0u};
__device__ __forceinline__ uint32_t sha1_k(int t) {
  return t < 20 ? 0x5a827999u : t < 40 ? 0x6ed9eba1u : t < 60 ? 0x8f1bbcdcu : 0xca62c1d6u;
}
__device__ __forceinline__ uint32_t rol32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
__device__ __forceinline__ uint32_t sha1_f(int t, uint32_t b, uint32_t c, uint32_t d) {  // f.circom:60-73
  return t < 20 ? ((b & c) | (~b & d)) : (t < 40 || t >= 60) ? (b ^ c ^ d) : ((b & c) | (b & d) | (c & d));
}

// core lane: in_row holds the message bits as 32-byte elements (MSB first per word)
__device__ __forceinline__ void sha1_core_lane(const uint8_t* in_row, const ShaJob& job, uint32_t* core,
                                               int32_t* status) {
  uint32_t H[5];
#pragma unroll
  for (int j = 0; j < 5; j++) H[j] = SHA1_IV[j];
  bool bad = false;
  for (int m = 0; m < job.blocks; m++) {
    uint32_t* bc = core + job.core_off + m * SHA1_BLOCK_CORE;
    uint32_t W[80];
    for (int k = 0; k < 16; k++) {
      uint32_t w = 0;
      const uint4* e = reinterpret_cast<const uint4*>(in_row + 32ull * (job.in_off + m * 512 + k * 32));
      for (int q = 0; q < 32; q++) {
        uint4 lo = e[2 * q], hi = e[2 * q + 1];
        bad |= (lo.x > 1u) | ((lo.y | lo.z | lo.w | hi.x | hi.y | hi.z | hi.w) != 0u);
        w = (w << 1) | (lo.x & 1u);
      }
      W[k] = w;
    }
#pragma unroll
    for (int t = 16; t < 80; t++) W[t] = rol32(W[t - 3] ^ W[t - 8] ^ W[t - 14] ^ W[t - 16], 1);
#pragma unroll
    for (int j = 0; j < 5; j++) bc[j] = H[j];
#pragma unroll
    for (int t = 0; t < 80; t++) bc[5 + t] = W[t];
    uint32_t a = H[0], b = H[1], c = H[2], d = H[3], e = H[4];
#pragma unroll
    for (int t = 0; t < 80; t++) {
      const uint32_t tmp = rol32(a, 5) + sha1_f(t, b, c, d) + e + sha1_k(t) + W[t];
      e = d; d = c; c = rol32(b, 30); b = a; a = tmp;
      bc[85 + t] = a;
    }
    H[0] += a; H[1] += b; H[2] += c; H[3] += d; H[4] += e;
  }
  uint32_t* hout = core + job.core_off + job.blocks * SHA1_BLOCK_CORE;
#pragma unroll
  for (int j = 0; j < 5; j++) hout[j] = H[j];
  if (bad) lane_status(status, ST_INPUT_RANGE);
}

// ------------------------------------------------------------ closed-form signals of one block
// LDS view: h = Hin[5], w = W[80], a[t + 4] = A[t] for t = -4..80 (A[-1] = H1, A[-2..-4] = rotl2(H2..H4),
// so that B[t] = A[t-1], C[t] = rotl30(A[t-2]), D[t] = rotl30(A[t-3]), E[t] = rotl30(A[t-4]) for every t)
struct Sha1Blk {
  const uint32_t *h, *w, *a;
  __device__ __forceinline__ uint32_t A(int t) const { return a[t + 4]; }
  __device__ __forceinline__ uint32_t B(int t) const { return a[t + 3]; }
  __device__ __forceinline__ uint32_t C(int t) const { return rol32(a[t + 2], 30); }
  __device__ __forceinline__ uint32_t D(int t) const { return rol32(a[t + 1], 30); }
  __device__ __forceinline__ uint32_t E(int t) const { return rol32(a[t], 30); }
  __device__ __forceinline__ uint32_t R(int i) const {  // final register i (A..E after round 79)
    return i == 0 ? A(80) : i == 1 ? B(80) : i == 2 ? C(80) : i == 3 ? D(80) : E(80);
  }
};
__device__ __forceinline__ uint64_t s1_mbit(uint32_t x, uint32_t k) { return (x >> (31 - k)) & 1u; }  // MSB-first
__device__ __forceinline__ uint64_t s1_lbit(uint64_t x, uint32_t k) { return (x >> k) & 1u; }
__device__ __forceinline__ uint64_t s1_mask(uint64_t v, uint32_t n) { return n >= 64 ? v : v & ((1ull << n) - 1); }
// Bits2Num(L) of v: out | in[L] | sum[L]
__device__ __forceinline__ uint64_t s1_b2n(uint64_t v, uint32_t L, uint32_t j) {
  return j == 0 ? v : j <= L ? s1_lbit(v, j - 1) : s1_mask(v, j - L);
}
// Num2Bits(L) of v: out[L] | in | sum[L]
__device__ __forceinline__ uint64_t s1_n2b(uint64_t v, uint32_t L, uint32_t j) {
  return j < L ? s1_lbit(v, j) : j == L ? v : s1_mask(v, j - L);
}
// BinSum(N, 32) of words x[0..N-1] (operations.circom:9-29): out[32+N-1] | in[N][32] | GetSumOfNElements(N)
// (out | in[N] | sum[N-1]) | Bits2Num(32) x N | Num2Bits(32+N-1)
template <int N>
__device__ __forceinline__ uint32_t s1_pick(const uint32_t (&x)[N], uint32_t i) {  // x[i] by selects
  uint32_t r = 0;
#pragma unroll
  for (int k = 0; k < N; k++) r = i == (uint32_t)k ? x[k] : r;
  return r;
}
template <int N>
__device__ __forceinline__ uint64_t s1_binsum(const uint32_t (&x)[N], uint32_t j) {
  constexpr uint32_t O = 32 + N - 1;
  uint64_t S = 0;
#pragma unroll
  for (int i = 0; i < N; i++) S += x[i];
  if (j < O) return s1_lbit(S, j);
  j -= O;
  if (j < 32u * N) return s1_lbit(s1_pick<N>(x, j >> 5), j & 31);
  j -= 32 * N;
  if (j < 2u * N) {
    if (j == 0) return S;
    if (j <= (uint32_t)N) return s1_pick<N>(x, j - 1);
    uint64_t p = x[0];
#pragma unroll
    for (int k = 1; k < N; k++) p += (uint32_t)k <= j - N ? x[k] : 0u;
    return p;
  }
  j -= 2 * N;
  if (j < 65u * N) { const uint32_t i = j / 65; return s1_b2n(s1_pick<N>(x, i), 32, j - 65 * i); }
  return s1_n2b(S, O, j - 65 * N);
}

constexpr uint32_t SHA1_T_SIGS = 1861, SHA1_FSUM_SIGS = 298, SHA1_K_SIGS = 97;
constexpr uint32_t SHA1_OWN = 16352, SHA1_ROTL1 = 64 * 64, SHA1_XOR4 = 64 * 224, SHA1_ROTL30 = 80 * 64,
                   SHA1_KT = 80 * SHA1_K_SIGS, SHA1_TT = 80 * SHA1_T_SIGS, SHA1_FSUM = 5 * SHA1_FSUM_SIGS;
constexpr uint32_t SHA1_BLOCK_SIGNALS = SHA1_OWN + SHA1_ROTL1 + SHA1_XOR4 + SHA1_ROTL30 + SHA1_KT + SHA1_TT + SHA1_FSUM;
static_assert(SHA1_BLOCK_SIGNALS == 198034, "Sha1compression block size");

// T(t) (t.circom:8-57), local signal u
__device__ __forceinline__ uint64_t sha1_t_sig(const Sha1Blk& X, int t, uint32_t u) {
  const uint32_t a = X.A(t), b = X.B(t), c = X.C(t), d = X.D(t), e = X.E(t), k = sha1_k(t), w = X.w[t];
  const uint32_t r5 = rol32(a, 5), f = sha1_f(t, b, c, d);
  if (u < 256) {  // out | a | b | c | d | e | kT | w
    const uint32_t g = u >> 5, q = u & 31;
    const uint32_t v = g == 0 ? X.A(t + 1) : g == 1 ? a : g == 2 ? b : g == 3 ? c : g == 4 ? d : g == 5 ? e : g == 6 ? k : w;
    return s1_mbit(v, q);
  }
  u -= 256;
  if (u < 64) return s1_mbit(u < 32 ? r5 : a, u & 31);  // rotatel5: out | in
  u -= 64;
  if (u < 704) {  // fT: out | b | c | d | maj (out a b c mid) | parity (out a b c) | xor3 (out a b c mid) | ch (out a b c)
    const uint32_t g = u >> 5, q = u & 31;
    const uint32_t maj = (b & c) | (b & d) | (c & d), par = b ^ c ^ d, ch = (b & c) | (~b & d), mid = c & d;
    // selects, not an indexed local array (that would live in scratch memory)
    const uint32_t v = g == 0 ? f : g == 4 ? maj : (g == 8 || g == 17) ? mid : (g == 9 || g == 13) ? par : g == 18 ? ch
                     : (g == 1 || g == 5 || g == 10 || g == 14 || g == 19) ? b
                     : (g == 2 || g == 6 || g == 11 || g == 15 || g == 20) ? c : d;
    return s1_mbit(v, q);
  }
  u -= 704;
  if (u < 604) { const uint32_t x[5] = {r5, f, e, k, w}; return s1_binsum<5>(x, u); }
  u -= 604;
  const uint64_t S = (uint64_t)r5 + f + e + k + w;
  if (u < 71) return s1_b2n(S, 35, u);  // sum = Bits2Num(35)
  return sig_lastnbits32(S, u - 71);    // GetLastNBits(32)
}

// Sha1compression block signal s (sha1compression.circom:7-132)
__device__ __forceinline__ uint64_t sha1_block_sig(const Sha1Blk& X, uint32_t s) {
  if (s < SHA1_OWN) {
    if (s < 160) { const uint32_t i = s >> 5; return s1_lbit((uint64_t)X.h[i] + X.R((int)i), s & 31); }  // out
    if (s < 320) { s -= 160; return s1_mbit(X.h[s >> 5], s & 31); }                                       // hin
    if (s < 832) { s -= 320; return s1_mbit(X.w[s >> 5], s & 31); }                                       // inp
    s -= 832;
    if (s < 5 * 2592) {  // a, b, c, d, e [81][32]
      const uint32_t g = s / 2592, r = s - 2592 * g, t = r >> 5;
      const uint32_t v = g == 0 ? X.A((int)t) : g == 1 ? X.B((int)t) : g == 2 ? X.C((int)t) : g == 3 ? X.D((int)t) : X.E((int)t);
      return s1_mbit(v, r & 31);
    }
    s -= 5 * 2592;
    return s1_mbit(X.w[s >> 5], s & 31);  // w[80][32]
  }
  s -= SHA1_OWN;
  if (s < SHA1_ROTL1) {  // rotl1[i]: out = W[i+16] | in = rotr1(W[i+16])
    const uint32_t i = s >> 6, q = s & 63, wt = X.w[i + 16];
    return s1_mbit(q < 32 ? wt : rol32(wt, 31), q & 31);
  }
  s -= SHA1_ROTL1;
  if (s < SHA1_XOR4) {  // xor4[i]: out | a | b | c | d | mid | aTemp
    const uint32_t i = s / 224, q = s - 224 * i, t = i + 16, g = q >> 5;
    const uint32_t a = X.w[t - 3], b = X.w[t - 8], c = X.w[t - 14], d = X.w[t - 16];
    const uint32_t v = g == 0 ? (a ^ b ^ c ^ d) : g == 1 ? a : g == 2 ? b : g == 3 ? c : g == 4 ? d : g == 5 ? (b & c) : (a ^ b ^ c);
    return s1_mbit(v, q & 31);
  }
  s -= SHA1_XOR4;
  if (s < SHA1_ROTL30) {  // rotl30[t]: out = C[t+1] | in = B[t]
    const uint32_t t = s >> 6, q = s & 63;
    return s1_mbit(q < 32 ? X.C((int)t + 1) : X.B((int)t), q & 31);
  }
  s -= SHA1_ROTL30;
  if (s < SHA1_KT) {  // kT[t] = K(t): out[32] (MSB first) | Num2Bits(32)(K)
    const uint32_t t = s / SHA1_K_SIGS, q = s - SHA1_K_SIGS * t, k = sha1_k((int)t);
    return q < 32 ? s1_mbit(k, q) : s1_n2b(k, 32, q - 32);
  }
  s -= SHA1_KT;
  if (s < SHA1_TT) { const uint32_t t = s / SHA1_T_SIGS; return sha1_t_sig(X, (int)t, s - SHA1_T_SIGS * t); }
  s -= SHA1_TT;
  const uint32_t i = s / SHA1_FSUM_SIGS;  // fSum[i] = BinSum(2, 32)(Hin_i, R_i)
  const uint32_t x[2] = {X.h[i], X.R((int)i)};
  return s1_binsum<2>(x, s - SHA1_FSUM_SIGS * i);
}

// Sha1HashChunks(B) own signals + H(0..4): out[160] (MSB-first digest) | in[512B] (copies) | 5 x K-style constants
__device__ __forceinline__ uint64_t sha1_own_sig(const uint32_t* hout, int B, bool wrapper, uint32_t s, bool& is_copy) {
  is_copy = false;
  if (wrapper) {  // ShaHashChunks(B, 160) (hash.circom:32-68): out[160] | in[512B]
    if (s < 160) return s1_mbit(hout[s >> 5], s & 31);
    s -= 160;
    if (s < 512u * B) { is_copy = true; return s; }
    s -= 512u * B;
  }
  if (s < 160) return s1_mbit(hout[s >> 5], s & 31);
  s -= 160;
  if (s < 512u * B) { is_copy = true; return s; }
  s -= 512u * B;
  const uint32_t x = s / SHA1_K_SIGS, q = s - SHA1_K_SIGS * x, h = SHA1_IV[x];
  return q < 32 ? s1_mbit(h, q) : s1_n2b(h, 32, q - 32);
}

}  // namespace pzk
