// SHA-256 padded-block hasher on gfx950 (hasher/sha2/sha256/*.circom).
//
// Two phases:
//  * core  — one lane per (witness, hasher): the word-level SHA-256 state machine, storing
//            per block Hin[8], W[0..63], A[1..64], E[1..64] (200 words = 800 B).
//  * emit  — signal-parallel: every one of the 150,762 signals of a block
//            (Sha2_224_256Shedule 36,048 + Sha2_224_256Rounds(64) 114,714) is a closed-form
//            function of those 200 words, so consecutive lanes write consecutive 32-byte
//            elements (2 KiB per wave store pair) — the HBM-write-bound bulk of the witness.
#pragma once
#include "fr.hpp"
#include "layout.hpp"
#include "sha_prog.hpp"

namespace pzk {

__device__ __constant__ uint32_t SHA_K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
__device__ __constant__ uint32_t SHA_IV[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                              0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
// SHA-224 (sha224InitialValue.circom:10-20): the same blocks from another IV, 224 output bits
__device__ __constant__ uint32_t SHA224_IV[8] = {0xc1059ed8, 0x367cd507, 0x3070dd17, 0xf70e5939,
                                                 0xffc00b31, 0x68581511, 0x64f98fa7, 0xbefa4fa4};

__device__ __forceinline__ uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
__device__ __forceinline__ uint32_t bsig0(uint32_t a) { return rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22); }
__device__ __forceinline__ uint32_t bsig1(uint32_t e) { return rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25); }
__device__ __forceinline__ uint32_t ssig0(uint32_t w) { return rotr32(w, 7) ^ rotr32(w, 18) ^ (w >> 3); }
__device__ __forceinline__ uint32_t ssig1(uint32_t w) { return rotr32(w, 17) ^ rotr32(w, 19) ^ (w >> 10); }
__device__ __forceinline__ uint64_t mask_lo(int n) { return n >= 64 ? ~0ull : ((1ull << n) - 1); }

// ------------------------------------------------------------------- core kernel
// lane = (witness, job). Input bits are 32-byte elements; a non-bit input flags the lane.
__device__ __forceinline__ void sha_core_lane(const uint8_t* in_row, const ShaJob& job, uint32_t* core,
                                              int32_t* status) {
  uint32_t H[8];
#pragma unroll
  for (int j = 0; j < 8; j++) H[j] = job.algo == 2 ? SHA224_IV[j] : SHA_IV[j];
  bool bad = false;
  for (int m = 0; m < job.blocks; m++) {
    uint32_t* bc = core + job.core_off + m * SHA_BLOCK_CORE;
    uint32_t W[64];
    for (int k = 0; k < 16; k++) {
      uint32_t w = 0;
      const uint4* e = reinterpret_cast<const uint4*>(in_row + 32ull * (job.in_off + m * 512 + k * 32));
      for (int q = 0; q < 32; q++) {  // element q is bit 31-q of the word (MSB first)
        uint4 lo = e[2 * q], hi = e[2 * q + 1];
        bad |= (lo.x > 1u) | ((lo.y | lo.z | lo.w | hi.x | hi.y | hi.z | hi.w) != 0u);
        w = (w << 1) | (lo.x & 1u);
      }
      W[k] = w;
    }
#pragma unroll
    for (int k = 16; k < 64; k++) W[k] = ssig1(W[k - 2]) + W[k - 7] + ssig0(W[k - 15]) + W[k - 16];
#pragma unroll
    for (int j = 0; j < 8; j++) bc[j] = H[j];
#pragma unroll
    for (int k = 0; k < 64; k++) bc[8 + k] = W[k];
    uint32_t a = H[0], b = H[1], c = H[2], d = H[3], e = H[4], f = H[5], g = H[6], h = H[7];
#pragma unroll 8
    for (int k = 0; k < 64; k++) {
      uint32_t t1 = h + bsig1(e) + ((e & f) ^ (~e & g)) + SHA_K[k] + W[k];
      uint32_t t2 = bsig0(a) + ((a & b) ^ (a & c) ^ (b & c));
      h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
      bc[72 + k] = a;
      bc[136 + k] = e;
    }
    H[0] += a; H[1] += b; H[2] += c; H[3] += d; H[4] += e; H[5] += f; H[6] += g; H[7] += h;
  }
  uint32_t* hout = core + job.core_off + job.blocks * SHA_BLOCK_CORE;
#pragma unroll
  for (int j = 0; j < 8; j++) hout[j] = H[j];
  if (bad) lane_status(status, ST_INPUT_RANGE);
}

// ------------------------------------------------------------ closed-form signals
// GetSumOfNElements(32) fed with (1<<i)*bit_i(X): out | in[32] | sum[31]      (64 signals)
__device__ __forceinline__ uint64_t sig_getsum32(uint32_t X, uint32_t j) {
  if (j == 0) return X;
  if (j <= 32) return (uint64_t)(X & (1u << (j - 1)));
  return (uint64_t)X & mask_lo((int)j - 31);
}
// GetLastNBits(32) of V: div | out[32] | in | check[32] | GetLastBitUnsecure[32]  (162)
__device__ __forceinline__ uint64_t sig_lastnbits32(uint64_t V, uint32_t j) {
  if (j == 0) return V >> 32;
  if (j <= 32) return (V >> (j - 1)) & 1;
  if (j == 33) return V;
  if (j < 66) return V & mask_lo((int)j - 33);
  uint32_t q = (j - 66) / 3, r = (j - 66) - 3 * q;
  return r == 0 ? ((V >> q) & 1) : (r == 1 ? (V >> (q + 1)) : (V >> q));
}
// Bits2Num(32) of X: out | in[32] | sum[32]                                         (65)
__device__ __forceinline__ uint64_t sig_bits2num32(uint32_t X, uint32_t j) {
  if (j == 0) return X;
  if (j <= 32) return (X >> (j - 1)) & 1;
  return (uint64_t)X & mask_lo((int)j - 32);
}

// block core accessors (LDS copy): Hin[8] W[64] A[1..64] E[1..64]
struct ShaBlk {
  const uint32_t* c;
  __device__ __forceinline__ uint32_t Hin(int j) const { return c[j]; }
  __device__ __forceinline__ uint32_t W(int k) const { return c[8 + k]; }
  // A[k] for k = -3..64 (A[0] = Hin[0], A[-1] = Hin[1], ...)
  __device__ __forceinline__ uint32_t A(int k) const { return k > 0 ? c[72 + k - 1] : c[-k]; }
  __device__ __forceinline__ uint32_t E(int k) const { return k > 0 ? c[136 + k - 1] : c[4 - k]; }
};

constexpr uint32_t SCH_SIZE = 36048, RDS_SIZE = 114714, SHA_BLOCK_SIGNALS = SCH_SIZE + RDS_SIZE;

// Sha2_224_256Shedule (sha256Schedule.circom:11-72), local signal s
__device__ __forceinline__ uint64_t sha_sched_sig(const ShaBlk& B, uint32_t s) {
  if (s < 64) return B.W(s);                                   // outWords
  if (s < 576) { s -= 64; return (B.W(s >> 5) >> (s & 31)) & 1; }  // chunkBits[16][32]
  if (s < 2624) { s -= 576; return (B.W(s >> 5) >> (s & 31)) & 1; } // outBits[64][32]
  if (s < 3648) { s -= 2624; return sig_getsum32(B.W(s >> 6), s & 63); } // sumN[16]
  s -= 3648;
  uint32_t r = s / 675, j = s - r * 675;
  uint32_t m = r + 16;
  uint32_t wk = B.W(m - 15), wl = B.W(m - 2);
  if (j < 64) return sig_getsum32(ssig0(wk), j);
  if (j < 128) return sig_getsum32(ssig1(wl), j - 64);
  if (j < 448) {
    j -= 128;
    uint32_t i = j / 10, q = j - 10 * i;
    uint32_t w, x, y, z;
    if (q < 5) {  // s0Xor[r][i]
      w = wk; x = (w >> ((i + 7) & 31)) & 1; y = (w >> ((i + 18) & 31)) & 1; z = i < 29 ? (w >> (i + 3)) & 1 : 0;
    } else {      // s1Xor[r][i]
      q -= 5;
      w = wl; x = (wl >> ((i + 17) & 31)) & 1; y = (wl >> ((i + 19) & 31)) & 1; z = i < 22 ? (wl >> (i + 10)) & 1 : 0;
    }
    // XOR3_v2: out | x, y, z | tmp
    switch (q) {
      case 0: return x ^ y ^ z;
      case 1: return x;
      case 2: return y;
      case 3: return z;
      default: return y & z;
    }
  }
  if (j < 610) {
    uint64_t V = (uint64_t)ssig1(wl) + B.W(m - 7) + ssig0(wk) + B.W(m - 16);
    return sig_lastnbits32(V, j - 448);
  }
  return sig_bits2num32(B.W(m), j - 610);
}

// Sha2_224_256CompressInner (sha256Compress.circom:11-96), round k, local signal s (1548)
__device__ __forceinline__ uint64_t sha_compress_sig(const ShaBlk& B, int k, uint32_t s) {
  uint32_t a = B.A(k), b = B.A(k - 1), c = B.A(k - 2), d = B.A(k - 3);
  uint32_t e = B.E(k), f = B.E(k - 1), g = B.E(k - 2), h = B.E(k - 3);
  if (s < 194) {  // outputs
    if (s < 32) return (B.A(k + 1) >> s) & 1;
    if (s < 64) return (a >> (s - 32)) & 1;
    if (s < 96) return (b >> (s - 64)) & 1;
    if (s == 96) return c;
    if (s < 129) return (B.E(k + 1) >> (s - 97)) & 1;
    if (s < 161) return (e >> (s - 129)) & 1;
    if (s < 193) return (f >> (s - 161)) & 1;
    return g;
  }
  if (s < 390) {  // inputs
    if (s == 194) return B.W(k);
    if (s == 195) return SHA_K[k];
    if (s < 228) return (a >> (s - 196)) & 1;
    if (s < 260) return (b >> (s - 228)) & 1;
    if (s < 292) return (c >> (s - 260)) & 1;
    if (s == 292) return d;
    if (s < 325) return (e >> (s - 293)) & 1;
    if (s < 357) return (f >> (s - 325)) & 1;
    if (s < 389) return (g >> (s - 357)) & 1;
    return h;
  }
  uint32_t ch = (e & f) ^ (~e & g);
  if (s < 422) return (ch >> (s - 390)) & 1;
  uint32_t S1 = bsig1(e), S0 = bsig0(a), mj = (a & b) ^ (a & c) ^ (b & c);
  uint64_t ovE = (uint64_t)d + h + S1 + ch + SHA_K[k] + B.W(k);
  uint64_t ovA = (uint64_t)h + S1 + ch + SHA_K[k] + B.W(k) + S0 + mj;
  if (s == 422) return ovE;
  if (s == 423) return ovA;
  if (s < 808) {
    uint32_t q = (s - 424) >> 6, j = (s - 424) & 63;
    uint32_t X = q == 0 ? c : q == 1 ? g : q == 2 ? S0 : q == 3 ? S1 : q == 4 ? mj : ch;
    return sig_getsum32(X, j);
  }
  if (s < 1224) {
    uint32_t t = s - 808, i = t / 13, q = t - 13 * i;
    if (q < 3) {  // Bits2: lo | hi | xy
      uint32_t xy = ((a >> i) & 1) + ((b >> i) & 1) + ((c >> i) & 1);
      return q == 0 ? (xy & 1) : q == 1 ? ((xy >> 1) & 1) : xy;
    }
    uint32_t x, y, z;
    if (q < 8) { q -= 3; x = (a >> ((i + 2) & 31)) & 1; y = (a >> ((i + 13) & 31)) & 1; z = (a >> ((i + 22) & 31)) & 1; }
    else { q -= 8; x = (e >> ((i + 6) & 31)) & 1; y = (e >> ((i + 11) & 31)) & 1; z = (e >> ((i + 25) & 31)) & 1; }
    switch (q) {
      case 0: return x ^ y ^ z;
      case 1: return x;
      case 2: return y;
      case 3: return z;
      default: return y & z;
    }
  }
  if (s < 1386) return sig_lastnbits32(ovE, s - 1224);
  return sig_lastnbits32(ovA, s - 1386);
}

// Sha2_224_256Rounds(64) (sha256Rounds.circom:12-125), local signal s (114,714)
__device__ __forceinline__ uint64_t sha_rounds_sig(const ShaBlk& B, uint32_t s) {
  constexpr uint32_t OWN = 13258, N1 = 65;
  if (s < OWN) {
    if (s < 256) {  // outHash[j][i]
      uint32_t j = s >> 5, i = s & 31;
      uint32_t X = j < 4 ? B.A(64 - (int)j) : B.E(64 - (int)(j - 4));
      return ((B.Hin(j) + X) >> i) & 1;
    }
    if (s < 320) return B.W(s - 256);
    if (s < 576) { s -= 320; return (B.Hin(s >> 5) >> (s & 31)) & 1; }
    s -= 576;
    if (s < 3 * N1 * 32) {  // a, b, c [65][32]
      uint32_t arr = s / (N1 * 32), t = s - arr * N1 * 32, k = t >> 5, i = t & 31;
      return (B.A((int)k - (int)arr) >> i) & 1;
    }
    s -= 3 * N1 * 32;
    if (s < N1) return B.A((int)s - 3);  // dd
    s -= N1;
    if (s < 3 * N1 * 32) {
      uint32_t arr = s / (N1 * 32), t = s - arr * N1 * 32, k = t >> 5, i = t & 31;
      return (B.E((int)k - (int)arr) >> i) & 1;
    }
    s -= 3 * N1 * 32;
    if (s < N1) return B.E((int)s - 3);  // hh
    s -= N1;
    if (s < 64) return SHA_K[s];          // ROUND_KEYS
    return B.Hin(s - 64);                 // hashWords
  }
  s -= OWN;
  if (s < 64) return SHA_K[s];                              // roundKeys
  if (s < 128) return sig_getsum32(B.Hin(3), s - 64);       // sumDd
  if (s < 192) return sig_getsum32(B.Hin(7), s - 128);      // sumHh
  if (s < 704) { s -= 192; return sig_getsum32(B.Hin(s >> 6), s & 63); } // sum[8]
  s -= 704;
  if (s < 64 * 1548) { uint32_t k = s / 1548; return sha_compress_sig(B, (int)k, s - k * 1548); }
  s -= 64 * 1548;
  if (s < 8 * 162) {  // modulo[8]
    uint32_t j = s / 162;
    uint32_t X = j < 4 ? B.A(64 - (int)j) : B.E(64 - (int)(j - 4));
    return sig_lastnbits32((uint64_t)B.Hin(j) + X, s - j * 162);
  }
  s -= 8 * 162;
  uint32_t q = s >> 6;  // sumA sumB sumC sumE sumF sumG
  uint32_t X = q < 3 ? B.A(64 - (int)q) : B.E(64 - (int)(q - 3));
  return sig_getsum32(X, s & 63);
}

// word-table entry e of a block (sha_prog.hpp layout)
__device__ __forceinline__ uint64_t sha_spread(uint32_t x) {  // bit i -> bit 2i
  uint64_t v = x;
  v = (v | (v << 16)) & 0x0000FFFF0000FFFFull;
  v = (v | (v << 8)) & 0x00FF00FF00FF00FFull;
  v = (v | (v << 4)) & 0x0F0F0F0F0F0F0F0Full;
  v = (v | (v << 2)) & 0x3333333333333333ull;
  v = (v | (v << 1)) & 0x5555555555555555ull;
  return v;
}
__device__ __forceinline__ uint64_t sha_wt_entry(const ShaBlk& B, int e) {
  if (e < 64) return B.W(e);
  if (e < sha_wt_e(-3)) return B.A(e - 67);
  if (e <= sha_wt_e(64)) return B.E(e - 135);
  if (e < SHA_WT_K) return 0;  // unused slots
  if (e < SHA_WT_SCH) return SHA_K[e - SHA_WT_K];
  if (e < SHA_WT_CMP) {
    const int r = (e - SHA_WT_SCH) / SHA_SCH_WORDS, q = (e - SHA_WT_SCH) - r * SHA_SCH_WORDS, m = r + 16;
    const uint32_t wk = B.W(m - 15), wl = B.W(m - 2);
    switch (q) {
      case SW_X7: return rotr32(wk, 7);
      case SW_Y18: return rotr32(wk, 18);
      case SW_Z3: return wk >> 3;
      case SW_T0: return rotr32(wk, 18) & (wk >> 3);
      case SW_S0: return ssig0(wk);
      case SW_X17: return rotr32(wl, 17);
      case SW_Y19: return rotr32(wl, 19);
      case SW_Z10: return wl >> 10;
      case SW_T1: return rotr32(wl, 19) & (wl >> 10);
      case SW_S1: return ssig1(wl);
      default: return (uint64_t)ssig1(wl) + B.W(m - 7) + ssig0(wk) + B.W(m - 16);
    }
  }
  if (e < SHA_WT_FF32) {
    const int k = (e - SHA_WT_CMP) / SHA_CMP_WORDS, q = (e - SHA_WT_CMP) - k * SHA_CMP_WORDS;
    const uint32_t a = B.A(k), b = B.A(k - 1), c = B.A(k - 2), d = B.A(k - 3);
    const uint32_t ee = B.E(k), f = B.E(k - 1), g = B.E(k - 2), h = B.E(k - 3);
    const uint32_t ch = (ee & f) ^ (~ee & g), mj = (a & b) ^ (a & c) ^ (b & c);
    switch (q) {
      case CW_CH: return ch;
      case CW_S1: return bsig1(ee);
      case CW_S0: return bsig0(a);
      case CW_MJ: return mj;
      case CW_OVE: return (uint64_t)d + h + bsig1(ee) + ch + SHA_K[k] + B.W(k);
      case CW_OVA: return (uint64_t)h + bsig1(ee) + ch + SHA_K[k] + B.W(k) + bsig0(a) + mj;
      case CW_R2: return rotr32(a, 2);
      case CW_R13: return rotr32(a, 13);
      case CW_R22: return rotr32(a, 22);
      case CW_T0: return rotr32(a, 13) & rotr32(a, 22);
      case CW_R6: return rotr32(ee, 6);
      case CW_R11: return rotr32(ee, 11);
      case CW_R25: return rotr32(ee, 25);
      case CW_T1: return rotr32(ee, 11) & rotr32(ee, 25);
      default: return sha_spread(a ^ b ^ c) | (sha_spread(mj) << 1);
    }
  }
  const int j = (e - SHA_WT_FF32) & 7;
  const uint32_t hj = j < 4 ? B.A(-j) : B.E(4 - j);
  const uint32_t xj = j < 4 ? B.A(64 - j) : B.E(64 - (j - 4));
  return e < SHA_WT_FF64 ? (uint64_t)(uint32_t)(hj + xj) : (uint64_t)hj + xj;
}

__device__ __forceinline__ uint64_t sha_block_sig(const ShaBlk& B, uint32_t s) {
  return s < SCH_SIZE ? sha_sched_sig(B, s) : sha_rounds_sig(B, s - SCH_SIZE);
}

}  // namespace pzk
