// SHA-256 block program: every one of the 150,762 signals of a Sha2_224_256Shedule +
// Sha2_224_256Rounds(64) block (sha256Schedule.circom:11-72, sha256Rounds.circom:12-125,
// sha256Compress.circom:11-96) is a bit field of one 64-bit word of a per-block WORD TABLE:
//
//   value = mode == EXTRACT ? (word >> lo) & mask(n)      (bits, shifted sums, whole words)
//                           : word & (mask(n) << lo)      (GetSumOfNElements partial sums)
//
// The word table (SHA_WT_SIZE u64, built in LDS per block by k_emit_sha from the 200-word SHA
// core) holds W, A, E, the round keys and, per round, the derived words the templates
// decompose: the XOR3 operands (rotations/shifts), their AND ("tmp"), the sigma outputs, ch, maj,
// the Bits2 sums (2-bit fields), the carry-extended sums (ovE, ovA, V) and the feed-forward sums.
// The per-signal descriptors (u32) are built once on the host (sha_program(), builder.cpp) and
// shared by every block of every witness, so the emitter does one descriptor load, one LDS read
// and a bit-field extract per 32-byte element.
#pragma once
#include <stdint.h>

namespace pzk {

// ---- word table layout
constexpr int SHA_WT_W = 0;                         // W[k], k < 64
__host__ __device__ constexpr int sha_wt_a(int k) { return 67 + k; }    // A(k), k = -3..64 (A(-j) = Hin[j])
__host__ __device__ constexpr int sha_wt_e(int k) { return 135 + k; }   // E(k), k = -3..64 (E(-j) = Hin[4+j])
constexpr int SHA_WT_K = 203;                       // round keys K[k]
constexpr int SHA_WT_SCH = 267;                     // schedule round r < 48: 11 words
constexpr int SHA_SCH_WORDS = 11;
enum { SW_X7, SW_Y18, SW_Z3, SW_T0, SW_S0, SW_X17, SW_Y19, SW_Z10, SW_T1, SW_S1, SW_V };
constexpr int SHA_WT_CMP = SHA_WT_SCH + 48 * SHA_SCH_WORDS;  // compress round k < 64: 15 words
constexpr int SHA_CMP_WORDS = 15;
enum { CW_CH, CW_S1, CW_S0, CW_MJ, CW_OVE, CW_OVA, CW_R2, CW_R13, CW_R22, CW_T0, CW_R6, CW_R11, CW_R25, CW_T1, CW_XY };
constexpr int SHA_WT_FF32 = SHA_WT_CMP + 64 * SHA_CMP_WORDS;   // (Hin[j] + X_j) mod 2^32, j < 8
constexpr int SHA_WT_FF64 = SHA_WT_FF32 + 8;                   // Hin[j] + X_j (no wrap)
constexpr int SHA_WT_SIZE = SHA_WT_FF64 + 8;                   // 1771 words = 14,168 B of LDS

// ---- descriptor
constexpr uint32_t SHA_D_EXTRACT = 0, SHA_D_MASK = 1;
__host__ __device__ constexpr uint32_t sha_desc(int idx, int lo, int n, uint32_t mode) {
  return (uint32_t)idx | ((uint32_t)lo << 11) | ((uint32_t)n << 17) | (mode << 24);
}
__host__ __device__ inline uint64_t sha_desc_apply(uint32_t d, uint64_t v) {
  const uint32_t lo = (d >> 11) & 63, n = (d >> 17) & 127;
  const uint64_t m = n >= 64 ? ~0ull : ((1ull << n) - 1);
  return (d >> 24) ? (v & (m << lo)) : ((v >> lo) & m);
}

// signal ranges of a block (for the per-chunk derived-word ranges)
constexpr uint32_t SHA_BLOCK_SIGNALS_COUNT = 36048 + 114714;
constexpr uint32_t SHA_SCH_ROUND0 = 3648, SHA_SCH_ROUND_SIGS = 675;
constexpr uint32_t SHA_RDS_CMP0 = 36048 + 13258 + 704, SHA_CMP_SIGS = 1548;

}  // namespace pzk
