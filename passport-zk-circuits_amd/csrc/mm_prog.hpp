// BigMultModP(64,K,K,K) block layout (bigInt.circom:206-272) as sections: a signal is addressed
// as (section << 24) | index within the section, located from compile-time section starts
// (mm_locate<K>, no memory access), and k_emit_mm switches on the section.
#pragma once
#include <stdint.h>

namespace pzk {

enum MMSection : uint32_t {
  MM_Q, MM_R, MM_XYN,                          // own: div[K+1] | mod[K] | in1, in2, modulus
  MM_MOUT, MM_MCOPY, MM_KARA,                  // mult = BigMultOverflow: out | in1, in2 | KaratsubaOverflow
  MM_MODCHK,                                   // modChecks[K] = Num2Bits(64)
  MM_GT0, MM_GTIN,                             // greaterThan: out | in[2][K]
  MM_LE0, MM_LEIN, MM_LERES, MM_LT,            // lessEqThan: out | in | result[K] | (LessThan(64), IsEqual) x K
  MM_M2OUT, MM_M2IN, MM_TMPM, MM_TMPR,         // mult2 = BigMultNonEqualOverflow(K+1, K)
  MM_ISZIN, MM_CARRY, MM_RANGE,                // isZero = BigIntIsZero: in | carry | carryRangeChecks
  MM_SECTIONS
};

__host__ __device__ constexpr int mm_log_ceil(int n) { int i = 0; while (n) { n >>= 1; i++; } return i; }
__host__ __device__ constexpr uint32_t mm_kara_size(int N) { return N == 1 ? 4 : 4 * N + 3 * mm_kara_size(N / 2); }
// number of signals of section sec of a BigMultModP(64,K,K,K) block (order as in the template)
__host__ __device__ constexpr uint32_t mm_section_size(int K, int sec) {
  const int BASE = 2 * K, DIV = K + 1, RL = 128 + mm_log_ceil(K + DIV - 1) + 3 - 64;
  switch (sec) {
    case MM_Q: return DIV;
    case MM_R: return K;
    case MM_XYN: return 3 * K;
    case MM_MOUT: return BASE - 1;
    case MM_MCOPY: return 2 * K;
    case MM_KARA:  // KaratsubaOverflow(K) for K = 2^m, else BigMultNonEqualOverflow(K, K) (bigIntOverflow.circom:38-72)
      return (K & (K - 1)) == 0 ? mm_kara_size(K) : (2 * K - 1) + 2 * K + K * K + (2 * K - 1) * K;
    case MM_MODCHK: return 129 * K;
    case MM_GT0: return 1;
    case MM_GTIN: return 2 * K;
    case MM_LE0: return 1;
    case MM_LEIN: return 2 * K;
    case MM_LERES: return K;
    case MM_LT: return 140 * K;
    case MM_M2OUT: return DIV + K - 1;
    case MM_M2IN: return DIV + K;
    case MM_TMPM: return DIV * K;
    case MM_TMPR: return (DIV + K - 1) * K;
    case MM_ISZIN: return BASE - 1;
    case MM_CARRY: return BASE - 2;
    default: return (BASE - 2) * (2 * RL + 1);
  }
}
struct MMStarts { uint32_t v[MM_SECTIONS + 1]; };
__host__ __device__ constexpr MMStarts mm_starts(int K) {
  MMStarts r{};
  uint32_t a = 0;
  for (int i = 0; i <= (int)MM_SECTIONS; i++) {
    r.v[i] = a;
    if (i < (int)MM_SECTIONS) a += mm_section_size(K, i);
  }
  return r;
}
__host__ __device__ constexpr uint32_t mm_section_start(int K, int sec) { return mm_starts(K).v[sec]; }
// (section << 24) | index of block signal s: branch-free count of the (compile-time) section
// starts <= s
template <int K>
__device__ __forceinline__ uint32_t mm_locate(uint32_t s) {
  constexpr MMStarts S = mm_starts(K);
  uint32_t sec = 0, st = 0;
#pragma unroll
  for (int i = 1; i < (int)MM_SECTIONS; i++) {
    const bool ge = s >= S.v[i];
    sec += ge ? 1u : 0u;
    st = ge ? S.v[i] : st;
  }
  return (sec << 24) | (s - st);
}

}  // namespace pzk
