// Small device helpers shared by the core kernels (register path and ECDSA path).
#pragma once
#include "fr.hpp"
#include "layout.hpp"

namespace pzk {

// ----------------------------------------------------------------------------- helpers
__device__ __forceinline__ bool in_is_u64(const uint8_t* e) {
  const uint4* q = reinterpret_cast<const uint4*>(e);
  uint4 a = q[0], b = q[1];
  return (a.z | a.w | b.x | b.y | b.z | b.w) == 0;
}
__device__ __forceinline__ uint64_t in_u64(const uint8_t* e) { return *reinterpret_cast<const uint64_t*>(e); }
__device__ __forceinline__ uint32_t in_bit(const uint8_t* row, int idx, bool& bad) {
  const uint4* q = reinterpret_cast<const uint4*>(row + 32ull * idx);
  uint4 a = q[0], b = q[1];
  bad |= (a.x > 1u) | ((a.y | a.z | a.w | b.x | b.y | b.z | b.w) != 0u);
  return a.x & 1u;
}
__device__ __forceinline__ void set_status(int32_t* st, int32_t code) {
  lane_status(st, code);
}
// integer from bits (bit k of the number = get(k)), L <= 254
template <typename F>
__device__ __forceinline__ fr bits_to_fr(int L, F get) {
  fr r = fr_zero();
  for (int j = 0; j < L; j++) r.v[j >> 5] |= get(j) << (j & 31);
  return r;
}
// signed 128-bit (lo, hi two's complement) -> normal-form Fr (negative x -> p - |x|)
__device__ __forceinline__ fr fr_from_i128(uint64_t lo, uint64_t hi) {
  bool neg = (int64_t)hi < 0;
  if (neg) { lo = ~lo + 1; hi = ~hi + (lo == 0); }
  fr m = fr_zero();
  m.v[0] = (uint32_t)lo; m.v[1] = (uint32_t)(lo >> 32); m.v[2] = (uint32_t)hi; m.v[3] = (uint32_t)(hi >> 32);
  return neg ? fr_sub(fr_zero(), m) : m;
}

// Software 128/64 -> 64 division (Hacker's Delight divlu), requires u1 < v and v normalised.
__device__ __forceinline__ uint64_t divlu(uint64_t u1, uint64_t u0, uint64_t v, uint64_t* rem) {
  const uint64_t b = 1ull << 32;
  uint64_t vn1 = v >> 32, vn0 = v & 0xffffffffull;
  uint64_t un1 = u0 >> 32, un0 = u0 & 0xffffffffull;
  uint64_t q1 = u1 / vn1, rhat = u1 - q1 * vn1;
  while (q1 >= b || q1 * vn0 > b * rhat + un1) { q1--; rhat += vn1; if (rhat >= b) break; }
  uint64_t un21 = u1 * b + un1 - q1 * v;
  uint64_t q0 = un21 / vn1;
  rhat = un21 - q0 * vn1;
  while (q0 >= b || q0 * vn0 > b * rhat + un0) { q0--; rhat += vn1; if (rhat >= b) break; }
  *rem = un21 * b + un0 - q0 * v;
  return q1 * b + q0;
}

}  // namespace pzk
