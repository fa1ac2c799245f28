// BN254 scalar field Fr on gfx950: 8 x 32-bit limbs, Montgomery form (R = 2^256).
//
// The witness is exported in NORMAL form (the .wtns contract); values
// that are Fr products are carried in Montgomery form inside the core kernels and
// converted once, in the emit kernels, right before the 32-byte store.
//
// Multiplication is CIOS with the "no final carry" shortcut (fr_mul), or FIPS (fr_mul_fast) that is valid because the
// top word of p (0x30644e72) is < (2^32-1)/2 - 1: each step is one v_mad_u64_u32
// (32x32 + 64 -> 64) per limb product. p < 2^254 also lets additions skip the
// 257th bit.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pzk {

struct fr { uint32_t v[8]; };

constexpr uint32_t P_[8] = {0xf0000001u, 0x43e1f593u, 0x79b97091u, 0x2833e848u,
                                                 0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
// R^2 mod p
constexpr uint32_t R2_[8] = {0xae216da7u, 0x1bb8e645u, 0xe35c59e3u, 0x53fe3ab1u,
                                                  0x53bb8085u, 0x8c49833du, 0x7f4e44a5u, 0x0216d0b1u};
// R mod p (Montgomery one)
constexpr uint32_t R1_[8] = {0x4ffffffbu, 0xac96341cu, 0x9f60cd29u, 0x36fc7695u,
                                                  0x7879462eu, 0x666ea36fu, 0x9a07df2fu, 0x0e0a77c1u};
constexpr uint32_t PINV = 0xefffffffu;  // -p^-1 mod 2^32

__device__ __forceinline__ fr fr_zero() { fr r; for (int i = 0; i < 8; i++) r.v[i] = 0; return r; }
__device__ __forceinline__ fr fr_u64(uint64_t x) {
  fr r = fr_zero(); r.v[0] = (uint32_t)x; r.v[1] = (uint32_t)(x >> 32); return r;
}
__device__ __forceinline__ fr fr_const(const uint32_t (&c)[8]) { fr r; for (int i = 0; i < 8; i++) r.v[i] = c[i]; return r; }
__device__ __forceinline__ fr fr_mont_one() { return fr_const(R1_); }

// bit i of a's limbs (a run-time a.v[i >> 5] puts `a` in scratch: select by AND/OR masks instead)
__device__ __forceinline__ uint32_t fr_bit(const fr& a, int i) {
  uint32_t r = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) r |= a.v[k] & (0u - (uint32_t)((i >> 5) == k));
  return (r >> (i & 31)) & 1u;
}

__device__ __forceinline__ bool fr_is_zero(const fr& a) {
  uint32_t o = 0; for (int i = 0; i < 8; i++) o |= a.v[i]; return o == 0;
}
__device__ __forceinline__ bool fr_eq(const fr& a, const fr& b) {
  uint32_t o = 0; for (int i = 0; i < 8; i++) o |= a.v[i] ^ b.v[i]; return o == 0;
}

// r = a - p if a >= p (a < 2p)
__device__ __forceinline__ fr fr_reduce_once(const fr& a) {
  fr t; uint64_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t d = (uint64_t)a.v[i] - P_[i] - br;
    t.v[i] = (uint32_t)d; br = (d >> 32) & 1;
  }
  // per-limb selects: `br ? a : t` on the structs is a select between two addresses, which keeps a
  // caller's fr array (pos_core_lane's state) from being promoted to registers (scratch)
#pragma unroll
  for (int i = 0; i < 8; i++) t.v[i] = br ? a.v[i] : t.v[i];
  return t;
}

__device__ __forceinline__ fr fr_add(const fr& a, const fr& b) {
  fr r; uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) { uint64_t s = (uint64_t)a.v[i] + b.v[i] + c; r.v[i] = (uint32_t)s; c = s >> 32; }
  return fr_reduce_once(r);
}

__device__ __forceinline__ fr fr_sub(const fr& a, const fr& b) {
  fr r; uint64_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) { uint64_t d = (uint64_t)a.v[i] - b.v[i] - br; r.v[i] = (uint32_t)d; br = (d >> 32) & 1; }
  if (br) {
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) { uint64_t s = (uint64_t)r.v[i] + P_[i] + c; r.v[i] = (uint32_t)s; c = s >> 32; }
  }
  return r;
}

__device__ __forceinline__ fr fr_neg(const fr& a) { return fr_sub(fr_zero(), a); }

// Throughput form of the Montgomery product for the emitters (pos_img_fill in poseidon.hpp,
// regemit.hpp), FIPS order (product scanning with the reduction interleaved
// per column): column k accumulates a_j*b_(k-j) and m_j*p_(k-j) into a 96-bit accumulator, each
// 32x32 product being one v_mad_u64_u32 into the accumulator's low 64 bits whose carry-out (vcc)
// goes into the top word — 2 VALU per product, no register moves. The carry read is 2 wait states
// after its write (s_nop 1), the spacing hipcc itself keeps on gfx950 between a VALU write of VCC
// and a VALU carry-in read. Measured on MI355X
// (tools/fieldbench): 1,200 cycles per wave64 product per SIMD against 1,554 for operand-scanning
// CIOS (whose carries cost ~3 moves per product). On a dependent chain at one wave per SIMD the
// carry pad makes it slower (1,233 ns against 1,091 ns), so the latency-bound cores keep fr_mul. A column sums at most 16 products plus the carry-in (< 2^69).
__device__ __forceinline__ void fr_mac(uint64_t& acc, uint32_t& top, uint32_t x, uint32_t y) {
  asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\ts_nop 1\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
      : "+v"(acc), "+v"(top) : "v"(x), "v"(y) : "vcc");
}
// same with y a wave-uniform constant (the modulus words) in an SGPR
__device__ __forceinline__ void fr_mac_s(uint64_t& acc, uint32_t& top, uint32_t x, uint32_t y) {
  asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\ts_nop 1\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
      : "+v"(acc), "+v"(top) : "v"(x), "s"(y) : "vcc");
}
__device__ __forceinline__ fr fr_mul_fast(const fr& a, const fr& b) {
  uint32_t m[8];
  fr r;
  uint64_t acc = 0;
  uint32_t top = 0;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const int j0 = k < 8 ? 0 : k - 7, j1 = k < 8 ? k : 7;
#pragma unroll
    for (int j = j0; j <= j1; j++) {
      fr_mac(acc, top, a.v[j], b.v[k - j]);
      if (j < k && j < 8 && k - j < 8) fr_mac_s(acc, top, m[j], P_[k - j]);
    }
    if (k < 8) {
      m[k] = (uint32_t)acc * PINV;
      fr_mac_s(acc, top, m[k], P_[0]);  // clears the column's low word
    } else {
      r.v[k - 8] = (uint32_t)acc;
    }
    acc = (acc >> 32) | ((uint64_t)top << 32);
    top = 0;
  }
  return fr_reduce_once(r);
}

// (a dedicated FIPS squaring, 36 instead of 64 operand products but doubled per column, measured
// slower than fr_mul_fast(a, a): 1,289 vs 1,200 cycles)
__device__ __forceinline__ fr fr_sqr_fast(const fr& a) { return fr_mul_fast(a, a); }

// a*2^-256 mod p (Montgomery -> normal form): the reduction half of fr_mul_fast
__device__ __forceinline__ fr fr_from_mont_fast(const fr& a) {
  uint32_t m[8];
  fr r;
  uint64_t acc = 0;
  uint32_t top = 0;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    if (k < 8) acc += a.v[k];  // < 2^64: the carry-in is < 2^37 here
#pragma unroll
    for (int j = (k < 8 ? 0 : k - 7); j < (k < 8 ? k : 8); j++) fr_mac_s(acc, top, m[j], P_[k - j]);
    if (k < 8) {
      m[k] = (uint32_t)acc * PINV;
      fr_mac_s(acc, top, m[k], P_[0]);
    } else {
      r.v[k - 8] = (uint32_t)acc;
    }
    acc = (acc >> 32) | ((uint64_t)top << 32);
    top = 0;
  }
  return fr_reduce_once(r);
}
// The general fr_mul / fr_sqr / fr_from_mont below stay operand-scanning CIOS: the latency-bound cores
// (one wave per SIMD on a dependent chain) run them faster than the FIPS form. (The round-2 "FIPS hang"
// of the EC table walker was not this product: the walker had become a callable function whose far
// branches the compiler expanded through its unsaved return-address registers)
// Montgomery product a*b*2^-256 mod p
__device__ __forceinline__ fr fr_mul(const fr& a, const fr& b) {
#ifdef PZK_FR_FIPS_ALL
  return fr_mul_fast(a, b);
#endif
  uint32_t t[8];
#pragma unroll
  for (int j = 0; j < 8; j++) t[j] = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t s = (uint64_t)a.v[0] * b.v[i] + t[0];
    uint32_t C = (uint32_t)(s >> 32);
    uint32_t t0 = (uint32_t)s;
    uint32_t m = t0 * PINV;
    uint64_t s2 = (uint64_t)m * P_[0] + t0;
    uint32_t C2 = (uint32_t)(s2 >> 32);
#pragma unroll
    for (int j = 1; j < 8; j++) {
      s = (uint64_t)a.v[j] * b.v[i] + t[j] + C;
      C = (uint32_t)(s >> 32);
      s2 = (uint64_t)m * P_[j] + (uint32_t)s + C2;
      C2 = (uint32_t)(s2 >> 32);
      t[j - 1] = (uint32_t)s2;
    }
    t[7] = C + C2;
  }
  fr r;
#pragma unroll
  for (int j = 0; j < 8; j++) r.v[j] = t[j];
  return fr_reduce_once(r);
}

// Montgomery square: 28 cross products (doubled) + 8 squares, then REDC — 100 instead of 128
// 32x32 products (measured 12 % faster than fr_mul(a, a) on MI355X, tools/fieldbench)
__device__ __forceinline__ fr fr_sqr(const fr& a) {
#ifdef PZK_FR_FIPS_ALL
  return fr_mul_fast(a, a);
#endif
  uint32_t t[16];
#pragma unroll
  for (int j = 0; j < 16; j++) t[j] = 0;
#pragma unroll
  for (int i = 0; i < 7; i++) {
    uint32_t c = 0;
#pragma unroll
    for (int j = i + 1; j < 8; j++) {
      uint64_t s = (uint64_t)a.v[i] * a.v[j] + t[i + j] + c;
      t[i + j] = (uint32_t)s; c = (uint32_t)(s >> 32);
    }
    t[i + 8] = c;
  }
#pragma unroll
  for (int j = 15; j > 0; j--) t[j] = (t[j] << 1) | (t[j - 1] >> 31);
  t[0] <<= 1;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t s = (uint64_t)a.v[i] * a.v[i] + t[2 * i] + c;
    t[2 * i] = (uint32_t)s;
    uint64_t s2 = (s >> 32) + t[2 * i + 1];
    t[2 * i + 1] = (uint32_t)s2; c = (uint32_t)(s2 >> 32);
  }
  uint32_t hc = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint32_t m = t[i] * PINV, cc = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      uint64_t s = (uint64_t)m * P_[j] + t[i + j] + cc;
      t[i + j] = (uint32_t)s; cc = (uint32_t)(s >> 32);
    }
    uint64_t s = (uint64_t)t[i + 8] + cc + hc;
    t[i + 8] = (uint32_t)s; hc = (uint32_t)(s >> 32);
  }
  fr r;
#pragma unroll
  for (int j = 0; j < 8; j++) r.v[j] = t[8 + j];
  return fr_reduce_once(r);
}
__device__ __forceinline__ fr fr_to_mont(const fr& a) { return fr_mul(a, fr_const(R2_)); }
__device__ __forceinline__ fr fr_from_mont(const fr& a) { fr one = fr_zero(); one.v[0] = 1; return fr_mul(a, one); }

// a^(p-2) in Montgomery form; inverse of 0 is 0 (IsZero semantics, comparators.circom:17).
// FAST = the FIPS product (throughput form, for kernels with many independent lanes per SIMD)
template <bool FAST = false>
__device__ __forceinline__ fr fr_inv(const fr& a) {
  auto mul = [](const fr& x, const fr& y) { return FAST ? fr_mul_fast(x, y) : fr_mul(x, y); };
  auto sqr = [](const fr& x) { return FAST ? fr_mul_fast(x, x) : fr_sqr(x); };
  // exponent p-2 (254 bits, 127 ones), square-and-multiply MSB->LSB on a wave-uniform bit: 253 squarings +
  // 126 products. A 4-bit window table saves ~50 products, but a fr[16] selected by a run-time nibble is
  // lowered to a 512-byte scratch array (every kernel calling this got 528 B of scratch per lane, whose
  // spills reached HBM: 6.9x the algorithmic traffic of k_bjj_core, 1.5x of k_emit_flow)
  fr r = a;
  for (int wi = 7; wi >= 0; wi--) {
    const uint32_t e = wi == 7 ? 0x30644e72u : wi == 6 ? 0xe131a029u : wi == 5 ? 0xb85045b6u : wi == 4 ? 0x8181585du
                     : wi == 3 ? 0x2833e848u : wi == 2 ? 0x79b97091u : wi == 1 ? 0x43e1f593u : 0xefffffffu;
    for (int b = wi == 7 ? 28 : 31; b >= 0; b--) {  // bit 253 (word 7, bit 29) is the leading one: r = a
      r = sqr(r);
      if ((e >> b) & 1u) r = mul(r, a);
    }
  }
  return r;
}

// a^(p-2) by a 4-bit sliding window: the odd powers a^1 .. a^15 in registers, then 49 windows (252 squarings +
// 49 products + 8 for the table = 309 products against fr_inv's 379). The windows are constants (a uniform loop) and
// pick their table entry by masks: no run-time array indexing, so no scratch. Windows of p - 2 MSB first; the first
// window is a^3.
template <bool FAST = false>
__device__ __forceinline__ fr fr_inv_sw(const fr& a) {
  auto mul = [](const fr& x, const fr& y) { return FAST ? fr_mul_fast(x, y) : fr_mul(x, y); };
  auto sqr = [](const fr& x) { return FAST ? fr_mul_fast(x, x) : fr_sqr(x); };
  static constexpr uint8_t SQ[49] = {7, 3, 7, 2, 5, 6, 1, 8, 1, 7, 10, 6, 2, 7, 6, 7, 5, 3, 8, 9, 3, 8, 3, 5, 7,
                                     6, 3, 8, 8, 6, 2, 6, 1, 8, 6, 8, 1, 8, 3, 3, 6, 4, 5, 4, 4, 4, 4, 4, 4};
  static constexpr uint8_t WV[49] = {3, 1, 9, 3, 7, 11, 1, 9, 1, 13, 5, 13, 3, 5, 1, 11, 13, 5, 3, 5, 3, 11, 5, 5, 3,
                                     15, 5, 9, 15, 13, 3, 11, 1, 9, 5, 15, 1, 15, 5, 3, 9, 15, 15, 15, 15, 15, 15, 15, 15};
  const fr a2 = sqr(a);
  const fr t3 = mul(a, a2), t5 = mul(t3, a2), t7 = mul(t5, a2), t9 = mul(t7, a2), t11 = mul(t9, a2),
           t13 = mul(t11, a2), t15 = mul(t13, a2);
  fr r = t3;
  for (int s = 0; s < 49; s++) {
    for (int q = 0; q < SQ[s]; q++) r = sqr(r);
    const int v = WV[s];
    fr t;  // masked OR of the eight entries (a select chain on the structs is lowered to a scratch array)
#pragma unroll
    for (int k = 0; k < 8; k++)
      t.v[k] = (a.v[k] & (0u - (uint32_t)(v == 1))) | (t3.v[k] & (0u - (uint32_t)(v == 3))) |
               (t5.v[k] & (0u - (uint32_t)(v == 5))) | (t7.v[k] & (0u - (uint32_t)(v == 7))) |
               (t9.v[k] & (0u - (uint32_t)(v == 9))) | (t11.v[k] & (0u - (uint32_t)(v == 11))) |
               (t13.v[k] & (0u - (uint32_t)(v == 13))) | (t15.v[k] & (0u - (uint32_t)(v == 15)));
    r = mul(r, t);
  }
  return r;
}

// Batch inversion (Montgomery's trick) over n values in a caller-provided array.
// x[i] := x[i]^-1 (0 stays 0); scratch must hold n elements.
template <typename Acc>
__device__ __forceinline__ void fr_batch_inv(Acc x, Acc scratch, int n) {
  fr acc = fr_mont_one();
  for (int i = 0; i < n; i++) {
    fr xi = x(i);
    scratch(i) = acc;
    if (!fr_is_zero(xi)) acc = fr_mul(acc, xi);
  }
  fr inv = fr_inv(acc);
  for (int i = n - 1; i >= 0; i--) {
    fr xi = x(i);
    if (!fr_is_zero(xi)) {
      fr r = fr_mul(inv, scratch(i));
      inv = fr_mul(inv, xi);
      x(i) = r;
    }
  }
}

// ---- cross-lane moves of a field element (ds_bpermute per limb)
__device__ __forceinline__ fr fr_shfl(const fr& a, int src, int width) {
  fr r;
#pragma unroll
  for (int k = 0; k < 8; k++) r.v[k] = (uint32_t)__shfl((int)a.v[k], src, width);
  return r;
}
__device__ __forceinline__ fr fr_shfl_up(const fr& a, unsigned d) {
  fr r;
#pragma unroll
  for (int k = 0; k < 8; k++) r.v[k] = (uint32_t)__shfl_up((int)a.v[k], d, 64);
  return r;
}
__device__ __forceinline__ fr fr_shfl_down(const fr& a, unsigned d) {
  fr r;
#pragma unroll
  for (int k = 0; k < 8; k++) r.v[k] = (uint32_t)__shfl_down((int)a.v[k], d, 64);
  return r;
}

// Batched inversion across a G-lane group (G a power of two dividing 64): given each lane's product acc, return the
// product of the OTHER lanes' values and the group total, by an inclusive prefix scan and suffix scan (2 log2 G + 1
// products per lane; the gather-all loop it replaces took 2 G).
template <int G>
__device__ __forceinline__ void fr_group_others(const fr& acc, fr& others, fr& total) {
  static_assert(G >= 2 && G <= 64 && (G & (G - 1)) == 0, "G: a power of two <= 64");
  const int l = (int)(threadIdx.x & (G - 1));
  auto up = [](const fr& a, int d) { fr r; for (int k = 0; k < 8; k++) r.v[k] = (uint32_t)__shfl_up((int)a.v[k], d, G); return r; };
  auto down = [](const fr& a, int d) { fr r; for (int k = 0; k < 8; k++) r.v[k] = (uint32_t)__shfl_down((int)a.v[k], d, G); return r; };
  fr p = acc, s = acc;
#pragma unroll
  for (int d = 1; d < G; d <<= 1) {
    const fr u = up(p, d), v = down(s, d);
    if (l >= d) p = fr_mul(p, u);
    if (l + d < G) s = fr_mul(s, v);
  }
  fr pe = up(p, 1), se = down(s, 1);
  if (l == 0) pe = fr_mont_one();
  if (l == G - 1) se = fr_mont_one();
  others = fr_mul(pe, se);
  total = fr_shfl(p, G - 1, G);
}

// ---- wave-contiguous element stores
// Emitters produce one 32-byte element per lane. Stored directly that is 32 B per lane per
// store pair; staged through LDS it becomes two 1 KiB fully contiguous wave stores of 16 B per
// lane, which the MI355X write path sustains ~19 % faster (k_emit_sha measurement).
struct El { uint4 lo, hi; };
__device__ __forceinline__ El el_zero() { return El{make_uint4(0u, 0u, 0u, 0u), make_uint4(0u, 0u, 0u, 0u)}; }
__device__ __forceinline__ El el_u64(uint64_t v) {
  return El{make_uint4((uint32_t)v, (uint32_t)(v >> 32), 0u, 0u), make_uint4(0u, 0u, 0u, 0u)};
}
__device__ __forceinline__ El el_fr(const fr& a) {
  return El{make_uint4(a.v[0], a.v[1], a.v[2], a.v[3]), make_uint4(a.v[4], a.v[5], a.v[6], a.v[7])};
}
__device__ __forceinline__ El el_load(const uint8_t* src) {
  const uint4* s = reinterpret_cast<const uint4*>(src);
  return El{s[0], s[1]};
}
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// All 64 lanes of the wave call this; lane l holds element l of the wave's run starting at
// wave_out; only the first nvalid elements are stored. stage: SW uint4 of LDS per wave — 128, or 64 (half the LDS,
// the two 1 KiB stores staged one after the other: for kernels whose LDS bounds their workgroups per CU)
template <int SW = 128>
__device__ __forceinline__ void wave_store(uint8_t* wave_out, const El& e, uint32_t nvalid, uint4* stage) {
  const uint32_t lane = threadIdx.x & 63;
  uint4* d = reinterpret_cast<uint4*>(wave_out);
  if constexpr (SW == 128) {
    stage[2 * lane] = e.lo;
    stage[2 * lane + 1] = e.hi;
    wave_sync();
    const uint4 a = stage[lane], b = stage[64 + lane];
    if (lane < 2 * nvalid) d[lane] = a;
    if (64 + lane < 2 * nvalid) d[64 + lane] = b;
    wave_sync();
  } else {
    static_assert(SW == 64, "stage: 128 or 64 uint4 per wave");
#pragma unroll
    for (uint32_t h = 0; h < 2; h++) {
      if ((lane >> 5) == h) {
        stage[2 * (lane & 31)] = e.lo;
        stage[2 * (lane & 31) + 1] = e.hi;
      }
      wave_sync();
      const uint4 a = stage[lane];
      if (64 * h + lane < 2 * nvalid) d[64 * h + lane] = a;
      wave_sync();
    }
  }
}
// for (q < count) out[q] = f(q), wave-contiguous; f(q) is evaluated only for q < count
template <int SW = 128, typename F>
__device__ __forceinline__ void emit_run(uint8_t* out, uint32_t count, uint4* stage_block, F f) {
  const uint32_t lane = threadIdx.x & 63;
  uint4* stage = stage_block + (threadIdx.x >> 6) * SW;
  for (uint32_t q0 = threadIdx.x - lane; q0 < count; q0 += blockDim.x) {
    const uint32_t q = q0 + lane;
    const El e = q < count ? f(q) : el_zero();
    wave_store<SW>(out + 32ull * q0, e, count - q0 < 64 ? count - q0 : 64, stage);
  }
}

// 32-byte normal-form store of a small non-negative integer
__device__ __forceinline__ void store_u64(uint8_t* dst, uint64_t v) {
  uint4* d = reinterpret_cast<uint4*>(dst);
  d[0] = make_uint4((uint32_t)v, (uint32_t)(v >> 32), 0u, 0u);
  d[1] = make_uint4(0u, 0u, 0u, 0u);
}
__device__ __forceinline__ void store_fr(uint8_t* dst, const fr& a) {
  uint4* d = reinterpret_cast<uint4*>(dst);
  d[0] = make_uint4(a.v[0], a.v[1], a.v[2], a.v[3]);
  d[1] = make_uint4(a.v[4], a.v[5], a.v[6], a.v[7]);
}
__device__ __forceinline__ fr load_fr(const uint8_t* src) {
  const uint4* s = reinterpret_cast<const uint4*>(src);
  uint4 a = s[0], b = s[1];
  fr r; r.v[0] = a.x; r.v[1] = a.y; r.v[2] = a.z; r.v[3] = a.w; r.v[4] = b.x; r.v[5] = b.y; r.v[6] = b.z; r.v[7] = b.w;
  return r;
}

// Core kernels are latency-bound chains with one wave per SIMD; they share CUs with the
// bandwidth-bound emitters of other streams. Raising their wave priority makes the SIMD arbiter
// issue their instructions first, so the chains are not starved by emitter waves.
__device__ __forceinline__ void core_priority() { __builtin_amdgcn_s_setprio(3); }

// lane status: keep the smallest nonzero check code, so the value reported for a lane that fails
// several checks does not depend on which kernel or stream reached it first
__device__ __forceinline__ void lane_status(int32_t* st, int32_t code) {
  if (!st) return;
  int32_t old = *(volatile int32_t*)st;
  while (old == 0 || old > code) {
    int32_t seen = atomicCAS(st, old, code);
    if (seen == old) return;
    old = seen;
  }
}

}  // namespace pzk
