// BN254 Fr spread over a DPP quad: four consecutive lanes (lane & ~3 .. lane | 3) hold one field element, lane q of
// the quad its words 2q and 2q + 1 (one 64-bit digit). Used where a chain of dependent Fr products is the critical
// path and too few independent chains exist to fill the chip (k_smt_chain4: one SMT proof's Poseidon levels): a
// product is ~4x shorter on a quad than on one lane, and the chain gets four times as many waves.
//
// Every cross-lane move inside a quad is a DPP quad_perm (a VALU operand modifier, no LDS round trip); moves between
// the quads of one 16-lane row are DPP row_ror. All functions here must be called by every lane of a quad (they
// exchange operands inside it); with the ballot-based carry resolution, by every lane of the wave.
//
// Products are row-wise CIOS (Montgomery, R = 2^256): iteration j broadcasts word j of the first operand to the quad,
// every lane adds its digit's share of a_j * b and of m * p (m = the accumulator's lowest word * -p^-1, broadcast from
// quad lane 0), and the accumulator shifts down one word (the lowest word is zero by construction: quad lane 3
// receives quad lane 0's zero word through the rotation). Per lane the accumulator is three words: positions 2q and
// 2q + 1 and a pending carry (<= 3) at 2q + 2 that belongs to the next lane; it is resolved once, at the end.
//
// Ranges: p < 2^254 and R / p > 5.28, so with a, b < 2p the product is < (4p^2 + Rp) / R < 1.76p: products of
// inputs below 2p stay below 2p without a final subtraction. fq_canon brings a value < 2p to [0, p) (stores, hashes).
#pragma once
#include <type_traits>
#include "fr.hpp"

namespace pzk {

struct fq { uint32_t lo, hi; };  // this lane's digit of a quad-spread element

constexpr int qperm(int a, int b, int c, int d) { return a | (b << 2) | (c << 4) | (d << 6); }
constexpr int DPP_ROW_ROR = 0x120;  // + n: row_ror:n (rotate right by n lanes within each row of 16)

template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xF, 0xF, true);
}
template <int Q>  // lane Q of the quad, to every lane of the quad
__device__ __forceinline__ uint32_t qbcast(uint32_t x) { return dpp<qperm(Q, Q, Q, Q)>(x); }
__device__ __forceinline__ uint32_t qnext(uint32_t x) { return dpp<qperm(1, 2, 3, 0)>(x); }  // lane q <- lane q + 1
__device__ __forceinline__ uint32_t qprev(uint32_t x) { return dpp<qperm(3, 0, 1, 2)>(x); }  // lane q <- lane q - 1
template <int Q>
__device__ __forceinline__ fq fq_bcast(const fq& a) { return fq{qbcast<Q>(a.lo), qbcast<Q>(a.hi)}; }
// lane L of the 16-lane row, to every lane of the row (row_newbcast, gfx90a+)
template <int L>
__device__ __forceinline__ uint32_t rbcast(uint32_t x) { return dpp<0x150 + L>(x); }
// word J (0..7) of the element held by quad Q of the row, to every lane of the row
template <int Q, int J>
__device__ __forceinline__ uint32_t rword(const fq& a) { return rbcast<4 * Q + (J >> 1)>((J & 1) ? a.hi : a.lo); }
// word J of the element of this lane's own quad, to every lane of the quad
template <int J>
__device__ __forceinline__ uint32_t qword(const fq& a) { return qbcast<(J >> 1)>((J & 1) ? a.hi : a.lo); }
// the element of the quad N quads before this one in the 16-lane row (row_ror:4N: lane i <- lane (i - 4N) & 15), so
// quad k gets quad (k - N) & 3's
template <int N>
__device__ __forceinline__ fq fq_from_quad(const fq& a) {
  static_assert(N >= 1 && N <= 3, "quad offset");
  return fq{dpp<DPP_ROW_ROR + 4 * N>(a.lo), dpp<DPP_ROW_ROR + 4 * N>(a.hi)};
}

// per-lane constants: the lane's quad index and its digit of p
struct QLane {
  int q;
  uint32_t p0, p1;
  __device__ __forceinline__ static QLane make() {
    QLane c;
    c.q = (int)(threadIdx.x & 3);
    c.p0 = c.q == 0 ? P_[0] : c.q == 1 ? P_[2] : c.q == 2 ? P_[4] : P_[6];
    c.p1 = c.q == 0 ? P_[1] : c.q == 1 ? P_[3] : c.q == 2 ? P_[5] : P_[7];
    return c;
  }
};

__device__ __forceinline__ fq fq_zero() { return fq{0u, 0u}; }
// the lane's digit of a one-lane element (constant index q: no scratch)
__device__ __forceinline__ fq fq_digit(const fr& a, int q) {
  // masks, not a select chain (which the compiler turns into an indexed scratch array)
  const uint32_t m0 = 0u - (uint32_t)(q == 0), m1 = 0u - (uint32_t)(q == 1), m2 = 0u - (uint32_t)(q == 2),
                 m3 = 0u - (uint32_t)(q == 3);
  fq r;
  r.lo = (a.v[0] & m0) | (a.v[2] & m1) | (a.v[4] & m2) | (a.v[6] & m3);
  r.hi = (a.v[1] & m0) | (a.v[3] & m1) | (a.v[5] & m2) | (a.v[7] & m3);
  return r;
}
// the whole element on every lane of the quad
__device__ __forceinline__ fr fq_gather(const fq& a) {
  fr r;
  r.v[0] = qbcast<0>(a.lo); r.v[1] = qbcast<0>(a.hi);
  r.v[2] = qbcast<1>(a.lo); r.v[3] = qbcast<1>(a.hi);
  r.v[4] = qbcast<2>(a.lo); r.v[5] = qbcast<2>(a.hi);
  r.v[6] = qbcast<3>(a.lo); r.v[7] = qbcast<3>(a.hi);
  return r;
}

// Carry resolution over the quads of a wave: lane l has a carry-out g (bit) and passes an incoming carry on iff p;
// returns the carry INTO each lane. Lane 3 of a quad neither generates nor propagates across the quad boundary
// (callers' ranges guarantee the top lane's carry-out is 0). Every lane of the wave must call it.
__device__ __forceinline__ uint32_t quad_carry_in(bool g, bool p) {
  constexpr uint64_t NOT_TOP = 0x7777777777777777ull;
  const uint64_t G = __ballot(g) & NOT_TOP, P = __ballot(p) & NOT_TOP;
  const uint64_t B = G | P, C = (G + B) ^ G ^ B;  // carry-lookahead by integer addition
  const uint32_t lane = threadIdx.x & 63;
  return (uint32_t)(C >> lane) & 1u;
}

// (lo, hi, x2) with x2 pending at the next lane's position -> normalised digits (value < 2^256)
__device__ __forceinline__ fq fq_settle(uint32_t x0, uint32_t x1, uint32_t x2) {
  const uint32_t cin = qprev(x2);  // quad lane 0 gets lane 3's pending word, 0 for values < 2^256
  uint64_t s = (uint64_t)x0 + cin;
  x0 = (uint32_t)s;
  s = (uint64_t)x1 + (uint32_t)(s >> 32);
  x1 = (uint32_t)s;
  const bool g = (s >> 32) != 0, pr = (x0 & x1) == 0xffffffffu;
  const uint32_t c = quad_carry_in(g, pr);
  s = (uint64_t)x0 + c;
  x0 = (uint32_t)s;
  x1 += (uint32_t)(s >> 32);
  return fq{x0, x1};
}

// Montgomery product a * b * 2^-256 mod p (a, b < 2p: result < 2p, normalised)
__device__ __forceinline__ fq fq_mul(const fq& a, const fq& b, const QLane& c) {
  uint32_t x0 = 0, x1 = 0, x2 = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const uint32_t src = (j & 1) ? a.hi : a.lo;
    const uint32_t aj = (j >> 1) == 0 ? qbcast<0>(src) : (j >> 1) == 1 ? qbcast<1>(src)
                      : (j >> 1) == 2 ? qbcast<2>(src) : qbcast<3>(src);
    const uint64_t X = (uint64_t)aj * b.lo + x0;
    uint64_t Y = (uint64_t)aj * b.hi + (X >> 32);
    Y += x1;  // <= 2^64 - 1: (2^32 - 1)^2 + 2 (2^32 - 1)
    const uint32_t lx = (uint32_t)X;
    const uint32_t m = qbcast<0>(lx) * PINV;
    const uint64_t Z = (uint64_t)m * c.p0 + lx;
    uint64_t W = (uint64_t)m * c.p1 + (Z >> 32);
    W += (uint32_t)Y;
    const uint32_t nx = qnext((uint32_t)Z);  // lane 3 <- lane 0's word, zero by the choice of m
    x0 = (uint32_t)W;
    const uint64_t S = (uint64_t)x2 + (uint32_t)(Y >> 32) + (uint32_t)(W >> 32) + nx;
    x1 = (uint32_t)S;
    x2 = (uint32_t)(S >> 32);
  }
  return fq_settle(x0, x1, x2);
}

// The same product with 64-bit iterations (digit J of a broadcast per step, product scanning inside the lane's two
// columns with fr_mac's 96-bit accumulator: one v_mad_u64_u32 + one carry add per 32 x 32 product), shifting one
// whole lane per step
__device__ __forceinline__ fq fq_mul64(const fq& a, const fq& b, const QLane& c) {
  uint32_t u0 = 0, u1 = 0, u2 = 0;  // the lane's digit (positions 0, 1) and its pending word at position 2
#pragma unroll
  for (int J = 0; J < 4; J++) {
    const uint32_t a0 = J == 0 ? qbcast<0>(a.lo) : J == 1 ? qbcast<1>(a.lo) : J == 2 ? qbcast<2>(a.lo) : qbcast<3>(a.lo);
    const uint32_t a1 = J == 0 ? qbcast<0>(a.hi) : J == 1 ? qbcast<1>(a.hi) : J == 2 ? qbcast<2>(a.hi) : qbcast<3>(a.hi);
    uint64_t acc = (uint64_t)u0 | ((uint64_t)u1 << 32);
    uint32_t top = u2;
    fr_mac(acc, top, a0, b.lo);  // position 0
    const uint32_t m0 = qbcast<0>((uint32_t)acc) * PINV;
    fr_mac(acc, top, m0, c.p0);
    const uint32_t w0 = (uint32_t)acc;  // quad lane 0: zero
    acc = (acc >> 32) | ((uint64_t)top << 32);
    top = 0;
    fr_mac(acc, top, a0, b.hi);  // position 1
    fr_mac(acc, top, a1, b.lo);
    fr_mac(acc, top, m0, c.p1);
    const uint32_t m1 = qbcast<0>((uint32_t)acc) * PINV;
    fr_mac(acc, top, m1, c.p0);
    const uint32_t w1 = (uint32_t)acc;  // quad lane 0: zero
    acc = (acc >> 32) | ((uint64_t)top << 32);
    top = 0;
    fr_mac(acc, top, a1, b.hi);  // positions 2, 3 (the next lane's digit)
    fr_mac(acc, top, m1, c.p1);
    // shift one lane: the next lane's (w0, w1) comes down (quad lane 3 gets lane 0's zeros)
    const uint64_t nx = (uint64_t)qnext(w0) | ((uint64_t)qnext(w1) << 32);
    const uint64_t s = acc + nx;
    u0 = (uint32_t)s;
    u1 = (uint32_t)(s >> 32);
    u2 = top + (s < acc ? 1u : 0u);
  }
  return fq_settle(u0, u1, u2);
}

// Lazy sum of products, reduced once: K * 2^-256 + sum_r a_r * b_r * 2^-256 (mod p), for NR rows. A(r, j, J) gives
// word j of row r's first operand, broadcast (J: std::integral_constant<int, j>, for compile-time DPP controls);
// b[r] is this lane's digit of row r's second operand; k the lane's digit of the constant K (< p).
// Per lane two column accumulators of 96 bits: E at the digit's even position 2q, O at the odd one 2q + 1. Each
// iteration adds the rows' a_j * b and m * p into them (fr_mac: one v_mad_u64_u32 + one carry add per product);
// the frame then shifts one word: E <- O + (E >> 32), O <- the next lane's E word 0 (quad lane 0's is zero).
// Result < (K + sum_r |a_r| |b_r| + R p) / R; the caller keeps it below 2^256.
// The rows' products of one iteration: 2 NR v_mad_u64_u32 into the two columns, each with its own SGPR carry-out
// pair, then the 2 NR carry adds into the columns' top words. A VALU write of an SGPR needs two wait states before a
// VALU reads it as a carry-in; with the adds after all the products that spacing is there without s_nop for NR >= 2
// (NR = 1 pads one). Every register a later DPP reads (E's low word) is written at least two instructions before
// the block ends.
template <int NR>
__device__ __forceinline__ void fq_rows_mac(const uint32_t* a, const fq* b, uint64_t& e, uint32_t& et, uint64_t& o,
                                            uint32_t& ot) {
  static_assert(NR == 1 || NR == 2 || NR == 3, "rows");
  uint64_t c0, c1, c2, c3, c4, c5;
  if constexpr (NR == 1) {
    asm("v_mad_u64_u32 %0, %4, %6, %7, %0\n\t"
        "v_mad_u64_u32 %1, %5, %6, %8, %1\n\t"
        "s_nop 0\n\t"
        "v_addc_co_u32_e64 %2, %4, 0, %2, %4\n\t"
        "v_addc_co_u32_e64 %3, %5, 0, %3, %5"
        : "+v"(e), "+v"(o), "+v"(et), "+v"(ot), "=&s"(c0), "=&s"(c1)
        : "v"(a[0]), "v"(b[0].lo), "v"(b[0].hi));
  } else if constexpr (NR == 2) {
    asm("v_mad_u64_u32 %0, %4, %8, %10, %0\n\t"
        "v_mad_u64_u32 %1, %5, %8, %11, %1\n\t"
        "v_mad_u64_u32 %0, %6, %9, %12, %0\n\t"
        "v_mad_u64_u32 %1, %7, %9, %13, %1\n\t"
        "v_addc_co_u32_e64 %2, %4, 0, %2, %4\n\t"
        "v_addc_co_u32_e64 %3, %5, 0, %3, %5\n\t"
        "v_addc_co_u32_e64 %2, %6, 0, %2, %6\n\t"
        "v_addc_co_u32_e64 %3, %7, 0, %3, %7"
        : "+v"(e), "+v"(o), "+v"(et), "+v"(ot), "=&s"(c0), "=&s"(c1), "=&s"(c2), "=&s"(c3)
        : "v"(a[0]), "v"(a[1]), "v"(b[0].lo), "v"(b[0].hi), "v"(b[1].lo), "v"(b[1].hi));
  } else {
    asm("v_mad_u64_u32 %0, %4, %10, %13, %0\n\t"
        "v_mad_u64_u32 %1, %5, %10, %14, %1\n\t"
        "v_mad_u64_u32 %0, %6, %11, %15, %0\n\t"
        "v_mad_u64_u32 %1, %7, %11, %16, %1\n\t"
        "v_mad_u64_u32 %0, %8, %12, %17, %0\n\t"
        "v_mad_u64_u32 %1, %9, %12, %18, %1\n\t"
        "v_addc_co_u32_e64 %2, %4, 0, %2, %4\n\t"
        "v_addc_co_u32_e64 %3, %5, 0, %3, %5\n\t"
        "v_addc_co_u32_e64 %2, %6, 0, %2, %6\n\t"
        "v_addc_co_u32_e64 %3, %7, 0, %3, %7\n\t"
        "v_addc_co_u32_e64 %2, %8, 0, %2, %8\n\t"
        "v_addc_co_u32_e64 %3, %9, 0, %3, %9"
        : "+v"(e), "+v"(o), "+v"(et), "+v"(ot), "=&s"(c0), "=&s"(c1), "=&s"(c2), "=&s"(c3), "=&s"(c4), "=&s"(c5)
        : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(b[0].lo), "v"(b[0].hi), "v"(b[1].lo), "v"(b[1].hi), "v"(b[2].lo),
          "v"(b[2].hi));
  }
  (void)c2; (void)c3; (void)c4; (void)c5;
}
template <int NR, class A, int J>
__device__ __forceinline__ void fq_dot_a(A& aw, uint32_t* a) {
  if constexpr (NR > 0) {
    a[NR - 1] = aw(NR - 1, std::integral_constant<int, J>{});
    fq_dot_a<NR - 1, A, J>(aw, a);
  }
}
template <int NR, class A, int J = 0>
__device__ __forceinline__ void fq_dot_iter(A& aw, const fq* b, const QLane& c, uint64_t& e, uint32_t& et, uint64_t& o,
                                            uint32_t& ot) {
  if constexpr (J < 8) {
    uint32_t a[NR];
    fq_dot_a<NR, A, J>(aw, a);
    fq_rows_mac<NR>(a, b, e, et, o, ot);
    const uint32_t m = qbcast<0>((uint32_t)e) * PINV;
    const uint32_t mm[1] = {m};
    const fq pp[1] = {fq{c.p0, c.p1}};
    fq_rows_mac<1>(mm, pp, e, et, o, ot);
    // shift one word: the odd column becomes the even one (plus the even column's carry), the next lane's even word
    // becomes this lane's odd column
    const uint32_t nx = qnext((uint32_t)e);
    const uint64_t hi = (e >> 32) | ((uint64_t)et << 32);
    const uint64_t s = o + hi;
    et = ot + (s < o ? 1u : 0u);
    e = s;
    o = nx;
    ot = 0;
    fq_dot_iter<NR, A, J + 1>(aw, b, c, e, et, o, ot);
  }
}
// (E, O) -> normalised digits
__device__ __forceinline__ fq fq_settle_eo(uint64_t e, uint32_t et, uint64_t o, uint32_t ot) {
  // positions: 2q: e.lo; 2q + 1: e.hi + o.lo; 2q + 2: et + o.hi; 2q + 3: ot
  const uint32_t x0 = (uint32_t)e;
  uint64_t s = (e >> 32) + (uint32_t)o;
  const uint32_t x1 = (uint32_t)s;
  s = (uint64_t)et + (uint32_t)(o >> 32) + (s >> 32);
  const uint32_t y0 = (uint32_t)s, y1 = ot + (uint32_t)(s >> 32);  // pending at the next lane's digit
  const uint32_t c0 = qprev(y0), c1 = qprev(y1);                      // quad lane 0 gets lane 3's: 0 below 2^256
  s = (uint64_t)x0 + c0;
  const uint32_t z0 = (uint32_t)s;
  s = (uint64_t)x1 + c1 + (s >> 32);
  const uint32_t z1 = (uint32_t)s;
  const bool g = (s >> 32) != 0, pr = (z0 & z1) == 0xffffffffu;
  const uint32_t cin = quad_carry_in(g, pr);
  s = (uint64_t)z0 + cin;
  return fq{(uint32_t)s, z1 + (uint32_t)(s >> 32)};
}
template <int NR, class A>
__device__ __forceinline__ fq fq_dot(A aw, const fq (&b)[NR], const fq& k, const QLane& c) {
  uint64_t e = k.lo, o = k.hi;
  uint32_t et = 0, ot = 0;
  fq_dot_iter<NR, A, 0>(aw, b, c, e, et, o, ot);
  return fq_settle_eo(e, et, o, ot);
}
// a * b * 2^-256 with a from this lane's quad
__device__ __forceinline__ fq fq_mulq(const fq& a, const fq& b, const QLane& c) {
  const fq bb[1] = {b};
  return fq_dot<1>([&](int, auto J) { return qword<decltype(J)::value>(a); }, bb, fq_zero(), c);
}

// a - p if a >= p (a < 2p): the canonical representative
__device__ __forceinline__ fq fq_canon(const fq& a, const QLane& c) {
  uint64_t d = (uint64_t)a.lo - c.p0;
  const uint32_t d0 = (uint32_t)d;
  const uint32_t b1 = (uint32_t)(d >> 32) & 1u;
  d = (uint64_t)a.hi - c.p1 - b1;
  const uint32_t d1 = (uint32_t)d;
  const bool g = ((d >> 32) & 1u) != 0, pr = (d0 | d1) == 0;
  const uint32_t bin = quad_carry_in(g, pr);
  // the digit minus the incoming borrow, and the borrow out of the whole quad (lane 3's)
  d = (uint64_t)d0 - bin;
  const uint32_t e0 = (uint32_t)d;
  d = (uint64_t)d1 - ((uint32_t)(d >> 32) & 1u);
  const uint32_t e1 = (uint32_t)d;
  const uint32_t bout = (g || (pr && bin)) ? 1u : 0u;
  const bool lt = qbcast<3>(bout) != 0;  // a < p: keep a
  return lt ? a : fq{e0, e1};
}

// a + b (no reduction; callers keep the sum < 2^256)
__device__ __forceinline__ fq fq_add_raw(const fq& a, const fq& b) {
  uint64_t s = (uint64_t)a.lo + b.lo;
  const uint32_t s0 = (uint32_t)s;
  s = (uint64_t)a.hi + b.hi + (uint32_t)(s >> 32);
  const uint32_t s1 = (uint32_t)s;
  const bool g = (s >> 32) != 0, pr = (s0 & s1) == 0xffffffffu;
  const uint32_t c = quad_carry_in(g, pr);
  s = (uint64_t)s0 + c;
  return fq{(uint32_t)s, s1 + (uint32_t)(s >> 32)};
}

}  // namespace pzk
