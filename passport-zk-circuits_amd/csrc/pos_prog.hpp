// Poseidon block program. A PoseidonHash(n) block (poseidon.circom:214-226 + PoseidonEx
// :80-209) of width t = n + 1 is emitted from a per-(permutation, witness) IMAGE of normal-form
// field elements rebuilt in LDS: the S-box layer inputs and powers (Sigma, :10-21), the Ark
// outputs (:23-33), the Mix / MixLast / MixS GetSumOfNElements rows as PREFIX SUMS
// (:35-78) and, beside them, each row's products 1..t-1 (product 0 is the first prefix sum), the
// partial-round states, the hash inputs/output and a zero. Every signal of the block is then a
// COPY of one image element, one u16 descriptor per signal, built once per width on the host
// (pos_program(), builder.cpp) in the template's signal order.
#pragma once
#include <stdint.h>

namespace pzk {

__host__ __device__ constexpr int pos_rp(int t) { return t == 2 ? 56 : t == 3 ? 57 : t == 4 ? 56 : 60; }

// Order: the S-box parts, partial-round states, hash inputs / output first, the GetSum rows and products (the part
// only a block with its Mix signals kept reads: every O0 block, none of the O2-shaped map's) last, from fs on — so a
// mapped block that keeps no GetSum signal needs an LDS image of fs elements only (t = 6: 27 KB instead of 63 KB).
struct PosImg {  // element offsets inside the image of width t
  int t, rp;
  int in, p2, p4, p5, ark, pin, pp2, pp4, pp5, pin0, inp, hash, zero, fs, ls, ps, pr, size;
  __host__ __device__ constexpr PosImg(int t_)
      : t(t_), rp(pos_rp(t_)),
        in(0), p2(8 * t_), p4(16 * t_), p5(24 * t_), ark(32 * t_),
        pin(39 * t_),                      // partial-round states Y_0..Y_RP
        pp2(pin + (rp + 1) * t_), pp4(pp2 + rp), pp5(pp4 + rp), pin0(pp5 + rp),
        inp(pin0 + rp), hash(inp + 5), zero(hash + 1),
        fs(zero + 1),                      // full mix rows (f < 7, i < t): t prefix sums each
        ls(fs + 7 * t_ * t_),              // mixLast row
        ps(ls + t_),                       // partial mix rows (r < RP): t prefix sums each
        pr(ps + rp * t_),                  // products 1..t-1 of GetSum row r (7t full, mixLast, RP partial)
        size(pr + (7 * t_ + 1 + rp) * (t_ - 1)) {}
  // image index of product j >= 1 of GetSum row `row` (rows numbered as in pos_img_fill's phase B)
  __host__ __device__ constexpr int prod(int row, int j) const { return pr + row * (t - 1) + j - 1; }
};

enum : uint32_t {
  PI_X = 1,     // S-box inputs x (full rounds; partial rounds' state 0)
  PI_ST = 2,    // the other partial-round states and Y_RP
  PI_MIX = 4,   // the GetSum rows: products, prefix sums (full mix, mixLast, partial mix)
  PI_MISC = 8,  // hash inputs / output, the zero
  PI_ALL = 15
};
__host__ __device__ inline uint32_t pos_img_need_t(int t, uint32_t d) {  // the image part descriptor d reads
  const PosImg I(t);
  if ((int)d < I.p2) return PI_X;    // S-box inputs of the full layers
  if ((int)d < I.pin) return 0;      // S-box powers, Ark outputs (always filled)
  if ((int)d < I.pp2) {              // partial-round states: state 0 is the S-box input
    const int k = (int)d - I.pin, r = k / t;
    return (r < I.rp && k - r * t == 0) ? PI_X : PI_ST;
  }
  if ((int)d < I.inp) return 0;      // partial S-box powers and Ark outputs
  if ((int)d < I.fs) return PI_MISC; // hash inputs / output, the zero
  return PI_MIX;                     // GetSum rows and products
}

__host__ __device__ constexpr uint16_t pos_desc(int idx) { return (uint16_t)idx; }

}  // namespace pzk
