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

struct PosImg {  // element offsets inside the image of width t
  int t, rp;
  int in, p2, p4, p5, ark, fs, ls, pin, pp2, pp4, pp5, pin0, ps, inp, hash, zero, pr, size;
  __host__ __device__ constexpr PosImg(int t_)
      : t(t_), rp(pos_rp(t_)),
        in(0), p2(8 * t_), p4(16 * t_), p5(24 * t_), ark(32 * t_),
        fs(39 * t_),                       // full mix rows (f < 7, i < t): t prefix sums each
        ls(39 * t_ + 7 * t_ * t_),         // mixLast row
        pin(ls + t_),                      // partial-round states Y_0..Y_RP
        pp2(pin + (rp + 1) * t_), pp4(pp2 + rp), pp5(pp4 + rp), pin0(pp5 + rp),
        ps(pin0 + rp),                     // partial mix rows (r < RP): t prefix sums each
        inp(ps + rp * t_), hash(inp + 5), zero(hash + 1),
        pr(zero + 1),                      // products 1..t-1 of GetSum row r (7t full, mixLast, RP partial)
        size(pr + (7 * t_ + 1 + rp) * (t_ - 1)) {}
  // image index of product j >= 1 of GetSum row `row` (rows numbered as in pos_img_fill's phase B)
  __host__ __device__ constexpr int prod(int row, int j) const { return pr + row * (t - 1) + j - 1; }
};

__host__ __device__ constexpr uint16_t pos_desc(int idx) { return (uint16_t)idx; }

}  // namespace pzk
