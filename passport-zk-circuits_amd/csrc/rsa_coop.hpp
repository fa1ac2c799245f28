// Cooperative RSA core: G lanes per witness, Barrett reduction.
//
// PowerMod(64,K,65537) (bigInt.circom:280-340) is 17 dependent BigMultModP per witness
// (bigInt.circom:206-272). One lane per witness leaves the chip nearly idle (2048 witnesses = 32
// waves) while the emitters wait for it, so here the G lanes of a witness share each multiplication:
//
//   * the product x*y, the Barrett estimate q3 = floor(floor(u / b^(k-1)) * mu / b^(k+1)) and the
//     convolution q*n are column sums split over the G lanes (column i -> lane i mod G);
//   * the serial glue (carry propagation, at most two Barrett corrections, the BigIntIsZero
//     carry chain) runs on the witness's first lane;
//   * mu = floor(b^(2k) / n) is computed once per witness (Knuth D), k = significant limbs of n.
//
// Barrett needs u = x*y < b^(2k); that holds for every multiplication of a passing witness
// (operands are remainders, and the signature is < n). Any other input (signature >= n, a 1-limb
// modulus) takes the exact serial Knuth D on the first lane instead, so quotient, remainder and
// carries are the ones long_div (bigIntFunc.circom:190-232) defines for EVERY input, as before.
// Output: the per-witness RSA core layout (MM_CORE_WORDS: x, y, q, r, IsEqual inverse slots
// (filled by k_rsa_inv), carries).
#pragma once
#include "core_util.hpp"
#include "fr.hpp"
#include "layout.hpp"

namespace pzk {

template <int K>
__host__ __device__ constexpr int rsa2_lds_words() { return 19 * K + 25; }

// Knuth D, serial (one lane): q = floor(a / b) (na - nb + 1 words), r = a mod b (nb words);
// a: na words, b: nb >= 2 words with b[nb-1] != 0. un: na + 1 words of scratch, vn: nb words.
__device__ inline void kd_div(const uint64_t* a, int na, const uint64_t* b, int nb, uint64_t* q, uint64_t* r,
                              uint64_t* un, uint64_t* vn) {
  const int s = __builtin_clzll(b[nb - 1]);
  for (int i = nb - 1; i > 0; i--) vn[i] = (b[i] << s) | (s ? b[i - 1] >> (64 - s) : 0ull);
  vn[0] = b[0] << s;
  un[na] = s ? a[na - 1] >> (64 - s) : 0ull;
  for (int i = na - 1; i > 0; i--) un[i] = (a[i] << s) | (s ? a[i - 1] >> (64 - s) : 0ull);
  un[0] = a[0] << s;
  const uint64_t vtop = vn[nb - 1], vsec = vn[nb - 2];
  for (int j = na - nb; j >= 0; j--) {
    uint64_t qhat, rhat;
    bool ovf = false;
    if (un[j + nb] >= vtop) {
      qhat = ~0ull;
      rhat = un[j + nb - 1] + vtop;
      ovf = rhat < vtop;
    } else {
      qhat = divlu(un[j + nb], un[j + nb - 1], vtop, &rhat);
    }
    while (!ovf) {
      uint64_t ph = __umul64hi(qhat, vsec), pl = qhat * vsec;
      if (ph > rhat || (ph == rhat && pl > un[j + nb - 2])) {
        qhat--;
        uint64_t r2 = rhat + vtop;
        ovf = r2 < rhat;
        rhat = r2;
      } else {
        break;
      }
    }
    uint64_t carry = 0, borrow = 0;
    for (int i = 0; i < nb; i++) {
      uint64_t pl = qhat * vn[i], ph = __umul64hi(qhat, vn[i]);
      pl += carry; ph += pl < carry; carry = ph;
      uint64_t t = un[i + j], d = t - pl, b1 = t < pl, d2 = d - borrow;
      b1 += d < borrow;
      un[i + j] = d2; borrow = b1;
    }
    uint64_t t = un[j + nb], d = t - carry, b1 = t < carry, d2 = d - borrow;
    b1 += d < borrow;
    un[j + nb] = d2;
    if (b1) {  // add back
      qhat--;
      uint64_t c = 0;
      for (int i = 0; i < nb; i++) {
        uint64_t s1 = un[i + j] + vn[i], c1 = s1 < vn[i], s2 = s1 + c;
        c1 += s2 < s1;
        un[i + j] = s2; c = c1;
      }
      un[j + nb] += c;
    }
    q[j] = qhat;
  }
  if (r)
    for (int i = 0; i < nb; i++) r[i] = s ? (un[i] >> s) | (un[i + 1] << (64 - s)) : un[i];
}

// column sums of a*b (a: na words, b: nb words) for columns i = g, g+G, ... < ncol; 3 words each
template <int G>
__device__ __forceinline__ void col_sums(const uint64_t* a, int na, const uint64_t* b, int nb, uint64_t* cs, int ncol,
                                         int g) {
  for (int i = g; i < ncol; i += G) {
    U192 acc;
    const int lo = i - (nb - 1) > 0 ? i - (nb - 1) : 0, hi = i < na - 1 ? i : na - 1;
    for (int j = lo; j <= hi; j++) acc.mac(a[j], b[i - j]);
    cs[3 * i] = acc.a0; cs[3 * i + 1] = acc.a1; cs[3 * i + 2] = acc.a2;
  }
}

// carry-propagating walk over 3-word column sums: word i of the sum, i = 0, 1, ...
struct ColWalk {
  const uint64_t* cs;
  int ncol;
  uint64_t c0 = 0, c1 = 0;
  __device__ __forceinline__ uint64_t next(int i) {
    if (i >= ncol) { uint64_t t = c0; c0 = c1; c1 = 0; return t; }
    uint64_t t0 = cs[3 * i] + c0, cc = t0 < c0;
    uint64_t t1 = cs[3 * i + 1] + c1, cc1 = t1 < c1, t1b = t1 + cc;
    cc1 += t1b < t1;
    c0 = t1b; c1 = cs[3 * i + 2] + cc1;
    return t0;
  }
};

// The G lanes of a witness cooperate; every lane of the block reaches every barrier.
template <int K, int G>
__global__ void __launch_bounds__(64) k_rsa_core2(DevLayout L, const uint8_t* inputs, uint64_t* rsa_core,
                                                  int32_t* status, uint32_t batch) {
  core_priority();
  constexpr int WPB = 64 / G, LW = rsa2_lds_words<K>(), MMW = MM_CORE_WORDS(K);
  extern __shared__ uint64_t lds2[];
  const int g = threadIdx.x % G, wl = threadIdx.x / G;
  const uint32_t w = blockIdx.x * WPB + wl;
  const bool live = w < batch;
  uint64_t* n = lds2 + wl * LW;   // K
  uint64_t* mu = n + K;           // K + 2
  uint64_t* x = mu + K + 2;       // K
  uint64_t* y = x + K;            // K
  uint64_t* u = y + K;            // 2K + 2: product, then remainder
  uint64_t* cs = u + 2 * K + 2;   // 3 x 2K: x*y column sums
  uint64_t* c2 = cs + 6 * K;      // 3 x (2K + 4): q1*mu / q*n column sums; Knuth D scratch
  uint64_t* q = c2 + 6 * K + 12;  // K + 3
  uint64_t* flag = q + K + 3;     // [0]: Barrett path for this multiplication
  const uint8_t* row = inputs + 32ull * (uint64_t)(live ? w : 0) * L.n_inputs;
  uint64_t* core = rsa_core + (size_t)(live ? w : 0) * L.rsa_core_words;
  bool bad = false, badz = false;
  for (int i = g; i < K; i += G) {
    const uint8_t* e = row + 32ull * (L.reg.in_pk + i);
    bad |= !in_is_u64(e);
    n[i] = in_u64(e);
  }
  __syncthreads();
  int nb = K;
  while (nb > 1 && n[nb - 1] == 0) nb--;
  const bool nzero = n[nb - 1] == 0;
  if (g == 0 && nb >= 2) {  // mu = floor(b^(2 nb) / n): nb + 2 words
    for (int i = 0; i < 2 * nb; i++) c2[i] = 0;
    c2[2 * nb] = 1;
    for (int i = 0; i < K + 2; i++) mu[i] = 0;
    kd_div(c2, 2 * nb + 1, n, nb, mu, nullptr, c2 + 2 * nb + 2, c2 + 4 * nb + 4);
  }
  __syncthreads();
  const int NM = L.reg.n_modmul;
  for (int k = 0; k < NM; k++) {
    uint64_t* mc = core + (size_t)k * MMW;
    // operands from the PowerMod schedule (e.g. 65537: muls[k] = muls[k-1].mod^2, muls[0] = base^2, then
    // resultMuls[0] = base * muls[15].mod; bigInt.circom:299-327)
    for (int i = g; i < K; i += G) {
      uint64_t xi;
      const int sx = L.reg.mm_x[k], sy = L.reg.mm_y[k];
      if (sx < 0) {
        const uint8_t* e = row + 32ull * (L.reg.in_sig + i);
        bad |= !in_is_u64(e);
        xi = in_u64(e);
      } else {
        xi = core[(size_t)sx * MMW + 3 * K + 1 + i];
      }
      const uint64_t yi = sy == sx ? xi : core[(size_t)sy * MMW + 3 * K + 1 + i];  // squaring, or a muls remainder
      x[i] = xi; y[i] = yi;
      if (live) { mc[i] = xi; mc[K + i] = yi; }
    }
    __syncthreads();
    col_sums<G>(x, K, y, K, cs, 2 * K - 1, g);  // raw column sums, kept for the carries
    __syncthreads();
    if (g == 0) {
      ColWalk cw{cs, 2 * K - 1};
      bool fast = nb >= 2;
      for (int i = 0; i < 2 * K + 1; i++) {
        u[i] = cw.next(i);
        if (i >= 2 * nb) fast &= u[i] == 0;  // Barrett domain: u < b^(2 nb)
      }
      flag[0] = fast;
    }
    __syncthreads();
    const bool fast = flag[0] != 0;
    // Barrett estimate: q1 = u[nb-1 .. 2nb] (nb + 2 words), q3 = (q1 * mu) >> 64 (nb + 1)
    const int nq = nb + 2, nc = 2 * nq - 1;
    if (fast) col_sums<G>(u + (nb - 1), nq, mu, nq, c2, nc, g);
    __syncthreads();
    if (g == 0) {
      for (int i = 0; i < K + 3; i++) q[i] = 0;
      if (fast) {
        ColWalk cw{c2, nc};
        for (int i = 0; i <= nc; i++) {
          const uint64_t t = cw.next(i);
          if (i >= nb + 1) q[i - (nb + 1)] = t;
        }
      } else if (!nzero) {
        // exact quotient/remainder of the 2K-word product; quotient words above K are dropped,
        // as long_div's K+1-word output does (the carry check then fails, as it must)
        uint64_t* qb = c2;              // 2K words
        uint64_t* un = c2 + 2 * K;      // 2K + 1
        uint64_t* vn = c2 + 4 * K + 1;  // nb
        uint64_t* rr = c2 + 5 * K + 1;  // nb
        if (nb >= 2) {
          kd_div(u, 2 * K, n, nb, qb, rr, un, vn);
        } else {
          uint64_t rem = 0;
          for (int i = 2 * K - 1; i >= 0; i--) qb[i] = divlu(rem, u[i], n[0], &rem);
          rr[0] = rem;
        }
        const int nqb = 2 * K - nb + 1;
        for (int i = 0; i < K + 1 && i < nqb; i++) q[i] = qb[i];
        for (int i = 0; i < 2 * K + 1; i++) u[i] = i < nb ? rr[i] : 0ull;
      }
    }
    __syncthreads();
    // q * n, all columns (q: K + 1 words, n: nb words)
    col_sums<G>(q, K + 1, n, nb, c2, K + nb, g);
    __syncthreads();
    if (g == 0) {
      if (fast) {
        // r = u - q3 n >= 0 (q3 <= q), then at most two corrections (Barrett, u < b^(2 nb))
        ColWalk cw{c2, K + nb};
        uint64_t br = 0;
        for (int i = 0; i < 2 * K + 1; i++) {
          const uint64_t pw = cw.next(i), a = u[i], d = a - pw;
          uint64_t b1 = a < pw;
          const uint64_t d2 = d - br;
          b1 += d < br;
          u[i] = d2; br = b1;
        }
        int corr = 0;
        for (; corr < 3; corr++) {  // while r >= n
          int i = 2 * K;
          for (; i >= nb; i--) if (u[i]) break;
          bool ge = true;
          if (i < nb)
            for (i = nb - 1; i >= 0; i--)
              if (u[i] != n[i]) { ge = u[i] > n[i]; break; }
          if (!ge) break;
          uint64_t b = 0;
          for (int j = 0; j < 2 * K + 1; j++) {
            const uint64_t nj = j < nb ? n[j] : 0ull, a = u[j], d = a - nj;
            uint64_t b1 = a < nj;
            const uint64_t d2 = d - b;
            b1 += d < b;
            u[j] = d2; b = b1;
          }
          for (int j = 0; j < K + 3; j++) if (++q[j]) break;
        }
        bad |= corr >= 3 || br != 0;  // outside Barrett's bounds: cannot happen for u < b^(2 nb)
        if (corr)  // columns of the corrected quotient's product: + corr * n_i
          for (int i = 0; i < nb; i++) {
            const uint64_t lo = (uint64_t)corr * n[i], hi = __umul64hi((uint64_t)corr, n[i]);
            const uint64_t s0 = c2[3 * i] + lo, cy = s0 < lo, s1 = c2[3 * i + 1] + hi;
            uint64_t cy1 = s1 < hi;
            const uint64_t s1b = s1 + cy;
            cy1 += s1b < s1;
            c2[3 * i] = s0; c2[3 * i + 1] = s1b; c2[3 * i + 2] += cy1;
          }
      }
      if (live) {
        uint64_t* qo = mc + 2 * K;      // q[K+1]
        uint64_t* ro = mc + 3 * K + 1;  // r[K]
        for (int i = 0; i <= K; i++) qo[i] = q[i];
        for (int i = 0; i < K; i++) ro[i] = i < nb ? u[i] : 0ull;
      }
      // BigIntIsZero carries (bigIntComparators.circom:105-129): c_i = (d_i + c_{i-1}) / 2^64 exactly,
      // d_i = conv(x,y)_i - conv(q,n)_i - r_i (signed, 256-bit two's complement)
      uint64_t* cr = mc + 8 * K + 1;  // (2K-2) x (lo, hi)
      uint64_t clo = 0, chi = 0;
      for (int i = 0; i < 2 * K - 1; i++) {
        const uint64_t a0 = cs[3 * i], a1 = cs[3 * i + 1], a2 = cs[3 * i + 2];
        uint64_t b0 = 0, b1 = 0, b2 = 0;
        if (i < K + nb) { b0 = c2[3 * i]; b1 = c2[3 * i + 1]; b2 = c2[3 * i + 2]; }
        uint64_t s0, s1, s2, s3, brr;
        s0 = a0 - b0; brr = a0 < b0;
        uint64_t t1 = a1 - b1, br1 = a1 < b1; s1 = t1 - brr; br1 += t1 < brr; brr = br1;
        uint64_t t2 = a2 - b2, br2 = a2 < b2; s2 = t2 - brr; br2 += t2 < brr; brr = br2;
        s3 = 0 - brr;
        const uint64_t rr = i < nb ? u[i] : 0ull;
        uint64_t v0 = s0 - rr, bb = s0 < rr; s0 = v0;
        uint64_t v1 = s1 - bb; bb = s1 < bb; s1 = v1;
        uint64_t v2 = s2 - bb; bb = s2 < bb; s2 = v2; s3 -= bb;
        const uint64_t csx = (int64_t)chi < 0 ? ~0ull : 0ull;  // sign extension of the carry
        const uint64_t w0 = s0 + clo;
        const uint64_t cc = w0 < s0, w1 = s1 + chi;
        uint64_t cc1 = w1 < s1;
        const uint64_t w1b = w1 + cc;
        cc1 += w1b < w1;
        const uint64_t w2 = s2 + csx;
        uint64_t cc2 = w2 < s2;
        const uint64_t w2b = w2 + cc1;
        cc2 += w2b < w2;
        const uint64_t w3 = s3 + csx + cc2;
        if (i < 2 * K - 2) {
          badz |= w0 != 0;  // exact division by 2^64
          clo = w1b; chi = w2b;
          badz |= !((w3 == 0 && (int64_t)w2b >= 0) || (w3 == ~0ull && (int64_t)w2b < 0));
          if (live) { cr[2 * i] = clo; cr[2 * i + 1] = chi; }
        } else {
          badz |= (w0 | w1b | w2b | w3) != 0;  // in[last] + carry[last-1] === 0
        }
      }
    }
    __syncthreads();
  }
  if (live && status) {
    if (bad || nzero) lane_status(status + w, ST_INPUT_RANGE);
    if (badz) lane_status(status + w, ST_BIGISZERO);
  }
}

}  // namespace pzk
