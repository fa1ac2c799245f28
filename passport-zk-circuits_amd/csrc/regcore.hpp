// Core (sequential, per-witness) kernels of the RegisterIdentityBuilder path.
//
// Each computes the compact per-witness state from which the emit kernels regenerate
// every signal in closed form:
//   * k_prep      — Poseidon inputs that are linear/bit functions of the inputs and digests
//   * k_rsa_core  — PowerMod(64,K,65537) (bigInt.circom:280-340): per BigMultModP the operands,
//                   the exact quotient/remainder (any exact long division yields the unique
//                   result that long_div, bigIntFunc.circom:190-232, must produce for a passing
//                   witness), the K IsEqual inverses (one batched Fermat inversion per modmul) and
//                   the 2K-2 signed BigIntIsZero carries. Per-lane 64-bit limb arrays live in LDS.
//   * k_bjj_core  — BabyjubjubBase8Multiplication (babyjubjub/curve.circom:143-171) as an
//                   extended-coordinate ladder (no inversion on the critical path) followed by
//                   ONE batched inversion that yields every affine point and IsZero inverse.
//   * k_smt_prep / k_smt_chain — SMTVerifier(80) (SMTVerifier.circom:109-176): level hashes
//                   whose child is 0 (every level at or above the insertion level) are
//                   independent Poseidon tasks; only the levels below run sequentially.
#pragma once
#include "fr.hpp"
#include "layout.hpp"
#include "poseidon.hpp"
#include "sha.hpp"
#include "core_util.hpp"
#include "pss.hpp"

namespace pzk {

// ============================================================================ k_prep
// wave = witness. Runs after k_sha_core (needs the SA digest). The Bits2Num chunks (AA key,
// dg1) are assembled 64 bits per ballot: lane l reads input element base +- (64 q + l), so each
// load instruction of the wave covers 2 KiB of one input row (one lane per witness read a
// 32-byte element per bit from 64 rows 185 KB apart: 2.5 ms per 2048 witnesses on the chain).
__device__ __forceinline__ fr wave_bits_fr(const uint8_t* row, int base, int L, int dir, bool& bad) {
  const int lane = threadIdx.x & 63;
  fr v = fr_zero();
  for (int q = 0; 64 * q < L; q++) {  // wave-uniform
    const int k = 64 * q + lane;
    uint32_t b = 0;
    if (k < L) b = in_bit(row, dir > 0 ? base + k : base + L - 1 - k, bad);
    const uint64_t m = __ballot(b);
    v.v[2 * q] = (uint32_t)m;
    v.v[2 * q + 1] = (uint32_t)(m >> 32);
  }
  return v;
}

#ifndef PZK_TEMPLATE_KERNELS_ONLY  // defined once, in kernels.hip
__global__ void __launch_bounds__(64) k_prep(DevLayout L, const uint8_t* inputs, const uint32_t* sha_core, ValueStore vs, int32_t* status) {
  core_priority();
  const uint32_t w = blockIdx.x;
  if (w >= vs.batch) return;  // whole wave
  const int lane = threadIdx.x;
  const RegInfo& R = L.reg;
  const uint8_t* row = inputs + 32ull * (uint64_t)w * L.n_inputs;
  bool bad = false;
  if (lane == 0) vs.at(R.v_one, w) = fr_mont_one();
  // pubkeyHasherRsa inputs: tempModulus[i] + pk[3i+2] = pk[3i]*2^128 + pk[3i+1]*2^64 + pk[3i+2]
  // (passportVerificationBuilder.circom:182-191), in field arithmetic; lane i computes input i
  if (R.ecdsa) {
    // ECDSA: pubkeyHasher = Poseidon2(x mod 2^FD, y mod 2^FD), FD = min(N CS, 248) (passportVerificationBuilder.circom:193-230)
    if (lane < 2) {
      const int a = lane, N = R.ec_nl, CS = R.ec_cs, FD = N * CS > 248 ? 248 : N * CS;
      fr v = fr_zero();
      for (int j = 0; j < N; j++) {
        const uint8_t* e = row + 32ull * (R.in_pk + N * a + j);
        bad |= !in_is_u64(e) || (CS < 64 && (in_u64(e) >> CS) != 0);
        const uint64_t x = in_u64(e);
        for (int k = 0; k < CS && CS * j + k < FD; k += 32) {  // 32-bit pieces of the chunk below bit FD
          const int bit = CS * j + k;
          uint32_t piece = (uint32_t)(x >> k);
          if (bit + 32 > FD) piece &= (1u << (FD - bit)) - 1u;
          v.v[bit >> 5] = piece;
        }
      }
      vs.at(a ? R.v_pky : R.v_pkx, w) = fr_to_mont(v);
    }
  } else if (lane < 5) {
    const int i = lane;
    fr two64 = fr_zero(); two64.v[2] = 1;
    fr two128 = fr_zero(); two128.v[4] = 1;
    two64 = fr_to_mont(two64); two128 = fr_to_mont(two128);
    fr a = fr_to_mont(load_fr(row + 32ull * (R.in_pk + 3 * i)));
    fr b = fr_to_mont(load_fr(row + 32ull * (R.in_pk + 3 * i + 1)));
    fr c = fr_to_mont(load_fr(row + 32ull * (R.in_pk + 3 * i + 2)));
    vs.at(R.v_pk + i, w) = fr_add(fr_add(fr_mul(a, two128), fr_mul(b, two64)), c);
  }
  if (R.aa && R.aa_ec) {  // EC key: x, y low HASH_SIZE bits (identity.circom:70-81)
    const int xy = R.aa_f - R.aa_hs;
    for (int a = 0; a < 2; a++) {
      fr v = wave_bits_fr(row, R.in_dg15 + R.aa_shift + a * R.aa_f + xy, R.aa_hs, -1, bad);
      if (lane == 0) vs.at(R.v_aa + a, w) = fr_to_mont(v);
    }
  } else if (R.aa) {
    // AA key chunks: Bits2Num(200) x4 + Bits2Num(224), in[L-1-i] = dg15[AA_SHIFT + 200 j + i] (identity.circom:31-45)
    for (int j = 0; j < 5; j++) {
      fr v = wave_bits_fr(row, R.in_dg15 + R.aa_shift + j * 200, j < 4 ? 200 : 224, -1, bad);
      if (lane == 0) vs.at(R.v_aa + j, w) = fr_to_mont(v);
    }
  }
  // dg1 chunks: Bits2Num(186|190), in[j] = dg1[i*chunk + j] (identity.circom:95-101)
  for (int i = 0; i < 4; i++) {
    fr v = wave_bits_fr(row, R.in_dg1 + i * R.dg1_chunk, R.dg1_chunk, +1, bad);
    if (lane == 0) vs.at(R.v_dg1 + i, w) = fr_to_mont(v);
  }
  // signedAttributesNum = Bits2Num(252)(saHash[0..251]) (passportVerificationBuilder.circom:165-172)
  if (lane == 0) {
    const ShaJob job = L.sha[R.j_sa];
    const uint32_t* H = sha_core + (size_t)w * L.sha_core_words + job.hout;
    // the hash's first 252 bits, or an HT < 252-bit hash shifted up by 252 - HT: 92 for SHA-1, 28 for SHA-224
    // (passportVerificationBuilder.circom:164-177)
    const int sh = job.algo == 1 ? 92 : job.algo == 2 ? 28 : 0;
    fr sn = bits_to_fr(252, [&](int k) { return k < sh ? 0u : (H[(k - sh) >> 5] >> (31 - ((k - sh) & 31))) & 1u; });
    vs.at(R.v_sanum, w) = fr_to_mont(sn);
  }
  if (__ballot(bad) && lane == 0) set_status(status ? status + w : nullptr, ST_INPUT_RANGE);
}
#endif

// ============================================================================ RSA core

// 192-bit unsigned accumulator
struct U192 {
  uint64_t a0 = 0, a1 = 0, a2 = 0;
  __device__ __forceinline__ void mac(uint64_t x, uint64_t y) {
    uint64_t lo = x * y, hi = __umul64hi(x, y);
    uint64_t s = a0 + lo; uint64_t c = s < lo; a0 = s;
    uint64_t t = a1 + hi; uint64_t c2 = t < hi; uint64_t t2 = t + c; c2 += t2 < t; a1 = t2;
    a2 += c2;
  }
};

// per-lane LDS arrays, [index][lane] so a wave's accesses hit consecutive banks
template <int NL>
struct LaneArr {
  uint64_t* base;
  int lane;
  __device__ __forceinline__ uint64_t& operator[](int i) const { return base[i * NL + lane]; }
};

template <int K>
__host__ __device__ constexpr int rsa_lds_words() { return 7 * K + 2; }

// 128/64 -> 64 division by a normalised v with a precomputed reciprocal
// vinv = floor((2^128 - 1) / v) - 2^64 (Moller & Granlund, "Improved division by invariant
// integers", Alg. 4); requires u1 < v. Two multiplications instead of a software divide.
__device__ __forceinline__ uint64_t div_preinv(uint64_t u1, uint64_t u0, uint64_t v, uint64_t vinv, uint64_t* rem) {
  uint64_t q0 = vinv * u1, q1 = __umul64hi(vinv, u1);
  uint64_t s0 = q0 + u0;
  q1 += u1 + 1 + (s0 < q0);
  q0 = s0;
  uint64_t r = u0 - q1 * v;
  if (r > q0) { q1--; r += v; }
  if (r >= v) { q1++; r -= v; }
  *rem = r;
  return q1;
}

// RSA core for one witness lane: the 17 BigMultModP of PowerMod(65537) (bigInt.circom:206-272,
// 280-340) — operands, quotient and remainder of the exact product (Knuth D with a
// precomputed reciprocal of the divisor's top word), and the BigIntIsZero carries. The IsEqual
// inverses are left to k_rsa_inv (one batched inversion per witness over all 17 x K of them).
// LDS: per-lane arrays [index][lane]; colsum: the x*y column sums, SoA [(3 i + c)][witness].
template <int K, int NL>
__device__ void rsa_lane(const DevLayout& L, const uint8_t* row, uint64_t* core, uint64_t* colsum, uint32_t cs_stride,
                         int32_t* status, uint64_t* lds, int lane) {
  LaneArr<NL> n{lds, lane}, x{lds + K * NL, lane}, y{lds + 2 * K * NL, lane}, u{lds + 3 * K * NL, lane},
      q{lds + (5 * K + 1) * NL, lane}, vn{lds + (6 * K + 2) * NL, lane};
  auto CS = [&](int i, int c) -> uint64_t& { return colsum[(size_t)(3 * i + c) * cs_stride]; };
  bool bad = false, badz = false;
  for (int i = 0; i < K; i++) {
    const uint8_t* e = row + 32ull * (L.reg.in_pk + i);
    bad |= !in_is_u64(e);
    n[i] = in_u64(e);
  }
  int nb = K;
  while (nb > 1 && n[nb - 1] == 0) nb--;
  const int s = __builtin_clzll(n[nb - 1] | 1ull);
  for (int i = nb - 1; i > 0; i--) vn[i] = (n[i] << s) | (s ? n[i - 1] >> (64 - s) : 0ull);
  vn[0] = n[0] << s;
  const uint64_t vtop = vn[nb - 1], vsec = nb > 1 ? vn[nb - 2] : 0ull;
  uint64_t vinv_r;
  const uint64_t vinv = vtop ? divlu(~vtop, ~0ull, vtop, &vinv_r) : 0ull;  // a zero modulus is flagged below
  constexpr int MMW = MM_CORE_WORDS(K);
  const int NM = L.reg.n_modmul;
  for (int k = 0; k < NM; k++) {
    uint64_t* mc = core + (size_t)k * MMW;
    // operands (exp_to_bits(65537) = [16,2,0,16]): muls[k] = muls[k-1].mod^2 with muls[0] = base^2;
    // resultMuls[0] = base * muls[15].mod (bigInt.circom:299-327)
    for (int i = 0; i < K; i++) {
      uint64_t xi;
      const int sx = L.reg.mm_x[k], sy = L.reg.mm_y[k];
      if (sx < 0) {
        const uint8_t* e = row + 32ull * (L.reg.in_sig + i);
        bad |= !in_is_u64(e);
        xi = in_u64(e);
      } else {
        xi = core[(size_t)sx * MMW + 3 * K + 1 + i];
      }
      uint64_t yi = sy == sx ? xi : core[(size_t)sy * MMW + 3 * K + 1 + i];
      x[i] = xi; y[i] = yi;
      mc[i] = xi; mc[K + i] = yi;
    }
    // exact product as 2K words; the raw column sums are kept for the carries
    {
      uint64_t c0 = 0, c1 = 0;
      for (int i = 0; i < 2 * K; i++) {
        U192 acc;
        int lo = i < K ? 0 : i - K + 1, hi = i < K ? i : K - 1;
        for (int j = lo; j <= hi; j++) acc.mac(x[j], y[i - j]);
        if (i < 2 * K - 1) { CS(i, 0) = acc.a0; CS(i, 1) = acc.a1; CS(i, 2) = acc.a2; }
        uint64_t t0 = acc.a0 + c0; uint64_t cc = t0 < c0;
        uint64_t t1 = acc.a1 + c1; uint64_t cc1 = t1 < c1; uint64_t t1b = t1 + cc; cc1 += t1b < t1;
        u[i] = t0; c0 = t1b; c1 = acc.a2 + cc1;
      }
    }
    // normalise into 2K+1 words
    u[2 * K] = s ? u[2 * K - 1] >> (64 - s) : 0ull;
    if (s) {
      for (int i = 2 * K - 1; i > 0; i--) u[i] = (u[i] << s) | (u[i - 1] >> (64 - s));
      u[0] = u[0] << s;
    }
    for (int j = 0; j <= K; j++) q[j] = 0;
    for (int j = 2 * K - nb; j >= 0 && vtop; j--) {
      uint64_t ujn = u[j + nb], ujn1 = u[j + nb - 1];
      uint64_t qhat, rhat;
      bool rhat_ovf = false;
      if (ujn >= vtop) {
        qhat = ~0ull;
        rhat = ujn1 + vtop;
        rhat_ovf = rhat < ujn1;
      } else {
        qhat = div_preinv(ujn, ujn1, vtop, vinv, &rhat);
      }
      if (nb > 1) {
        for (int it = 0; it < 2 && !rhat_ovf; it++) {
          uint64_t plo = qhat * vsec, phi = __umul64hi(qhat, vsec);
          uint64_t u2 = u[j + nb - 2];
          if (phi > rhat || (phi == rhat && plo > u2)) {
            qhat--;
            uint64_t r2 = rhat + vtop;
            rhat_ovf = r2 < rhat;
            rhat = r2;
          } else {
            break;
          }
        }
      }
      uint64_t borrow = 0, carry = 0;
      for (int i = 0; i < nb; i++) {
        uint64_t plo = qhat * vn[i], phi = __umul64hi(qhat, vn[i]);
        plo += carry; phi += plo < carry; carry = phi;
        uint64_t t = u[i + j];
        uint64_t d = t - plo; uint64_t b1 = t < plo;
        uint64_t d2 = d - borrow; uint64_t b2 = d < borrow;
        u[i + j] = d2; borrow = b1 + b2;
      }
      uint64_t t = u[j + nb];
      uint64_t d = t - carry; uint64_t b1 = t < carry;
      uint64_t d2 = d - borrow; uint64_t b2 = d < borrow;
      u[j + nb] = d2;
      if (b1 + b2) {  // add back
        qhat--;
        uint64_t cy = 0;
        for (int i = 0; i < nb; i++) {
          uint64_t a = u[i + j], vb = vn[i];
          uint64_t sm = a + vb; uint64_t ca = sm < a; uint64_t sm2 = sm + cy; uint64_t cb = sm2 < sm;
          u[i + j] = sm2; cy = ca + cb;
        }
        u[j + nb] += cy;
      }
      q[j] = qhat;
    }
    uint64_t* qo = mc + 2 * K;      // q[K+1]
    uint64_t* ro = mc + 3 * K + 1;  // r[K]
    for (int i = 0; i <= K; i++) qo[i] = q[i];
    for (int i = 0; i < K; i++) {
      uint64_t r = 0;
      if (i < nb) r = s ? (u[i] >> s) | (u[i + 1] << (64 - s)) : u[i];
      ro[i] = r;
    }
    // BigIntIsZero carries (bigIntComparators.circom:105-129): c_i = (d_i + c_{i-1}) / 2^64 exactly,
    // d_i = conv(x,y)_i - conv(q,n)_i - r_i   (signed, 256-bit two's complement)
    uint64_t* cr = mc + 8 * K + 1;  // (2K-2) x (lo, hi)
    {
      uint64_t clo = 0, chi = 0;  // signed 128 carry
      for (int i = 0; i < 2 * K - 1; i++) {
        U192 a, b;
        a.a0 = CS(i, 0); a.a1 = CS(i, 1); a.a2 = CS(i, 2);
        int lo2 = i < K ? 0 : i - K + 1, hi2 = i < K + 1 ? i : K;
        for (int j = lo2; j <= hi2 && j <= K; j++) if (i - j < K) b.mac(q[j], n[i - j]);
        // s = a - b - r_i + c (256-bit)
        uint64_t s0, s1, s2, s3, br;
        s0 = a.a0 - b.a0; br = a.a0 < b.a0;
        uint64_t t1 = a.a1 - b.a1; uint64_t br1 = a.a1 < b.a1; s1 = t1 - br; br1 += t1 < br; br = br1;
        uint64_t t2 = a.a2 - b.a2; uint64_t br2 = a.a2 < b.a2; s2 = t2 - br; br2 += t2 < br; br = br2;
        s3 = 0 - br;
        uint64_t rr = i < K ? ro[i] : 0ull;
        uint64_t u0 = s0 - rr; uint64_t bb = s0 < rr; s0 = u0;
        uint64_t u1 = s1 - bb; bb = s1 < bb; s1 = u1;
        uint64_t u2 = s2 - bb; bb = s2 < bb; s2 = u2; s3 -= bb;
        uint64_t csx = (int64_t)chi < 0 ? ~0ull : 0ull;  // sign extension of the carry
        uint64_t v0 = s0 + clo; uint64_t cc = v0 < s0;
        uint64_t v1 = s1 + chi; uint64_t cc1 = v1 < s1; uint64_t v1b = v1 + cc; cc1 += v1b < v1;
        uint64_t v2 = s2 + csx; uint64_t cc2 = v2 < s2; uint64_t v2b = v2 + cc1; cc2 += v2b < v2;
        uint64_t v3 = s3 + csx + cc2;
        if (i < 2 * K - 2) {
          badz |= v0 != 0;  // exact division by 2^64
          clo = v1b; chi = v2b;
          badz |= !((v3 == 0 && (int64_t)v2b >= 0) || (v3 == ~0ull && (int64_t)v2b < 0));
          cr[2 * i] = clo; cr[2 * i + 1] = chi;
        } else {
          badz |= (v0 | v1b | v2b | v3) != 0;  // in[last] + carry[last-1] === 0
        }
      }
    }
  }
  if (bad || !vtop) set_status(status, ST_INPUT_RANGE);
  if (badz) set_status(status, ST_BIGISZERO);
}

template <int K, int NL>
__global__ void __launch_bounds__(NL) k_rsa_core(DevLayout L, const uint8_t* inputs, uint64_t* rsa_core, uint64_t* colsum,
                                                 int32_t* status, uint32_t batch) {
  core_priority();
  extern __shared__ uint64_t lds_rsa[];
  uint32_t w = blockIdx.x * NL + threadIdx.x;
  if (w >= batch) return;
  rsa_lane<K, NL>(L, inputs + 32ull * (uint64_t)w * L.n_inputs, rsa_core + (size_t)w * L.rsa_core_words, colsum + w,
                  batch, status ? status + w : nullptr, lds_rsa, threadIdx.x);
}

// IsEqual inverses of (r_i - n_i) for every limb of every BigMultModP (BigLessEqThan,
// bigIntComparators.circom:50-75; IsZero.inv = 1/in or 0, comparators.circom:17): one wave per
// witness, one batched inversion over the 17 x K differences. Lane l takes a contiguous run of
// elements; the run products are combined across the wave with shuffles, and the wave totals of the workgroup's
// RI_WAVES witnesses are inverted together by wave 0 (one Fr inversion per wave was ~85 % of the kernel's VALU).
// Output: normal form, in each BigMultModP's inv slots.
#ifndef PZK_RI_WAVES  // witnesses (waves) per k_rsa_inv workgroup (A/B builds)
#define PZK_RI_WAVES 8
#endif
constexpr int RI_WAVES = PZK_RI_WAVES;
// f(integral_constant<int, J>) for J = J0 .. N - 1, unrolled by construction (register arrays indexed by J stay in
// registers; a #pragma unroll of the same loop leaves them in scratch once the body is large)
template <int J, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (J < N) {
    f(std::integral_constant<int, J>{});
    static_for<J + 1, N>(f);
  }
}
template <int K>
__global__ void __launch_bounds__(64 * RI_WAVES) k_rsa_inv(DevLayout L, const uint8_t* inputs, uint64_t* rsa_core,
                                                           uint32_t batch) {
  core_priority();
  // the run's exclusive prefix products stay in registers ([element of the run]): parked in the core's inverse
  // slots they cost a write and a read of 32 B per IsEqual, and each read waited for the run's stores
  // (up to 20 multiplications: 65537, 3, 37187; a longer PowerMod schedule parks them in the slots as before)
  // (up to 12 per lane, RSA-2048 / 3072: 20 multiplications; RSA-4096 and a longer PowerMod schedule park them in the
  // slots)
  constexpr int PER_MAX = (20 * K + 63) / 64 < 12 ? (20 * K + 63) / 64 : 12;
  __shared__ fr s_tot[RI_WAVES];
  __shared__ fr s_out[RI_WAVES][64];  // element-order staging of the stores
  const int wv = (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63);
  const uint32_t w0 = blockIdx.x * RI_WAVES + (uint32_t)wv;
  const bool live = w0 < batch;  // a wave past the batch takes part in the barriers only, and stores nothing
  const uint32_t w = live ? w0 : batch - 1;
  // (the layout's fields as locals: a lambda below that reached the by-value kernel argument put a copy of it in scratch)
  const int NE = L.reg.n_modmul * K, PER = (NE + 63) / 64, in_pk = (int)L.reg.in_pk;
  constexpr int MMW = MM_CORE_WORDS(K);
  const uint8_t* row = inputs + 32ull * (uint64_t)w * L.n_inputs;
  uint64_t* core = rsa_core + (size_t)w * L.rsa_core_words;
  const int e0 = lane * PER, e1 = !live ? e0 : e0 + PER < NE ? e0 + PER : NE;
  auto diff = [=](int e) -> fr {  // (r_i - n_i) in Montgomery form
    const int k = e / K, i = e - k * K;
    const uint64_t a = core[(size_t)k * MMW + 3 * K + 1 + i], b = in_u64(row + 32ull * (in_pk + i));
    fr d = a >= b ? fr_u64(a - b) : fr_sub(fr_zero(), fr_u64(b - a));
    return fr_to_mont(d);
  };
  auto slot = [=](int e) -> uint8_t* {
    const int k = e / K, i = e - k * K;
    return reinterpret_cast<uint8_t*>(core + (size_t)k * MMW + 4 * K + 1 + 4 * i);
  };
  const bool in_reg = PER <= PER_MAX;  // grid-uniform
  fr pr[PER_MAX];
  fr acc = fr_mont_one();
  if (in_reg) {
    static_for<0, PER_MAX>([&](auto J) __attribute__((always_inline)) {
      const int e = e0 + J();
      if (e < e1) {
        const fr d = diff(e);
        pr[J()] = acc;  // exclusive prefix within the run
        if (!fr_is_zero(d)) acc = fr_mul_fast(acc, d);
      }
    });
  } else {
    for (int e = e0; e < e1; e++) {
      const fr d = diff(e);
      store_fr(slot(e), acc);
      if (!fr_is_zero(d)) acc = fr_mul_fast(acc, d);
    }
  }
  // exclusive prefix / suffix products of the run products across the wave (log-step scans)
  fr incl = acc, sincl = acc;
  for (int d = 1; d < 64; d <<= 1) {
    fr a = fr_shfl_up(incl, d), b = fr_shfl_down(sincl, d);
    if (lane >= d) incl = fr_mul_fast(incl, a);
    if (lane + d < 64) sincl = fr_mul_fast(sincl, b);
  }
  fr pre = fr_shfl_up(incl, 1), suf = fr_shfl_down(sincl, 1);
  if (lane == 0) pre = fr_mont_one();
  if (lane == 63) suf = fr_mont_one();
  // the workgroup's wave totals inverted together (lane k of wave 0: wave k's total; a dead wave's is 1)
  if (lane == 63) s_tot[wv] = incl;
  __syncthreads();
  if (wv == 0) {
    const fr t = lane < RI_WAVES ? s_tot[lane] : fr_mont_one();
    fr t_others, t_all;
    fr_group_others<RI_WAVES>(t, t_others, t_all);
    const fr t_inv = fr_mul_fast(fr_inv<true>(t_all), t_others);  // = 1 / total of wave `lane`
    if (lane < RI_WAVES) s_tot[lane] = t_inv;  // (read above, by this wave only)
  }
  __syncthreads();
  fr inv = fr_mul_fast(fr_mul_fast(s_tot[wv], pre), suf);  // = 1 / (this run's product)
  if (!in_reg) {
    if (!live) return;
    for (int e = e1 - 1; e >= e0; e--) {
      const fr d = diff(e);
      fr r = fr_zero();
      if (!fr_is_zero(d)) { r = fr_mul_fast(inv, load_fr(slot(e))); inv = fr_mul_fast(inv, d); }
      store_fr(slot(e), fr_from_mont(r));
    }
    return;
  }
  static_for<0, PER_MAX>([&](auto J) __attribute__((always_inline)) {
    constexpr int j = PER_MAX - 1 - J();
    const int e = e0 + j;
    if (e < e1) {
      const fr d = diff(e);
      fr r = fr_zero();
      if (!fr_is_zero(d)) { r = fr_mul_fast(inv, pr[j]); inv = fr_mul_fast(inv, d); }
      pr[j] = fr_from_mont(r);
    }
  });
  // written out in element order, 64 consecutive 32-byte inverse slots per store instruction: lane l's run is
  // elements [l PER, (l + 1) PER), so storing from the loop above put 64 partial lines of 64 different slots in
  // flight per iteration, and L2 wrote most lines twice (2.0x the inverse bytes, pmc_r4c3)
  for (int t = 0; t < (NE + 63) / 64; t++) {  // (the same step count in every wave: NE is the instance's)
    static_for<0, PER_MAX>([&](auto J) __attribute__((always_inline)) {
      const int e = e0 + J();
      if (e < e1 && (e >> 6) == t) s_out[wv][e & 63] = pr[J()];
    });
    __syncthreads();
    const int e = 64 * t + lane;
    if (live && e < NE) store_fr(slot(e), s_out[wv][lane]);
    __syncthreads();
  }
}

// ============================================================================ RSA EM checks
// RsaVerifyPkcs1v15 (rsa.circom:47-71) on EM = PowerMod.out (last BigMultModP remainder), and
// BigMultModP's BigGreaterThan(modulus, mod) (bigInt.circom:241-245) for every multiplication.
// One lane per witness; reads the RSA core, the SA digest (SHA core) and the pubkey input.
constexpr uint64_t RSA_EM4 = 217300885422736416ull, RSA_EM5 = 938447882527703397ull;  // rsa.circom:53-54
constexpr uint64_t RSA_EM6 = 0xFFFFFFFF00303130ull;  // num2bits_6: remainsBits (rsa.circom:59-62), ones (:65-67)

#ifndef PZK_TEMPLATE_KERNELS_ONLY  // defined once, in kernels.hip
__global__ void __launch_bounds__(64) k_rsa_check(DevLayout L, const uint8_t* inputs, const uint32_t* sha_core,
                                                  const uint64_t* rsa_core, int32_t* status, uint32_t batch) {
  const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= batch || !status) return;
  const int K = L.reg.K;
  const uint8_t* row = inputs + 32ull * (uint64_t)w * L.n_inputs;
  const uint64_t* core = rsa_core + (size_t)w * L.rsa_core_words;
  const uint64_t* em = core + (size_t)(L.reg.n_modmul - 1) * MM_CORE_WORDS(K) + 3 * K + 1;
  const ShaJob& J = L.sha[L.reg.j_sa];
  const uint32_t* H = sha_core + (size_t)w * L.sha_core_words + J.hout;
  bool hash_bad = false;
  for (int i = 0; i < 4; i++) {  // hashed_chunks[i] = digest bits [64(3-i), 64(4-i)) as a number
    const int wd = 3 - i;
    hash_bad |= (((uint64_t)H[2 * wd] << 32) | H[2 * wd + 1]) != em[i];
  }
  bool pad_bad = em[6] != RSA_EM6;
  for (int i = 7; i < K - 1; i++) pad_bad |= em[i] != ~0ull;
  bool gt_bad = false;
  for (int m = 0; m < L.reg.n_modmul; m++) {  // mod < modulus, limb-wise from the top
    const uint64_t* r = core + (size_t)m * MM_CORE_WORDS(K) + 3 * K + 1;
    int cmp = 0;
    for (int i = K - 1; i >= 0 && cmp == 0; i--) {
      uint64_t n = in_u64(row + 32ull * (L.reg.in_pk + i));
      cmp = n > r[i] ? 1 : n < r[i] ? -1 : 0;
    }
    gt_bad |= cmp != 1;
  }
  if (L.reg.pss_s8) {
    pss_check(pss_view(L, rsa_core, sha_core, w), status + w);
  } else if (J.algo == 1) {
    // RsaVerifyPkcs1v15(64,K,65537,160) (rsa.circom:73-109): EM limb 2 = 0x05000414 | first digest word,
    // limbs 3, 4 = DigestInfo, then 0xFF.. padding and the 00 01 top limb; digest words 1-4 are not constrained
    const uint64_t em2 = em[2];
    if ((uint32_t)em2 != H[0]) lane_status(status + w, ST_RSA_HASH);
    if ((em2 >> 32) != 83887124ull || em[3] != 650212878678426138ull || em[4] != 18446744069417738544ull)
      lane_status(status + w, ST_RSA_PREFIX);
    bool pb = em[K - 1] != 562949953421311ull;
    for (int i = 5; i < K - 1; i++) pb |= em[i] != ~0ull;
    if (pb) lane_status(status + w, ST_RSA_PAD);
  } else {
    if (hash_bad) lane_status(status + w, ST_RSA_HASH);
    if (em[4] != RSA_EM4 || em[5] != RSA_EM5) lane_status(status + w, ST_RSA_PREFIX);
    if (pad_bad) lane_status(status + w, ST_RSA_PAD);
  }
  if (gt_bad) lane_status(status + w, ST_BIGMOD_GT);
}
#endif

// ============================================================================ BabyJubJub core
// twisted Edwards a x^2 + y^2 = 1 + d x^2 y^2, a = 168700, d = 168696 (babyjubjub/curve.circom:62-70)
struct ExtPt { fr X, Y, Z, T; };

template <class PM = FrMulInline>
__device__ __forceinline__ ExtPt bjj_dbl(const ExtPt& P, const fr& A) {  // dbl-2008-hwcd
  fr a = PM::sqr(P.X), b = PM::sqr(P.Y), c = PM::sqr(P.Z);
  c = fr_add(c, c);
  fr d = PM::mul(A, a);
  fr xy = fr_add(P.X, P.Y);
  fr e = fr_sub(fr_sub(PM::sqr(xy), a), b);
  fr g = fr_add(d, b), f = fr_sub(g, c), h = fr_sub(d, b);
  return ExtPt{PM::mul(e, f), PM::mul(g, h), PM::mul(f, g), PM::mul(e, h)};
}
template <class PM = FrMulInline>
__device__ __forceinline__ ExtPt bjj_add_affine(const ExtPt& P, const fr& x2, const fr& y2, const fr& t2d, const fr& A) {
  // add-2008-hwcd with Z2 = 1, t2d = d * x2 * y2
  fr a = PM::mul(P.X, x2), b = PM::mul(P.Y, y2), c = PM::mul(P.T, t2d), d = P.Z;
  fr e = fr_sub(fr_sub(PM::mul(fr_add(P.X, P.Y), fr_add(x2, y2)), a), b);
  fr f = fr_sub(d, c), g = fr_add(d, c), h = fr_sub(b, PM::mul(A, a));
  return ExtPt{PM::mul(e, f), PM::mul(g, h), PM::mul(f, g), PM::mul(e, h)};
}

// Base8 (babyjubjub/get.circom:9-10), normal form; 1/Base8.x (IsZero of adders' in2)
constexpr uint32_t BJJ_B8X[8] = {0xbb957051u, 0x2893f3f6u, 0x0534e0b6u, 0x2ab8d801u,
                                 0x9d6277c1u, 0x4eacb2e0u, 0xd63e739bu, 0x0bb77a6au};
constexpr uint32_t BJJ_B8Y[8] = {0x872d7d8bu, 0x4b3c257au, 0xb9e13377u, 0xfce0051fu,
                                 0xd16bf9edu, 0x25572e1cu, 0xf7a0b249u, 0x25797203u};
constexpr uint32_t BJJ_INV_B8X[8] = {0x7bc45854u, 0x42cd5135u, 0x5936d873u, 0x5dc5f319u,
                                     0x40d1c783u, 0x40e2c828u, 0xcaabb2bdu, 0x0b1a7dddu};
constexpr uint64_t BJJ_A = 168700, BJJ_D = 168696;

// the same constants in Montgomery form (R = 2^256), as literals: a kernel that sets them from these keeps no
// registers for them (the compiler rematerialises literal moves)
constexpr uint32_t BJJ_M_A[8] = {0xfff261e0u, 0x95accf61u, 0x9df7d378u, 0x24780d65u,
                                 0x7e906ae8u, 0xe0ac11b0u, 0x16d3def3u, 0x0f35db22u};
constexpr uint32_t BJJ_M_D[8] = {0xaff261f5u, 0x2735f484u, 0x9a2e0f63u, 0x70ba1b57u,
                                 0x1e2caa8cu, 0xff41c9a9u, 0x8fe6025fu, 0x07704a8eu};
constexpr uint32_t BJJ_M_B8X[8] = {0x1a89fa86u, 0x0a8fc7bcu, 0xe9e48627u, 0xa7d9d786u,
                                   0x65bea369u, 0xee6158b4u, 0x2f874519u, 0x14a0ff6du};
constexpr uint32_t BJJ_M_B8Y[8] = {0x0d0201aau, 0xb83342d2u, 0xcdcfeac7u, 0x2ffef2f7u,
                                   0x25a6e625u, 0xbfa79a94u, 0xc3a44b70u, 0x0dfb859du};
constexpr uint32_t BJJ_M_B8TD[8] = {0x0f1b2ee0u, 0x10c75c99u, 0xc23309edu, 0x83d5e20cu,
                                    0xe93991cfu, 0x3fc6be6bu, 0xb5195112u, 0x03a44577u};

struct BjjConsts {
  fr A, D, B8x, B8y, B8t_d;  // Montgomery
  __device__ __forceinline__ void init() {
    A = fr_to_mont(fr_u64(BJJ_A)); D = fr_to_mont(fr_u64(BJJ_D));
    B8x = fr_to_mont(fr_const(BJJ_B8X)); B8y = fr_to_mont(fr_const(BJJ_B8Y));
    B8t_d = fr_mul(fr_mul(D, B8x), B8y);
  }
  __device__ __forceinline__ void init_literal() {
    A = fr_const(BJJ_M_A); D = fr_const(BJJ_M_D);
    B8x = fr_const(BJJ_M_B8X); B8y = fr_const(BJJ_M_B8Y); B8t_d = fr_const(BJJ_M_B8TD);
  }
};

// Fixed-base table for the segment start points: T[w][v] = v * 2^(8w) * Base8, w < 32, v < 256,
// affine (x, y) and t2d = d*x*y, Montgomery form. Built once per instance (k_bjj_table).
template <class PM = FrMulInline>
__device__ __forceinline__ ExtPt bjj_add(const ExtPt& P, const ExtPt& Q, const BjjConsts& C) {  // add-2008-hwcd
  fr a = PM::mul(P.X, Q.X), b = PM::mul(P.Y, Q.Y), c = PM::mul(PM::mul(P.T, C.D), Q.T), d = PM::mul(P.Z, Q.Z);
  fr e = fr_sub(fr_sub(PM::mul(fr_add(P.X, P.Y), fr_add(Q.X, Q.Y)), a), b);
  fr f = fr_sub(d, c), g = fr_add(d, c), h = fr_sub(b, PM::mul(C.A, a));
  return ExtPt{PM::mul(e, f), PM::mul(g, h), PM::mul(f, g), PM::mul(e, h)};
}

#ifndef PZK_TEMPLATE_KERNELS_ONLY  // defined once, in kernels.hip
__global__ void __launch_bounds__(256) k_bjj_table(fr* table) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;  // (w, v)
  if (idx >= BJJ_TABLE_WINDOWS * 256) return;
  const int wi = idx >> 8, v = idx & 255;
  BjjConsts C;
  C.init();
  fr* out = table + 3 * (size_t)idx;
  if (v == 0) { out[0] = fr_zero(); out[1] = fr_zero(); out[2] = fr_zero(); return; }
  ExtPt base{C.B8x, C.B8y, fr_mont_one(), fr_mul(C.B8x, C.B8y)};
  for (int k = 0; k < 8 * wi; k++) base = bjj_dbl(base, C.A);
  ExtPt acc = base;  // v * base, MSB-first double-and-add from the top set bit
  for (int bit = 30 - __clz(v); bit >= 0; bit--) {
    acc = bjj_dbl(acc, C.A);
    if ((v >> bit) & 1) acc = bjj_add(acc, base, C);
  }
  fr zi = fr_inv(acc.Z);
  fr x = fr_mul(acc.X, zi), y = fr_mul(acc.Y, zi);
  out[0] = x; out[1] = y; out[2] = fr_mul(fr_mul(C.D, x), y);
}
#endif


// segment start of the ladder below: A_{i0-1} = p * Base8, p = sk >> (254 - i0) (an i0-bit prefix), summed from the
// fixed-base table (8-bit windows; the top window of a prefix may be partial)
template <class PM = FrMulInline>
__device__ __forceinline__ void bjj_seg_start(const fr& sk, int i0, const fr* table, const BjjConsts& C, bool& have,
                                              ExtPt& A) {
  have = false;
  A = ExtPt{fr_zero(), fr_zero(), fr_zero(), fr_zero()};
  for (int wi = 0; 8 * wi < i0; wi++) {
    uint32_t v = 0;
    for (int b = 0; b < 8 && 8 * wi + b < i0; b++) v |= fr_bit(sk, 254 - i0 + 8 * wi + b) << b;
    if (!v) continue;
    const fr* e = table + 3 * (size_t)(wi * 256 + v);
    if (!have) { A = ExtPt{e[0], e[1], fr_mont_one(), PM::mul(e[0], e[1])}; have = true; }
    else A = bjj_add_affine<PM>(A, e[0], e[1], e[2], C.A);
  }
}
// The same start points with the table additions of each lane pair (seg, SEGS - 1 - seg) balanced: prefix lengths grow
// with seg, so the lane with the shorter prefix also sums the top windows of its partner's and hands that partial sum
// over (a wave shuffle and one general addition): a lane's additions go from up to SEGS - 1 windows (SEGS = 32: 31)
// to about half. The sums start from the identity (0 : 1 : 1 : 0) — the addition law is complete on BabyJubJub
// (a a square, d not) — so Z differs from bjj_seg_start's but the affine point and `have` do not.
template <int SEGS, int SEG_LEN, class PM = FrMulInline>
__device__ __forceinline__ void bjj_seg_start_paired(const fr& sk, int seg, const fr* table, const BjjConsts& C,
                                                     bool& have, ExtPt& A) {
  static_assert(SEGS % 2 == 0 && SEG_LEN % 8 == 0, "lane pairs of whole windows");
  constexpr int NWIN = SEG_LEN / 8;  // windows per segment of prefix
  const int p = SEGS - 1 - seg;
  const bool helper = seg < p;
  const int n_own = NWIN * seg, n_p = NWIN * p, n_lo = helper ? n_own : n_p;
  const int half = (n_own + n_p + 1) / 2, h = half - n_lo;  // h: the longer prefix's windows the helper sums
  const int own_end = helper ? n_own : n_own - h;
  const ExtPt id{fr_zero(), fr_mont_one(), fr_mont_one(), fr_zero()};
  ExtPt Ao = id, Ah = id;
  bool ho = false, hh = false;
  for (int k = 0; k < half; k++) {
    const bool mine = k < own_end;
    if (!mine && !(helper && k - own_end < h)) continue;
    const int i0x = SEG_LEN * (mine ? seg : p), wi = mine ? k : n_p - h + (k - own_end);
    uint32_t v = 0;
    for (int b = 0; b < 8; b++) v |= fr_bit(sk, 254 - i0x + 8 * wi + b) << b;
    if (!v) continue;
    const fr* e = table + 3 * (size_t)(wi * 256 + v);
    const ExtPt cur = bjj_add_affine<PM>(mine ? Ao : Ah, e[0], e[1], e[2], C.A);
    if (mine) { Ao = cur; ho = true; }
    else { Ah = cur; hh = true; }
  }
  auto xo = [](const fr& a) { fr r; for (int k = 0; k < 8; k++) r.v[k] = (uint32_t)__shfl_xor((int)a.v[k], SEGS - 1, 64); return r; };
  const ExtPt got{xo(Ah.X), xo(Ah.Y), xo(Ah.Z), xo(Ah.T)};
  const bool gh = __shfl_xor((int)hh, SEGS - 1, 64) != 0;
  if (!helper && gh) {
    Ao = ho ? bjj_add<PM>(Ao, got, C) : got;
    ho = true;
  }
  have = ho;
  A = Ao;
}
// ladder step i (curve.circom:156-168): D_i = 2 A_{i-1} when A_{i-1} exists (the (0,0) sentinel otherwise: D = 0),
// A_i = D_i + Base8 when bit 253 - i of sk is set, else D_i
template <class PM = FrMulInline>
__device__ __forceinline__ void bjj_step(const fr& sk, int i, const BjjConsts& C, bool& have, ExtPt& A, bool& haveD,
                                         ExtPt& D) {
  const uint32_t bit = fr_bit(sk, 253 - i);
  haveD = i > 0 && have;
  D = haveD ? bjj_dbl<PM>(A, C.A) : ExtPt{fr_zero(), fr_zero(), fr_zero(), fr_zero()};
  if (bit) {
    if (haveD) A = bjj_add_affine<PM>(D, C.B8x, C.B8y, C.B8t_d, C.A);
    else { A.X = C.B8x; A.Y = C.B8y; A.Z = fr_mont_one(); A.T = PM::mul(C.B8x, C.B8y); }
    have = true;
  } else {
    if (haveD) A = D;
    have = haveD;
  }
}

// BabyjubjubBase8Multiplication (babyjubjub/curve.circom:143-171): MSB-first double-and-add over
// the 254 bits of sk with the (0,0) sentinel for "no point yet". The ladder is cut into BJJ_SEGS
// segments of BJJ_SEG_LEN steps, one lane each (BJJ_SEGS adjacent lanes = one witness): a segment
// starts from A_{i0-1} = (sk >> (254 - i0)) * Base8, summed from the fixed-base table, so the
// segments run in parallel. The affine outputs need 1/Z of every point (and 1/x of every D):
// one batched inversion per witness across its lanes (wave shuffles), and one Fr inversion per workgroup: wave 0
// inverts the BJJ_WG_WAVES * 64 / BJJ_SEGS witness totals at once (a Fr inversion per witness group was ~40 % of
// the kernel's VALU).
// scratch: SoA [elem][lane], 9 * SEG_LEN elements per lane (X,Y,Z of D and A, 3 prefixes).
// SEGS (8 / 16 / 32 lanes per witness, SEG_LEN = 256 / SEGS steps each) trades the segment-start
// table sums (up to i0 / 8 affine additions) against ladder length and occupancy.
constexpr int BJJ_WG_WAVES = 4;
template <int BJJ_SEGS>
__global__ void __launch_bounds__(64 * BJJ_WG_WAVES) k_bjj_core(DevLayout L, ValueStore vs, const fr* table,
                                                               fr* bjj_core, fr* scratch, uint32_t batch,
                                                               bool paired) {
  constexpr int BJJ_SEG_LEN = BJJ_SCRATCH_STEPS / BJJ_SEGS, NW = 64 * BJJ_WG_WAVES / BJJ_SEGS;
  static_assert(64 % BJJ_SEGS == 0 && BJJ_SEG_LEN * BJJ_SEGS >= BJJ_STEPS, "segments must cover the ladder");
  static_assert(NW <= 64 && (NW & (NW - 1)) == 0, "the workgroup's witness totals: one per lane of wave 0");
  __shared__ fr s_tot[NW];
  core_priority();
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t nlanes = batch * BJJ_SEGS;
  const uint32_t w = tid / BJJ_SEGS;
  const int seg = (int)(tid % BJJ_SEGS);
  if (blockIdx.x * (uint32_t)NW >= batch) return;  // whole workgroups only (no lane of it is live)
  const bool live = w < batch;  // a lane group past the batch takes part in the workgroup's barriers only
  BjjConsts C;
  C.init();
  const int NS = BJJ_STEPS;
  const int i0 = seg * BJJ_SEG_LEN, i1 = i0 + BJJ_SEG_LEN < NS ? i0 + BJJ_SEG_LEN : NS, ns = i1 - i0;
  auto S = [&](int e) -> fr& { return scratch[(size_t)e * nlanes + tid]; };
  // batched inversion of Z(D_i), Z(A_i), X(D_i) over the segment, then across the BJJ_SEGS lanes
  auto elem = [&](int qi) -> fr {
    int j = qi / 3, kind = qi - 3 * j;
    return kind == 0 ? S(3 * j + 2) : kind == 1 ? S(3 * BJJ_SEG_LEN + 3 * j + 2) : S(3 * j);
  };
  const int NQ = 3 * ns, PRE = 6 * BJJ_SEG_LEN;
  fr acc = fr_mont_one();
  if (live) {
    const fr sk = fr_from_mont(vs.at(L.reg.v_sk, w));
    bool have;
    ExtPt A;
    if (paired) bjj_seg_start_paired<BJJ_SEGS, BJJ_SEG_LEN, CoreMul>(sk, seg, table, C, have, A);
    else bjj_seg_start<CoreMul>(sk, i0, table, C, have, A);
    // projective coords of D_i (local elems 0..3ns) and A_i (3ns..6ns): [X, Y, Z] per step
    for (int j = 0; j < ns; j++) {
      ExtPt D;
      bool haveD;
      bjj_step<CoreMul>(sk, i0 + j, C, have, A, haveD, D);
      if (haveD) { S(3 * j) = D.X; S(3 * j + 1) = D.Y; S(3 * j + 2) = D.Z; }
      else { S(3 * j) = fr_zero(); S(3 * j + 1) = fr_zero(); S(3 * j + 2) = fr_zero(); }
      const int o = 3 * BJJ_SEG_LEN + 3 * j;
      if (have) { S(o) = A.X; S(o + 1) = A.Y; S(o + 2) = A.Z; }
      else { S(o) = fr_zero(); S(o + 1) = fr_zero(); S(o + 2) = fr_zero(); }
    }
    for (int qi = 0; qi < NQ; qi++) {
      fr e = elem(qi);
      S(PRE + qi) = acc;
      if (!fr_is_zero(e)) acc = CoreMul::mul(acc, e);
    }
  }
  fr others, total;
  fr_group_others<BJJ_SEGS>(acc, others, total);
  // the workgroup's witness totals inverted together (lane k of wave 0: witness group k; a dead group's total is 1)
  const int g = (int)(threadIdx.x / BJJ_SEGS);
  if (seg == 0) s_tot[g] = total;
  __syncthreads();
  if (threadIdx.x < 64) {
    const fr t = threadIdx.x < NW ? s_tot[threadIdx.x] : fr_mont_one();
    fr t_others, t_all;
    fr_group_others<NW>(t, t_others, t_all);
    const fr t_inv = fr_mul(fr_inv_sw(t_all), t_others);  // = 1 / total of group threadIdx.x
    if (threadIdx.x < NW) s_tot[threadIdx.x] = t_inv;  // (read above, by this wave only)
  }
  __syncthreads();
  if (!live) return;
  fr inv = fr_mul(s_tot[g], others);  // = 1 / acc
  fr* out = bjj_core + (size_t)w * L.bjj_core_fr;
  for (int qi = NQ - 1; qi >= 0; qi--) {
    fr e = elem(qi);
    fr r = fr_zero();
    if (!fr_is_zero(e)) { r = CoreMul::mul(inv, S(PRE + qi)); inv = CoreMul::mul(inv, e); }
    const int j = qi / 3, kind = qi - 3 * j;
    fr* o = out + 5 * (i0 + j);  // Dx, Dy, Ax, Ay, inv(Dx)
    if (kind == 0) { o[0] = CoreMul::mul(S(3 * j), r); o[1] = CoreMul::mul(S(3 * j + 1), r); }
    else if (kind == 1) { o[2] = CoreMul::mul(S(3 * BJJ_SEG_LEN + 3 * j), r); o[3] = CoreMul::mul(S(3 * BJJ_SEG_LEN + 3 * j + 1), r); }
    else { o[4] = CoreMul::mul(S(3 * j + 2), r); }  // 1/x = Z / X
  }
  if (i1 == NS) {
    vs.at(L.reg.v_bjj, w) = out[5 * (NS - 1) + 2];
    vs.at(L.reg.v_bjj + 1, w) = out[5 * (NS - 1) + 3];
  }
}

// The same ladder and outputs without the scratch array (k_bjj_core keeps 74 KB of points and prefix products per
// witness in global memory, 6x its algorithmic traffic): the forward pass keeps only the step prefix products (LDS,
// SL per lane) and two checkpoints of the ladder state (registers: the segment start and the state before step CK);
// the backward pass recomputes step j's D and A from the nearer checkpoint (SL = 4: 2 + 1 + 2 + 1 extra steps).
// Same per-lane segments as k_bjj_core, SEGS lanes per witness.
#ifndef PZK_BJJ_RC_WPE  // waves per SIMD the register allocation must allow (A/B builds)
#define PZK_BJJ_RC_WPE 2
#endif
template <int BJJ_SEGS>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(PZK_BJJ_RC_WPE))) k_bjj_core_rc(DevLayout L, ValueStore vs, const fr* table, fr* bjj_core,
                                                   uint32_t batch) {
  constexpr int SL = BJJ_SCRATCH_STEPS / BJJ_SEGS, CK = SL / 2;
  static_assert(64 % BJJ_SEGS == 0 && SL * BJJ_SEGS >= BJJ_STEPS && SL >= 2, "segments must cover the ladder");
  __shared__ fr pre[SL][64];  // prefix product before step j, per lane
  core_priority();
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t w = tid / BJJ_SEGS;
  const int seg = (int)(tid % BJJ_SEGS);
  if (w >= batch) return;  // whole lane groups only (64 % BJJ_SEGS == 0)
  BjjConsts C;
  C.init_literal();
  const int NS = BJJ_STEPS;
  const int i0 = seg * SL, i1 = i0 + SL < NS ? i0 + SL : NS, ns = i1 - i0;
  const fr sk = fr_from_mont(vs.at(L.reg.v_sk, w));
  bool have0, have1;
  ExtPt A0, A1;
  bjj_seg_start(sk, i0, table, C, have0, A0);
  have1 = have0;
  A1 = A0;
  // forward: the ladder, prefix products of the inverted elements (Z(D_i), Z(A_i), X(D_i); zeros skipped)
  fr acc = fr_mont_one();
  {
    bool have = have0;
    ExtPt A = A0;
    for (int j = 0; j < ns; j++) {
      if (j == CK) { have1 = have; A1 = A; }
      bool haveD;
      ExtPt D;
      bjj_step(sk, i0 + j, C, have, A, haveD, D);
      pre[j][threadIdx.x] = acc;
      const fr e1 = have ? A.Z : fr_zero();
      if (!fr_is_zero(D.Z)) acc = fr_mul(acc, D.Z);
      if (!fr_is_zero(e1)) acc = fr_mul(acc, e1);
      if (!fr_is_zero(D.X)) acc = fr_mul(acc, D.X);
    }
  }
  fr others, total;
  fr_group_others<BJJ_SEGS>(acc, others, total);
  fr inv = fr_mul(fr_inv_sw(total), others);  // = 1 / acc
  fr* out = bjj_core + (size_t)w * L.bjj_core_fr;
  fr last_x = fr_zero(), last_y = fr_zero();
  for (int j = ns - 1; j >= 0; j--) {
    const int jb = j >= CK ? CK : 0;
    bool have = j >= CK ? have1 : have0, haveD = false;
    ExtPt A = j >= CK ? A1 : A0, D;
    for (int k = jb; k <= j; k++) bjj_step(sk, i0 + k, C, have, A, haveD, D);
    const fr e0 = D.Z, e1 = have ? A.Z : fr_zero(), e2 = D.X;
    const fr q0 = pre[j][threadIdx.x];
    const fr q1 = fr_is_zero(e0) ? q0 : fr_mul(q0, e0);
    const fr q2 = fr_is_zero(e1) ? q1 : fr_mul(q1, e1);
    fr r0 = fr_zero(), r1 = fr_zero(), r2 = fr_zero();
    if (!fr_is_zero(e2)) { r2 = fr_mul(inv, q2); inv = fr_mul(inv, e2); }
    if (!fr_is_zero(e1)) { r1 = fr_mul(inv, q1); inv = fr_mul(inv, e1); }
    if (!fr_is_zero(e0)) { r0 = fr_mul(inv, q0); inv = fr_mul(inv, e0); }
    fr* o = out + 5 * (i0 + j);  // Dx, Dy, Ax, Ay, inv(Dx)
    const fr ax = fr_mul(A.X, r1), ay = fr_mul(A.Y, r1);
    o[0] = fr_mul(D.X, r0);
    o[1] = fr_mul(D.Y, r0);
    o[2] = ax;
    o[3] = ay;
    o[4] = fr_mul(D.Z, r2);  // 1/x = Z / X
    if (j == ns - 1) { last_x = ax; last_y = ay; }
  }
  if (i1 == NS) {
    vs.at(L.reg.v_bjj, w) = last_x;
    vs.at(L.reg.v_bjj + 1, w) = last_y;
  }
}

// ============================================================================ SMT
// flags per level (u32 in the SMT core): bit0 levIns, bit1 done, bit2 st_top, bit3 st_inew, bit4 lrbit, bit5 isZero
// SMT core (Fr): [inv(sibling) normal][80] [root Montgomery][80] [flags][80] [j, inv(root_in - root_0)]
// SMT_PREP_LANES lanes per witness, SMT_LEVELS / SMT_PREP_LANES levels each: the sibling inverses
// are one batched inversion per witness (segment prefix products per lane, the segment totals
// combined by shuffles, one Fr inversion shared by the group, as in k_bjj_core); the SMTLevIns /
// SMTVerifierSM chains are integer recurrences over the 80 isZero bits, which every lane of the
// group rebuilds from the gathered bit mask and writes for its own levels. The workgroup's SMT_PREP_WAVES * 64 / G
// witness totals are inverted together by wave 0 (round 6), with FIPS products.
constexpr int SMT_PREP_WAVES = 4;
#ifndef PZK_TEMPLATE_KERNELS_ONLY  // defined once, in kernels.hip
__global__ void __launch_bounds__(64 * SMT_PREP_WAVES) k_smt_prep(DevLayout L, const uint8_t* inputs, ValueStore vs,
                                                                 fr* smt_core, int32_t* status, uint32_t batch) {
  core_priority();
  constexpr int G = SMT_PREP_LANES, NL = SMT_LEVELS / SMT_PREP_LANES, NW = 64 * SMT_PREP_WAVES / SMT_PREP_LANES;
  static_assert(SMT_LEVELS % SMT_PREP_LANES == 0 && 64 % SMT_PREP_LANES == 0 && NL <= 32, "level split");
  static_assert(NW <= 64 && (NW & (NW - 1)) == 0, "the workgroup's witness totals: one per lane of wave 0");
  __shared__ fr s_tot[NW];
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t w0 = tid / G;
  const int seg = (int)(tid % G), i0 = seg * NL;
  const bool live = w0 < batch;  // a lane group past the batch takes part in the barriers only, and stores nothing
  const uint32_t w = live ? w0 : batch - 1;
  const RegInfo& R = L.reg;
  const uint8_t* row = inputs + 32ull * (uint64_t)w * L.n_inputs;
  fr* core = smt_core + (size_t)w * L.smt_core_fr;
  uint32_t* flags = reinterpret_cast<uint32_t*>(core + 2 * SMT_LEVELS);
  const fr key = fr_from_mont(vs.at(R.v_smt_key, w));
  // inverses of the siblings (SMTLevIns isZero, SMTVerifier.circom:47-50), batched
  fr sm[NL];
  uint32_t zmask = 0;  // bit k: sibling i0 + k is zero
  // (the forward pass runs twice, before and after the workgroup's inversion: arrays kept across its barriers and its
  // register-hungry inversion went to scratch)
  auto forward = [&](bool park) {  // park: the exclusive prefixes go to the inverse slots (read back below)
    fr a = fr_mont_one();
#pragma unroll
    for (int k = 0; k < NL; k++) {
      const fr sn = load_fr(row + 32ull * (R.in_br + i0 + k));
      const bool z = fr_is_zero(sn);
      zmask |= (uint32_t)z << k;
      sm[k] = fr_to_mont(sn);
      if (park) core[i0 + k] = a;
      if (!z) a = fr_mul_fast(a, sm[k]);
    }
    return a;
  };
  const fr acc = live ? forward(false) : fr_mont_one();
  fr others, total;
  fr_group_others<G>(acc, others, total);
  const int g = (int)(threadIdx.x / G);
  if (seg == 0) s_tot[g] = total;
  __syncthreads();
  if (threadIdx.x < 64) {
    const fr t = threadIdx.x < NW ? s_tot[threadIdx.x] : fr_mont_one();
    fr t_others, t_all;
    fr_group_others<NW>(t, t_others, t_all);
    const fr t_inv = fr_mul_fast(fr_inv_sw<true>(t_all), t_others);  // = 1 / total of group threadIdx.x
    if (threadIdx.x < NW) s_tot[threadIdx.x] = t_inv;  // (read above, by this wave only)
  }
  __syncthreads();
  if (!live) return;
  fr inv = fr_mul_fast(s_tot[g], others);  // = 1 / acc
  zmask = 0;
  forward(true);
#pragma unroll
  for (int k = NL - 1; k >= 0; k--) {
    fr r = fr_zero();
    if (!((zmask >> k) & 1)) { r = fr_mul_fast(inv, core[i0 + k]); inv = fr_mul_fast(inv, sm[k]); }
    core[i0 + k] = fr_from_mont(r);
  }
  // the group's isZero bits, levels 0..79
  uint32_t zm[G];
#pragma unroll
  for (int t = 0; t < G; t++) zm[t] = (uint32_t)__shfl((int)zmask, t, G);
  auto iz = [&](int i) -> int {
    int r = 0;
#pragma unroll
    for (int t = 0; t < G; t++) r |= (i / NL == t) ? (int)((zm[t] >> (i - t * NL)) & 1u) : 0;
    return r;
  };
  if (seg == G - 1 && !iz(SMT_LEVELS - 1)) set_status(status ? status + w : nullptr, ST_SMT_LAST);
  // SMTLevIns (SMTVerifier.circom:39-65): done[i-1] = lev[i] + done[i], from the top
  uint32_t levm[3] = {0, 0, 0}, donem[3] = {0, 0, 0};
  auto setb = [](uint32_t* m, int i, int v) { m[i >> 5] |= (uint32_t)(v & 1) << (i & 31); };
  auto getb = [](const uint32_t* m, int i) -> int { return (int)((m[i >> 5] >> (i & 31)) & 1u); };
  {
    int lev = 1 - iz(SMT_LEVELS - 2), done = lev;  // lev[79], done[78]
    setb(levm, SMT_LEVELS - 1, lev);
    setb(donem, SMT_LEVELS - 2, done);
    for (int i = SMT_LEVELS - 2; i > 0; i--) {
      lev = (1 - done) * (1 - iz(i - 1));
      setb(levm, i, lev);
      done = lev + done;  // done[i - 1]
      setb(donem, i - 1, done);
    }
    setb(levm, 0, 1 - done);
  }
  // SMTVerifierSM chain and the insertion level j
  int prev_top = 1, j = SMT_LEVELS;
  for (int i = 0; i < SMT_LEVELS; i++) {
    const int lv = getb(levm, i), st_inew = prev_top * lv, st_top = prev_top - st_inew;
    if (st_inew) j = i;
    if (i >= i0 && i < i0 + NL) {
      const int lr = (int)fr_bit(key, i);
      flags[i] = (uint32_t)lv | ((uint32_t)getb(donem, i) << 1) | ((uint32_t)(st_top & 1) << 2) |
                 ((uint32_t)(st_inew & 1) << 3) | ((uint32_t)lr << 4) | ((uint32_t)iz(i) << 5);
    }
    prev_top = st_top;
  }
  if (seg == 0) reinterpret_cast<uint32_t*>(core + 3 * SMT_LEVELS)[0] = (uint32_t)j;
  // level hashes whose child is 0 (i >= j): inputs known now
  const int from = j < SMT_LEVELS ? j : 0;
#pragma unroll
  for (int k = 0; k < NL; k++) {
    const int i = i0 + k;
    if (i < from) continue;
    const int lr = (int)fr_bit(key, i);
    vs.at(R.v_smt_lr + 2 * i, w) = lr ? sm[k] : fr_zero();
    vs.at(R.v_smt_lr + 2 * i + 1, w) = lr ? fr_zero() : sm[k];
  }
}
#endif

// sequential part: levels j-1 .. 0, then all roots and the isEqual inverse. SMT_CHAIN_LANES lanes per
// witness run each level hash as a cooperative permutation (pos_perm_group: lane k < 3 holds state
// element k) whose hash comes back to every lane of the group by its butterfly. What the rounds read is staged in
// LDS first — the width-3 constants, the group's left/right bits, the level tasks' core offsets — so no round
// issues a global load (one issued after the round-state stores would wait for them: gfx9 vmcnt counts both).
// The siblings are the one global read: level i - 1's is loaded when level i starts and converted when level i
// ends, one wait per level (round 5: staging all 80 per lane group took 40 KB of the 63 KB of LDS a chain
// workgroup held beside the emitters on every CU it ran on).
// PM: the product policy (PZK_CHAIN_MUL=inline|call|fips, A/B; poseidon.hpp FrMulInline / FrMulCall / FrMulFips)
#ifndef PZK_TEMPLATE_KERNELS_ONLY  // defined once, in kernels.hip
template <class PM>
__global__ void __launch_bounds__(64) k_smt_chain(DevLayout L, PosConsts K, const int32_t* level_task, const uint8_t* inputs,
                                                 ValueStore vs, fr* pos_core, fr* smt_core, const uint32_t* order,
                                                 int32_t* status, uint32_t batch) {
  core_priority();
  constexpr int G = SMT_CHAIN_LANES, NG = 64 / G;
  static_assert(G == 4 && 64 % G == 0, "PoseidonHash(2) groups are 4 lanes (t = 3)");
  using KL = PosConstsLds<3>;
  __shared__ fr kc[KL::SIZE];
  __shared__ uint8_t lrs[NG][SMT_LEVELS];
  __shared__ int32_t lv_core[SMT_LEVELS];
  KL::stage(kc, K);
  for (int i = threadIdx.x; i < SMT_LEVELS; i += blockDim.x) lv_core[i] = L.pos[level_task[i]].core_off;
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t g = tid / G;
  const int jl = (int)(tid % G), gi = (int)(threadIdx.x / G);
  const bool live = g < batch;  // whole lane groups only; every thread takes part in the barrier
  const uint32_t w = live ? (order ? order[g] : g) : 0;  // k_smt_order: lane groups by proof depth, deepest first
  const RegInfo& R = L.reg;
  const uint8_t* row = inputs + 32ull * (uint64_t)w * L.n_inputs;
  fr* core = smt_core + (size_t)w * L.smt_core_fr;
  const uint32_t* flags = reinterpret_cast<const uint32_t*>(core + 2 * SMT_LEVELS);
  const int j = live ? (int)reinterpret_cast<const uint32_t*>(core + 3 * SMT_LEVELS)[0] : 0;
  const int top = j < SMT_LEVELS ? j : SMT_LEVELS;
  for (int i = jl; i < top; i += G) lrs[gi][i] = (uint8_t)((flags[i] >> 4) & 1);
  __syncthreads();
  if (!live) return;
  const KL Kl{kc};
  const fr leaf = vs.at(R.v_leaf, w);
  fr child = leaf;  // root_j = leaf
  fr* pcore = pos_core + (size_t)w * L.pos_core_elems;
  const uint8_t* sib_row = row + 32ull * R.in_br;
  fr sib = top > 0 ? fr_to_mont(load_fr(sib_row + 32ull * (top - 1))) : fr_zero();
  for (int i = top - 1; i >= 0; i--) {
    const fr sib_next_raw = i > 0 ? load_fr(sib_row + 32ull * (i - 1)) : fr_zero();  // before this level's stores
    const bool lr = lrs[gi][i] != 0;
    const fr lv = lr ? sib : child, rv = lr ? child : sib;  // Switcher (SMTVerifier.circom): the level's L / R
    if (jl == 0) {
      vs.at(R.v_smt_lr + 2 * i, w) = lv;
      vs.at(R.v_smt_lr + 2 * i + 1, w) = rv;
    }
    child = pos_perm_group<3, G, KL, PM>(Kl, jl == 1 ? lv : jl == 2 ? rv : fr_zero(), pcore + lv_core[i], jl);
    if (jl == 0) vs.at(R.v_smt_h + i, w) = child;  // root_i = H_i (st_top = 1 below j)
    sib = fr_to_mont(sib_next_raw);
  }
  if (jl != 0) return;  // lane 0 wrote every level hash this kernel made
  // roots of every level: root_i = st_top_i * H_i + st_inew_i * leaf (SMTVerifier.circom:104-106)
  fr* roots = core + SMT_LEVELS;
  for (int i = 0; i < SMT_LEVELS; i++) {
    uint32_t f = flags[i];
    fr r = fr_zero();
    if (f & 4) r = vs.at(R.v_smt_h + i, w);
    if (f & 8) r = fr_add(r, leaf);
    roots[i] = r;
  }
  // isEqual(root_0, root): inverse of root - root_0
  fr rin = fr_to_mont(load_fr(row + 32ull * R.in_root));
  fr dlt = fr_sub(rin, roots[0]);
  core[3 * SMT_LEVELS + 1] = fr_inv_sw(dlt);
  // smtVerifier.isVerified === 1 where the circuit asserts it (identityStateVerifier.circom:46; the register
  // circuit leaves it commented out, passportVerificationBuilder.circom:240)
  if (R.smt_check && !fr_is_zero(dlt)) set_status(status ? status + w : nullptr, ST_ISV_ROOT);
}
#endif

}  // namespace pzk
