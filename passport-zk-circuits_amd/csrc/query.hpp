// QueryIdentity(80) (identityManagement/queryIdentity.circom:37-229): the query-specific
// small templates, evaluated in closed form per signal, and the per-witness prep kernel.
//
// The circuit's heavy parts reuse the register path's machinery: PoseidonHash blocks (k_pos_core / k_emit_pos),
// the identity-state SMTVerifier(80) (k_smt_prep / k_smt_chain + the SMT regions), the BabyJubJub key
// (k_bjj_core / k_emit_bjj), Bits2Num / Num2Bits (k_emit_bits). What is left are a few thousand signals of
// comparators, date codecs and the citizenship list, all small integers or single field products of input
// elements: they are emitted by k_emit_gen through query_small() below, each signal from the input row and a
// handful of value-store slots that k_qry_prep fills (DG1 fields, the citizenship's list index and the 240
// IsEqual inverses of CitizenshipCheck, one batched inversion per witness).
#pragma once
#include "bufs.hpp"
#include "core_util.hpp"
#include "ec_emit.hpp"
#include "fr.hpp"
#include "layout.hpp"
#include "regcore.hpp"
#include "query_layout.hpp"

namespace pzk {

static __constant__ const uint32_t Q_COUNTRY[240] = {
#include "../data/citizenship_codes.inc"
};

// ---- field values as plain integers (fr limbs, normal form)
__device__ __forceinline__ fr q_u128(uint64_t lo, uint64_t hi) {
  fr r = fr_zero();
  r.v[0] = (uint32_t)lo; r.v[1] = (uint32_t)(lo >> 32); r.v[2] = (uint32_t)hi; r.v[3] = (uint32_t)(hi >> 32);
  return r;
}
__device__ __forceinline__ uint32_t q_word(const fr& a, int k) {  // select chain (no run-time register indexing)
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r |= a.v[i] & (0u - (uint32_t)(k == i));
  return r;
}
__device__ __forceinline__ uint32_t q_bit(const fr& a, int i) { return (q_word(a, i >> 5) >> (i & 31)) & 1u; }
__device__ __forceinline__ fr q_mask(const fr& a, int nbits) {  // a mod 2^nbits
  fr r = a;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const int lo = 32 * i;
    if (nbits <= lo) r.v[i] = 0;
    else if (nbits < lo + 32) r.v[i] &= (1u << (nbits - lo)) - 1u;
  }
  return r;
}
// 1/d in normal form for a signed integer d (IsZero: 1/0 = 0)
__device__ __forceinline__ fr q_inv_signed(const fr* T, int64_t d) {
  if (d > -256 && d < 256) return inv_small_signed(T, (int)d);
  const fr x = d >= 0 ? fr_u64((uint64_t)d) : fr_sub(fr_zero(), fr_u64((uint64_t)(-d)));
  return fr_from_mont(fr_inv(fr_to_mont(x)));
}
__device__ __forceinline__ fr q_signed(int64_t d) {
  return d >= 0 ? fr_u64((uint64_t)d) : fr_sub(fr_zero(), fr_u64((uint64_t)(-d)));
}

// LessThan(L) block (comparators.circom:46-57) signal e: out | in[2] | Num2Bits(L+1)(v = in0 + 2^L - in1);
// v given (a field value; for in-domain inputs a non-negative (L+1)-bit integer)
__device__ __forceinline__ El q_lt_sig(int e, int L, const El& in0, const El& in1, const fr& v) {
  if (e == 0) return el_u64(1u - q_bit(v, L));
  if (e == 1) return in0;
  if (e == 2) return in1;
  e -= 3;                                  // Num2Bits(L+1): out[L+1] | in | sum[L+1]
  if (e <= L) return el_u64(q_bit(v, e));
  if (e == L + 1) return el_fr(v);
  return el_fr(q_mask(v, e - (L + 1)));    // sum[i] = v mod 2^(i+1)
}
// small-integer LessThan(L): v = a + 2^L - b
__device__ __forceinline__ El q_lt_small(int e, int L, int64_t a, int64_t b) {
  return q_lt_sig(e, L, el_fr(q_signed(a)), el_fr(q_signed(b)), q_signed(a + (1ll << L) - b));
}
// 64-bit LessThan(64): v = a + 2^64 - b for a, b < 2^65 given as (lo, hi)
__device__ __forceinline__ fr q_v64(uint64_t alo, uint64_t ahi, uint64_t blo, uint64_t bhi) {
  const uint64_t lo = alo - blo, borrow = alo < blo;
  return q_u128(lo, ahi - bhi - borrow + 1);
}

// ---- dates: "YYMMDD" as UTF-8 bytes, big-endian (dateDecoder.circom, dateEncoder.circom)
struct QDate { int d, m, y; };
__device__ __forceinline__ QDate q_dec(uint64_t e) {
  return QDate{(int)(((e >> 8) & 15) * 10 + (e & 15)), (int)(((e >> 24) & 15) * 10 + ((e >> 16) & 15)),
               (int)(((e >> 40) & 15) * 10 + ((e >> 32) & 15))};
}
__device__ __forceinline__ uint64_t q_enc1(int v) { return (uint64_t)(v / 10) * 256 + (uint64_t)(v % 10) + 12336; }
__device__ __forceinline__ uint64_t q_enc(const QDate& q) {
  return (q_enc1(q.y) << 32) + (q_enc1(q.m) << 16) + q_enc1(q.d);
}
// DateDecoder block (17): day, month, year | dateEncoded | DateEncoder: encoded | day, month, year |
// dayDecimals, dayRest, monthDecimals, monthRest, yearDecimals, yearRest, dayEncoded, monthEncoded, yearEncoded
__device__ __forceinline__ El q_datedec_sig(int s, uint64_t e) {
  const QDate q = q_dec(e);
  switch (s) {
    case 0: case 5: return el_u64((uint64_t)q.d);
    case 1: case 6: return el_u64((uint64_t)q.m);
    case 2: case 7: return el_u64((uint64_t)q.y);
    case 3: return el_u64(e);
    case 4: return el_u64(q_enc(q));
    case 8: return el_u64((uint64_t)(q.d / 10));
    case 9: return el_u64((uint64_t)(q.d % 10));
    case 10: return el_u64((uint64_t)(q.m / 10));
    case 11: return el_u64((uint64_t)(q.m % 10));
    case 12: return el_u64((uint64_t)(q.y / 10));
    case 13: return el_u64((uint64_t)(q.y % 10));
    case 14: return el_u64(q_enc1(q.d));
    case 15: return el_u64(q_enc1(q.m));
    default: return el_u64(q_enc1(q.y));
  }
}
__device__ __forceinline__ int q_dil_out(int fd, int sd, int fm, int sm, int fy, int sy) {
  return (fy < sy) | ((fy == sy) & (fm < sm)) | ((fy == sy) & (fm == sm) & (fd < sd));
}
// DateIsLess block (109, dateComparison.circom:5-58): out | firstDay, secondDay, firstMonth, secondMonth,
// firstYear, secondYear | isYearLess, isMonthLess, isDayLess, isYearEqual, isMonthEqual, isLess1, isLess2, temp,
// isLess3 | yearLess, monthLess, dayLess (LessThan(8)), yearEqual, monthEqual (IsEqual), greaterThen (GreaterThan(3))
__device__ __forceinline__ El q_dil_sig(int s, const fr* T, int fd, int sd, int fm, int sm, int fy, int sy) {
  const int yl = fy < sy, ml = fm < sm, dl = fd < sd, ye = fy == sy, me = fm == sm;
  const int x = yl + (ye & ml) + (ye & me & dl);
  if (s < 16) {
    switch (s) {
      case 0: return el_u64(x > 0);
      case 1: return el_u64((uint64_t)fd);
      case 2: return el_u64((uint64_t)sd);
      case 3: return el_u64((uint64_t)fm);
      case 4: return el_u64((uint64_t)sm);
      case 5: return el_u64((uint64_t)fy);
      case 6: return el_u64((uint64_t)sy);
      case 7: case 12: return el_u64(yl);
      case 8: return el_u64(ml);
      case 9: return el_u64(dl);
      case 10: return el_u64(ye);
      case 11: return el_u64(me);
      case 13: return el_u64(ye & ml);
      case 14: return el_u64(ye & me);
      default: return el_u64(ye & me & dl);
    }
  }
  if (s < 38) return q_lt_small(s - 16, 8, fy, sy);
  if (s < 60) return q_lt_small(s - 38, 8, fm, sm);
  if (s < 82) return q_lt_small(s - 60, 8, fd, sd);
  if (s < 88) return iseq_sig(s - 82, (uint64_t)fy, (uint64_t)sy, q_inv_signed(T, (int64_t)sy - fy));
  if (s < 94) return iseq_sig(s - 88, (uint64_t)fm, (uint64_t)sm, q_inv_signed(T, (int64_t)sm - fm));
  // GreaterThan(3)(x, 0): out | in[2] | LessThan(3)(0, x)
  if (s == 94) return el_u64(x > 0);
  if (s == 95) return el_u64((uint64_t)x);
  if (s == 96) return el_u64(0);
  return q_lt_small(s - 97, 3, 0, x);
}
__device__ __forceinline__ int q_edil_out(uint64_t e1, uint64_t e2) {
  const QDate a = q_dec(e1), b = q_dec(e2);
  return q_dil_out(a.d, b.d, a.m, b.m, a.y, b.y);
}
// EncodedDateIsLess block (146, dateComparisonEncoded.circom:6-29): out | first, second | firstDateDecoder,
// secondDateDecoder, dateIsLess
__device__ __forceinline__ El q_edil_sig(int s, const fr* T, uint64_t e1, uint64_t e2) {
  const QDate a = q_dec(e1), b = q_dec(e2);
  if (s == 0) return el_u64(q_dil_out(a.d, b.d, a.m, b.m, a.y, b.y));
  if (s == 1) return el_u64(e1);
  if (s == 2) return el_u64(e2);
  if (s < 3 + (int)Q_SZ_DATEDEC) return q_datedec_sig(s - 3, e1);
  if (s < 3 + 2 * (int)Q_SZ_DATEDEC) return q_datedec_sig(s - 3 - (int)Q_SZ_DATEDEC, e2);
  return q_dil_sig(s - 3 - 2 * (int)Q_SZ_DATEDEC, T, a.d, b.d, a.m, b.m, a.y, b.y);
}
// EncodedDateIsLessNormalized block (440, dateComparisonEncodedNormalized.circom:13-53): out | first, second,
// currentDate | CENTURY | firstDateDecoder, secondDateDecoder, firstDateNormalization, secondDateNormalization (EDIL
// against currentDate), dateIsLess over years + 100 * normalization
__device__ __forceinline__ El q_ediln_sig(int s, const fr* T, uint64_t e1, uint64_t e2, uint64_t cur) {
  const QDate a = q_dec(e1), b = q_dec(e2);
  const int n1 = q_edil_out(e1, cur), n2 = q_edil_out(e2, cur);
  const int ya = a.y + 100 * n1, yb = b.y + 100 * n2;
  constexpr int D1 = 5, D2 = D1 + (int)Q_SZ_DATEDEC, N1 = D2 + (int)Q_SZ_DATEDEC, N2 = N1 + (int)Q_SZ_EDIL,
                DL = N2 + (int)Q_SZ_EDIL;
  switch (s) {
    case 0: return el_u64(q_dil_out(a.d, b.d, a.m, b.m, ya, yb));
    case 1: return el_u64(e1);
    case 2: return el_u64(e2);
    case 3: return el_u64(cur);
    case 4: return el_u64(100);
    default: break;
  }
  if (s < D2) return q_datedec_sig(s - D1, e1);
  if (s < N1) return q_datedec_sig(s - D2, e2);
  if (s < N2) return q_edil_sig(s - N1, T, e1, cur);
  if (s < DL) return q_edil_sig(s - N2, T, e2, cur);
  return q_dil_sig(s - DL, T, a.d, b.d, a.m, b.m, ya, yb);
}

// the dates and conditions of one witness (inputs < 2^64 in the evaluated domain)
struct QView {
  const uint8_t* row;
  int ts, ic;  // input offsets of timestamp / identityCounter (after dg1, whose length depends on TD1 / TD3)
  __device__ __forceinline__ uint64_t in(int k) const { return in_u64(row + 32ull * k); }
};
__device__ __forceinline__ QView q_view(const DevLayout& L, const uint8_t* inputs, uint32_t w) {
  const bool td1 = L.reg.q_td1 != 0;
  return QView{inputs + 32ull * (uint64_t)w * L.n_inputs, q_in_ts(td1), q_in_ic(td1)};
}
// condition k of the ForceEqualIfEnabled checks (queryIdentity.circom:109-188); exp / birth: DG1 dates
__device__ __forceinline__ int q_cond(const QView& Q, int k, uint64_t exp, uint64_t birth) {
  switch (k) {
    case 0: return Q.in(Q.ts) >= Q.in(QI_TSLO);
    case 1: return Q.in(Q.ts) < Q.in(QI_TSHI);
    case 2: return Q.in(Q.ic) >= Q.in(QI_ICLO);
    case 3: return Q.in(Q.ic) < Q.in(QI_ICHI);
    case 4: return q_edil_out(Q.in(QI_EDLO), exp);
    case 5: return q_edil_out(exp, Q.in(QI_EDHI));
    case 6: { const uint64_t c = Q.in(QI_CUR), lo = Q.in(QI_BDLO);
      const QDate a = q_dec(lo), b = q_dec(birth);
      return q_dil_out(a.d, b.d, a.m, b.m, a.y + 100 * q_edil_out(lo, c), b.y + 100 * q_edil_out(birth, c)); }
    default: { const uint64_t c = Q.in(QI_CUR), hi = Q.in(QI_BDHI);
      const QDate a = q_dec(birth), b = q_dec(hi);
      return q_dil_out(a.d, b.d, a.m, b.m, a.y + 100 * q_edil_out(birth, c), b.y + 100 * q_edil_out(hi, c)); }
  }
}

// one signal of a query region (emit_small, regemit.hpp)
__device__ __forceinline__ El query_small(const DevLayout& L, const Bufs& B, const Region& R, uint32_t w, uint32_t s) {
  const RegInfo& G = L.reg;
  const QView Q = q_view(L, B.inputs, w);
  const bool td1 = G.q_td1 != 0;
  const int fcit = q_f_cit(td1);
  auto V = [&](int slot) { return fr_from_mont_fast(B.vs.at(slot, w)); };
  auto IN = [&](int k) { return el_load(Q.row + 32ull * k); };
  auto dg_u64 = [&](int k) { const fr v = V(G.q_dgf + k); return (uint64_t)v.v[0] | ((uint64_t)v.v[1] << 32); };
  const uint64_t sel = Q.in(QI_SEL);
  switch (R.kind) {
    case RK_Q_OUT: {
      if (s == 0) return (sel & 1) ? el_fr(V(G.q_nul)) : el_zero();
      const int k = (int)s - 1;
      if (!td1) return ((sel >> Q_OUT_SEL[k]) & 1) ? el_fr(V(G.q_dgf + k)) : el_zero();
      // TD1: fields 0-5, PoseidonHash(1) of documentNumber / personalNumber, documentType
      const int slot = k == 6 ? G.q_doch : k == 7 ? G.q_persh : G.q_dgf + (k == 8 ? 8 : k);
      return ((sel >> Q1_OUT_SEL[k]) & 1) ? el_fr(V(slot)) : el_zero();
    }
    case RK_Q_SQ: {
      const fr x = fr_to_mont(load_fr(Q.row + 32ull * QI_EVDATA));
      return el_fr(fr_from_mont_fast(fr_mul_fast(x, x)));
    }
    case RK_Q_CMP: {  // GreaterEqThan(64) (even) / LessThan(64) (odd) of (timestamp | identityCounter, bound)
      const int k = R.a[0];
      const int xi = k < 2 ? Q.ts : Q.ic, yi = k == 0 ? QI_TSLO : k == 1 ? QI_TSHI : k == 2 ? QI_ICLO : QI_ICHI;
      const uint64_t x = Q.in(xi), y = Q.in(yi);
      if (k & 1) return q_lt_sig((int)s, 64, IN(xi), IN(yi), q_v64(x, 0, y, 0));
      // out | in[2] | LessThan(64)(in[1], in[0] + 1)
      if (s == 0) return el_u64(x >= y);
      if (s == 1) return IN(xi);
      if (s == 2) return IN(yi);
      const uint64_t x1 = x + 1, x1h = x1 == 0;
      return q_lt_sig((int)s - 3, 64, IN(yi), el_fr(q_u128(x1, x1h)), q_v64(y, 0, x1, x1h));
    }
    case RK_Q_FEIE: {  // enabled, in[2] | IsEqual(in[0] = condition, in[1] = 1)
      const int k = R.a[0];
      const uint64_t c = (uint64_t)q_cond(Q, k, dg_u64(1), dg_u64(0));
      switch (s) {
        case 0: return el_u64((sel >> (8 + k)) & 1);
        case 2: case 5: return el_u64(1);
        case 7: case 8: return el_u64(1 - c);
        default: return el_u64(c);  // in[0], IsEqual.out, IsEqual.in[0], IsZero.out
      }
    }
    case RK_Q_EDIL: {
      const uint64_t exp = dg_u64(1);
      return R.a[0] == 0 ? q_edil_sig((int)s, B.inv_small, Q.in(QI_EDLO), exp)
                         : q_edil_sig((int)s, B.inv_small, exp, Q.in(QI_EDHI));
    }
    case RK_Q_EDILN: {
      const uint64_t birth = dg_u64(0), cur = Q.in(QI_CUR);
      return R.a[0] == 0 ? q_ediln_sig((int)s, B.inv_small, Q.in(QI_BDLO), birth, cur)
                         : q_ediln_sig((int)s, B.inv_small, birth, Q.in(QI_BDHI), cur);
    }
    case RK_Q_CIT: {  // citizenship, blacklist | validCheck[241], bitmask[240]
      if (s == 0) return el_fr(V(G.q_dgf + fcit));
      if (s == 1) return IN(QI_CMASK);
      if (s < 243) return el_u64((uint32_t)(s - 2) > B.vs.at(G.q_cidx, w).v[0]);
      const fr m = load_fr(Q.row + 32ull * QI_CMASK);
      return el_u64(q_bit(m, 239 - (int)(s - 243)));
    }
    default: {  // RK_Q_CITEQ: isEqual[i] (COUNTRY_ARR[i], citizenship), isEqual2[i] (1, bitmask[i])
      const uint32_t i = s / 12, r = s % 12;
      if (r < 6) return iseq_sig((int)r, Q_COUNTRY[i], dg_u64(fcit), V(G.q_cinv + (int)i));
      const fr m = load_fr(Q.row + 32ull * QI_CMASK);
      const uint32_t bm = q_bit(m, 239 - (int)i);
      const fr pm1 = fr_sub(fr_zero(), fr_u64(1));
      switch (r - 6) {
        case 1: return el_u64(1);
        case 4: case 5: return bm ? el_zero() : el_fr(pm1);  // in = bm - 1, inv = 1 / (bm - 1)
        default: return el_u64(bm);                          // out, in[1], IsZero.out
      }
    }
  }
}

// ============================================================================ k_qry_prep
// wave = witness, QP_WAVES witnesses per workgroup. DG1DataExtractor fields and the dg1 commitment chunks (Bits2Num
// over input bits, 64 per ballot as in k_prep), the citizenship's list index and the 240 IsEqual inverses (one batched
// inversion across the wave, whose single field inversion is shared by the workgroup's witnesses: wave 0 inverts
// the QP_WAVES wave totals at once — a wave inverting its own total spent ~75 % of the kernel's VALU on it), and the
// checks of the query templates: ForceEqualIfEnabled (19), DateDecoder re-encoding (20), CitizenshipCheck (21, 22),
// LessThan(8) ranges of the date comparisons (1), input range (64).
constexpr int QP_WAVES = 8;
#ifndef PZK_TEMPLATE_KERNELS_ONLY  // defined once, in kernels.hip
__global__ void __launch_bounds__(64 * QP_WAVES) k_qry_prep(DevLayout L, const uint8_t* inputs, ValueStore vs,
                                                            int32_t* status) {
  core_priority();
  __shared__ fr s_tot[QP_WAVES];
  const int wv = (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63);
  const uint32_t w0 = blockIdx.x * QP_WAVES + (uint32_t)wv;
  const bool live = w0 < vs.batch;  // a wave past the batch takes part in the barriers only
  const uint32_t w = live ? w0 : vs.batch - 1;
  const RegInfo& R = L.reg;
  const QView Q = q_view(L, inputs, w);
  const bool td1 = R.q_td1 != 0;
  bool bad = false;
  const bool wr = live && lane == 0;  // a wave past the batch stores nothing
  if (wr) vs.at(R.v_one, w) = fr_mont_one();
  uint64_t f64[9];
#pragma unroll
  for (int k = 0; k < 9; k++) {
    if (k == 8 && !td1) { f64[k] = 0; continue; }
    const int Lk = td1 ? Q1_DGX_L[k] : Q_DGX_L[k], Sk = td1 ? Q1_DGX_SHIFT[k] : Q_DGX_SHIFT[k];
    const fr v = wave_bits_fr(Q.row, QI_DG1 + Sk, Lk, -1, bad);
    f64[k] = (uint64_t)v.v[0] | ((uint64_t)v.v[1] << 32);
    if (wr) vs.at(R.q_dgf + k, w) = fr_to_mont(v);
  }
  const int CH = q_chunk(td1);
  for (int i = 0; i < 4; i++) {  // dg1Chunking[i] = Bits2Num(186 | 190), in[j] = dg1[CH i + j] (queryIdentity.circom:192-198)
    const fr v = wave_bits_fr(Q.row, QI_DG1 + CH * i, CH, +1, bad);
    if (wr) vs.at(R.v_dg1 + i, w) = fr_to_mont(v);
  }
  // CitizenshipCheck: index of the citizenship in COUNTRY_ARR and 1 / (citizenship - COUNTRY_ARR[i])
  const uint64_t cit = f64[q_f_cit(td1)];
  int first = 240;
  fr d[4], pre[4];
  // (run before and after the workgroup's inversion: arrays kept across its barriers went to scratch)
  auto forward = [&]() {
    fr a = fr_mont_one();
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int i = lane + 64 * j;
      const bool has = i < 240;
      const uint32_t ci = has ? Q_COUNTRY[i] : 0u;
      d[j] = has ? fr_to_mont(fr_sdiff(cit, ci)) : fr_zero();
      pre[j] = a;
      if (!fr_is_zero(d[j])) a = fr_mul(a, d[j]);
    }
    return a;
  };
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const int i = lane + 64 * j;
    const bool has = i < 240;
    const uint64_t m = __ballot(has && (has ? Q_COUNTRY[i] : 0u) == cit);
    if (m && first == 240) first = 64 * j + __builtin_ctzll(m);
  }
  const fr acc = forward();
  fr others, total;
  fr_group_others<64>(acc, others, total);
  // the workgroup's totals inverted together: lane k of wave 0 holds wave k's total (a lane past QP_WAVES one)
  if (lane == 0) s_tot[wv] = live ? total : fr_mont_one();
  __syncthreads();
  if (wv == 0) {
    const fr t = lane < QP_WAVES ? s_tot[lane] : fr_mont_one();
    fr t_others, t_all;
    fr_group_others<QP_WAVES>(t, t_others, t_all);
    const fr t_inv = fr_mul(fr_inv_sw<true>(t_all), t_others);  // = 1 / total of wave `lane`
    if (lane < QP_WAVES) s_tot[lane] = t_inv;  // (read above, by this wave only)
  }
  __syncthreads();
  if (!live) return;
  fr inv = fr_mul(s_tot[wv], others);  // = 1 / acc
  forward();
#pragma unroll
  for (int j = 3; j >= 0; j--) {
    const int i = lane + 64 * j;
    fr r = fr_zero();
    if (!fr_is_zero(d[j])) { r = fr_mul(inv, pre[j]); inv = fr_mul(inv, d[j]); }
    if (i < 240) vs.at(R.q_cinv + i, w) = r;
  }
  if (lane != 0) return;
  { fr ix = fr_zero(); ix.v[0] = (uint32_t)first; vs.at(R.q_cidx, w) = ix; }
  int32_t* st = status ? status + w : nullptr;
  // inputs read as 64-bit integers: bounds, dates, timestamp, counter (the evaluated domain)
  const int u64_in[11] = {QI_CUR, QI_TSLO, QI_TSHI, QI_ICLO, QI_ICHI, QI_BDLO, QI_BDHI, QI_EDLO, QI_EDHI, Q.ts, Q.ic};
  for (int k = 0; k < 11; k++) bad |= !in_is_u64(Q.row + 32ull * u64_in[k]);
  if (bad) set_status(st, ST_INPUT_RANGE);
  const uint64_t exp = f64[1], birth = f64[0], cur = Q.in(QI_CUR);
  // DateDecoder: dateEncoder.encoded === dateEncoded (dateDecoder.circom:22) for every decoded date
  const uint64_t dates[7] = {Q.in(QI_EDLO), exp, Q.in(QI_EDHI), Q.in(QI_BDLO), birth, Q.in(QI_BDHI), cur};
  for (int k = 0; k < 7; k++)
    if (q_enc(q_dec(dates[k])) != dates[k]) set_status(st, ST_DATE);
  // LessThan(8) of the date comparisons: Num2Bits(9) of a + 256 - b (comparators.circom:52-54)
  auto lt8_ok = [](int a, int b) { const int v = a + 256 - b; return v >= 0 && v < 512; };
  auto dil_ok = [&](const QDate& a, const QDate& b, int ya, int yb) {
    return lt8_ok(ya, yb) && lt8_ok(a.m, b.m) && lt8_ok(a.d, b.d);
  };
  bool rng = true;
  const uint64_t pairs[4][2] = {{Q.in(QI_EDLO), exp}, {exp, Q.in(QI_EDHI)}, {Q.in(QI_BDLO), birth}, {birth, Q.in(QI_BDHI)}};
  for (int k = 0; k < 4; k++) {
    const QDate a = q_dec(pairs[k][0]), b = q_dec(pairs[k][1]);
    rng &= dil_ok(a, b, a.y, b.y);
    if (k >= 2) {
      const QDate c = q_dec(cur);
      rng &= dil_ok(a, c, a.y, c.y) && dil_ok(b, c, b.y, c.y);
      rng &= dil_ok(a, b, a.y + 100 * q_edil_out(pairs[k][0], cur), b.y + 100 * q_edil_out(pairs[k][1], cur));
    }
  }
  if (!rng) set_status(st, ST_NUM2BITS);
  // ForceEqualIfEnabled: (1 - cond) * selector[8 + k] === 0 (comparators.circom:42)
  const uint64_t sel = Q.in(QI_SEL);
  for (int k = 0; k < 8; k++)
    if (((sel >> (8 + k)) & 1) && !q_cond(Q, k, exp, birth)) set_status(st, ST_QUERY);
  // CitizenshipCheck (citizenshipCheck.circom:271,274)
  if (first == 240) set_status(st, ST_CIT_LIST);
  else if (q_bit(load_fr(Q.row + 32ull * QI_CMASK), 239 - first)) set_status(st, ST_CIT_BLACKLIST);
}
#endif

}  // namespace pzk
