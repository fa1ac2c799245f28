// Emit (signal-parallel) generators of the RegisterIdentityBuilder regions.
//
// Every function maps a region-local signal index to its value in closed form from the
// per-witness cores (regcore.hpp, sha.hpp, poseidon.hpp) — no sequential dependency, so
// consecutive lanes store consecutive 32-byte witness elements.
#pragma once
#include "bufs.hpp"
#include "fr.hpp"
#include "layout.hpp"
#include "poseidon.hpp"
#include "regcore.hpp"
#include "sha.hpp"
#include "mm_prog.hpp"
#include "ec_emit.hpp"
#include "pss.hpp"
#include "mapsink.hpp"
#include "query.hpp"

namespace pzk {


// ------------------------------------------------------------------ 256-bit helpers
struct W256 { uint32_t v[8]; };
__device__ __forceinline__ W256 w_zero() { W256 r; for (int i = 0; i < 8; i++) r.v[i] = 0; return r; }
__device__ __forceinline__ W256 w_u64(uint64_t x) { W256 r = w_zero(); r.v[0] = (uint32_t)x; r.v[1] = (uint32_t)(x >> 32); return r; }
__device__ __forceinline__ W256 w_mask(const W256& a, int nbits) {  // a mod 2^nbits
  W256 r = a;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    int lo = 32 * i;
    if (nbits <= lo) r.v[i] = 0;
    else if (nbits < lo + 32) r.v[i] &= (1u << (nbits - lo)) - 1u;
  }
  return r;
}
// word k of a (select chain: a runtime index into a register array would go to scratch, and a
// scratch load inside an emit loop waits for every store in flight)
__device__ __forceinline__ uint32_t w_word(const W256& a, int k) {
  // AND/OR with lane masks rather than selects, which LLVM folds back into a scratch lookup
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r |= a.v[i] & (0u - (uint32_t)(k == i));
  return r;
}
__device__ __forceinline__ uint32_t w_bit(const W256& a, int i) { return (w_word(a, i >> 5) >> (i & 31)) & 1u; }
__device__ __forceinline__ void store_w(uint8_t* dst, const W256& a) {
  uint4* d = reinterpret_cast<uint4*>(dst);
  d[0] = make_uint4(a.v[0], a.v[1], a.v[2], a.v[3]);
  d[1] = make_uint4(a.v[4], a.v[5], a.v[6], a.v[7]);
}
__device__ __forceinline__ El el_w(const W256& a) {
  return El{make_uint4(a.v[0], a.v[1], a.v[2], a.v[3]), make_uint4(a.v[4], a.v[5], a.v[6], a.v[7])};
}
__device__ __forceinline__ W256 w_from_fr(const fr& a) { W256 r; for (int i = 0; i < 8; i++) r.v[i] = a.v[i]; return r; }
__device__ __forceinline__ fr fr_from_w(const W256& a) { fr r; for (int i = 0; i < 8; i++) r.v[i] = a.v[i]; return r; }
__device__ __forceinline__ void copy_el(uint8_t* dst, const uint8_t* src) {
  const uint4* s4 = reinterpret_cast<const uint4*>(src);
  uint4* d4 = reinterpret_cast<uint4*>(dst);
  d4[0] = s4[0]; d4[1] = s4[1];
}
__device__ __forceinline__ const uint32_t* sha_hout(const DevLayout& L, const Bufs& B, uint32_t w, int job) {
  const ShaJob& J = L.sha[job];
  return B.sha_core + (size_t)w * L.sha_core_words + J.hout;
}
__device__ __forceinline__ uint32_t digest_bit(const uint32_t* H, int i) { return (H[i >> 5] >> (31 - (i & 31))) & 1u; }

// ------------------------------------------------------------------ generic small regions
// returns true and writes the element; the value source is per kind
__device__ __forceinline__ El emit_small(const DevLayout& L, const Bufs& B, const Region& R, uint32_t w, uint32_t s) {
  const RegInfo& G = L.reg;
  const uint8_t* row = B.inputs + 32ull * (uint64_t)w * L.n_inputs;
  const fr* smt = B.smt_core + (size_t)w * L.smt_core_fr;
  const uint32_t* flags = reinterpret_cast<const uint32_t*>(smt + 2 * SMT_LEVELS);
  auto V = [&](int slot) { return fr_from_mont_fast(B.vs.at(slot, w)); };
  switch (R.kind) {
    case RK_ONE: return el_u64(1);
    case RK_INCOPY: return el_load(row + 32ull * ((uint64_t)R.a[0] + s));
    case RK_VALUE: {
      int slot = R.a[0] >= 0 ? R.a[0] + (int)s : R.a[0] == -2 ? -2 : R.a[1 + s];
      if (slot < 0) return el_u64(0);
      else return el_fr(V(slot));
    }
    case RK_DIGEST: return el_u64(digest_bit(sha_hout(L, B, w, R.a[0]), (int)s));
    case RK_TEMPMOD: {
      const uint8_t* a = row + 32ull * (R.a[0] + 3 * s);
      const uint8_t* b = row + 32ull * (R.a[0] + 3 * s + 1);
      if (in_is_u64(a) && in_is_u64(b)) {
        uint64_t la = in_u64(a), lb = in_u64(b);
        W256 r = w_zero();
        r.v[2] = (uint32_t)lb; r.v[3] = (uint32_t)(lb >> 32); r.v[4] = (uint32_t)la; r.v[5] = (uint32_t)(la >> 32);
        return el_w(r);
      } else {
        fr t64 = fr_zero(); t64.v[2] = 1;
        fr t128 = fr_zero(); t128.v[4] = 1;
        fr v = fr_add(fr_mul_fast(fr_to_mont(load_fr(a)), fr_to_mont(t128)), fr_mul_fast(fr_to_mont(load_fr(b)), fr_to_mont(t64)));
        return el_fr(fr_from_mont_fast(v));
      }
    }
    case RK_HCHUNK: {  // chunk s = digest bits [cs (n-1-s), cs (n-s)) as a number (rsa.circom:84-91, ecdsa.circom:30-38)
      const uint32_t* H = sha_hout(L, B, w, R.a[0]);
      const int n = R.a[1], cs = R.a[2], i = n - 1 - (int)s;
      return el_u64(cs == 64 ? ((uint64_t)H[2 * i] << 32) | H[2 * i + 1] : H[i]);
    }
    case RK_RSA_OUT: {
      const uint64_t* mc = B.rsa_core + (size_t)w * L.rsa_core_words + (size_t)(G.n_modmul - 1) * MM_CORE_WORDS(G.K);
      return el_u64(mc[3 * G.K + 1 + s]);
    }
    case RK_SMT_OWN: {  // isVerified | root, leaf, key, siblings[80] | value
      if (s == 0) {
        fr r0 = fr_from_mont_fast(smt[SMT_LEVELS]);
        return el_u64(fr_eq(r0, load_fr(row + 32ull * R.a[0])) ? 1 : 0);
      } else if (s == 1) return el_load(row + 32ull * R.a[0]);
      else if (s == 3) return el_fr(V(G.v_smt_key));
      else if (s == 2 || s == 84) return el_fr(V(G.v_smt_val));
      else return el_load(row + 32ull * (R.a[1] + s - 4));
    }
    case RK_SMTHASH: {
      int lv = R.a[0];
      if (lv < 0) return el_fr(s == 0 ? V(G.v_leaf) : s == 1 ? V(G.v_smt_key) : V(G.v_smt_val));
      else return el_fr(s == 0 ? V(G.v_smt_h + lv) : V(G.v_smt_lr + 2 * lv + (int)s - 1));
    }
    case RK_LEVINS: {  // levIns[80] | siblings[80] | done[79] | isZero[80] (out, in, inv)
      if (s < 80) { return el_u64(flags[s] & 1); }
      if (s < 160) { return el_load(row + 32ull * (R.a[0] + s - 80)); }
      if (s < 239) { return el_u64((flags[s - 160] >> 1) & 1); }
      uint32_t i = (s - 239) / 3, k = (s - 239) % 3;
      if (k == 0) return el_u64((flags[i] >> 5) & 1);
      else if (k == 1) return el_load(row + 32ull * (R.a[0] + i));
      else return el_fr(smt[i]);
    }
    case RK_SM: {  // st_top, st_inew | levIns, prev_top
      uint32_t i = s >> 2, k = s & 3;
      uint32_t v = k == 0 ? (flags[i] >> 2) & 1 : k == 1 ? (flags[i] >> 3) & 1 : k == 2 ? flags[i] & 1
                                                                              : (i == 0 ? 1u : (flags[i - 1] >> 2) & 1);
      return el_u64(v);
    }
    case RK_SMT_LEVEL: {  // root | st_top, st_inew, sibling, new1leaf, lrbit, child | fromProof
      int i = R.a[0];
      uint32_t f = flags[i];
      switch (s) {
        case 0: return el_fr(fr_from_mont_fast(smt[SMT_LEVELS + i]));
        case 1: return el_u64((f >> 2) & 1);
        case 2: return el_u64((f >> 3) & 1);
        case 3: return el_load(row + 32ull * (R.a[1] + i));
        case 4: return el_fr(V(G.v_leaf));
        case 5: return el_u64((f >> 4) & 1);
        case 6: return el_fr(i == SMT_LEVELS - 1 ? fr_zero() : fr_from_mont_fast(smt[SMT_LEVELS + i + 1]));
        default: return el_fr((f & 4) ? V(G.v_smt_h + i) : fr_zero());
      }
    }
    case RK_SWITCHER: {  // out[2] | bool, in[2] | aux
      int i = R.a[0];
      uint32_t lr = (flags[i] >> 4) & 1;
      if (s < 2) { return el_fr(V(G.v_smt_lr + 2 * i + (int)s)); }
      if (s == 2) { return el_u64(lr); }
      fr child = i == SMT_LEVELS - 1 ? fr_zero() : fr_from_mont_fast(smt[SMT_LEVELS + i + 1]);
      fr sib = load_fr(row + 32ull * (R.a[1] + i));
      if (s == 3) return el_fr(child);
      else if (s == 4) return el_load(row + 32ull * (R.a[1] + i));
      else return el_fr(lr ? fr_sub(sib, child) : fr_zero());
    }
    case RK_ISEQ_ROOT: {  // out | in[2] | IsZero(out, in, inv)
      fr r0 = fr_from_mont_fast(smt[SMT_LEVELS]);
      fr rin = load_fr(row + 32ull * R.a[0]);
      uint32_t eq = fr_eq(r0, rin);
      if (s == 0 || s == 3) return el_u64(eq);
      else if (s == 1) return el_fr(r0);
      else if (s == 2) return el_load(row + 32ull * R.a[0]);
      else if (s == 4) return el_fr(fr_sub(rin, r0));
      else return el_fr(fr_from_mont_fast(smt[3 * SMT_LEVELS + 1]));
    }
    case RK_BJJ_OWN: {  // out[2] | scalar | base8[2]
      const fr* bc = B.bjj_core + (size_t)w * L.bjj_core_fr + 5 * (BJJ_STEPS - 1);
      if (s < 2) return el_fr(fr_from_mont_fast(bc[2 + s]));
      else if (s == 2) return el_fr(V(G.v_sk));
      else {
        W256 r; for (int i = 0; i < 8; i++) r.v[i] = s == 3 ? BJJ_B8X[i] : BJJ_B8Y[i];
        return el_w(r);
      }
    }
    case RK_PSS_OWN: case RK_PSS_B2N8: case RK_PSS_MGF: case RK_PSS_CTR: case RK_PSS_XOR:
      return pss_small(pss_view(L, B.rsa_core, B.sha_core, w), R, s);
    default: return ec_small(L, B, R, w, s);
  }
}

// ------------------------------------------------------------------ Bits2Num / Num2Bits (+ AliasCheck)
// one workgroup per (region, witness): the L-bit value is assembled in LDS first.
// CompConstant(p-1) part i (compconstant.circom:28-46): a = 2^i, b = 2^128 - 2^i
__device__ __forceinline__ void alias_part(const W256& bits, int i, uint64_t& lo, uint64_t& hi) {
  W256 pm1; for (int k = 0; k < 8; k++) pm1.v[k] = P_[k];
  pm1.v[0] -= 1;
  const uint32_t cl = w_bit(pm1, 2 * i), cm = w_bit(pm1, 2 * i + 1);  // (pm1.v[run-time index] went to scratch)
  uint32_t sl = w_bit(bits, 2 * i), sm = w_bit(bits, 2 * i + 1);
  // which of {0, a, b}
  int sel;
  if (!cm && !cl) sel = (sm | sl) ? 2 : 0;
  else if (!cm && cl) sel = sm ? 2 : (sl ? 0 : 1);
  else if (cm && !cl) sel = sm ? (sl ? 2 : 0) : 1;
  else sel = (sm & sl) ? 0 : 1;
  uint64_t alo = i < 64 ? (1ull << i) : 0, ahi = i >= 64 ? (1ull << (i - 64)) : 0;
  if (sel == 0) { lo = 0; hi = 0; }
  else if (sel == 1) { lo = alo; hi = ahi; }
  else { lo = 0 - alo; hi = ~0ull - ahi + (alo == 0 ? 1 : 0); if (alo == 0) hi = 0 - ahi; }
}

__device__ __forceinline__ W256 u192_w(const uint64_t* a) {
  W256 r = w_zero();
  for (int i = 0; i < 3; i++) { r.v[2 * i] = (uint32_t)a[i]; r.v[2 * i + 1] = (uint32_t)(a[i] >> 32); }
  return r;
}

// AliasCheck block (908 signals) over bits of V; sout precomputed
__device__ __forceinline__ W256 alias_sig(const W256& V, const uint64_t* sout, uint32_t s) {
  if (s < 254) return w_u64(w_bit(V, s));                   // AliasCheck.in
  s -= 254;
  W256 so = u192_w(sout);
  if (s == 0) return w_u64(w_bit(so, 127));                 // CompConstant.out
  if (s < 255) return w_u64(w_bit(V, s - 1));               // CompConstant.in
  if (s < 382) { uint64_t lo, hi; alias_part(V, s - 255, lo, hi); W256 r = w_zero();
    r.v[0] = (uint32_t)lo; r.v[1] = (uint32_t)(lo >> 32); r.v[2] = (uint32_t)hi; r.v[3] = (uint32_t)(hi >> 32); return r; }
  if (s == 382) return so;                                  // sout
  s -= 383;                                                 // Num2Bits(135)(sout)
  if (s < 135) return w_u64(w_bit(so, s));
  if (s == 135) return so;
  return w_mask(so, (int)s - 135);
}

#ifndef PZK_TEMPLATE_KERNELS_ONLY  // defined once, in kernels.hip
__global__ void __launch_bounds__(256) k_emit_bits(DevLayout L, const Work* work, Bufs B) {
  __shared__ uint32_t val[8];
  __shared__ uint64_t sout[3];
  __shared__ fr inval;
  const Work wk = work[blockIdx.x];
  const uint32_t w = blockIdx.y;
  const Region R = L.regions[wk.region];
  const int Lb = R.a[0];
  const uint8_t* row = B.inputs + 32ull * (uint64_t)w * L.n_inputs;
  if (threadIdx.x < 8) val[threadIdx.x] = 0;
  if (threadIdx.x < 3) sout[threadIdx.x] = 0;
  __syncthreads();
  const bool b2n = R.kind == RK_BITS2NUM;
  const uint32_t* H = (b2n && R.a[1] == 1) ? sha_hout(L, B, w, R.a[4]) : nullptr;
  // bit sources: 0 input elements, 1 digest bits of SHA job a4 (index < 0: a zero, the SHA-1 passportHash
  // padding), 2 bits of EM limb a4 (RSA core)
  const uint64_t emw = (b2n && R.a[1] == 2)
      ? B.rsa_core[(size_t)w * L.rsa_core_words + (size_t)(L.reg.n_modmul - 1) * MM_CORE_WORDS(L.reg.K) + 3 * L.reg.K + 1 + R.a[4]]
      : 0ull;
  auto src_bit = [&](int j) -> uint32_t {
    int idx = R.a[2] + R.a[3] * j;
    if (R.a[1] == 1) return idx < 0 ? 0u : digest_bit(H, idx);
    if (R.a[1] == 2) return (uint32_t)(emw >> idx) & 1u;
    return *(row + 32ull * idx) & 1u;
  };
  if (b2n) {
    for (int j = threadIdx.x; j < Lb; j += blockDim.x)
      if (src_bit(j)) atomicOr(&val[j >> 5], 1u << (j & 31));
  } else if (threadIdx.x == 0) {
    fr v;
    if (R.a[1] == 0) v = fr_from_mont_fast(B.vs.at(R.a[2], w));
    else v = fr_u64(B.rsa_core[(size_t)w * L.rsa_core_words + (size_t)(L.reg.n_modmul - 1) * MM_CORE_WORDS(L.reg.K) +
                               3 * L.reg.K + 1 + R.a[2]]);
    inval = v;
    for (int i = 0; i < 8; i++) val[i] = v.v[i];
    // bits beyond L are ignored by Num2Bits' outputs; in === sum is checked against the full value
    W256 vv; for (int i = 0; i < 8; i++) vv.v[i] = v.v[i];
    W256 m = w_mask(vv, Lb);
    bool ok = true; for (int i = 0; i < 8; i++) ok &= m.v[i] == vv.v[i];
    if (!ok && B.status) lane_status(B.status + w, ST_NUM2BITS);
  }
  __syncthreads();
  W256 V; for (int i = 0; i < 8; i++) V.v[i] = val[i];
  if (Lb == 254) {
    // CompConstant's sum of its 127 parts: one part per thread, summed as four 32-bit columns in LDS (127 * 2^32
    // fits 64 bits), then one carry pass (a serial 127-step loop on thread 0 held the whole workgroup)
    __shared__ unsigned long long col[4];
    if (threadIdx.x < 4) col[threadIdx.x] = 0;
    __syncthreads();
    if (threadIdx.x < 127) {
      uint64_t lo, hi;
      alias_part(V, threadIdx.x, lo, hi);
      atomicAdd(&col[0], (unsigned long long)(uint32_t)lo);
      atomicAdd(&col[1], (unsigned long long)(lo >> 32));
      atomicAdd(&col[2], (unsigned long long)(uint32_t)hi);
      atomicAdd(&col[3], (unsigned long long)(hi >> 32));
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t l[6];
      uint64_t c = 0;
      for (int k = 0; k < 4; k++) { c += col[k]; l[k] = (uint32_t)c; c >>= 32; }
      l[4] = (uint32_t)c; l[5] = (uint32_t)(c >> 32);
      uint64_t acc[3];
      for (int k = 0; k < 3; k++) acc[k] = (uint64_t)l[2 * k] | ((uint64_t)l[2 * k + 1] << 32);
      sout[0] = acc[0]; sout[1] = acc[1]; sout[2] = acc[2];
      W256 so = u192_w(acc);
      if (w_bit(so, 127) && B.status) lane_status(B.status + w, ST_ALIAS);
    }
    __syncthreads();
  }
  const OutRow out = out_row(L, B.wtns, B.stride, w, R.off + wk.start);
  __shared__ uint4 stage[2 * 256];
  emit_run(out, wk.count, stage, [&](uint32_t q) -> El {
    uint32_t s = wk.start + q;
    if (s > 2u * Lb) return el_w(alias_sig(V, sout, s - 2 * Lb - 1));
    if (b2n) {
      if (s == 0) return el_w(V);
      if (s <= (uint32_t)Lb) {
        int idx = R.a[2] + R.a[3] * (int)(s - 1);
        return R.a[1] == 1 ? el_u64(idx < 0 ? 0u : digest_bit(H, idx)) : R.a[1] == 2 ? el_u64((emw >> idx) & 1u)
                                                                                  : el_load(row + 32ull * idx);
      }
      return el_w(w_mask(V, (int)(s - Lb)));
    }
    if (s < (uint32_t)Lb) return el_u64(w_bit(V, s));
    if (s == (uint32_t)Lb) return el_fr(inval);
    return el_w(w_mask(V, (int)(s - Lb)));
  });
}
#endif

// ------------------------------------------------------------------ PassportVerificationFlow
#ifndef PZK_TEMPLATE_KERNELS_ONLY  // defined once, in kernels.hip
__global__ void __launch_bounds__(256) k_emit_flow(DevLayout L, const Work* work, Bufs B) {
  __shared__ uint8_t eq[3 * 512 + 8], chain[3 * 512 + 8];  // 3 DG + 8 IsEqual, DG <= 512
  __shared__ fr invV;  // 1 / DG15_VERIFICATION (normal form): IsZero inverses of the scaled DG15 checks
  const Work wk = work[blockIdx.x];
  const uint32_t w = blockIdx.y;
  const Region R = L.regions[wk.region];
  const int jd1 = R.a[0], jd15 = R.a[1], jec = R.a[2], jsa = R.a[3], in_ec = R.a[4], in_sa = R.a[5];
  const int d1s = R.a[6], d15s = R.a[7], ecs = R.a[8], V = R.a[9];
  const int ecLen = (L.sha[jec].algo >= 3 ? 1024 : 512) * L.sha[jec].blocks;
  auto hbits = [&](int j) {
    const int a = L.sha[j].algo;
    return a == 1 ? 160 : a == 2 ? 224 : a == 3 ? 384 : a == 4 ? 512 : 256;
  };
  const int H = hbits(jd1), EH = hbits(jec), NC = 3 * H + 8;
  const uint8_t* row = B.inputs + 32ull * (uint64_t)w * L.n_inputs;
  const uint32_t* H1 = sha_hout(L, B, w, jd1);
  const uint32_t* H15 = jd15 >= 0 ? sha_hout(L, B, w, jd15) : nullptr;
  const uint32_t* HE = sha_hout(L, B, w, jec);
  auto ebit = [&](int i) -> uint32_t { return *(row + 32ull * (in_ec + i)) & 1u; };
  auto sbit = [&](int i) -> uint32_t { return *(row + 32ull * (in_sa + i)) & 1u; };
  auto pair = [&](int k, uint32_t& a, uint32_t& b) {  // IsEqual k: in[0], in[1]
    const int g = k < 3 * H ? k / H : 3, i = k - g * H;
    if (g == 0) { a = digest_bit(H1, i); b = ebit(d1s + i); }
    else if (g == 1) { a = H15 ? digest_bit(H15, i) * V : 0; b = ebit(d15s + i) * V; }
    else if (g == 2) { a = digest_bit(HE, i); b = sbit(ecs + i); }
    else { a = (i >= 4 ? 1u : 0u) * V; b = ebit(d15s - 24 + i) * V; }  // 0x0F prefix, MSB first
  };
  for (int k = threadIdx.x; k < NC; k += blockDim.x) { uint32_t a, b; pair(k, a, b); eq[k] = a == b; }
  if (threadIdx.x == 0) invV = V > 1 ? fr_from_mont_fast(fr_inv(fr_to_mont(fr_u64((uint64_t)V)))) : fr_u64(1);
  __syncthreads();
  if (threadIdx.x == 0) {
    uint8_t c = 1;
    for (int k = 0; k < NC; k++) { c &= eq[k]; chain[k] = c; }
    if (!c && B.status) lane_status(B.status + w, ST_FLOW);
  }
  __syncthreads();
  const OutRow out = out_row(L, B.wtns, B.stride, w, R.off + wk.start);
  const uint32_t o_d1 = 1, o_d15 = 1 + H, o_ec = 1 + 2 * H, o_eh = o_ec + ecLen, o_sa = o_eh + EH, o_v = o_sa + 1024,
                 o_eq = o_v + NC;
  __shared__ uint4 stage[2 * 256];
  emit_run(out, wk.count, stage, [&](uint32_t q) -> El {
    uint32_t s = wk.start + q;
    if (s == 0) return el_u64(chain[NC - 1]);
    if (s < o_d15) return el_u64(digest_bit(H1, s - o_d1));
    if (s < o_ec) return el_u64(H15 ? digest_bit(H15, s - o_d15) : 0);
    if (s < o_eh) return el_load(row + 32ull * (in_ec + s - o_ec));
    if (s < o_sa) return el_u64(digest_bit(HE, s - o_eh));
    if (s < o_v) return el_load(row + 32ull * (in_sa + s - o_sa));
    if (s < o_eq) return el_u64(chain[s - o_v]);
    uint32_t k = (s - o_eq) / 6, t = (s - o_eq) % 6;
    uint32_t a, b; pair(k, a, b);
    // IsEqual: out | in[0], in[1] | IsZero: out, in = in[1]-in[0], inv
    if (t == 0 || t == 3) return el_u64(a == b);
    if (t == 1) return el_u64(a);
    if (t == 2) return el_u64(b);
    // in = in[1] - in[0] in {-1, 0, 1} (scale 1) or {-V, 0, V} (DG15 checks, V = AA_SIGNATURE_ALGO)
    const int d = (int)b - (int)a, ad = d < 0 ? -d : d;
    const fr m = t == 4 ? fr_u64((uint64_t)ad) : ad <= 1 ? fr_u64((uint64_t)ad) : invV;
    return d >= 0 ? el_fr(m) : el_fr(fr_sub(fr_zero(), m));
  });
}
#endif

// ------------------------------------------------------------------ BigMultModP
// Karatsuba input table (K = 32): the in1/in2 values of every non-root KaratsubaOverflow node
// (bigIntHelpers.circom:11-53), level by level; node m of level l holds in1[N_l] then in2[N_l],
// N_l = K >> l. A value is a sum of up to 2^l limbs: lo 64 bits + a small high part. Level l
// starts at value kt_base(l) = sum_{i<l} 3^i 2 N_i (i >= 1): 0, 96, 240, 456, 780; 1266 in all.
constexpr int KT_K = 32, KT_LEVELS = 5, KT_VALUES = 1266;

struct MMCore {
  int K;
  const uint64_t *x, *y, *q, *r, *n, *inv, *cr;  // LDS
  const uint64_t *cxy, *cqn;                      // LDS: column sums of x*y (2K-1) and q*n (2K), 3 words each
  bool kara;                                      // x*y by KaratsubaOverflow (K = 2^m), else schoolbook
  const uint64_t* kt_lo;                          // LDS Karatsuba input table (K = 32 / 64; else null)
  const uint8_t* kt_hi;
  const uint32_t* ko;                             // LDS node outputs of the upper Karatsuba levels, 5 words each (ko5_at;
                                                  // K = 32 / 64; else null)
  __device__ __forceinline__ uint64_t X(int i) const { return i < K ? x[i] : 0; }
};
__device__ __forceinline__ U192 u192_at(const uint64_t* a, int i) { U192 r; r.a0 = a[3 * i]; r.a1 = a[3 * i + 1]; r.a2 = a[3 * i + 2]; return r; }
// a Karatsuba node output (< 2^139) in 5 LDS words: 20 instead of 24 bytes per value, so the mapped / O0 k_emit_mm<32>
// fits five workgroups per CU
__device__ __forceinline__ U192 ko5_at(const uint32_t* a, int i) {
  const uint32_t* p = a + 5 * i;
  U192 r;
  r.a0 = (uint64_t)p[0] | ((uint64_t)p[1] << 32);
  r.a1 = (uint64_t)p[2] | ((uint64_t)p[3] << 32);
  r.a2 = p[4];
  return r;
}
__device__ __forceinline__ void u192_addto(U192& a, const U192& b) {
  uint64_t s0 = a.a0 + b.a0; uint64_t c = s0 < b.a0;
  uint64_t s1 = a.a1 + b.a1; uint64_t c1 = s1 < b.a1; uint64_t s1b = s1 + c; c1 += s1b < s1;
  a.a0 = s0; a.a1 = s1b; a.a2 += b.a2 + c1;
}
__device__ __forceinline__ U192 u192_shfl_up(const U192& v, unsigned d) {
  U192 r;
  r.a0 = ((uint64_t)(uint32_t)__shfl_up((int)(uint32_t)(v.a0 >> 32), d, 64) << 32) | (uint32_t)__shfl_up((int)(uint32_t)v.a0, d, 64);
  r.a1 = ((uint64_t)(uint32_t)__shfl_up((int)(uint32_t)(v.a1 >> 32), d, 64) << 32) | (uint32_t)__shfl_up((int)(uint32_t)v.a1, d, 64);
  r.a2 = ((uint64_t)(uint32_t)__shfl_up((int)(uint32_t)(v.a2 >> 32), d, 64) << 32) | (uint32_t)__shfl_up((int)(uint32_t)v.a2, d, 64);
  return r;
}

// U192 += (alo + ahi 2^64) * (blo + bhi 2^64), ahi, bhi < 2^8
__device__ __forceinline__ void mac2(U192& acc, uint64_t alo, uint64_t ahi, uint64_t blo, uint64_t bhi) {
  acc.mac(alo, blo);
  uint64_t m1 = alo * bhi, m1h = __umul64hi(alo, bhi), m2 = blo * ahi, m2h = __umul64hi(blo, ahi);
  uint64_t s = acc.a1 + m1; uint64_t c = s < m1; uint64_t s2 = s + m2; c += s2 < s; acc.a1 = s2;
  acc.a2 += m1h + m2h + c + ahi * bhi;
}
__device__ __forceinline__ W256 u192w(const U192& a) {
  W256 r = w_zero();
  r.v[0] = (uint32_t)a.a0; r.v[1] = (uint32_t)(a.a0 >> 32); r.v[2] = (uint32_t)a.a1; r.v[3] = (uint32_t)(a.a1 >> 32);
  r.v[4] = (uint32_t)a.a2; r.v[5] = (uint32_t)(a.a2 >> 32);
  return r;
}
// signed 256-bit (two's complement in W256) -> normal-form field element
__device__ __forceinline__ W256 w_signed_to_fr(const W256& a) {
  if (!(a.v[7] >> 31)) return a;
  W256 m; uint64_t c = 1;
  for (int i = 0; i < 8; i++) { uint64_t t = (uint64_t)(~a.v[i]) + c; m.v[i] = (uint32_t)t; c = t >> 32; }
  return w_from_fr(fr_sub(fr_zero(), fr_from_w(m)));
}
__device__ __forceinline__ W256 w_sub(const W256& a, const W256& b) {
  W256 r; uint64_t br = 0;
  for (int i = 0; i < 8; i++) { uint64_t d = (uint64_t)a.v[i] - b.v[i] - br; r.v[i] = (uint32_t)d; br = (d >> 32) & 1; }
  return r;
}

// BigMultNonEqualOverflow(G, L) tmpResult[i][j] of a (G limbs) x b (L limbs), G >= L
// (bigIntHelpers.circom:55-124): a running sum along row i. Consecutive signals of a row sit in
// consecutive lanes, so each lane forms its own term and a segmented inclusive scan across the wave
// adds the earlier ones; the row's terms before this wave (if the row started in an earlier wave)
// are added by the wave's first lane.
__device__ __forceinline__ W256 bmneq_tmpr(const uint64_t* a, int G, const uint64_t* b, int L, uint32_t s) {
  const int i = s / L, j = s - i * L, lane = threadIdx.x & 63;
  auto term = [&](int t) -> U192 {
    U192 acc;
    if (i < G) { if (t <= i) acc.mac(a[i - t], b[t]); }
    else if (t < G + L - 1 - i) acc.mac(a[G - 1 - t], b[i + t - G + 1]);
    return acc;
  };
  U192 v = term(j);
  if (lane == 0)
    for (int t = 0; t < j; t++) u192_addto(v, term(t));
  for (unsigned dd = 1; dd < 64; dd <<= 1) {
    U192 o = u192_shfl_up(v, dd);
    if ((int)dd <= j && (unsigned)lane >= dd) u192_addto(v, o);
  }
  if (i < L ? j > i : (i >= G && j >= G + L - 1 - i)) return w_zero();
  return u192w(v);
}

// BigMultModP(64,K,K,K) block signal (bigInt.circom:206-272), addressed by the block program
// (mm_prog.hpp): section + index within the section, so the emitter does no range cascade.
__device__ __forceinline__ W256 mm_sig(const MMCore& C, uint32_t d) {
  const int K = C.K, DIV = K + 1;
  const uint32_t s = d & 0xFFFFFFu;
  auto le_result = [&](int upto) -> uint32_t {
    uint32_t res = 0;
    for (int i = 0; i <= upto; i++) {
      uint32_t lt = C.n[i] < C.r[i], e = C.n[i] == C.r[i];
      res = i == 0 ? lt + e : lt + e * res;
    }
    return res;
  };
  switch (d >> 24) {
    case MM_Q: return w_u64(C.q[s]);                                   // div[DIV]
    case MM_R: return w_u64(C.r[s]);                                   // mod[K]
    case MM_XYN: { int g = s / K, i = s - g * K; return w_u64(g == 0 ? C.x[i] : g == 1 ? C.y[i] : C.n[i]); }
    case MM_MOUT: return u192w(u192_at(C.cxy, (int)s));                // mult.out = x*y columns
    case MM_MCOPY: return w_u64(s < (uint32_t)K ? C.x[s] : C.y[s - K]);
    case MM_KARA: {  // K = 32 / 64 (KaratsubaOverflow) go to kara_el32 / kara_el64 (mm_el)
      // BigMultNonEqualOverflow(K, K) of x, y: out[2K-1] | in1[K], in2[K] | tmpMults[K][K] | tmpResult[2K-1][K]
      uint32_t e = s;
      if (e < (uint32_t)(2 * K - 1)) return u192w(u192_at(C.cxy, (int)e));
      e -= 2 * K - 1;
      if (e < (uint32_t)(2 * K)) return w_u64(e < (uint32_t)K ? C.x[e] : C.y[e - K]);
      e -= 2 * K;
      if (e < (uint32_t)(K * K)) { const uint32_t i = e / K, j = e - i * K; U192 acc; acc.mac(C.x[i], C.y[j]); return u192w(acc); }
      return bmneq_tmpr(C.x, K, C.y, K, e - K * K);
    }
    case MM_MODCHK: {  // Num2Bits(64)(mod_i): out[64] | in | sum[64]
      uint32_t i = s / 129, t = s - 129 * i;
      uint64_t v = C.r[i];
      if (t < 64) return w_u64((v >> t) & 1);
      if (t == 64) return w_u64(v);
      return w_u64(v & mask_lo((int)t - 64));
    }
    case MM_GT0: return w_u64(1 - le_result(K - 1));                   // greaterThan.out
    case MM_GTIN: case MM_LEIN: return w_u64(s < (uint32_t)K ? C.n[s] : C.r[s - K]);
    case MM_LE0: return w_u64(le_result(K - 1));
    case MM_LERES: return w_u64(le_result((int)s));
    case MM_LT: {
      uint32_t i = s / 140, t = s - 140 * i;
      uint64_t a = C.n[i], b = C.r[i];
      if (t < 134) {  // LessThan(64): out | in[2] | Num2Bits(65)(a + 2^64 - b)
        uint64_t vlo = a - b; uint32_t vhi = a >= b ? 1u : 0u;
        if (t == 0) return w_u64(1 - vhi);
        if (t == 1) return w_u64(a);
        if (t == 2) return w_u64(b);
        t -= 3;
        W256 v = w_zero(); v.v[0] = (uint32_t)vlo; v.v[1] = (uint32_t)(vlo >> 32); v.v[2] = vhi;
        if (t < 65) return w_u64(w_bit(v, t));
        if (t == 65) return v;
        return w_mask(v, (int)t - 65);
      }
      t -= 134;  // IsEqual: out | in[2] | IsZero(out, in, inv)
      if (t == 0 || t == 3) return w_u64(a == b);
      if (t == 1) return w_u64(a);
      if (t == 2) return w_u64(b);
      if (t == 4) return a <= b ? w_u64(b - a) : w_from_fr(fr_sub(fr_zero(), fr_u64(a - b)));
      W256 r; for (int k = 0; k < 8; k++) r.v[k] = (uint32_t)(C.inv[4 * i + (k >> 1)] >> (32 * (k & 1)));
      return r;
    }
    case MM_M2OUT: return u192w(u192_at(C.cqn, (int)s));               // mult2.out = q*n columns
    case MM_M2IN: return w_u64(s < (uint32_t)DIV ? C.q[s] : C.n[s - DIV]);
    case MM_TMPM: { uint32_t i = s / K, j = s - i * K; U192 acc; acc.mac(C.q[i], C.n[j]); return u192w(acc); }
    case MM_TMPR: return bmneq_tmpr(C.q, DIV, C.n, K, s);  // tmpResult of mult2 = q * n
    case MM_ISZIN: {  // BigIntIsZero.in = x*y - q*n - r (signed)
      const int i = s;
      W256 dd = w_sub(u192w(u192_at(C.cxy, i)), u192w(u192_at(C.cqn, i)));
      if (i < K) dd = w_sub(dd, w_u64(C.r[i]));
      return w_signed_to_fr(dd);
    }
    case MM_CARRY: return w_from_fr(fr_from_i128(C.cr[2 * s], C.cr[2 * s + 1]));
    default: {  // MM_RANGE: Num2Bits(RL)(carry + 2^(RL-1))
      const int MAXB = 128 + mm_log_ceil(2 * K);  // 2*64 + log_ceil(K + DIV - 1)
      const int RL = MAXB + 3 - 64;
      uint32_t per = 2 * RL + 1, i = s / per, t = s - per * i;
      uint64_t lo = C.cr[2 * i], hi = C.cr[2 * i + 1];
      uint64_t add_hi = 1ull << (RL - 1 - 64);
      uint64_t vhi = hi + add_hi;
      W256 v = w_zero();
      v.v[0] = (uint32_t)lo; v.v[1] = (uint32_t)(lo >> 32); v.v[2] = (uint32_t)vhi; v.v[3] = (uint32_t)(vhi >> 32);
      if (t < (uint32_t)RL) return w_u64(w_bit(v, t));
      if (t == (uint32_t)RL) return v;
      return w_mask(v, (int)t - RL);
    }
  }
}

// ---- section-specialised element functions of the BigMultModP emitter
// A 128-bit non-negative value (lo, hi) as an element, its bit t, and its low n bits (n in 1..128).
__device__ __forceinline__ El el_u128(uint64_t lo, uint64_t hi) {
  return El{make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)), make_uint4(0u, 0u, 0u, 0u)};
}
__device__ __forceinline__ uint32_t u128_bit(uint64_t lo, uint64_t hi, uint32_t t) {
  return (uint32_t)((t < 64 ? lo >> (t & 63) : hi >> (t & 63)) & 1u);
}
__device__ __forceinline__ El el_u128_low(uint64_t lo, uint64_t hi, uint32_t n) {
  const uint64_t ml = n >= 64 ? ~0ull : (1ull << n) - 1ull;
  const uint64_t mh = n >= 128 ? ~0ull : n > 64 ? (1ull << (n - 64)) - 1ull : 0ull;
  return el_u128(lo & ml, hi & mh);
}
// Num2Bits(L) block (bitify.circom:10-32) of a value < 2^128: out[L] | in | sum[L] (sum[j] = v mod 2^(j+1))
__device__ __forceinline__ El el_num2bits(uint64_t lo, uint64_t hi, uint32_t L, uint32_t t) {
  if (t < L) return el_u64(u128_bit(lo, hi, t));
  if (t == L) return el_u128(lo, hi);
  return el_u128_low(lo, hi, t - L);
}

// KaratsubaOverflow(32) signal from tables (K = KT_K): the node is found by a fixed five-step descent over the
// compile-time subtree sizes (no size switch, no loop), its inputs are Karatsuba table entries and the outputs of
// levels 1..KO_LEVELS come precomputed from LDS (ko, filled once per workgroup by k_emit_mm), so only the two
// deepest levels (<= 2 products per signal) are multiplied here (round 2 walked the tree per signal and formed each
// output as a convolution of up to 16 products per lane, the dominant VALU cost of the K = 32 emitter).
constexpr int KO_LEVELS = 3, KO_VALUES = 456;  // 3 x 32 + 9 x 16 + 27 x 8 node outputs (2N per node)
__device__ __forceinline__ int kt_level_base(int l) {  // first table entry of level l >= 1 (2N entries per node)
  return l == 1 ? 0 : l == 2 ? 96 : l == 3 ? 240 : l == 4 ? 456 : 780;
}
__device__ __forceinline__ El kara_el32(const MMCore& C, const uint32_t* ko, uint32_t s) {
  constexpr uint32_t SZ[6] = {mm_kara_size(32), mm_kara_size(16), mm_kara_size(8), mm_kara_size(4), mm_kara_size(2),
                              mm_kara_size(1)};
  int lvl = 0, m = 0;
  uint32_t p = s;
#pragma unroll
  for (int L = 0; L < 5; L++) {  // node at level L has 4 N_L own signals, then its 3 child subtrees of SZ[L + 1]
    const uint32_t own = 4u * (32u >> L);
    if (lvl == L && p >= own) {
      p -= own;
      const uint32_t c = (p >= SZ[L + 1] ? 1u : 0u) + (p >= 2 * SZ[L + 1] ? 1u : 0u);
      p -= c * SZ[L + 1];
      m = 3 * m + (int)c;
      lvl = L + 1;
    }
  }
  const int N = 32 >> lvl;
  if (p >= 2u * N) {  // in1[N] | in2[N]
    const int k = (int)p - 2 * N;
    if (lvl == 0) return el_u64(k < N ? C.x[k] : C.y[k - N]);
    const int i = kt_level_base(lvl) + m * 2 * N + k;
    return el_u128(C.kt_lo[i], C.kt_hi[i]);
  }
  if (p == 2u * N - 1) return el_zero();  // top coefficient (K(1).out[1] never assigned)
  if (lvl == 0) return el_w(u192w(u192_at(C.cxy, (int)p)));
  if (lvl <= KO_LEVELS) return el_w(u192w(ko5_at(ko, kt_level_base(lvl) + m * 2 * N + (int)p)));
  const int tb = kt_level_base(lvl) + m * 2 * N, lo = (int)p < N ? 0 : (int)p - N + 1, hi = (int)p < N ? (int)p : N - 1;
  U192 acc;
  for (int u = lo; u <= hi; u++)  // <= 2 terms (N <= 2)
    mac2(acc, C.kt_lo[tb + u], C.kt_hi[tb + u], C.kt_lo[tb + N + (int)p - u], C.kt_hi[tb + N + (int)p - u]);
  return el_w(u192w(acc));
}

// KaratsubaOverflow(64) signal (K = 64, RSA-4096), the K = 32 scheme one level deeper. LDS holds the in1/in2
// values of levels 1..K64_TL (K64_TL_VALUES, filled once per workgroup) and the node outputs of levels
// 1..K64_OL (ko). Deeper nodes' inputs (levels 5, 6: N = 2, 1) are sums of at most 4 level-4 entries, found by
// walking up the tree as offset masks (a child takes its parent's low half, high half, or their sum), so the
// table fits beside the block's core (3 workgroups per CU); output signals of levels 3..6 multiply <= 8 / 4 / 2 / 1
// pairs of such values. The round-2 walker this replaces summed limbs of x and y for every input and every
// product (91 k VALU instructions per wave).
constexpr int K64_TL = 4, K64_OL = 2;
__host__ __device__ constexpr int kt_base64(int l) {  // first table entry of level l >= 1 (2N entries per node)
  return l <= 1 ? 0 : l == 2 ? 192 : l == 3 ? 480 : l == 4 ? 912 : 1560;
}
constexpr int K64_TL_VALUES = kt_base64(K64_TL + 1), K64_OL_VALUES = kt_base64(K64_OL + 1);  // 1560, 480
__device__ __forceinline__ El kara_el64(const MMCore& C, const uint32_t* ko, uint32_t s) {
  constexpr uint32_t SZ[7] = {mm_kara_size(64), mm_kara_size(32), mm_kara_size(16), mm_kara_size(8),
                              mm_kara_size(4), mm_kara_size(2), mm_kara_size(1)};
  int lvl = 0, m = 0;
  uint32_t p = s;
#pragma unroll
  for (int L = 0; L < 6; L++) {  // node at level L has 4 N_L own signals, then its 3 child subtrees of SZ[L + 1]
    const uint32_t own = 4u * (64u >> L);
    if (lvl == L && p >= own) {
      p -= own;
      const uint32_t c = (p >= SZ[L + 1] ? 1u : 0u) + (p >= 2 * SZ[L + 1] ? 1u : 0u);
      p -= c * SZ[L + 1];
      m = 3 * m + (int)c;
      lvl = L + 1;
    }
  }
  const int N = 64 >> lvl;
  // input value k of in1 (op 0) or in2 (op 1) of node (lvl, m), lvl >= 1
  auto val = [&](int op, int k, uint64_t& lo, uint64_t& hi) {
    if (lvl <= K64_TL) {
      const int i = kt_base64(lvl) + m * 2 * N + op * N + k;
      lo = C.kt_lo[i]; hi = C.kt_hi[i];
      return;
    }
    uint32_t O = 1u << k;  // offsets into the level-K64_TL ancestor's N = 4 values
    int a = m, n = N;
    for (int l = lvl; l > K64_TL; l--) {
      const int c = a % 3;
      a /= 3;
      O = c == 0 ? O : c == 1 ? O << n : (O | (O << n));
      n *= 2;
    }
    const int tb = kt_base64(K64_TL) + a * 2 * n + op * n;
    lo = 0; hi = 0;
    while (O) {
      const int j = __builtin_ctz(O);
      O &= O - 1;
      const uint64_t v = C.kt_lo[tb + j];
      lo += v;
      hi += C.kt_hi[tb + j] + (lo < v ? 1u : 0u);
    }
  };
  if (p >= 2u * N) {  // in1[N] | in2[N]
    const int k = (int)p - 2 * N;
    if (lvl == 0) return el_u64(k < N ? C.x[k] : C.y[k - N]);
    uint64_t lo, hi;
    val(k >= N ? 1 : 0, k >= N ? k - N : k, lo, hi);
    return el_u128(lo, hi);
  }
  if (p == 2u * N - 1) return el_zero();  // top coefficient (K(1).out[1] never assigned)
  if (lvl == 0) return el_w(u192w(u192_at(C.cxy, (int)p)));
  if (lvl <= K64_OL) return el_w(u192w(ko5_at(ko, kt_base64(lvl) + m * 2 * N + (int)p)));
  const int lo_u = (int)p < N ? 0 : (int)p - N + 1, hi_u = (int)p < N ? (int)p : N - 1;
  U192 acc;
  for (int u = lo_u; u <= hi_u; u++) {
    uint64_t al, ah, bl, bh;
    val(0, u, al, ah);
    val(1, (int)p - u, bl, bh);
    mac2(acc, al, ah, bl, bh);
  }
  return el_w(u192w(acc));
}

template <int K, int SEC>
__device__ __forceinline__ El mm_el(const MMCore& C, uint32_t s) {
  if constexpr (SEC == MM_MODCHK) {  // Num2Bits(64)(mod_i): out[64] | in | sum[64]
    const uint32_t i = s / 129, t = s - 129 * i;
    return el_num2bits(C.r[i], 0, 64, t);
  } else if constexpr (SEC == MM_LT) {
    const uint32_t i = s / 140;
    uint32_t t = s - 140 * i;
    const uint64_t a = C.n[i], b = C.r[i];
    if (t < 134) {  // LessThan(64): out | in[2] | Num2Bits(65)(a + 2^64 - b)
      const uint64_t vlo = a - b, vhi = a >= b ? 1u : 0u;
      if (t < 3) return el_u64(t == 0 ? 1 - vhi : t == 1 ? a : b);
      return el_num2bits(vlo, vhi, 65, t - 3);
    }
    t -= 134;  // IsEqual: out | in[2] | IsZero(out, in, inv)
    if (t == 0 || t == 3) return el_u64(a == b);
    if (t == 1) return el_u64(a);
    if (t == 2) return el_u64(b);
    if (t == 4) return a <= b ? el_u64(b - a) : el_fr(fr_sub(fr_zero(), fr_u64(a - b)));
    const uint64_t* iv = C.inv + 4 * i;
    return El{make_uint4((uint32_t)iv[0], (uint32_t)(iv[0] >> 32), (uint32_t)iv[1], (uint32_t)(iv[1] >> 32)),
              make_uint4((uint32_t)iv[2], (uint32_t)(iv[2] >> 32), (uint32_t)iv[3], (uint32_t)(iv[3] >> 32))};
  } else if constexpr (SEC == MM_RANGE) {  // Num2Bits(RL)(carry + 2^(RL-1)), RL = 2*64 + log_ceil(2K) + 3 - 64
    constexpr uint32_t RL = 128 + mm_log_ceil(2 * K) + 3 - 64, PER = 2 * RL + 1;
    const uint32_t i = s / PER, t = s - PER * i;
    const uint64_t lo = C.cr[2 * i], hi = C.cr[2 * i + 1] + (1ull << (RL - 1 - 64));
    return el_num2bits(lo, hi, RL, t);
  } else if constexpr (SEC == MM_KARA && K == KT_K) {
    return kara_el32(C, C.ko, s);
  } else if constexpr (SEC == MM_KARA && K == 64) {
    return kara_el64(C, C.ko, s);
  } else if constexpr (SEC == MM_KARA) {
    static_assert((K & (K - 1)) != 0, "KaratsubaOverflow sizes have their own table path");
    return el_w(mm_sig(C, ((uint32_t)SEC << 24) | s));
  } else if constexpr (SEC == MM_Q) {
    return el_u64(C.q[s]);
  } else if constexpr (SEC == MM_R) {
    return el_u64(C.r[s]);
  } else if constexpr (SEC == MM_TMPM) {
    const uint32_t i = s / K, j = s - i * K;
    U192 acc;
    acc.mac(C.q[i], C.n[j]);
    return el_w(u192w(acc));
  } else {
    return el_w(mm_sig(C, ((uint32_t)SEC << 24) | s));
  }
}

#ifdef PZK_MM_PROF  // profiling build only (make EXTRA=-DPZK_MM_PROF): per-section clocks of wave 0 of every workgroup
static __device__ unsigned long long g_mm_prof[MM_SECTIONS + 2];
#define PZK_MM_CLK(v) const long long v = clock64()
#define PZK_MM_ACC(i, t0) do { const long long t1_ = clock64(); if (threadIdx.x == 0) atomicAdd(&g_mm_prof[i], (unsigned long long)(t1_ - (t0))); } while (0)
#else
#define PZK_MM_CLK(v)
#define PZK_MM_ACC(i, t0)
#endif

// the BigMultModP emitter's store stage: 64 uint4 per wave (wave_store's two-round form), which with the 5-word node
// outputs brings k_emit_mm<32> to 31 KB of LDS: five workgroups per CU instead of four
constexpr int MM_STAGE = 64;
// and its mapped kept-list segments: 896 signals (14 bitmap words), so the mapped k_emit_mm<32> also fits five per CU
constexpr uint32_t MM_SEG = 896;
template <int K, int SEC, int MM>
__device__ __forceinline__ void mm_sections(const MMCore C, const OutRow& out, uint4* stage) {
  if constexpr (SEC < (int)MM_SECTIONS) {
    constexpr MMStarts S = mm_starts(K);
    constexpr uint32_t a = S.v[SEC], n = S.v[SEC + 1] - S.v[SEC];
    PZK_MM_CLK(t0);
    // tmpResult rows (and BigMultNonEqualOverflow's, K != 32) are segmented scans across the wave (bmneq_tmpr)
    constexpr bool INDEP = !(SEC == MM_TMPR || (SEC == MM_KARA && (K & (K - 1)) != 0));
    emit_run<MM, INDEP, MM_STAGE, MM_SEG>(out.at(a), n, stage, [=](uint32_t q) { return mm_el<K, SEC>(C, q); });
    PZK_MM_ACC(SEC, t0);
    mm_sections<K, SEC + 1, MM>(C, out, stage);
  }
}

template <int K, int MM, int NT = 256>
__global__ void __launch_bounds__(NT) k_emit_mm(DevLayout L, const Work* work, Bufs B) {
  __shared__ uint64_t lds[MM_CORE_WORDS(K) + K + 3 * (4 * K - 1)];
  PZK_MM_CLK(tp);
  const Work wk = work[blockIdx.x];
  const uint32_t w = blockIdx.y;
  const Region R = L.regions[wk.region];
  const uint64_t* mc = B.rsa_core + (size_t)w * L.rsa_core_words + (size_t)R.a[0] * MM_CORE_WORDS(K);
  const uint8_t* row = B.inputs + 32ull * (uint64_t)w * L.n_inputs;
#ifdef PZK_MM_SERIAL_LOAD  // A/B builds: the round-3 load / write loops
  for (int i = threadIdx.x; i < MM_CORE_WORDS(K); i += blockDim.x) lds[i] = mc[i];
  for (int i = threadIdx.x; i < K; i += blockDim.x) lds[MM_CORE_WORDS(K) + i] = in_u64(row + 32ull * (R.a[1] + i));
#else
  // every load issued before any LDS write: a load / write loop waits out one HBM round trip per iteration, and
  // under the emitters' store stream that is several microseconds each (MM_CORE_WORDS(32) = 381: two per thread)
  constexpr int MM_NT = NT, CW = MM_CORE_WORDS(K), CL = (CW + MM_NT - 1) / MM_NT;
  uint64_t cv[CL];
#pragma unroll
  for (int k = 0; k < CL; k++) {
    const int i = threadIdx.x + k * MM_NT;
    cv[k] = mc[i < CW ? i : 0];
  }
  const uint64_t xin = in_u64(row + 32ull * (R.a[1] + (threadIdx.x < K ? threadIdx.x : 0)));
#pragma unroll
  for (int k = 0; k < CL; k++) {
    const int i = threadIdx.x + k * MM_NT;
    if (i < CW) lds[i] = cv[k];
  }
  if (threadIdx.x < K) lds[CW + threadIdx.x] = xin;
#endif
  __syncthreads();
  // column sums of x*y (2K-1) and q*n (2K), one thread per column
  uint64_t* cxy = lds + MM_CORE_WORDS(K) + K;
  uint64_t* cqn = cxy + 3 * (2 * K - 1);
  for (int c = threadIdx.x; c < 4 * K - 1; c += blockDim.x) {
    U192 acc;
    if (c < 2 * K - 1) {
      for (int j = c < K ? 0 : c - K + 1; j <= c && j < K; j++) acc.mac(lds[j], lds[K + (c - j)]);
      cxy[3 * c] = acc.a0; cxy[3 * c + 1] = acc.a1; cxy[3 * c + 2] = acc.a2;
    } else {
      const int i = c - (2 * K - 1);
      for (int j = i < K ? 0 : i - K + 1; j <= i && j <= K; j++) acc.mac(lds[2 * K + j], lds[MM_CORE_WORDS(K) + (i - j)]);
      cqn[3 * i] = acc.a0; cqn[3 * i + 1] = acc.a1; cqn[3 * i + 2] = acc.a2;
    }
  }
  __syncthreads();
  // Karatsuba input table (K = 32), level by level: a child's operand is the parent's low half,
  // high half, or their sum
  constexpr int KTN = K == KT_K ? KT_VALUES : K == 64 ? K64_TL_VALUES : 1;
  __shared__ uint64_t kt_lo[KTN];
  __shared__ uint8_t kt_hi[KTN];
  if (K == KT_K || K == 64) {
    int base = 0, pbase = 0, nodes = 3;
    for (int l = 1; l <= (K == KT_K ? KT_LEVELS : K64_TL); l++) {
      const int N = K >> l, cnt = nodes * 2 * N;
      for (int r = threadIdx.x; r < cnt; r += blockDim.x) {
        const int m = r / (2 * N), k = r - m * 2 * N, op = k >= N, u = k - op * N, p = m / 3, c = m - 3 * p;
        uint64_t alo, ahi, blo = 0, bhi = 0;
        if (l == 1) {
          const uint64_t* src = op ? lds + K : lds;  // x or y
          alo = src[u]; ahi = 0; if (c != 0) { blo = src[u + N]; bhi = 0; }
        } else {
          const int pi = pbase + p * 4 * N + op * 2 * N + u;  // parent node: in1[2N] then in2[2N]
          alo = kt_lo[pi]; ahi = kt_hi[pi];
          if (c != 0) { blo = kt_lo[pi + N]; bhi = kt_hi[pi + N]; }
        }
        uint64_t lo, hi;
        if (c == 0) { lo = alo; hi = ahi; }
        else if (c == 1) { lo = blo; hi = bhi; }
        else { lo = alo + blo; hi = ahi + bhi + (lo < alo); }
        kt_lo[base + r] = lo; kt_hi[base + r] = (uint8_t)hi;
      }
      __syncthreads();
      pbase = base;
      base += cnt;
      nodes *= 3;
    }
  }
  // outputs of the Karatsuba nodes of levels 1..KO_LEVELS (K = 32): out[s] = sum_u in1[u] in2[s - u] over the
  // node's table inputs, once per workgroup (kara_el32 reads them)
  constexpr int KON = K == KT_K ? 3 * KO_VALUES : K == 64 ? 3 * K64_OL_VALUES : 1;
  __shared__ uint32_t ko[(KON + 2) / 3 * 5];
  if (K == KT_K || K == 64) {
    for (int r = threadIdx.x; r < (K == KT_K ? KO_VALUES : K64_OL_VALUES); r += blockDim.x) {
      const int l = K == KT_K ? (r < 96 ? 1 : r < 240 ? 2 : 3) : (r < kt_base64(2) ? 1 : 2), N = K >> l;
      const int lb = K == KT_K ? kt_level_base(l) : kt_base64(l), rr = r - lb, m = rr / (2 * N);
      const int p = rr - m * 2 * N, tb = lb + m * 2 * N;
      U192 acc;
      if (p < 2 * N - 1)
        for (int u = p < N ? 0 : p - N + 1; u <= (p < N ? p : N - 1); u++)
          mac2(acc, kt_lo[tb + u], kt_hi[tb + u], kt_lo[tb + N + p - u], kt_hi[tb + N + p - u]);
      uint32_t* o = ko + 5 * r;
      o[0] = (uint32_t)acc.a0; o[1] = (uint32_t)(acc.a0 >> 32); o[2] = (uint32_t)acc.a1; o[3] = (uint32_t)(acc.a1 >> 32);
      o[4] = (uint32_t)acc.a2;
    }
    __syncthreads();
  }
  MMCore C{K, lds, lds + K, lds + 2 * K, lds + 3 * K + 1, lds + MM_CORE_WORDS(K), lds + 4 * K + 1, lds + 8 * K + 1,
           cxy, cqn, (K & (K - 1)) == 0, K == KT_K || K == 64 ? kt_lo : nullptr, K == KT_K || K == 64 ? kt_hi : nullptr,
           K == KT_K || K == 64 ? ko : nullptr};
  const OutRow out = out_row(L, B.wtns, B.stride, w, R.off + wk.start);
  __shared__ uint4 stage[MM_STAGE * (NT / 64)];
  PZK_MM_ACC(MM_SECTIONS, tp);  // prologue: core loads, column sums, Karatsuba input table
  // section by section, each with its own specialised element function (mm_el<K, SEC>): every
  // wave works inside one section, and each section starts wave-aligned, so a tmpResult row never
  // straddles the start of a wave (K = 32: two rows per wave; K = 64: one)
  // (mapped blocks with the sections merged into as few runs as the scan sections allow, one kept-list collection
  // per 1,664 signals instead of one per section, measured 4 % slower on the O2-shaped line: profiles/r5p)
  mm_sections<K, 0, MM>(C, out, stage);
}

// ------------------------------------------------------------------ BabyJubJub steps
// Two stages. (1) Per ladder step, the fourteen distinct field values its 60 signals are drawn
// from (coordinates, the adder's/doubler's products, the IsZero inverse, -x1 and -y1) are computed once, in
// normal form, into an LDS record: one thread per (step, value); five constants follow the records. (2) Every
// signal is then one read of the record array at an index chosen by integer selects (the choice depends on the
// step's bit and on x1 = 0: selecting 8-word values per signal instead took ~680 VALU per wave and element).
// Work items are step-aligned (BJJ_EMIT_STEPS steps each, builder_impl.hpp).
enum BjjRec { BR_X1, BR_Y1, BR_OX, BR_OY, BR_INV, BR_X1Y2, BR_Y1X2, BR_DELTA, BR_TAU, BR_XYD, BR_DELTAD, BR_TAUD,
              BR_NX1, BR_NY1, BR_N };
enum BjjConst { BC_ZERO, BC_ONE, BC_B8X, BC_B8Y, BC_INVB8X, BC_N };

__device__ __forceinline__ uint32_t bjj_step_of(uint32_t s) { return s < 46 ? 0 : 1 + (s - 46) / 60; }
__device__ __forceinline__ uint32_t bjj_sig_of(uint32_t i) { return i == 0 ? 0 : 46 + 60 * (i - 1); }

#ifndef PZK_TEMPLATE_KERNELS_ONLY  // defined once, in kernels.hip
// (at most 80 VGPRs: six workgroups per CU, as its LDS allows, instead of five at 88)
__global__ void __launch_bounds__(256, 6) k_emit_bjj(DevLayout L, const Work* work, Bufs B) {
  constexpr int CB = (BJJ_EMIT_STEPS + 1) * BR_N;  // the constants' base in rec
  __shared__ fr rec[CB + BC_N];
  __shared__ uint32_t bits[BJJ_EMIT_STEPS + 1], zx1[BJJ_EMIT_STEPS + 1];
  const Work wk = work[blockIdx.x];
  const uint32_t w = blockIdx.y;
  const Region R = L.regions[wk.region];
  const fr* core = B.bjj_core + (size_t)w * L.bjj_core_fr;
  const uint32_t i0 = bjj_step_of(wk.start), i1 = bjj_step_of(wk.start + wk.count - 1) + 1;
  const int base = i0 == 0 ? 0 : (int)i0 - 1;  // local record 0 = step base (predecessor of i0 when i0 > 0)
  const int nrec = (int)i1 - base;
  {
    fr skm = B.vs.at(L.reg.v_sk, w);
    fr sk = fr_from_mont_fast(skm);
    for (int j = threadIdx.x; j < nrec; j += blockDim.x) {
      int i = base + j;
      bits[j] = fr_bit(sk, 253 - i);
    }
    if (threadIdx.x < BC_N) {
      const int c = (int)threadIdx.x;
      rec[CB + c] = c == BC_ZERO ? fr_zero() : c == BC_ONE ? fr_u64(1) : c == BC_B8X ? fr_const(BJJ_B8X)
                  : c == BC_B8Y ? fr_const(BJJ_B8Y) : fr_const(BJJ_INV_B8X);
    }
  }
  __syncthreads();
  // value-major item order: the lanes of a wave compute the same record value for consecutive
  // steps (one or two branches of the switch per wave instead of all fourteen)
  for (int q = threadIdx.x; q < nrec * BR_N; q += blockDim.x) {
    const int v = q / nrec, j = q - v * nrec, i = base + j;
    const fr* P = core + 5 * i;
    fr r;
    if (v == BR_XYD || v == BR_DELTAD || v == BR_TAUD) {  // doubler of step i (doublers[i-1]) over A_{i-1}
      if (i == 0) r = fr_zero();
      else {
        fr xp = P[-3], yp = P[-2];  // core + 5(i-1) + 2, + 3
        fr xy = fr_mul_fast(xp, yp);
        if (v == BR_XYD) r = xy;
        else if (v == BR_DELTAD) r = fr_mul_fast(fr_sub(yp, fr_mul_fast(fr_to_mont(fr_u64(BJJ_A)), xp)), fr_add(xp, yp));
        else r = fr_sqr_fast(xy);
      }
    } else if (v == BR_OX || v == BR_OY) {
      r = P[v];
    } else {
      const bool bit = bits[j];
      fr x1 = i == 0 ? fr_zero() : P[0], y1 = i == 0 ? fr_zero() : P[1];
      fr x2 = bit ? fr_to_mont(fr_const(BJJ_B8X)) : fr_zero(), y2 = bit ? fr_to_mont(fr_const(BJJ_B8Y)) : fr_zero();
      switch (v) {
        case BR_X1: r = x1; zx1[j] = fr_is_zero(x1); break;
        case BR_Y1: r = y1; break;
        case BR_NX1: r = fr_sub(fr_zero(), x1); break;
        case BR_NY1: r = fr_sub(fr_zero(), y1); break;
        case BR_INV: r = i == 0 ? fr_zero() : P[4]; break;
        case BR_X1Y2: r = fr_mul_fast(x1, y2); break;
        case BR_Y1X2: r = fr_mul_fast(y1, x2); break;
        case BR_DELTA: r = fr_mul_fast(fr_sub(y1, fr_mul_fast(fr_to_mont(fr_u64(BJJ_A)), x1)), fr_add(x2, y2)); break;
        default: r = fr_mul_fast(fr_mul_fast(x1, y2), fr_mul_fast(y1, x2)); break;
      }
    }
    rec[j * BR_N + v] = fr_from_mont_fast(r);
  }
  __syncthreads();
  const OutRow out = out_row(L, B.wtns, B.stride, w, R.off + wk.start);
  __shared__ uint4 stage[2 * 256];
  emit_run(out, wk.count, stage, [&](uint32_t q) -> El {
    const uint32_t s = wk.start + q, i = bjj_step_of(s), t = s - bjj_sig_of(i);
    const int j = (int)i - base;
    const int rc = j * BR_N, rp = rc - BR_N;
    constexpr int ZERO = CB + BC_ZERO, ONE = CB + BC_ONE;
    int idx;
    if (t >= 46) {  // doublers[i-1]: out[2] = D_i | in[2] = A_{i-1} | adder out, in1, in2, beta, gamma, delta, tau
      const uint32_t u = t - 46;
      idx = u < 2 ? rc + BR_X1 + (int)u : u < 4 ? rp + BR_OX + (int)u - 2 : u < 6 ? rc + BR_X1 + (int)u - 4
          : u < 10 ? rp + BR_OX + (int)(u & 1) : u < 12 ? rc + BR_XYD : rc + (u == 12 ? BR_DELTAD : BR_TAUD);
    } else {
      const bool bit = bits[j] != 0, z1 = zx1[j] != 0, z2 = !bit;
      const int x1 = rc + BR_X1, y1 = rc + BR_Y1, x2 = bit ? CB + BC_B8X : ZERO, y2 = bit ? CB + BC_B8Y : ZERO;
      const int rawx = (!z1 && !z2) ? rc + BR_OX : ZERO, rawy = (!z1 && !z2) ? rc + BR_OY : ZERO;
      if (t < 2) idx = rc + BR_OX + (int)t;
      else if (t < 4) idx = t == 2 ? x1 : y1;
      else if (t < 6) idx = t == 4 ? x2 : y2;
      else if (t < 9) idx = t == 6 ? (z1 ? ONE : ZERO) : t == 7 ? x1 : rc + BR_INV;
      else if (t < 12) idx = t == 9 ? (z2 ? ONE : ZERO) : t == 10 ? x2 : (bit ? CB + BC_INVB8X : ZERO);
      else if (t < 22) {  // adder: out[2] | in1[2], in2[2] | beta, gamma, delta, tau
        const uint32_t u = t - 12;
        idx = u < 2 ? (u == 0 ? rawx : rawy) : u < 4 ? (u == 2 ? x1 : y1) : u < 6 ? (u == 4 ? x2 : y2)
            : rc + BR_X1Y2 + (int)(u - 6);
      } else {  // switchers L0, R0, L1, R1: out[2] | bool, in[2] | aux
        const uint32_t u = t - 22, sw = u / 6, k = u % 6;
        const bool cy = (sw >> 1) != 0;
        const int raw = cy ? rawy : rawx, in1c = cy ? y1 : x1, in2c = cy ? y2 : x2;
        const int l0 = z2 ? in1c : raw, l1 = z2 ? raw : in1c;
        if ((sw & 1) == 0) {
          // aux = z2 ? in1c - raw : 0, and raw = 0 when z2
          idx = k == 0 ? l0 : k == 1 ? l1 : k == 2 ? (z2 ? ONE : ZERO) : k == 3 ? raw : k == 4 ? in1c
              : (z2 ? in1c : ZERO);
        } else {
          // aux = z1 ? in2c - l0 : 0; with z1, raw = 0, so l0 = (z2 ? in1c : 0) and in2c = (z2 ? 0 : in2c)
          const int aux = !z1 ? ZERO : z2 ? rc + (cy ? BR_NY1 : BR_NX1) : in2c;
          idx = k == 0 ? (z1 ? in2c : l0) : k == 1 ? (z1 ? l0 : in2c) : k == 2 ? (z1 ? ONE : ZERO) : k == 3 ? l0
              : k == 4 ? in2c : aux;
        }
      }
    }
    return el_fr(rec[idx]);
  });
}
#endif

}  // namespace pzk
