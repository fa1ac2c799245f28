// Device kernels of the witness generator (unity build: every device header is included
// here; the host runtime in runtime.cpp launches them through the launch_* wrappers).
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include "poseidon.hpp"
#include "regcore.hpp"
#include "smt_chain4.hpp"
#include "pss.hpp"
#include "regemit.hpp"
#include "sha.hpp"
#include "sha1.hpp"
#include "sha512.hpp"
#include "sha_prog.hpp"
#include "mapsink.hpp"
#include "kernels.hpp"

namespace pzk {

// ------------------------------------------------------------------- value loads
// value-store slot <- input element (normal form -> Montgomery)
__global__ void k_load_values(const ValueLoad* loads, int n_loads, const uint8_t* inputs, uint64_t n_inputs,
                              fr* values, uint32_t batch) {
  uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
  int l = blockIdx.y;
  if (w >= batch || l >= n_loads) return;
  ValueLoad ld = loads[l];
  fr x = load_fr(inputs + 32ull * ((uint64_t)w * n_inputs + ld.in_off));
  values[(size_t)ld.slot * batch + w] = fr_to_mont(x);
}

// ------------------------------------------------------------------- SHA core
__global__ void __launch_bounds__(64, 1) k_sha_core(const ShaJob* jobs, int n_jobs, const uint8_t* inputs, uint64_t n_inputs,
                           const uint8_t* derived, uint64_t n_derived, uint32_t* sha_core, uint32_t core_words,
                           int32_t* status, uint32_t batch) {
  core_priority();
  uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
  int j = blockIdx.y;
  if (w >= batch || j >= n_jobs) return;
  const ShaJob& J = jobs[j];
  const uint8_t* row = J.src ? derived + 32ull * (uint64_t)w * n_derived : inputs + 32ull * (uint64_t)w * n_inputs;
  if (J.algo == 1) sha1_core_lane(row, J, sha_core + (size_t)w * core_words, status ? status + w : nullptr);
  else if (J.algo >= 3) sha512_core_lane(row, J, sha_core + (size_t)w * core_words, status ? status + w : nullptr);
  else sha_core_lane(row, J, sha_core + (size_t)w * core_words, status ? status + w : nullptr);
}

// ------------------------------------------------------------------- emit: SHA regions
__device__ __forceinline__ uint64_t sha_own_sig(const Region& R, const uint32_t* H /* (B+1)*8 in LDS */, uint32_t s,
                                                bool& is_copy, uint64_t& src) {
  const int B = R.a[1];
  const uint32_t inLen = 512u * B, O = R.a[4] == 224 ? 224u : 256u;  // SHA-224: out[224], its own IV
  is_copy = false;
  if (R.a[3]) {  // ShaHashChunks wrapper: out[O] | in[512B]
    if (s < O) { uint32_t j = s >> 5, i = s & 31; return (H[B * 8 + j] >> (31 - i)) & 1; }
    s -= O;
    if (s < inLen) { is_copy = true; src = (uint64_t)R.a[2] + s; return 0; }
    s -= inLen;
  }
  if (s < O) { uint32_t j = s >> 5, i = s & 31; return (H[B * 8 + j] >> (31 - i)) & 1; }
  s -= O;
  if (s < inLen) { is_copy = true; src = (uint64_t)R.a[2] + s; return 0; }
  s -= inLen;
  if (s < 256u * (B + 1)) { uint32_t m = s >> 8, j = (s >> 5) & 7, i = s & 31; return (H[m * 8 + j] >> i) & 1; }
  s -= 256u * (B + 1);
  return ((O == 224 ? SHA224_IV[s >> 5] : SHA_IV[s >> 5]) >> (s & 31)) & 1;
}

template <int SHA_U, int MM>  // descriptors loaded ahead of their stores (see stage 2); MM: store mode (mapsink.hpp)
__global__ void __launch_bounds__(EMIT_THREADS) k_emit_sha(DevLayout L, const Work* work, const uint8_t* inputs,
                                                          const uint8_t* derived, const uint32_t* sha_core,
                                                          uint8_t* wtns, size_t stride, int wit_major) {
  __shared__ uint32_t core[SHA_BLOCK_CORE + 8 * 65];  // RK_SHA_OWN: H_0..H_B, B <= 64
  __shared__ __attribute__((aligned(16))) uint64_t wt[SHA_WT_SIZE];
  // grid (witness, chunk): the blocks in flight together work on the same chunk of different
  // witnesses, so they share its slice of the block program in L2
  const Work wk = work[wit_major ? blockIdx.y : blockIdx.x];
  const uint32_t w = wit_major ? blockIdx.x : blockIdx.y;
  const Region R = L.regions[wk.region];
  const ShaJob job = L.sha[R.a[0]];
  const uint32_t* wc = sha_core + (size_t)w * L.sha_core_words + job.core_off;
  const OutRow out = out_row(L, wtns, stride, w, R.off + wk.start);
  if (R.kind == RK_SHA_BLOCK) {
    // stage 1: the word-table entries this chunk's signals read (base words, feed-forward sums,
    // and the derived words of the schedule / compress rounds the chunk overlaps)
    const uint32_t* bc = wc + R.a[1] * SHA_BLOCK_CORE;
    for (int i = threadIdx.x; i < SHA_BLOCK_CORE; i += blockDim.x) core[i] = bc[i];
    __syncthreads();
    const ShaBlk Bk{core};
    const uint32_t a = wk.start, b = wk.start + wk.count - 1;
    auto rng = [](uint32_t lo_sig, uint32_t per, int nr, uint32_t x) {  // round index of signal x, clamped
      return x < lo_sig ? 0 : (int)min((x - lo_sig) / per, (uint32_t)nr - 1);
    };
    const bool sch = a < SHA_SCH_ROUND0 + 48 * SHA_SCH_ROUND_SIGS && b >= SHA_SCH_ROUND0;
    const bool cmp = a < SHA_RDS_CMP0 + 64 * SHA_CMP_SIGS && b >= SHA_RDS_CMP0;
    const int r0 = sch ? rng(SHA_SCH_ROUND0, SHA_SCH_ROUND_SIGS, 48, a) : 0;
    const int r1 = sch ? rng(SHA_SCH_ROUND0, SHA_SCH_ROUND_SIGS, 48, b) + 1 : 0;
    const int k0 = cmp ? rng(SHA_RDS_CMP0, SHA_CMP_SIGS, 64, a) : 0;
    const int k1 = cmp ? rng(SHA_RDS_CMP0, SHA_CMP_SIGS, 64, b) + 1 : 0;
    const int n_base = SHA_WT_SCH, n_ff = 16, n_sch = (r1 - r0) * SHA_SCH_WORDS, n_cmp = (k1 - k0) * SHA_CMP_WORDS;
    for (int v = threadIdx.x; v < n_base + n_ff + n_sch + n_cmp; v += blockDim.x) {
      int e = v < n_base ? v
            : v < n_base + n_ff ? SHA_WT_FF32 + (v - n_base)
            : v < n_base + n_ff + n_sch ? SHA_WT_SCH + r0 * SHA_SCH_WORDS + (v - n_base - n_ff)
                                        : SHA_WT_CMP + k0 * SHA_CMP_WORDS + (v - n_base - n_ff - n_sch);
      wt[e] = sha_wt_entry(Bk, e);
    }
    __syncthreads();
    // stage 2: one descriptor, one LDS word, one bit-field extract per element
    // Two lanes per element (16 B each), so every wave store is 1 KiB contiguous: the element
    // is cheap enough to evaluate twice, and this store shape writes ~19 % faster than 32 B per
    // lane (emit_run stages through LDS for the emitters whose elements are expensive).
    // SHA_U descriptors are loaded before the SHA_U stores that use them (a global load issued
    // after a store waits for it: gfx9 vmcnt counts both)
    // Mapped: the kept elements' descriptors (desc_run), stored consecutively from their mapped index.
    const DescRun dr = desc_run<MM>(L, wtns, stride, w, wk, R.off + wk.start, L.sha_prog + wk.start);
    const uint32_t* prog = dr.prog;
    const uint32_t tot = 2 * dr.count;
    for (uint32_t base = threadIdx.x; base < tot; base += SHA_U * blockDim.x) {
      uint32_t d[SHA_U];
#pragma unroll
      for (int k = 0; k < SHA_U; k++) {
        const uint32_t h = base + k * blockDim.x;
        d[k] = h < tot ? prog[h >> 1] : 0u;
      }
#pragma unroll
      for (int k = 0; k < SHA_U; k++) {
        const uint32_t h = base + k * blockDim.x;
        const uint64_t v = (h & 1) ? 0 : sha_desc_apply(d[k], wt[d[k] & 2047]);
        store_half<MAP_O0>(dr.out, h, make_uint4((uint32_t)v, (uint32_t)(v >> 32), 0u, 0u), h < tot);
      }
    }
  } else {  // RK_SHA_OWN: H_0..H_B (H_m = Hin of block m, H_B = Hout)
    const int Bn = R.a[1];
    for (int i = threadIdx.x; i < 8 * (Bn + 1); i += blockDim.x) {
      int m = i >> 3, j = i & 7;
      core[i] = m < Bn ? wc[m * SHA_BLOCK_CORE + j] : wc[Bn * SHA_BLOCK_CORE + j];
    }
    __syncthreads();
    const uint8_t* in_row = job.src ? derived + 32ull * (uint64_t)w * L.n_derived : inputs + 32ull * (uint64_t)w * L.n_inputs;
    uint4* stage = reinterpret_cast<uint4*>(wt);  // the word table is not used on this path
    emit_run<MM>(out, wk.count, stage, [&](uint32_t q) {
      bool cp; uint64_t src = 0;
      uint64_t v = sha_own_sig(R, core, wk.start + q, cp, src);
      return cp ? el_load(in_row + 32ull * src) : el_u64(v);
    });
  }
}

// ------------------------------------------------------------------- emit: SHA-1 regions
// workgroup per (witness, chunk) of a region: the block's 165 core words go to LDS (with A[-4..-1]
// so that B..E of every round are A-history lookups), then one closed-form signal per lane.
__global__ void __launch_bounds__(EMIT_THREADS) k_emit_sha1(DevLayout L, const Work* work, const uint8_t* inputs,
                                                           const uint8_t* derived, const uint32_t* sha_core,
                                                           uint8_t* wtns, size_t stride) {
  __shared__ uint32_t wd[5 + 80 + 85];
  __shared__ uint4 stage[2 * EMIT_THREADS];
  const Work wk = work[blockIdx.y];
  const uint32_t w = blockIdx.x;
  const Region R = L.regions[wk.region];
  const ShaJob job = L.sha[R.a[0]];
  const uint32_t* wc = sha_core + (size_t)w * L.sha_core_words + job.core_off;
  const OutRow out = out_row(L, wtns, stride, w, R.off + wk.start);
  if (R.kind == RK_SHA1_BLOCK) {
    const uint32_t* bc = wc + R.a[1] * SHA1_BLOCK_CORE;
    for (int i = threadIdx.x; i < SHA1_BLOCK_CORE; i += blockDim.x) wd[i < 85 ? i : i + 5] = bc[i];
    if (threadIdx.x == 0) {
      wd[89] = bc[0]; wd[88] = bc[1];
      wd[87] = rol32(bc[2], 2); wd[86] = rol32(bc[3], 2); wd[85] = rol32(bc[4], 2);
    }
    __syncthreads();
    const Sha1Blk X{wd, wd + 5, wd + 85};
    emit_run(out, wk.count, stage, [&](uint32_t q) { return el_u64(sha1_block_sig(X, wk.start + q)); });
  } else {  // RK_SHA1_OWN
    const int Bn = R.a[1];
    const uint32_t* hout = wc + Bn * SHA1_BLOCK_CORE;
    const uint8_t* in_row = job.src ? derived + 32ull * (uint64_t)w * L.n_derived : inputs + 32ull * (uint64_t)w * L.n_inputs;
    emit_run(out, wk.count, stage, [&](uint32_t q) {
      bool cp;
      const uint64_t v = sha1_own_sig(hout, Bn, R.a[3] != 0, wk.start + q, cp);
      return cp ? el_load(in_row + 32ull * (R.a[2] + v)) : el_u64(v);
    });
  }
}

// ------------------------------------------------------------------- emit: SHA-384/512 regions
// workgroup per (witness, chunk) of a region: the block's 64-bit core words go to LDS (with the
// Hin words in front of A and E, so B..D / F..H of every round are history lookups), then one
// closed-form signal per lane (sha512.hpp), staged through LDS for wave-contiguous stores.
__device__ __forceinline__ El el_u128v(U128 v) {
  return El{make_uint4((uint32_t)v.lo, (uint32_t)(v.lo >> 32), (uint32_t)v.hi, (uint32_t)(v.hi >> 32)), make_uint4(0u, 0u, 0u, 0u)};
}
__global__ void __launch_bounds__(EMIT_THREADS) k_emit_sha512(DevLayout L, const Work* work, const uint8_t* inputs,
                                                             const uint8_t* derived, const uint32_t* sha_core,
                                                             uint8_t* wtns, size_t stride) {
  __shared__ uint64_t wd[8 + 80 + 84 + 84];
  __shared__ uint4 stage[2 * EMIT_THREADS];
  const Work wk = work[blockIdx.y];
  const uint32_t w = blockIdx.x;
  const Region R = L.regions[wk.region];
  const ShaJob job = L.sha[R.a[0]];
  const uint64_t* wc = reinterpret_cast<const uint64_t*>(sha_core + (size_t)w * L.sha_core_words + job.core_off);
  const OutRow out = out_row(L, wtns, stride, w, R.off + wk.start);
  if (R.kind == RK_SHA5_BLOCK) {
    const uint64_t* bc = wc + (size_t)R.a[1] * (SHA5_BLOCK_CORE / 2);  // Hin[8] W[80] A[1..80] E[1..80]
    for (int i = threadIdx.x; i < 8 + 80; i += blockDim.x) wd[i] = bc[i];
    for (int i = threadIdx.x; i < 80; i += blockDim.x) { wd[88 + 4 + i] = bc[88 + i]; wd[172 + 4 + i] = bc[168 + i]; }
    if (threadIdx.x < 4) {  // A[-3..0] = Hin[3..0], E[-3..0] = Hin[7..4]
      wd[88 + threadIdx.x] = bc[3 - threadIdx.x];
      wd[172 + threadIdx.x] = bc[7 - threadIdx.x];
    }
    __syncthreads();
    const Sha5Blk X{wd, wd + 8, wd + 88, wd + 172};  // A(t) = wd[88 + t + 3], E(t) = wd[172 + t + 3]
    emit_run(out, wk.count, stage, [&](uint32_t q) { return el_u128v(sha5_block_sig(X, wk.start + q)); });
  } else {  // RK_SHA5_OWN
    const int Bn = R.a[1], O = R.a[3];
    const uint8_t* in_row = job.src ? derived + 32ull * (uint64_t)w * L.n_derived : inputs + 32ull * (uint64_t)w * L.n_inputs;
    const uint64_t* iv = job.algo == 3 ? SHA384_IV_ : SHA512_IV_;
    auto hin = [&](int m, uint32_t j) -> uint64_t { return m < Bn ? wc[(size_t)m * (SHA5_BLOCK_CORE / 2) + j] : wc[(size_t)Bn * (SHA5_BLOCK_CORE / 2) + j]; };
    emit_run(out, wk.count, stage, [&](uint32_t q) {
      bool cp;
      const uint64_t v = sha5_own_sig(hin, Bn, O, iv, wk.start + q, cp, R.a[4] != 0);
      return cp ? el_load(in_row + 32ull * (R.a[2] + v)) : el_u64(v);
    });
  }
}

// ------------------------------------------------------------------- emit: generic small regions
// A work item packs up to GEN_PACK signals from up to GEN_MAX_PIECES region slices (most generic
// regions are a handful of signals: SMT levels, switchers, IsZero blocks). Thread q finds its
// piece by binary search over the piece prefix sums staged in LDS.
template <bool QRY>
__device__ __forceinline__ void emit_gen_body(const DevLayout& L, const Work* work, const Bufs& B) {
  __shared__ uint32_t cum[GEN_MAX_PIECES];
  const Work wk = work[blockIdx.x];
  const uint32_t w = blockIdx.y;
  const GenPiece* pc = L.gen_pieces + wk.region;
  const uint32_t np = wk.pad;
  for (uint32_t i = threadIdx.x; i < np; i += blockDim.x) cum[i] = pc[i].cum;
  __syncthreads();
  uint8_t* row = B.wtns + (size_t)w * B.stride;
  // two passes: every load of the thread's elements first, then every store. A load issued after
  // a store waits for that store (gfx9 vmcnt counts both), which under a saturated write path
  // would serialise each element on the store latency. Mapped (mapsink.hpp): the element's keep bit
  // and mapped index are loaded in the first pass too; a dropped element is not evaluated. PER stays small
  // enough for the loop to unroll: at 8 (GEN_PACK 2048) it did not, val[] / dst[] went to 272 B of scratch
  // per lane, and the spills doubled the kernel's HBM traffic.
  constexpr int PER = GEN_PACK / EMIT_THREADS;
  static_assert(PER <= 2, "k_emit_gen keeps PER elements per lane in registers");
  El val[PER];
  uint64_t dst[PER];
#pragma unroll
  for (int k = 0; k < PER; k++) {
    const uint32_t q = threadIdx.x + k * EMIT_THREADS;
    dst[k] = ~0ull;
    if (q < wk.count) {
      uint32_t lo = 0, hi = np - 1;
      while (lo < hi) {
        uint32_t mid = (lo + hi + 1) >> 1;
        if (cum[mid] <= q) lo = mid; else hi = mid - 1;
      }
      const GenPiece p = pc[lo];
      const Region& R = L.regions[p.region];
      const uint32_t s = p.start + (q - cum[lo]);
      uint32_t rank = 0;
      if (L.keep.bits && !map_keep_lane(L.keep, R.off + s, rank)) continue;
      val[k] = QRY ? query_small(L, B, R, w, s) : emit_small(L, B, R, w, s);
      dst[k] = L.keep.bits ? rank : R.off + s;
    }
  }
#pragma unroll
  for (int k = 0; k < PER; k++)
    if (dst[k] != ~0ull) {
      uint4* d = reinterpret_cast<uint4*>(row + 32ull * dst[k]);
      d[0] = val[k].lo; d[1] = val[k].hi;
    }
}

// (at most 96 VGPRs: five workgroups per CU instead of four at 112; LDS allows nine)
__global__ void __launch_bounds__(EMIT_THREADS, 5) k_emit_gen(DevLayout L, const Work* work, Bufs B) {
  emit_gen_body<false>(L, work, B);
}
// QueryIdentity's small regions (query.hpp): the same packed emitter with its own element function, so
// k_emit_gen keeps its register budget (one kernel for both took 192 VGPRs and 208 B of scratch per lane,
// against 112 and none)
__global__ void __launch_bounds__(EMIT_THREADS) k_emit_qry(DevLayout L, const Work* work, Bufs B) {
  emit_gen_body<true>(L, work, B);
}

// ------------------------------------------------------------------- signal map (.sym) gather
// out[k] = o0[map[k]] per witness row: 16 B per lane (two lanes per element), so every wave store is
// 1 KiB contiguous; the O0 reads follow the map (monotonic maps read mostly forward).
__global__ void __launch_bounds__(256) k_wtns_gather(const uint8_t* o0, size_t o0_stride, const uint32_t* map,
                                                     uint64_t out_size, uint8_t* out, size_t out_stride) {
  const uint32_t w = blockIdx.y;
  const uint4* src = reinterpret_cast<const uint4*>(o0 + o0_stride * w);
  uint4* dst = reinterpret_cast<uint4*>(out + out_stride * w);
  const uint64_t n2 = 2 * out_size;
  for (uint64_t h = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; h < n2; h += (uint64_t)gridDim.x * blockDim.x)
    dst[h] = src[2ull * map[h >> 1] + (h & 1)];
}

// ------------------------------------------------------------------- launchers
#define HIP_TRY(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return e_; } while (0)

hipError_t launch_wtns_gather(const uint8_t* o0, size_t o0_stride, const uint32_t* map, uint64_t out_size, uint8_t* out,
                              size_t out_stride, uint32_t batch, hipStream_t st) {
  const uint32_t blocks = (uint32_t)std::min<uint64_t>((2 * out_size + 255) / 256, 512);
  hipLaunchKernelGGL(k_wtns_gather, dim3(blocks, batch), dim3(256), 0, st, o0, o0_stride, map, out_size, out, out_stride);
  return hipGetLastError();
}

hipError_t launch_load_values(const ValueLoad* loads, int n, const uint8_t* inputs, uint64_t n_inputs, fr* values,
                              uint32_t batch, hipStream_t st) {
  if (n == 0) return hipSuccess;
  dim3 g((batch + 63) / 64, n);
  hipLaunchKernelGGL(k_load_values, g, dim3(64), 0, st, loads, n, inputs, n_inputs, values, batch);
  return hipGetLastError();
}

hipError_t launch_sha_core(const DevLayout& L, const uint8_t* inputs, const uint8_t* derived, uint32_t first,
                           uint32_t count, uint32_t* sha_core, int32_t* status, uint32_t batch, hipStream_t st) {
  if (count == 0) return hipSuccess;
  if (first + count > L.n_sha) return hipErrorInvalidValue;
  dim3 g((batch + 63) / 64, count);
  hipLaunchKernelGGL(k_sha_core, g, dim3(64), 0, st, L.sha + first, (int)count, inputs, L.n_inputs, derived,
                     L.n_derived, sha_core, L.sha_core_words, status, batch);
  return hipGetLastError();
}

hipError_t launch_pss(const DevLayout& L, int stage, const uint64_t* rsa_core, const uint32_t* sha_core,
                      uint8_t* derived, uint32_t batch, hipStream_t st) {
  if (stage == 0)
    hipLaunchKernelGGL(k_pss_mgf, dim3(((L.reg.pss_h > 256 ? 1024 : 512) * L.reg.n_mgf + 255) / 256, batch), dim3(256), 0, st,
                       L, rsa_core,
                       sha_core, derived);
  else
    hipLaunchKernelGGL(k_pss_mdash, dim3(4, batch), dim3(256), 0, st, L, rsa_core, sha_core, derived);
  return hipGetLastError();
}

hipError_t launch_prep(const DevLayout& L, const uint8_t* inputs, const uint32_t* sha_core, ValueStore vs,
                       int32_t* status, hipStream_t st) {
  hipLaunchKernelGGL(k_prep, dim3(vs.batch), dim3(64), 0, st, L, inputs, sha_core, vs, status);
  return hipGetLastError();
}

hipError_t launch_qry_prep(const DevLayout& L, const uint8_t* inputs, ValueStore vs, int32_t* status, hipStream_t st) {
  hipLaunchKernelGGL(k_qry_prep, dim3((vs.batch + QP_WAVES - 1) / QP_WAVES), dim3(64 * QP_WAVES), 0, st, L, inputs, vs,
                     status);
  return hipGetLastError();
}

hipError_t launch_rsa_check(const DevLayout& L, const uint8_t* inputs, const uint32_t* sha_core,
                            const uint64_t* rsa_core, int32_t* status, uint32_t batch, hipStream_t st) {
  if (!status) return hipSuccess;
  hipLaunchKernelGGL(k_rsa_check, dim3((batch + 63) / 64), dim3(64), 0, st, L, inputs, sha_core, rsa_core, status,
                     batch);
  return hipGetLastError();
}

hipError_t launch_bjj_table(fr* table, hipStream_t st) {
  hipLaunchKernelGGL(k_bjj_table, dim3(BJJ_TABLE_WINDOWS * 256 / 256), dim3(256), 0, st, table);
  return hipGetLastError();
}

hipError_t launch_bjj_core(const DevLayout& L, ValueStore vs, const fr* table, fr* bjj_core, fr* scratch,
                           hipStream_t st) {
  // scratch given: the round-3 kernel with its global scratch array (the default, bjj_uses_scratch);
  // PZK_BJJ_SEGS: lanes per witness (scratch 8 / 16 / 32, recompute 16 / 32 / 64), for tuning runs (runtime.cpp
  // validates it)
  static const int env_segs = getenv("PZK_BJJ_SEGS") ? atoi(getenv("PZK_BJJ_SEGS")) : 0;
  const int segs = env_segs ? env_segs : scratch ? BJJ_SEGS_DEFAULT : BJJ_RC_SEGS_DEFAULT;
  const uint32_t lanes = vs.batch * segs;
  if (scratch) {
    auto kern = segs == 8 ? k_bjj_core<8> : segs == 32 ? k_bjj_core<32> : k_bjj_core<16>;
    const uint32_t wg = 64 * BJJ_WG_WAVES;
    // PZK_BJJ_PAIRED=0 (A/B): every lane sums its own segment start (bjj_seg_start) instead of the balanced pairs
    static const bool paired = !getenv("PZK_BJJ_PAIRED") || atoi(getenv("PZK_BJJ_PAIRED")) != 0;
    hipLaunchKernelGGL(kern, dim3((lanes + wg - 1) / wg), dim3(wg), 0, st, L, vs, table, bjj_core, scratch, vs.batch,
                       paired);
  } else {
    auto kern = segs == 16 ? k_bjj_core_rc<16> : segs == 32 ? k_bjj_core_rc<32> : k_bjj_core_rc<64>;
    hipLaunchKernelGGL(kern, dim3((lanes + 63) / 64), dim3(64), 0, st, L, vs, table, bjj_core, vs.batch);
  }
  return hipGetLastError();
}

bool bjj_uses_scratch() {
  const char* v = getenv("PZK_BJJ");
  return v ? !strcmp(v, "scratch") : true;
}

hipError_t launch_smt_prep(const DevLayout& L, const uint8_t* inputs, ValueStore vs, fr* smt_core, int32_t* status,
                           hipStream_t st) {
  const uint32_t wg = 64 * SMT_PREP_WAVES;
  hipLaunchKernelGGL(k_smt_prep, dim3((vs.batch * SMT_PREP_LANES + wg - 1) / wg), dim3(wg), 0, st, L, inputs, vs, smt_core,
                     status, vs.batch);
  return hipGetLastError();
}

hipError_t launch_smt_chain(const DevLayout& L, const PosConsts& K, const int32_t* level_task, const uint8_t* inputs,
                            ValueStore vs, fr* pos_core, fr* smt_core, const uint32_t* order, int32_t* status,
                            hipStream_t st) {
  // PZK_CHAIN=lane (A/B): the round-5 chain, one cooperative permutation on 4 lanes per witness with one-lane
  // products (PZK_CHAIN_MUL=inline | call | fips picks its product); default: k_smt_chain4, 16 lanes per witness on
  // quad-spread products (smt_chain4.hpp)
  static const char* ch = getenv("PZK_CHAIN");
  if (!ch || strcmp(ch, "lane") != 0) {
    hipLaunchKernelGGL(k_smt_chain4, dim3((vs.batch * 16 + 255) / 256), dim3(256), 0, st, L, K, level_task, inputs, vs,
                       pos_core, smt_core, order, status, vs.batch);
    return hipGetLastError();
  }
  static const char* pm = getenv("PZK_CHAIN_MUL");
  const int mode = !pm ? 2 : !strcmp(pm, "call") ? 1 : !strcmp(pm, "fips") ? 2 : 0;
  hipLaunchKernelGGL(mode == 1 ? k_smt_chain<FrMulCall> : mode == 2 ? k_smt_chain<FrMulFips> : k_smt_chain<FrMulInline>,
                     dim3((vs.batch * SMT_CHAIN_LANES + 63) / 64),
                     dim3(64), 0, st, L, K, level_task, inputs, vs, pos_core, smt_core, order, status, vs.batch);
  return hipGetLastError();
}

hipError_t launch_qc_build(const PosConsts& K, fr* qc, hipStream_t st) {
  hipLaunchKernelGGL(k_qc_build, dim3(1), dim3(256), 0, st, K, qc);
  return hipGetLastError();
}

// Counting sort of the batch by SMT insertion level j (0..80, written by k_smt_prep), deepest first: one workgroup.
// k_smt_chain's lane groups then take witnesses in this order, so a wave holds proofs of (nearly) one depth and
// finishes after its own depth, not after the deepest of 16 random ones (with uniform depths 0-79 that halves the
// chain's SIMD time; the kernel itself still lasts as long as the deepest proof).
__global__ void __launch_bounds__(256) k_smt_order(const fr* smt_core, uint32_t smt_core_fr, uint32_t* order,
                                                    uint32_t batch) {
  constexpr int NB = SMT_LEVELS + 1;
  __shared__ uint32_t cnt[NB], at[NB];
  for (int i = threadIdx.x; i < NB; i += blockDim.x) cnt[i] = 0;
  __syncthreads();
  auto level = [&](uint32_t w) -> uint32_t {
    const uint32_t j = reinterpret_cast<const uint32_t*>(smt_core + (size_t)w * smt_core_fr + 3 * SMT_LEVELS)[0];
    return j < (uint32_t)SMT_LEVELS ? j : (uint32_t)SMT_LEVELS;  // no insertion level: the chain walks all 80
  };
  for (uint32_t w = threadIdx.x; w < batch; w += blockDim.x) atomicAdd(&cnt[level(w)], 1u);
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t sum = 0;
    for (int k = NB - 1; k >= 0; k--) { at[k] = sum; sum += cnt[k]; }  // deepest first
  }
  __syncthreads();
  for (uint32_t w = threadIdx.x; w < batch; w += blockDim.x) order[atomicAdd(&at[level(w)], 1u)] = w;
}
hipError_t launch_smt_order(const fr* smt_core, uint32_t smt_core_fr, uint32_t* order, uint32_t batch, hipStream_t st) {
  // 256 threads: one workgroup that fits beside the emitters' waves on any CU (a 1024-thread group waited
  // ~1.7 ms for a CU with 16 free wave slots inside the concurrent config-3 run)
  hipLaunchKernelGGL(k_smt_order, dim3(1), dim3(256), 0, st, smt_core, smt_core_fr, order, batch);
  return hipGetLastError();
}

// 1/k mod p (normal form) for k < 256: IsEqual inverses of small differences (ECDSA selections)
__global__ void k_inv_small(fr* out) {
  const int k = threadIdx.x;
  out[k] = k == 0 ? fr_zero() : fr_from_mont(fr_inv(fr_to_mont(fr_u64((uint64_t)k))));
}
hipError_t launch_inv_small(fr* out, hipStream_t st) {
  hipLaunchKernelGGL(k_inv_small, dim3(1), dim3(256), 0, st, out);
  return hipGetLastError();
}

hipError_t launch_emit(int emitter, const DevLayout& L, const Work* work, uint32_t n_work, const PosConsts& K,
                       const Bufs& B, uint32_t batch, int max_t, hipStream_t st) {
  if (n_work == 0) return hipSuccess;
  dim3 g(n_work, batch), blk(EMIT_THREADS);
  switch (emitter) {
    case E_GEN: case E_GENR: hipLaunchKernelGGL(k_emit_gen, g, blk, 0, st, L, work, B); break;
    case E_QRY: hipLaunchKernelGGL(k_emit_qry, g, blk, 0, st, L, work, B); break;
    case E_SHA: case E_SHAD:  // witness-major grid (see k_emit_sha)
    {  // PZK_SHA_U (8 / 16 / 32): prefetch depth, for tuning runs
      static const int u = getenv("PZK_SHA_U") ? atoi(getenv("PZK_SHA_U")) : 16;
      auto kern = L.keep.bits ? k_emit_sha<16, MAP_DIRECT>
                  : u == 8 ? k_emit_sha<8, MAP_O0> : u == 32 ? k_emit_sha<32, MAP_O0> : k_emit_sha<16, MAP_O0>;
      hipLaunchKernelGGL(kern, dim3(batch, n_work), blk, 0, st, L, work, B.inputs, B.derived, B.sha_core, B.wtns,
                         B.stride, 1);
      break;
    }
    case E_POS: return launch_emit_pos(L, work, n_work, K, B, batch, max_t, st);  // one launch per width (kernels_pos.hip)
    case E_BITS: hipLaunchKernelGGL(k_emit_bits, g, blk, 0, st, L, work, B); break;
    case E_FLOW: hipLaunchKernelGGL(k_emit_flow, g, blk, 0, st, L, work, B); break;
    case E_MM: return launch_emit_mm(L, work, n_work, B, batch, st);  // kernels_rsa.hip
    case E_ECR: return launch_emit_ecr(L, work, n_work, B, batch, st);  // kernels_ec*.hip
    case E_BJJ: hipLaunchKernelGGL(k_emit_bjj, g, blk, 0, st, L, work, B); break;
    case E_SHA5:
    case E_SHA5D:
      hipLaunchKernelGGL(k_emit_sha512, dim3(batch, n_work), blk, 0, st, L, work, B.inputs, B.derived, B.sha_core, B.wtns,
                         B.stride);
      break;
    case E_SHA1:  // witness-major grid, as k_emit_sha
      hipLaunchKernelGGL(k_emit_sha1, dim3(batch, n_work), blk, 0, st, L, work, B.inputs, B.derived, B.sha_core, B.wtns,
                         B.stride);
      break;
    case E_ECT: return launch_emit_ect(L, work, n_work, B, batch, st);
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace pzk
