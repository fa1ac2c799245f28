// PoseidonHash block emitter (k_emit_pos<t>, t = 2..6) and its launcher. Own translation unit (template
// kernels only from the shared headers), so it compiles in parallel with the other kernel units.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <stdio.h>

#define PZK_TEMPLATE_KERNELS_ONLY
#include "bufs.hpp"
#include "poseidon.hpp"
#include "mapsink.hpp"
#include "kernels.hpp"

namespace pzk {

#ifdef PZK_MM_PROF  // profiling build only: image fill / store clocks of wave 0 of every workgroup
static __device__ unsigned long long g_pos_prof[2];
#define PZK_POS_CLK(v) const long long v = clock64()
#define PZK_POS_ACC(i, t0) do { const long long t1_ = clock64(); if (threadIdx.x == 0) atomicAdd(&g_pos_prof[i], (unsigned long long)(t1_ - (t0))); } while (0)
#else
#define PZK_POS_CLK(v)
#define PZK_POS_ACC(i, t0)
#endif

// ------------------------------------------------------------------- emit: Poseidon
// A workgroup emits one PoseidonHash block (a Work item) for WPB consecutive witnesses: per witness it
// fills the permutation's value image in LDS (pos_img_fill), then stores the block's signals from it. The
// stores of witness k are still in flight while the image of witness k + 1 is computed, so one workgroup
// overlaps its own compute with its store drain; the block's descriptors are loaded once per WPB witnesses.
template <int T, int MM>
// (t <= 3: at most 96 VGPRs, so five workgroups fit on a CU as their LDS allows; wider blocks are LDS-bound at <= 4)
__global__ void __launch_bounds__(EMIT_THREADS, T <= 3 ? 5 : 1) k_emit_pos(DevLayout L, const Work* work, PosConsts K, ValueStore vs,
                                                          const fr* pos_core, uint8_t* wtns, size_t stride, uint32_t batch,
                                                          uint32_t wpb, bool kept_fill) {
  constexpr PosImg I(T);
  // the image: dynamic LDS of I.size elements, or I.fs when no block of the launch keeps a GetSum signal (mapped
  // layouts, DevLayout.pos_nomix: the image parts from fs on are never filled or read then)
  extern __shared__ uint4 pos_img_lds[];
  fr* img = reinterpret_cast<fr*>(pos_img_lds);
  const Work wk = work[blockIdx.x];
  const Region R = L.regions[wk.region];
  const PosTask& task = L.pos[R.a[0]];  // global: in_slot is indexed at run time
  // the block's descriptors go to LDS first: a global load inside the store loop would wait for
  // every store in flight (gfx9 vmcnt counts stores too)
  // (mapped: the kept elements' image indices, from the instance's compacted program, desc_run)
  __shared__ uint16_t prog[pos_hash_size_c(T - 1)];
  const DescRun dr0 = desc_run<MM>(L, wtns, stride, 0, wk, R.off + wk.start, nullptr);
  const uint32_t cnt = dr0.count;
  const uint32_t w0 = blockIdx.y * wpb, w1 = min(batch, w0 + wpb);
  // which of the workgroup's witnesses have zero inputs: tested before any store (wpb <= 64)
  uint64_t zmask = 0;
  for (uint32_t w = w0; w < w1; w++) zmask |= (uint64_t)pos_inputs_zero(task, vs, w) << (w - w0);
  // (an O0 workgroup whose witnesses are all zero blocks copies zero rows and needs no program)
  // mapped: the image parts the kept signals read (pos_img_need), so the fill skips the rest (the O2-shaped map keeps
  // the S-box powers of a block: no GetSum row, no partial-round state)
  __shared__ uint32_t need_s;
  if (MM == MAP_DIRECT && kept_fill) {
    if (threadIdx.x == 0) need_s = 0;
    __syncthreads();
    uint32_t need = 0;
    for (uint32_t i = threadIdx.x; i < cnt; i += blockDim.x) {
      const uint32_t d = dr0.prog[i];
      prog[i] = (uint16_t)d;
      need |= pos_img_need<T>(d);
    }
    if (need) atomicOr(&need_s, need);
  } else if (MM == MAP_DIRECT) {
    for (uint32_t i = threadIdx.x; i < cnt; i += blockDim.x) prog[i] = (uint16_t)dr0.prog[i];
  } else if (zmask != (w1 - w0 == 64 ? ~0ull : (1ull << (w1 - w0)) - 1)) {
    for (uint32_t i = threadIdx.x; i < cnt; i += blockDim.x) prog[i] = L.pos_prog[L.pos_prog_off[T] + wk.start + i];
  }
  __syncthreads();
  const uint32_t need = MM == MAP_DIRECT && kept_fill ? need_s : (uint32_t)PI_ALL;
  const uint32_t tot = 2 * cnt;
  for (uint32_t w = w0; w < w1; w++) {
    if ((zmask >> (w - w0)) & 1) {
      // zero inputs (the SMT levels below the insertion level): the block is the constant zero-input one (no core
      // was written for this witness), read from global memory (L2-resident): O0, a straight copy of the block's
      // zero row (K.Zrow); mapped, the kept elements gathered from the zero image through the compacted program.
      // U halves per lane loaded ahead of their stores.
      constexpr int U = 8;
      uint4* dst = reinterpret_cast<uint4*>(wtns + (size_t)w * stride) + 2 * dr0.out.g;
      const uint4* z = reinterpret_cast<const uint4*>(MM == MAP_O0 ? K.Zrow(T) + wk.start : K.Zimg(T));
      for (uint32_t h0 = threadIdx.x; h0 < tot; h0 += U * blockDim.x) {
        uint4 v[U];
#pragma unroll
        for (int k = 0; k < U; k++) {
          const uint32_t h = h0 + k * blockDim.x;
          v[k] = h < tot ? z[MM == MAP_O0 ? h : 2u * prog[h >> 1] + (h & 1)] : make_uint4(0u, 0u, 0u, 0u);
        }
#pragma unroll
        for (int k = 0; k < U; k++) {
          const uint32_t h = h0 + k * blockDim.x;
          if (h < tot) dst[h] = v[k];
        }
      }
      continue;
    }
    __syncthreads();  // every lane has read the previous witness's image
    PZK_POS_CLK(t0);
    pos_img_fill<T>(img, K, pos_core + (size_t)w * L.pos_core_elems + task.core_off, vs, task, w, need);
    PZK_POS_ACC(0, t0);
    PZK_POS_CLK(t1);
    // two lanes per element (16 B each, 1 KiB contiguous per wave store), each copying its half
    const OutRow out{wtns + (size_t)w * stride, dr0.out.g, KeepMap{nullptr, nullptr}};
    const uint4* im = reinterpret_cast<const uint4*>(img);
    for (uint32_t h = threadIdx.x; h < tot; h += blockDim.x)
      store_half<MAP_O0>(out, h, im[2u * prog[h >> 1] + (h & 1)], true);
    PZK_POS_ACC(1, t1);
  }
}

// The zero-input block of width T (setup, once per instance): the permutation of zeros on one lane, then its image.
// scratch: 2 + 512 Fr (a one-witness value store: slot 0 = every input, slot 1 = the hash; the core's states)
template <int T>
__global__ void __launch_bounds__(256) k_pos_zero_img(PosConsts K, fr* scratch, fr* zimg) {
  constexpr PosImg I(T);
  __shared__ fr img[I.size];
  __shared__ fr lines[4 * 64];
  PosTask task{};
  task.n = T - 1;
  task.out_slot = 1;
  task.smt_level = -1;
  const ValueStore vs{scratch, 1};
  fr* core = scratch + 4;  // 128-byte aligned (PosLineSink writes whole lines)
  if (threadIdx.x == 0) {
    scratch[0] = fr_zero();
    pos_core_lane<T>(K, task, vs, 0, PosLineSink{core, lines});
  }
  __threadfence();
  __syncthreads();
  pos_img_fill<T>(img, K, core, vs, task, 0);
  fr* out = zimg + pos_zimg_off(T);
  for (int i = threadIdx.x; i < I.size; i += blockDim.x) out[i] = img[i];
  if (threadIdx.x == 0) out[I.size] = vs.at(1, 0);
}

hipError_t launch_pos_zero_img(const PosConsts& K, fr* scratch, fr* zimg, hipStream_t st) {
  hipLaunchKernelGGL(k_pos_zero_img<2>, dim3(1), dim3(256), 0, st, K, scratch, zimg);
  hipLaunchKernelGGL(k_pos_zero_img<3>, dim3(1), dim3(256), 0, st, K, scratch, zimg);
  hipLaunchKernelGGL(k_pos_zero_img<4>, dim3(1), dim3(256), 0, st, K, scratch, zimg);
  hipLaunchKernelGGL(k_pos_zero_img<5>, dim3(1), dim3(256), 0, st, K, scratch, zimg);
  hipLaunchKernelGGL(k_pos_zero_img<6>, dim3(1), dim3(256), 0, st, K, scratch, zimg);
  return hipGetLastError();
}

// witnesses per workgroup (A/B: PZK_POS_WPB, default 1)
static uint32_t pos_wpb() {
  static const uint32_t v = [] {
    const char* e = getenv("PZK_POS_WPB");
    const int x = e ? atoi(e) : 1;
    return (uint32_t)(x < 1 ? 1 : x > 64 ? 64 : x);
  }();
  return v;
}

hipError_t launch_emit_pos(const DevLayout& L, const Work* work, uint32_t n_work, const PosConsts& K, const Bufs& B,
                           uint32_t batch, int t, hipStream_t st) {
#ifdef PZK_MM_PROF
  {
    static int n = 0;
    unsigned long long h[2];
    if (++n > 1 && hipDeviceSynchronize() == hipSuccess && hipMemcpyFromSymbol(h, HIP_SYMBOL(g_pos_prof), sizeof h) == hipSuccess)
      fprintf(stderr, "pos_prof launches=%d fill %llu store %llu\n", n - 1, h[0], h[1]);
  }
#endif
  if (n_work == 0) return hipSuccess;
  const uint32_t wpb = pos_wpb();
  static const bool kept_fill = getenv("PZK_POS_FULL") == nullptr;  // A/B: mapped blocks fill the whole image
  dim3 g(n_work, (batch + wpb - 1) / wpb), blk(EMIT_THREADS);
  // LDS image size (k_emit_pos): the part before the GetSum rows when the launch's blocks keep none of them. The
  // width-6 image is 63 KB, and beside the other emitters' workgroups (k_emit_sha 20 KB, k_emit_mm 32 KB, ... packed
  // onto every CU) such a workgroup waited for a CU with that much LDS free: k_emit_pos<6> ran 40x its standalone
  // time in the concurrent schedule and its stream paced the O2-shaped line (profiles/r6k)
  const bool small = L.keep.bits && kept_fill && ((L.pos_nomix >> t) & 1u);
  const size_t lds = 32ull * (small ? (size_t)PosImg(t).fs : (size_t)PosImg(t).size);
#define PZK_POS_LAUNCH(T_)                                                                                              \
  {                                                                                                                    \
    auto kern = L.keep.bits ? k_emit_pos<T_, MAP_DIRECT> : k_emit_pos<T_, MAP_O0>;                                     \
    static bool attr[2] = {false, false};                                                                              \
    if (!attr[L.keep.bits ? 1 : 0]) {                                                                                  \
      (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,                         \
                                32 * PosImg(T_).size);                                                                 \
      attr[L.keep.bits ? 1 : 0] = true;                                                                                \
    }                                                                                                                  \
    hipLaunchKernelGGL(kern, g, blk, lds, st, L, work, K, B.vs, B.pos_core, B.wtns, B.stride, batch, wpb, kept_fill);   \
  }
  switch (t) {
    case 2: PZK_POS_LAUNCH(2); break;
    case 3: PZK_POS_LAUNCH(3); break;
    case 4: PZK_POS_LAUNCH(4); break;
    case 5: PZK_POS_LAUNCH(5); break;
    case 6: PZK_POS_LAUNCH(6); break;
    default: return hipErrorInvalidValue;
  }
#undef PZK_POS_LAUNCH
  return hipGetLastError();
}

}  // namespace pzk
