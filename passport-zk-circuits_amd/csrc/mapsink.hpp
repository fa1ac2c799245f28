// Witness stores of the emit kernels, O0 or .sym-mapped.
//
// An emitter produces O0 elements: element q of a run is the signal with O0 index g + q. Without a map it
// is stored at row[g + q]. With a monotone map (pzk_instance_create_mapped, every kept signal's witness
// index increasing with its O0 index — the order circom gives the kept signals) the kept elements of any
// run are CONSECUTIVE in the mapped row, so the emitter writes the mapped witness directly: element
// g goes to row[rank(g)], rank(g) = number of kept signals below g, and dropped elements are not
// stored (emit_run skips the evaluation of a wave with no kept element). The map is a keep bitmap over the O0 indices (one u64 per 64
// signals) and the rank at every 64-signal boundary (one u32), read per wave with SCALAR loads: a wave's
// 64 consecutive elements span at most two bitmap words, the address is wave-uniform, and scalar loads
// are counted by lgkmcnt, so unlike a vector load they never wait for the wave's stores in flight (gfx9
// vmcnt counts loads and stores together; DESIGN.md §4.2 rule 1).
#pragma once
#include "fr.hpp"
#include "layout.hpp"

namespace pzk {

typedef __attribute__((address_space(4))) const uint64_t cu64_t;
typedef __attribute__((address_space(4))) const uint32_t cu32_t;

// bitmap words [i, i + 1] and their ranks: covers O0 indices [64 i, 64 i + 128)
struct MapWin {
  uint64_t w0, w1;
  uint32_t r0, r1;
  uint64_t base;
};
// g0: a wave-uniform O0 index (every lane passes the same value)
__device__ __forceinline__ MapWin map_win(const KeepMap& M, uint64_t g0) {
  const uint32_t i = __builtin_amdgcn_readfirstlane((uint32_t)(g0 >> 6));
  cu64_t* b = (cu64_t*)M.bits;
  cu32_t* r = (cu32_t*)M.rank;
  MapWin m;
  m.w0 = b[i];
  m.w1 = b[i + 1];
  m.r0 = r[i];
  m.r1 = r[i + 1];
  m.base = (uint64_t)i << 6;
  return m;
}
__device__ __forceinline__ bool map_keep(const MapWin& m, uint64_t g) {  // g in [base, base + 128)
  const uint32_t d = (uint32_t)(g - m.base);
  return ((d < 64 ? m.w0 : m.w1) >> (d & 63)) & 1;
}
__device__ __forceinline__ uint32_t map_rank(const MapWin& m, uint64_t g) {  // kept signals below g
  const uint32_t d = (uint32_t)(g - m.base);
  const uint64_t w = d < 64 ? m.w0 : m.w1;
  return (d < 64 ? m.r0 : m.r1) + (uint32_t)__popcll(w & ((1ull << (d & 63)) - 1));
}
// per-lane form (vector loads: only where no store of the wave is in flight yet, e.g. k_emit_gen's load pass)
__device__ __forceinline__ bool map_keep_lane(const KeepMap& M, uint64_t g, uint32_t& rank) {
  const uint64_t w = M.bits[g >> 6];
  rank = M.rank[g >> 6] + (uint32_t)__popcll(w & ((1ull << (g & 63)) - 1));
  return (w >> (g & 63)) & 1;
}

// Store modes: the hot emitters are compiled per mode (O0 / direct), so their O0 code is the plain store
// loop; the rest check the instance's map at run time (a wave-uniform branch).
enum { MAP_O0 = 0, MAP_DIRECT = 1, MAP_ANY = 2 };

// One emitter run's destination: O0 element g + q of the witness row `row`.
struct OutRow {
  uint8_t* row;  // the witness row (mapped: the compact row)
  uint64_t g;    // O0 index of element 0 of the run
  KeepMap map;   // map.bits == nullptr: O0, the identity
  __device__ OutRow at(uint64_t q) const { return OutRow{row, g + q, map}; }
};
__device__ __forceinline__ OutRow out_row(const DevLayout& L, uint8_t* wtns, size_t stride, uint32_t w, uint64_t g) {
  return OutRow{wtns + (size_t)w * stride, g, L.keep};
}

// Half h of element h / 2 of the run (16 B; the "two lanes per element" store shape: with all lanes of a
// wave storing consecutive halves, every wave store is 1 KiB contiguous; mapped, the kept halves of a wave
// are still consecutive). Called with a wave's 64 lanes on 64 consecutive h (h - lane wave-uniform); lanes
// with valid = false store nothing but take part.
template <int MM = MAP_ANY>
__device__ __forceinline__ void store_half(const OutRow& o, uint32_t h, const uint4& v, bool valid) {
  if (MM == MAP_O0 || (MM == MAP_ANY && !o.map.bits)) {
    if (valid) reinterpret_cast<uint4*>(o.row + 32ull * o.g)[h] = v;
    return;
  }
  const uint32_t lane = threadIdx.x & 63;
  const MapWin m = map_win(o.map, o.g + ((h - lane) >> 1));
  const uint64_t e = o.g + (h >> 1);
  if (valid && map_keep(m, e)) reinterpret_cast<uint4*>(o.row)[2ull * map_rank(m, e) + (h & 1)] = v;
}

// kept signals below O0 index g (wave-uniform g): the mapped row index of the first kept element at or after g
__device__ __forceinline__ uint32_t map_rank_at(const KeepMap& M, uint64_t g) {
  const uint32_t i = __builtin_amdgcn_readfirstlane((uint32_t)(g >> 6));
  const uint64_t w = ((cu64_t*)M.bits)[i];
  return ((cu32_t*)M.rank)[i] + (uint32_t)__popcll(w & ((1ull << (g & 63)) - 1));
}

// Block-wide (every thread calls it; it ends with __syncthreads): the kept elements among the run's O0 elements
// [a, a + n) (n > 0), ascending, as list[k] = payload(q) with q their offset from a; returns how many. Kept element
// k goes to mapped row index map_rank_at(o.g + a) + k. Each wave takes whole bitmap words (scalar loads: the
// address is wave-uniform), a lane per bit, and places its kept bit by the word's rank + the set bits below it.
template <typename T, typename P>
__device__ __forceinline__ uint32_t kept_collect(const OutRow& o, uint32_t a, uint32_t n, T* list, P payload) {
  const uint64_t lo = o.g + a, hi = lo + n;
  const uint32_t r0 = map_rank_at(o.map, lo), nk = map_rank_at(o.map, hi) - r0;
  const uint32_t lane = threadIdx.x & 63, nw = blockDim.x >> 6;
  const uint32_t i0 = (uint32_t)(lo >> 6), i1 = (uint32_t)((hi - 1) >> 6);
  for (uint32_t i = i0 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); i <= i1; i += nw) {
    const uint32_t iu = __builtin_amdgcn_readfirstlane(i);
    const uint64_t word = ((cu64_t*)o.map.bits)[iu];
    const uint32_t rk = ((cu32_t*)o.map.rank)[iu];
    const uint64_t e = ((uint64_t)iu << 6) + lane;
    if (((word >> lane) & 1) && e >= lo && e < hi)
      list[rk + (uint32_t)__popcll(word & ((1ull << lane) - 1)) - r0] = payload((uint32_t)(e - lo));
  }
  __syncthreads();
  return nk;
}

// the kept-offset list of mapped emit_run segments (one LDS array per kernel, whichever element functions it runs).
// 26 bitmap words, sized for occupancy: with 2,048 the mapped k_emit_mm<32> took 40,984 B of LDS (24 B over a
// quarter of the CU's 160 KiB: three workgroups per CU instead of four) and the mapped k_emit_sha 21,152 B (seven
// instead of the eight its registers allow)
constexpr uint32_t MAP_SEG = 1664;
template <uint32_t SEG = MAP_SEG>
__device__ __forceinline__ uint16_t* map_seg_list() {
  __shared__ uint16_t klist[SEG];
  return klist;
}

// for (q < count) out[q] = f(q), wave-contiguous (fr.hpp emit_run).
// Mapped (block-wide: every thread of the workgroup calls it): the run is taken in segments of MAP_SEG O0
// elements; per segment the kept offsets are collected into LDS (kept_collect) and the waves evaluate f on the
// KEPT elements only, 64 per wave instruction, stored contiguously at the segment's mapped index (the kept
// elements of a run are consecutive in a monotone map). LANE_INDEP = false: f scans across the wave's lanes
// (regemit.hpp bmneq_tmpr needs 64 consecutive q per wave), so every element of a wave with a kept one is
// evaluated in O0 order and the kept ones are compacted through the stage.
template <int MM = MAP_ANY, bool LANE_INDEP = true, int SW = 128, uint32_t SEG = MAP_SEG, typename F>
__device__ __forceinline__ void emit_run(const OutRow& o, uint32_t count, uint4* stage_block, F f) {
  if (MM == MAP_O0 || (MM == MAP_ANY && !o.map.bits)) {
    emit_run<SW>(o.row + 32ull * o.g, count, stage_block, f);
    return;
  }
  const uint32_t lane = threadIdx.x & 63;
  uint4* stage = stage_block + (threadIdx.x >> 6) * SW;
  if constexpr (LANE_INDEP) {
    uint16_t* klist = map_seg_list<SEG>();
    for (uint32_t a = 0; a < count; a += SEG) {
      const uint32_t n = min(SEG, count - a);
      const uint32_t r0 = map_rank_at(o.map, o.g + a);
      const uint32_t nk = kept_collect(o, a, n, klist, [](uint32_t q) { return (uint16_t)q; });
      uint8_t* dst = o.row + 32ull * r0;
      for (uint32_t k0 = threadIdx.x - lane; k0 < nk; k0 += blockDim.x) {
        const uint32_t k = k0 + lane;
        const El e = k < nk ? f(a + klist[k]) : el_zero();
        wave_store<SW>(dst + 32ull * k0, e, nk - k0 < 64 ? nk - k0 : 64, stage);
      }
      __syncthreads();  // klist is rewritten by the next segment
    }
  } else {
    for (uint32_t q0 = threadIdx.x - lane; q0 < count; q0 += blockDim.x) {
      const uint32_t q = q0 + lane;
      const MapWin m = map_win(o.map, o.g + q0);
      const bool keep = q < count && map_keep(m, o.g + q);
      const uint64_t mask = __ballot(keep);
      if (mask == 0) continue;  // wave-uniform
      const El e = q < count ? f(q) : el_zero();
      const uint32_t pos = (uint32_t)__popcll(mask & ((1ull << lane) - 1)), nk = (uint32_t)__popcll(mask);
      uint4* d = reinterpret_cast<uint4*>(o.row + 32ull * map_rank(m, o.g + q0));
      if constexpr (SW == 128) {
        if (keep) {
          stage[2 * pos] = e.lo;
          stage[2 * pos + 1] = e.hi;
        }
        wave_sync();
        const uint4 a = stage[lane], b = stage[64 + lane];
        if (lane < 2 * nk) d[lane] = a;
        if (64 + lane < 2 * nk) d[64 + lane] = b;
        wave_sync();
      } else {
#pragma unroll
        for (uint32_t h = 0; h < 2; h++) {  // kept elements 32 h .. 32 h + 31
          if (keep && (pos >> 5) == h) {
            stage[2 * (pos & 31)] = e.lo;
            stage[2 * (pos & 31) + 1] = e.hi;
          }
          wave_sync();
          const uint4 a = stage[lane];
          if (64 * h + lane < 2 * nk) d[64 * h + lane] = a;
          wave_sync();
        }
      }
    }
  }
}

// A descriptor-driven emitter's work item (k_emit_sha block programs, k_emit_pos, k_emit_ect): O0, its
// descriptors are prog[0 .. count) and it stores at O0 index g; mapped, the instance's compacted program
// (DevLayout.mprog, built by pzk_instance_create_mapped) holds the kept elements' descriptors at Work.pad, and
// they go to consecutive mapped indices from rank(g). Either way the store loop is the O0 loop.
struct DescRun {
  const uint32_t* prog;  // mapped: L.mprog + Work.pad
  uint32_t count;        // elements to store
  OutRow out;            // identity store: row + 32 * (out.g + k)
};
template <int MM>
__device__ __forceinline__ DescRun desc_run(const DevLayout& L, uint8_t* wtns, size_t stride, uint32_t w, const Work& wk,
                                            uint64_t g, const uint32_t* o0_prog) {
  uint8_t* row = wtns + (size_t)w * stride;
  if (MM == MAP_O0 || (MM == MAP_ANY && !L.keep.bits)) return DescRun{o0_prog, wk.count, OutRow{row, g, KeepMap{nullptr, nullptr}}};
  const uint32_t r0 = map_rank_at(L.keep, g), r1 = map_rank_at(L.keep, g + wk.count);
  return DescRun{L.mprog + wk.pad, r1 - r0, OutRow{row, r0, KeepMap{nullptr, nullptr}}};
}

}  // namespace pzk
