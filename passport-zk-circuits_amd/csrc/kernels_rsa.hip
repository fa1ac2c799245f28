// RSA kernels: the BigMultModP cores of PowerMod (cooperative Barrett / Knuth D), the batched IsEqual
// inversions, and the BigMultModP block emitter, with their launchers. Own translation unit (template
// kernels only from the shared headers), so it compiles in parallel with kernels.hip.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define PZK_TEMPLATE_KERNELS_ONLY
#include "regemit.hpp"
#include "rsa_coop.hpp"
#include "kernels.hpp"

namespace pzk {

#define HIP_TRY(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return e_; } while (0)

// RSA core: the cooperative Barrett kernel (rsa_coop.hpp) by default; PZK_RSA_CORE=lane selects
// the one-lane-per-witness Knuth D kernel (regcore.hpp) for A/B measurements.
template <int K, int G>
static hipError_t launch_rsa_core2(const DevLayout& L, const uint8_t* inputs, uint64_t* rsa_core, int32_t* status,
                                   uint32_t batch, hipStream_t st) {
  constexpr int WPB = 64 / G;
  const size_t lds = sizeof(uint64_t) * rsa2_lds_words<K>() * WPB;
  HIP_TRY(hipFuncSetAttribute((const void*)k_rsa_core2<K, G>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL((k_rsa_core2<K, G>), dim3((batch + WPB - 1) / WPB), dim3(64), lds, st, L, inputs, rsa_core, status,
                     batch);
  return hipGetLastError();
}

template <int K, int NL>
static hipError_t launch_rsa_lane(const DevLayout& L, const uint8_t* inputs, uint64_t* rsa_core, uint64_t* colsum,
                                  int32_t* status, uint32_t batch, hipStream_t st) {
  const size_t lds = sizeof(uint64_t) * rsa_lds_words<K>() * NL;
  HIP_TRY(hipFuncSetAttribute((const void*)k_rsa_core<K, NL>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL((k_rsa_core<K, NL>), dim3((batch + NL - 1) / NL), dim3(NL), lds, st, L, inputs, rsa_core, colsum,
                     status, batch);
  return hipGetLastError();
}

static bool rsa_core_lane() {
  static const int v = [] {
    const char* e = getenv("PZK_RSA_CORE");
    return e && e[0] == 'l' ? 1 : 0;
  }();
  return v;
}

hipError_t launch_rsa_core(const DevLayout& L, const uint8_t* inputs, uint64_t* rsa_core, uint64_t* colsum,
                           int32_t* status, uint32_t batch, hipStream_t st) {
  const bool lane = rsa_core_lane() && colsum;
  if (L.reg.K == 48) {  // RSA-3072 (SIGNATURE_TYPE 14): cooperative core only
    HIP_TRY((launch_rsa_core2<48, 16>(L, inputs, rsa_core, status, batch, st)));
    hipLaunchKernelGGL(k_rsa_inv<48>, dim3((batch + RI_WAVES - 1) / RI_WAVES), dim3(64 * RI_WAVES), 0, st, L, inputs,
                       rsa_core, batch);
  } else if (L.reg.K == 32) {
    HIP_TRY((lane ? launch_rsa_lane<32, 64>(L, inputs, rsa_core, colsum, status, batch, st)
                  : launch_rsa_core2<32, 8>(L, inputs, rsa_core, status, batch, st)));
    hipLaunchKernelGGL(k_rsa_inv<32>, dim3((batch + RI_WAVES - 1) / RI_WAVES), dim3(64 * RI_WAVES), 0, st, L, inputs,
                       rsa_core, batch);
  } else {
    HIP_TRY((lane ? launch_rsa_lane<64, 32>(L, inputs, rsa_core, colsum, status, batch, st)
                  : launch_rsa_core2<64, 16>(L, inputs, rsa_core, status, batch, st)));
    hipLaunchKernelGGL(k_rsa_inv<64>, dim3((batch + RI_WAVES - 1) / RI_WAVES), dim3(64 * RI_WAVES), 0, st, L, inputs,
                       rsa_core, batch);
  }
  return hipGetLastError();
}

hipError_t launch_emit_mm(const DevLayout& L, const Work* work, uint32_t n_work, const Bufs& B, uint32_t batch,
                          hipStream_t st) {
#ifdef PZK_MM_PROF
  {  // cumulative per-section clocks (wave 0 of each workgroup), printed at every launch after a sync
    static int n = 0;
    if (++n > 1) {
      unsigned long long h[MM_SECTIONS + 2];
      if (hipDeviceSynchronize() == hipSuccess && hipMemcpyFromSymbol(h, HIP_SYMBOL(g_mm_prof), sizeof h) == hipSuccess) {
        fprintf(stderr, "mm_prof launches=%d", n - 1);
        for (int i = 0; i <= (int)MM_SECTIONS; i++) fprintf(stderr, " %llu", h[i]);
        fprintf(stderr, "\n");
      }
    }
  }
#endif
  if (n_work == 0) return hipSuccess;
  const bool m = L.keep.bits != nullptr;  // store mode (mapsink.hpp)
  // O0 K = 32: eight waves per workgroup (35 KB of LDS, three per CU by registers: 24 waves instead of 5 x 4 = 20, the
  // prologue's column sums and tables on twice the threads): config 3 +1.0 % on one box, k_emit_sha's share of
  // the chip up with it (profiles/r5z). PZK_MM_THREADS=256 restores four waves.
  static const bool wide = !getenv("PZK_MM_THREADS") || atoi(getenv("PZK_MM_THREADS")) != 256;
  const bool w512 = wide && !m && L.reg.K == 32;
  dim3 g(n_work, batch), blk(w512 ? 512 : EMIT_THREADS);
  auto kern = w512 ? k_emit_mm<32, MAP_O0, 512>
            : L.reg.K == 32 ? (m ? k_emit_mm<32, MAP_DIRECT> : k_emit_mm<32, MAP_O0>)
            : L.reg.K == 48 ? (m ? k_emit_mm<48, MAP_DIRECT> : k_emit_mm<48, MAP_O0>)
                            : (m ? k_emit_mm<64, MAP_DIRECT> : k_emit_mm<64, MAP_O0>);
  hipLaunchKernelGGL(kern, g, blk, 0, st, L, work, B);
  return hipGetLastError();
}

}  // namespace pzk
