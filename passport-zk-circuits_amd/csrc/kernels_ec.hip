// ECDSA kernels (ec_core.hpp) and their launchers; a separate translation unit from kernels.hip so the
// two compile in parallel. Compiled once per curve: this file for PZK_EC_CURVE 0 (secp256r1), and
// kernels_ec_bp.hip / kernels_ec_p224.hip / kernels_ec_bp384.hip include it with PZK_EC_CURVE 1 / 2 / 3
// (brainpoolP256r1 / secp224r1 / brainpoolP384r1). The curve-0 unit also defines the public launchers,
// which dispatch on the instance's curve.
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include "bufs.hpp"
#include "ec_core.hpp"
#include "kernels.hpp"

namespace pzk {
inline namespace PZK_EC_NS {

#define HIP_TRY(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return e_; } while (0)

hipError_t launch_ec_core_cv(const DevLayout& L, const uint8_t* inputs, const uint32_t* sha_core, uint64_t* ec_core,
                          uint64_t* ec_jac, fr* ec_inv, int32_t* status, uint32_t batch, hipStream_t st) {
  hipLaunchKernelGGL(k_ec_scalars, dim3((batch + 63) / 64), dim3(64), 0, st, L, inputs, sha_core, ec_core, status, batch);
  HIP_TRY(hipGetLastError());
  hipLaunchKernelGGL(k_ec_chain, dim3((2 * batch + 63) / 64), dim3(64), 0, st, L, inputs, ec_core, ec_jac, batch);
  HIP_TRY(hipGetLastError());
  hipLaunchKernelGGL(k_ec_final, dim3((batch + 63) / 64), dim3(64), 0, st, ec_jac, batch);
  HIP_TRY(hipGetLastError());
  hipLaunchKernelGGL(k_ec_affine, dim3((batch * EC_AFF_GROUPS + 63) / 64), dim3(64), 0, st, ec_core, ec_jac, status,
                     batch);
  HIP_TRY(hipGetLastError());
  hipLaunchKernelGGL(k_ec_link, dim3((batch * EC_LINK_ITEMS + 63) / 64), dim3(64), 0, st, L, inputs, ec_core, ec_jac,
                     status, batch);
  HIP_TRY(hipGetLastError());
  hipLaunchKernelGGL(k_ec_inv, dim3((batch * ECG.n_inv + 63) / 64), dim3(64), 0, st, ec_core, ec_inv, batch);
  return hipGetLastError();
}

hipError_t launch_ec_table_cv(const DevLayout& L, int type, const int32_t* ops, uint32_t n_ops, const uint64_t* ec_core,
                           uint8_t* ec_tab, int32_t* status, uint32_t batch, hipStream_t st) {
  if (n_ops == 0) return hipSuccess;
  dim3 g((batch + 63) / 64, n_ops);
  switch (type) {
    case ECT_DBL: hipLaunchKernelGGL(k_ec_table<ECT_DBL>, g, dim3(64), 0, st, L, ops, ec_core, ec_tab, status, batch); break;
    case ECT_ADD: hipLaunchKernelGGL(k_ec_table<ECT_ADD>, g, dim3(64), 0, st, L, ops, ec_core, ec_tab, status, batch); break;
    default: hipLaunchKernelGGL(k_ec_table<ECT_MM>, g, dim3(64), 0, st, L, ops, ec_core, ec_tab, status, batch); break;
  }
  return hipGetLastError();
}

hipError_t launch_emit_ect_cv(const DevLayout& L, const Work* work, uint32_t n_work, const Bufs& B, uint32_t batch,
                           hipStream_t st) {
  if (n_work == 0) return hipSuccess;
  static const int prefetch = getenv("PZK_ECT_PREFETCH") ? atoi(getenv("PZK_ECT_PREFETCH")) : 1;
  static const int u = getenv("PZK_ECT_U") ? atoi(getenv("PZK_ECT_U")) : 16;  // isolated P-256: 8 / 16 / 32 = 22.6 / 21.7 / 41.0 ms
  auto kern = L.keep.bits ? k_emit_ect<MAP_DIRECT, 16>
              : u == 16 ? k_emit_ect<MAP_O0, 16> : u == 32 ? k_emit_ect<MAP_O0, 32> : k_emit_ect<MAP_O0, 8>;
  // witnesses per workgroup (A/B switch PZK_ECT_WPB; the next witness's table loads behind this one's stores)
  static const uint32_t wpb = getenv("PZK_ECT_WPB") ? (uint32_t)atoi(getenv("PZK_ECT_WPB")) : 4u;
  if (wpb < 1 || wpb > 64) return hipErrorInvalidValue;
  hipLaunchKernelGGL(kern, dim3(n_work, (batch + wpb - 1) / wpb), dim3(ECT_NT), 0, st, L, work, B.ec_tab, B.wtns,
                     B.stride, prefetch, wpb, batch);
  return hipGetLastError();
}

hipError_t launch_emit_ecr_cv(const DevLayout& L, const Work* work, uint32_t n_work, const Bufs& B, uint32_t batch,
                              hipStream_t st) {
  if (n_work == 0) return hipSuccess;
  hipLaunchKernelGGL((L.keep.bits ? k_emit_ecr<MAP_DIRECT> : k_emit_ecr<MAP_O0>), dim3(n_work, batch), dim3(256), 0, st, L, work, B);
  return hipGetLastError();
}

}  // namespace PZK_EC_NS

#if PZK_EC_CURVE == 0
#define PZK_EC_DECL(ns)                                                                                                   \
  namespace ns {                                                                                                        \
  hipError_t launch_ec_core_cv(const DevLayout& L, const uint8_t* inputs, const uint32_t* sha_core, uint64_t* ec_core,  \
                               uint64_t* ec_jac, fr* ec_inv, int32_t* status, uint32_t batch, hipStream_t st);          \
  hipError_t launch_ec_table_cv(const DevLayout& L, int type, const int32_t* ops, uint32_t n_ops,                       \
                                const uint64_t* ec_core, uint8_t* ec_tab, int32_t* status, uint32_t batch,              \
                                hipStream_t st);                                                                        \
  hipError_t launch_emit_ect_cv(const DevLayout& L, const Work* work, uint32_t n_work, const Bufs& B, uint32_t batch,   \
                                hipStream_t st);                                                                        \
  hipError_t launch_emit_ecr_cv(const DevLayout& L, const Work* work, uint32_t n_work, const Bufs& B, uint32_t batch,   \
                                hipStream_t st);                                                                        \
  }
PZK_EC_DECL(ec_c1)
PZK_EC_DECL(ec_c2)
PZK_EC_DECL(ec_c3)
#undef PZK_EC_DECL

#define PZK_EC_DISPATCH(call)                         \
  switch (L.reg.ec_curve) {                           \
    case 1: return ec_c1::call;                       \
    case 2: return ec_c2::call;                       \
    case 3: return ec_c3::call;                       \
    default: return ec_c0::call;                      \
  }
hipError_t launch_ec_core(const DevLayout& L, const uint8_t* inputs, const uint32_t* sha_core, uint64_t* ec_core,
                          uint64_t* ec_jac, fr* ec_inv, int32_t* status, uint32_t batch, hipStream_t st) {
  PZK_EC_DISPATCH(launch_ec_core_cv(L, inputs, sha_core, ec_core, ec_jac, ec_inv, status, batch, st))
}
hipError_t launch_ec_table(const DevLayout& L, int type, const int32_t* ops, uint32_t n_ops, const uint64_t* ec_core,
                           uint8_t* ec_tab, int32_t* status, uint32_t batch, hipStream_t st) {
  PZK_EC_DISPATCH(launch_ec_table_cv(L, type, ops, n_ops, ec_core, ec_tab, status, batch, st))
}
hipError_t launch_emit_ect(const DevLayout& L, const Work* work, uint32_t n_work, const Bufs& B, uint32_t batch,
                           hipStream_t st) {
  PZK_EC_DISPATCH(launch_emit_ect_cv(L, work, n_work, B, batch, st))
}
hipError_t launch_emit_ecr(const DevLayout& L, const Work* work, uint32_t n_work, const Bufs& B, uint32_t batch,
                           hipStream_t st) {
  PZK_EC_DISPATCH(launch_emit_ecr_cv(L, work, n_work, B, batch, st))
}
#undef PZK_EC_DISPATCH
#endif
}  // namespace pzk
