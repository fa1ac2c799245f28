// Poseidon permutation core, t cooperating lanes per permutation, and the launcher of both cores. Own
// translation unit (template kernels only from the shared headers), so it compiles in parallel with kernels.hip.
#include <hip/hip_runtime.h>
#include <stdlib.h>

#define PZK_TEMPLATE_KERNELS_ONLY
#include "bufs.hpp"
#include "poseidon.hpp"
#include "kernels.hpp"

namespace pzk {

// kernels_pos1.hip
hipError_t launch_pos_core1(int t, const PosConsts& K, const PosTask* tasks, uint32_t n_tasks, ValueStore vs, fr* pos_core,
                            uint32_t core_elems, const fr* smt_core, uint32_t smt_core_fr, const uint32_t* order,
                            hipStream_t st);

#define HIP_TRY(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return e_; } while (0)

// ------------------------------------------------------------------- Poseidon core
// wave = 64 witnesses of one task. SMT level tasks below the insertion level depend on the
// chain and are left to k_smt_chain.
template <int T>
__global__ void __launch_bounds__(256) k_pos_core(PosConsts K, const PosTask* tasks, ValueStore vs, fr* pos_core,
                                                  uint32_t core_elems, const fr* smt_core, uint32_t smt_core_fr,
                                                  const uint32_t* order) {
  core_priority();
  constexpr int G = T <= 4 ? 4 : 8;
  const uint32_t gid = (blockIdx.x * blockDim.x + threadIdx.x) / G;  // (witness) of this lane group
  const int j = threadIdx.x & (G - 1);
  if (gid >= vs.batch) return;  // whole groups (batch rows are group-aligned)
  const PosTask& task = tasks[blockIdx.y];
  const uint32_t w = (order && task.smt_level >= 0) ? order[gid] : gid;  // SMT levels: depth order (k_pos_core1)
  if (task.smt_level >= 0) {
    int jl = (int)reinterpret_cast<const uint32_t*>(smt_core + (size_t)w * smt_core_fr + 3 * SMT_LEVELS)[0];
    if (task.smt_level < jl) return;  // whole group: same witness
  }
  if (pos_inputs_zero(task, vs, w)) {  // whole group: the constant zero-input hash (k_pos_core1)
    if (j == 0) vs.at(task.out_slot, w) = K.Zhash(T);
    return;
  }
  pos_core_group<T, G>(K, task, vs, w, pos_core + (size_t)w * core_elems, j);
}

hipError_t launch_pos_core(const PosConsts& K, const PosTask* d_tasks, const PosTask* h_tasks, uint32_t first,
                           uint32_t count, ValueStore vs, fr* pos_core, uint32_t core_elems, const fr* smt_core,
                           uint32_t smt_core_fr, const uint32_t* order, hipStream_t st) {
  // group consecutive tasks of equal t into one launch (blockIdx.y = task)
  uint32_t i = 0;
  while (i < count) {
    int t = h_tasks[first + i].n + 1;
    uint32_t j = i;
    while (j < count && h_tasks[first + j].n + 1 == t) j++;
    const PosTask* tp = d_tasks + first + i;
    if (j - i >= 8) {  // many tasks: one lane per permutation
      HIP_TRY(launch_pos_core1(t, K, tp, j - i, vs, pos_core, core_elems, smt_core, smt_core_fr, order, st));
      i = j;
      continue;
    }
    const uint32_t G = t <= 4 ? 4 : 8;
    dim3 g((vs.batch * G + 255) / 256, j - i);
    switch (t) {
      case 2: hipLaunchKernelGGL(k_pos_core<2>, g, dim3(256), 0, st, K, tp, vs, pos_core, core_elems, smt_core, smt_core_fr, order); break;
      case 3: hipLaunchKernelGGL(k_pos_core<3>, g, dim3(256), 0, st, K, tp, vs, pos_core, core_elems, smt_core, smt_core_fr, order); break;
      case 4: hipLaunchKernelGGL(k_pos_core<4>, g, dim3(256), 0, st, K, tp, vs, pos_core, core_elems, smt_core, smt_core_fr, order); break;
      case 5: hipLaunchKernelGGL(k_pos_core<5>, g, dim3(256), 0, st, K, tp, vs, pos_core, core_elems, smt_core, smt_core_fr, order); break;
      case 6: hipLaunchKernelGGL(k_pos_core<6>, g, dim3(256), 0, st, K, tp, vs, pos_core, core_elems, smt_core, smt_core_fr, order); break;
      default: return hipErrorInvalidValue;
    }
    HIP_TRY(hipGetLastError());
    i = j;
  }
  return hipSuccess;
}

}  // namespace pzk
