// Poseidon permutation core, one lane per permutation (launches with many tasks of one width: the SMT
// level hashes), and its launcher; own translation unit so it compiles in parallel with kernels_pos.hip.
#include <hip/hip_runtime.h>

#define PZK_TEMPLATE_KERNELS_ONLY
#include "bufs.hpp"
#include "poseidon.hpp"
#include "kernels.hpp"

namespace pzk {

// lane per permutation: for launches with many tasks (the 80 SMT level hashes), where the
// batch x tasks lanes already fill the chip and the cooperative form only adds shuffles
template <int T>
__global__ void __launch_bounds__(64) k_pos_core1(PosConsts K, const PosTask* tasks, ValueStore vs, fr* pos_core,
                                                  uint32_t core_elems, const fr* smt_core, uint32_t smt_core_fr,
                                                  const uint32_t* order) {
  core_priority();
  __shared__ fr lines[4 * 64];
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= vs.batch) return;
  const PosTask& task = tasks[blockIdx.y];
  // SMT level hashes take the witnesses in k_smt_order's depth order, so the lanes of a wave agree on whether
  // the level is theirs (below the insertion level) or the chain's, and whole waves leave together
  const uint32_t w = (order && task.smt_level >= 0) ? order[g] : g;
  if (task.smt_level >= 0) {
    int jl = (int)reinterpret_cast<const uint32_t*>(smt_core + (size_t)w * smt_core_fr + 3 * SMT_LEVELS)[0];
    if (task.smt_level < jl) return;
  }
  // zero inputs: the hash is the constant one, and the emitter copies the constant image instead of reading a core
  if (pos_inputs_zero(task, vs, w)) {
    vs.at(task.out_slot, w) = K.Zhash(T);
    return;
  }
  const PosLineSink out{pos_core + (size_t)w * core_elems + task.core_off, lines + threadIdx.x};
  pos_core_lane<T>(K, task, vs, w, out);
}

hipError_t launch_pos_core1(int t, const PosConsts& K, const PosTask* tp, uint32_t n_tasks, ValueStore vs, fr* pos_core,
                            uint32_t core_elems, const fr* smt_core, uint32_t smt_core_fr, const uint32_t* order,
                            hipStream_t st) {
  dim3 g1((vs.batch + 63) / 64, n_tasks);
  switch (t) {
    case 2: hipLaunchKernelGGL(k_pos_core1<2>, g1, dim3(64), 0, st, K, tp, vs, pos_core, core_elems, smt_core, smt_core_fr, order); break;
    case 3: hipLaunchKernelGGL(k_pos_core1<3>, g1, dim3(64), 0, st, K, tp, vs, pos_core, core_elems, smt_core, smt_core_fr, order); break;
    case 4: hipLaunchKernelGGL(k_pos_core1<4>, g1, dim3(64), 0, st, K, tp, vs, pos_core, core_elems, smt_core, smt_core_fr, order); break;
    case 5: hipLaunchKernelGGL(k_pos_core1<5>, g1, dim3(64), 0, st, K, tp, vs, pos_core, core_elems, smt_core, smt_core_fr, order); break;
    case 6: hipLaunchKernelGGL(k_pos_core1<6>, g1, dim3(64), 0, st, K, tp, vs, pos_core, core_elems, smt_core, smt_core_fr, order); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace pzk
