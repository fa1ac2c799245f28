// Launch wrappers shared between kernels.hip (device code) and runtime.cpp (host runtime).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fr.hpp"
#include "layout.hpp"

namespace pzk {

constexpr int EMIT_THREADS = 256;  // emit kernels' workgroup size

struct ValueLoad {
  int32_t slot;    // value-store slot
  int32_t in_off;  // input element offset
};

struct PosConsts;
struct ValueStore;
struct Bufs;

hipError_t launch_load_values(const ValueLoad* loads, int n, const uint8_t* inputs, uint64_t n_inputs, fr* values,
                              uint32_t batch, hipStream_t st);
// SHA jobs [first, first + count); a job with src = 1 reads its message from the derived row
hipError_t launch_sha_core(const DevLayout& L, const uint8_t* inputs, const uint8_t* derived, uint32_t first,
                           uint32_t count, uint32_t* sha_core, int32_t* status, uint32_t batch, hipStream_t st);
// RSA-PSS derived messages (pss.hpp): stage 0 = MGF1 blocks (after the RSA core), 1 = M' (after the MGF1 hashes)
hipError_t launch_pss(const DevLayout& L, int stage, const uint64_t* rsa_core, const uint32_t* sha_core,
                      uint8_t* derived, uint32_t batch, hipStream_t st);
hipError_t launch_pos_core(const PosConsts& K, const PosTask* d_tasks, const PosTask* h_tasks, uint32_t first,
                           uint32_t count, ValueStore vs, fr* pos_core, uint32_t core_elems, const fr* smt_core,
                           uint32_t smt_core_fr, const uint32_t* order, hipStream_t st);  // order: k_smt_order's
hipError_t launch_prep(const DevLayout& L, const uint8_t* inputs, const uint32_t* sha_core, ValueStore vs,
                       int32_t* status, hipStream_t st);
hipError_t launch_rsa_check(const DevLayout& L, const uint8_t* inputs, const uint32_t* sha_core,
                            const uint64_t* rsa_core, int32_t* status, uint32_t batch, hipStream_t st);
hipError_t launch_rsa_core(const DevLayout& L, const uint8_t* inputs, uint64_t* rsa_core, uint64_t* colsum,
                           int32_t* status, uint32_t batch, hipStream_t st);
hipError_t launch_bjj_table(fr* table, hipStream_t st);
hipError_t launch_wtns_gather(const uint8_t* o0, size_t o0_stride, const uint32_t* map, uint64_t out_size, uint8_t* out,
                              size_t out_stride, uint32_t batch, hipStream_t st);
// whether the BabyJubJub core runs the kernel with its global scratch array (launch_bjj_core: when it is given one):
// by default yes — QueryIdentity (the core is on its latency-critical chain) and, since round 5, the register
// circuit too (k_bjj_core_rc recomputes the ladder instead, 1.35x instead of 6x its bytes but twice the VALU:
// configs 3 / 4 / O2-shaped +1.0 / +0.7 / +5.7 % with the scratch kernel, profiles/r5e); PZK_BJJ=scratch|rc (A/B)
bool bjj_uses_scratch();
hipError_t launch_bjj_core(const DevLayout& L, ValueStore vs, const fr* table, fr* bjj_core, fr* scratch,
                           hipStream_t st);
hipError_t launch_smt_prep(const DevLayout& L, const uint8_t* inputs, ValueStore vs, fr* smt_core, int32_t* status,
                           hipStream_t st);
// query: QueryIdentity's chain or the register circuit's (both default to FIPS products, PZK_CHAIN_MUL overrides)
hipError_t launch_smt_chain(const DevLayout& L, const PosConsts& K, const int32_t* level_task, const uint8_t* inputs,
                            ValueStore vs, fr* pos_core, fr* smt_core, const uint32_t* order, int32_t* status,
                            hipStream_t st);
// the quad SMT chain's constant table (smt_chain4.hpp), once per instance
hipError_t launch_qc_build(const PosConsts& K, fr* qc, hipStream_t st);
// witnesses ordered by SMT insertion level (the chain's length), deepest first, for k_smt_chain's lane groups
hipError_t launch_smt_order(const fr* smt_core, uint32_t smt_core_fr, uint32_t* order, uint32_t batch, hipStream_t st);
// QueryIdentity prep (query.hpp): DG1 fields, dg1 chunks, citizenship inverses, the query checks
hipError_t launch_qry_prep(const DevLayout& L, const uint8_t* inputs, ValueStore vs, int32_t* status, hipStream_t st);
hipError_t launch_ec_core(const DevLayout& L, const uint8_t* inputs, const uint32_t* sha_core, uint64_t* ec_core,
                          uint64_t* ec_jac, fr* ec_inv, int32_t* status, uint32_t batch, hipStream_t st);
hipError_t launch_emit_ecr(const DevLayout& L, const Work* work, uint32_t n_work, const Bufs& B, uint32_t batch,
                           hipStream_t st);
hipError_t launch_ec_table(const DevLayout& L, int type, const int32_t* ops, uint32_t n_ops, const uint64_t* ec_core,
                           uint8_t* ec_tab, int32_t* status, uint32_t batch, hipStream_t st);
hipError_t launch_inv_small(fr* out, hipStream_t st);
hipError_t launch_emit_ect(const DevLayout& L, const Work* work, uint32_t n_work, const Bufs& B, uint32_t batch,
                           hipStream_t st);
hipError_t launch_emit_pos(const DevLayout& L, const Work* work, uint32_t n_work, const PosConsts& K, const Bufs& B,
                           uint32_t batch, int t, hipStream_t st);
// the zero-input Poseidon images and hashes of t = 2..6 (poseidon.hpp pos_zimg_off), once per instance;
// scratch: 2 + 512 Fr of device memory; sequential launches on st
hipError_t launch_pos_zero_img(const PosConsts& K, fr* scratch, fr* zimg, hipStream_t st);
hipError_t launch_emit_mm(const DevLayout& L, const Work* work, uint32_t n_work, const Bufs& B, uint32_t batch,
                          hipStream_t st);
hipError_t launch_emit(int emitter, const DevLayout& L, const Work* work, uint32_t n_work, const PosConsts& K,
                       const Bufs& B, uint32_t batch, int max_t, hipStream_t st);

}  // namespace pzk
