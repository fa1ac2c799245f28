// Host-side layout builder: walks the template tree of an instance (at region granularity)
// and produces the region table, the per-kernel work lists, the SHA jobs, the Poseidon task
// DAG and the value-store map. Pure host C++.
#pragma once
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <array>
#include <string>
#include <vector>

#include "../../include/pzkwit.h"
#include "kernels.hpp"
#include "layout.hpp"

namespace pzk {

struct InputGroup {
  std::string name;
  uint64_t offset, length;
};

struct Layout {
  uint64_t wit_size = 0, n_inputs = 0;
  uint64_t n_derived = 0;  // derived SHA message elements per witness (RSA-PSS)
  uint32_t n_outputs = 0, n_public = 0;
  std::vector<InputGroup> inputs;
  std::vector<Region> regions;
  std::vector<Work> work[E_COUNT];  // per emit kernel
  std::vector<GenPiece> gen_pieces;  // pieces of the packed emitters' work items
  std::vector<uint32_t> sha_prog;    // SHA block program: one descriptor per block signal (sha_prog.hpp)
  std::vector<uint16_t> pos_prog;    // Poseidon block programs, t = 2..6 (pos_prog.hpp)
  uint32_t pos_prog_off[POS_MAX_T + 1] = {};
  std::vector<std::array<uint32_t, 3>> pos_emit_groups;  // (t, first work, works) of work[E_POS]
  // emission that reads the SMT chain's output (k_smt_chain): the SMT level Poseidon blocks are the groups
  // [pos_chain_group, end) of pos_emit_groups, the SMT regions of E_GEN the work items [gen_chain_work, end); the
  // rest of both emitters can run before the chain ends (register runtime: the post-chain stream)
  uint32_t pos_chain_group = 0, gen_chain_work = 0;
  std::vector<ShaJob> sha;
  uint32_t sha_core_words = 0;
  std::vector<PosTask> pos;            // sorted by level, then t
  std::vector<uint32_t> pos_level_start;
  uint32_t pos_core_elems = 0;
  int max_t = 2;
  uint32_t n_values = 0;
  std::vector<ValueLoad> loads;
  // RegisterIdentityBuilder only
  bool is_register = false;
  RegInfo reg{};
  pzk_params params{};
  std::vector<int> out_slots;
  uint32_t rsa_core_words = 0, bjj_core_fr = 0, smt_core_fr = 0;
  // QueryIdentity(80) (builder_query.cpp, query.hpp)
  bool is_query = false;
  // ECDSA (SIGNATURE_TYPE 20)
  bool is_ecdsa = false;
  std::vector<uint32_t> ec_prog;      // per-type descriptor programs (ec_walk.hpp)
  uint32_t ec_prog_off[3] = {}, ec_tab_n[3] = {};
  std::vector<uint32_t> ec_tab_off;   // per table op
  uint32_t ec_tab_entries = 0;
  std::vector<int32_t> ec_ops[3];     // table ops per type (k_ec_table launches)
};

bool build_layout(const pzk_params& p, Layout& L, std::string& why);
bool build_query(const pzk_params& p, Layout& L, std::string& why);

// chunk size of one emit workgroup (signals)
constexpr uint32_t EMIT_CHUNK = 4096;
// signals per work item of a chunked emitter (PZK_CHUNK_<e> overrides, for tuning runs)
inline uint32_t emit_chunk(int e) {
  char name[32];
  snprintf(name, sizeof name, "PZK_CHUNK_%d", e);
  const char* v = getenv(name);
  if (v) return (uint32_t)atoi(v);
  return (e == E_MM || e == E_ECT) ? (1u << 30) : EMIT_CHUNK;  // whole block per workgroup
}

}  // namespace pzk
