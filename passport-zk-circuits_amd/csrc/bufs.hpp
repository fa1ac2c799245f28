// Per-batch device pointers handed to every emit kernel.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "fr.hpp"
#include "poseidon.hpp"

namespace pzk {

struct Bufs {
  const uint8_t* inputs;
  const uint32_t* sha_core;
  const uint64_t* rsa_core;
  const fr* pos_core;
  const fr* bjj_core;
  const fr* smt_core;
  ValueStore vs;
  uint8_t* wtns;
  size_t stride;
  int32_t* status;
  // ECDSA (ec_common.hpp)
  const uint64_t* ec_core;
  const fr* ec_inv;       // IsEqual inverses, normal form
  const uint8_t* ec_tab;  // value tables of the table ops
  const fr* inv_small;    // 1/k mod p, k < 256, normal form
  const uint8_t* derived; // derived SHA message elements (RSA-PSS, pss.hpp), n_derived per witness
};

}  // namespace pzk
