// Layout builder (see builder.hpp). Template sizes follow the circom sources cited inline;
// every offset here is re-derived independently of the CPU oracle, and the parity tests
// compare the two layouts element by element.
#include "builder_impl.hpp"

#include <algorithm>
#include <map>

namespace pzk {

namespace {

bool build_poseidon(const pzk_params& p, Layout& L, std::string& why) {
  int n = p.size_arg;
  if (n < 1 || n > 5) { why = "PoseidonHash(n): n must be 1..5 (Poseidon parameters shipped for t = 2..6)"; return false; }
  Builder b(L);
  L.n_inputs = n;
  L.n_outputs = 1;
  L.inputs.push_back({"in", 0, (uint64_t)n});
  std::vector<int> slots;
  for (int i = 0; i < n; i++) { int s = b.value(); slots.push_back(s); L.loads.push_back(ValueLoad{s, i}); }
  b.region(RK_ONE, 1);
  b.poseidon(n, slots, 0);  // main = PoseidonHash(n): [1, out, in[n], PoseidonEx]
  b.finalize();
  return true;
}

bool build_sha256(const pzk_params& p, Layout& L, std::string& why) {
  int B = p.size_arg;
  if (B < 1 || B > 64) { why = "Sha256HashChunks(blocks): blocks must be 1..64"; return false; }
  Builder b(L);
  L.n_inputs = 512ull * B;
  L.n_outputs = 256;
  L.inputs.push_back({"in", 0, L.n_inputs});
  b.region(RK_ONE, 1);
  b.sha256(0, B, false);
  b.finalize();
  return true;
}

}  // namespace

bool build_register(const pzk_params& p, Layout& L, std::string& why);

bool build_layout(const pzk_params& p, Layout& L, std::string& why) {
  L = Layout();
  switch (p.circuit) {
    case PZK_CIRCUIT_POSEIDON: return build_poseidon(p, L, why);
    case PZK_CIRCUIT_SHA256: return build_sha256(p, L, why);
    case PZK_CIRCUIT_REGISTER: return build_register(p, L, why);
    default: why = "unknown circuit family"; return false;
  }
}

}  // namespace pzk
