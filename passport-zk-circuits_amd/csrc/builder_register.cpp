// RegisterIdentityBuilder layout (registerIdentityBuilder.circom:41-196) — see builder.hpp.
#include "builder.hpp"

namespace pzk {

bool build_register(const pzk_params& p, Layout& L, std::string& why) {
  (void)p; (void)L;
  why = "RegisterIdentityBuilder layout: not built in this library version";
  return false;
}

}  // namespace pzk
