// Host ASan/UBSan driver for the EF.SOD preprocessor (passport-zk-circuits_amd/csrc/passport.cpp), which
// parses untrusted DER: reads records "<len dg1><dg1><len dg15><dg15><len sod><sod>" (u32 little-endian
// lengths) from stdin, parses each with pzk_passport_parse and prints one line per record:
// "ok <name>" or "err". Built by tools/fuzz/Makefile with -fsanitize=address,undefined; any sanitizer
// report aborts the run (tests/test_passport_fuzz.py feeds it mutated SOD files).
#include "../../passport-zk-circuits_amd/csrc/passport.cpp"

#include <cstdio>

namespace pzk {
int api_fail(int code, const std::string&) { return code; }
}
extern "C" int pzk_layout_query(const pzk_params*, pzk_info*, uint32_t*) { return PZK_E_PARAMS; }

static bool read_blob(std::vector<uint8_t>& v) {
  uint32_t n;
  if (fread(&n, 4, 1, stdin) != 1) return false;
  v.resize(n);
  return n == 0 || fread(v.data(), 1, n, stdin) == n;
}

int main() {
  std::vector<uint8_t> a, b, c;
  while (read_blob(a) && read_blob(b) && read_blob(c)) {
    pzk_passport_src src{a.data(), a.size(), b.data(), b.size(), c.data(), c.size()};
    pzk_passport_info info;
    if (pzk_passport_parse(&src, &info) == 0) printf("ok %s\n", info.name);
    else printf("err\n");
  }
  return 0;
}
