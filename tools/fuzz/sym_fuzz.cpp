// Host ASan/UBSan driver for the product's host-side input handling that needs no device: the .sym parser, the
// layout builders and the mapped-layout program compaction (passport-zk-circuits_amd/csrc/host_api.cpp,
// builder*.cpp) behind pzk_sym_check / pzk_layout_query / pzk_layout_region. Reads records from stdin:
//   u8 mode, pzk_params (12 x i32), then for mode 0 a u32 length + that many bytes of .sym text;
// mode 0: pzk_sym_check, and on success the map's emission program (parse_sym + map_program over the layout);
// mode 1: pzk_layout_query + pzk_layout_region of every region.
// Prints one line per record: "ok <n>" (mode 0: mapped witness size, mode 1: witness size) or "err <code>".
// Built by tools/fuzz/Makefile with -fsanitize=address,undefined (-fno-sanitize-recover): any report aborts the
// run (tests/test_host_fuzz.py).
#include <cstdio>
#include <string>
#include <vector>

#include "../../include/pzkwit.h"
#include "../../passport-zk-circuits_amd/csrc/host_api.hpp"

namespace pzk {
static thread_local std::string g_msg;
int api_fail(int code, const std::string& msg) { g_msg = msg; return code; }
}  // namespace pzk

static bool read_n(void* p, size_t n) { return n == 0 || fread(p, 1, n, stdin) == n; }

int main() {
  uint8_t mode;
  while (read_n(&mode, 1)) {
    pzk_params prm;
    if (!read_n(&prm, sizeof prm)) break;
    if (mode == 0) {
      uint32_t len;
      if (!read_n(&len, 4)) break;
      std::vector<char> text(len);
      if (!read_n(text.data(), len)) break;
      uint64_t ws = 0;
      const int rc = pzk_sym_check(&prm, text.data(), len, &ws);
      if (rc) { printf("err %d\n", rc); continue; }
      // the emission program a mapped instance would upload (no device: the host half only)
      pzk::Layout L;
      std::string why;
      std::vector<uint32_t> inv;
      if (!pzk::build_layout(prm, L, why) || !pzk::parse_sym(text.data(), len, L.wit_size, inv, why)) {
        printf("err mismatch\n");
        return 2;
      }
      pzk::MapProgram mp;
      pzk::map_program(L, inv, false, mp);
      printf("ok %llu %s %zu\n", (unsigned long long)ws, mp.direct ? "direct" : "gather", mp.mprog.size());
    } else {
      pzk_info info;
      uint32_t nreg = 0;
      const int rc = pzk_layout_query(&prm, &info, &nreg);
      if (rc) { printf("err %d\n", rc); continue; }
      uint64_t end = 0;
      for (uint32_t i = 0; i < nreg; i++) {
        uint64_t off;
        uint32_t len, kind;
        if (pzk_layout_region(&prm, i, &off, &len, &kind)) { printf("err region\n"); return 2; }
        if (off + len > end) end = off + len;
        if (i > 4) break;  // every region query rebuilds the layout: sample the first few
      }
      printf("ok %llu\n", (unsigned long long)info.witness_size);
    }
    fflush(stdout);
  }
  return 0;
}
