// Host-only half of the C-ABI (no device code, no HIP runtime calls): .sym parsing, the mapped-layout program
// compaction, and the entry points that only build a layout (pzk_sym_check, pzk_layout_query,
// pzk_layout_region). Split from runtime.cpp so that tools/fuzz builds it with the host sanitizers.
#pragma once
#include <stdint.h>

#include <exception>
#include <new>
#include <string>
#include <vector>

#include "builder.hpp"

namespace pzk {

int api_fail(int code, const std::string& msg);  // sets pzk_last_error(), returns code (runtime.cpp)

constexpr int PIPELINE_SETS_MAX = 6;  // scratch sets an instance can rotate over
// scratch sets = calls in flight: PZK_NSETS (A/B), else 6 for QueryIdentity (its calls are one long chain each:
// 196.7k -> 229.3k -> 238.1k witnesses/s with four chain streams and three / four / six sets, profiles/r5h, r5i),
// 3 for the others
int nsets_env(bool query = false);

// circom .sym text -> inv[k] = O0 index of output witness element k (inv[0] = 0)
bool parse_sym(const char* text, size_t len, uint64_t o0_size, std::vector<uint32_t>& inv, std::string& why);

// A mapped instance's emission program (runtime.cpp pzk_instance_create_mapped): for a monotone map (every map
// circom writes) the emitters write the kept signals directly (mapsink.hpp): the keep bitmap over the O0 indices
// (+ 2 zero words past the end: a wave's window reads words i, i + 1), the kept count below every 64-signal
// boundary, and each descriptor-driven work item's kept descriptors compacted in O0 order (Work.pad = their
// offset in mprog). Any other map (or force_gather) takes the O0 staging + gather path (direct = false).
struct MapProgram {
  bool direct = false;
  std::vector<uint64_t> bits;
  std::vector<uint32_t> rank, mprog;
  std::vector<Work> work[E_COUNT];  // the work lists of E_SHA, E_SHAD, E_POS, E_ECT with Work.pad set
  uint32_t pos_nomix = 0;           // bit t: no kept signal of a width-t Poseidon block reads a GetSum row (pos_prog.hpp)
};
void map_program(const Layout& lay, const std::vector<uint32_t>& inv, bool force_gather, MapProgram& out);

// Exceptions never cross the C ABI (pzkwit.h: every function returns 0 or a negative PZK_E_* code): each entry point
// runs its implementation under guarded(), which maps a host allocation failure to PZK_E_NOMEM and any other
// exception to PZK_E_ARG, with the reason in pzk_last_error().
template <class F>
static int guarded(F&& f) {
  try {
    return f();
  } catch (const std::bad_alloc&) {
    return api_fail(PZK_E_NOMEM, "host memory allocation failed");
  } catch (const std::exception& e) {
    return api_fail(PZK_E_ARG, std::string("internal error: ") + e.what());
  } catch (...) {
    return api_fail(PZK_E_ARG, "internal error");
  }
}

}  // namespace pzk
