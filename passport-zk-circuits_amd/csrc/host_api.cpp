// Host-only half of the C-ABI (host_api.hpp).
#include <string.h>

#include <algorithm>

#include "../../include/pzkwit.h"
#include "host_api.hpp"
#include "pos_prog.hpp"

namespace pzk {

int nsets_env(bool query) {
  const char* e = getenv("PZK_NSETS");
  const int v = e ? atoi(e) : query ? 6 : 3;
  return v < 2 ? 2 : v > PIPELINE_SETS_MAX ? PIPELINE_SETS_MAX : v;
}

// circom .sym text ("signal_idx,witness_idx,component_idx,name" per line; witness_idx -1 = eliminated)
// -> inv[k] = O0 index of output witness element k (inv[0] = 0, the constant 1). Signal indices are the
// --O0 numbering (1 .. o0_size - 1); witness indices must cover 1 .. max, each by one or
// more signals (several signals on one index: the lowest signal index is emitted).
bool parse_sym(const char* text, size_t len, uint64_t o0_size, std::vector<uint32_t>& inv, std::string& why) {
  std::vector<int64_t> w_of;  // witness index -> signal index
  size_t i = 0;
  uint64_t line = 0;
  auto num = [&](int64_t& v) -> bool {
    bool neg = false, any = false;
    v = 0;
    if (i < len && text[i] == '-') { neg = true; i++; }
    while (i < len && text[i] >= '0' && text[i] <= '9') { v = v * 10 + (text[i] - '0'); i++; any = true; if (v > (1ll << 40)) return false; }
    if (neg) v = -v;
    return any;
  };
  while (i < len) {
    line++;
    if (text[i] == '\n' || text[i] == '\r') { i++; continue; }
    int64_t sig, wit, comp;
    if (!num(sig) || i >= len || text[i++] != ',' || !num(wit) || i >= len || text[i++] != ',' || !num(comp)) {
      why = "sym line " + std::to_string(line) + ": expected signal_idx,witness_idx,component_idx,name";
      return false;
    }
    while (i < len && text[i] != '\n') i++;
    if (sig < 1 || (uint64_t)sig >= o0_size) {
      why = "sym line " + std::to_string(line) + ": signal index " + std::to_string(sig) + " outside 1.." +
            std::to_string(o0_size - 1);
      return false;
    }
    if (wit == -1) continue;
    // kept signals get distinct-or-shared indices 1..n, n <= the O0 signal count: anything above is not a .sym of
    // this instance (and must not size w_of)
    if (wit < 1 || (uint64_t)wit >= o0_size) {
      why = "sym line " + std::to_string(line) + ": witness index " + std::to_string(wit) + " outside 1.." +
            std::to_string(o0_size - 1);
      return false;
    }
    if ((uint64_t)wit >= w_of.size()) w_of.resize(wit + 1, -1);
    // circom's simplification can merge equal signals onto one witness index (snarkjs loadSymbols joins
    // their names with '|'): they carry one value, so the lowest signal index stands for all of them
    if (w_of[wit] == -1 || sig < w_of[wit]) w_of[wit] = sig;
  }
  if (w_of.size() < 2) { why = "sym: no signal is kept"; return false; }
  inv.assign(w_of.size(), 0);
  for (size_t k = 1; k < w_of.size(); k++) {
    if (w_of[k] < 0) { why = "sym: witness index " + std::to_string(k) + " is not assigned"; return false; }
    inv[k] = (uint32_t)w_of[k];
  }
  return true;
}

void map_program(const Layout& lay, const std::vector<uint32_t>& inv, bool force_gather, MapProgram& out) {
  out = MapProgram();
  bool monotone = true;
  for (size_t k = 1; k < inv.size() && monotone; k++) monotone = inv[k] > inv[k - 1];
  if (!monotone || force_gather) return;
  out.direct = true;
  const size_t nw = lay.wit_size / 64 + 3;
  out.bits.assign(nw, 0);
  out.rank.assign(nw, 0);
  for (uint32_t g : inv) out.bits[g >> 6] |= 1ull << (g & 63);
  for (size_t i = 1; i < nw; i++) out.rank[i] = out.rank[i - 1] + (uint32_t)__builtin_popcountll(out.bits[i - 1]);
  auto kept = [&](uint64_t g) { return (out.bits[g >> 6] >> (g & 63)) & 1; };
  bool mix_t[POS_MAX_T + 1] = {};
  auto kept_in = [&](uint64_t a, uint64_t n) {
    uint64_t c = 0;
    for (uint64_t g = a; g < a + n; g++) c += kept(g);
    return c;
  };
  for (int e : {E_SHA, E_SHAD, E_POS, E_ECT}) {
    std::vector<Work>& wl = out.work[e];
    wl = lay.work[e];
    if (e == E_SHA || e == E_SHAD) {
      // SHA block chunks hold EMIT_CHUNK O0 signals; with a map keeping a fifth of them a workgroup would build its
      // word table for ~800 stores. Consecutive chunks of a block merge until they hold EMIT_CHUNK kept signals
      // (the O2-shaped line: 188k -> 200k witnesses/s at 16,384-signal chunks, profiles/r5i)
      std::vector<Work> merged;
      uint64_t kept_cur = 0;
      for (const Work& wk : wl) {
        const uint64_t k = kept_in(lay.regions[wk.region].off + wk.start, wk.count);
        Work* last = merged.empty() ? nullptr : &merged.back();
        if (last && last->region == wk.region && lay.regions[wk.region].kind == RK_SHA_BLOCK &&
            last->start + last->count == wk.start && kept_cur + k <= EMIT_CHUNK) {
          last->count += wk.count;
          kept_cur += k;
        } else {
          merged.push_back(wk);
          kept_cur = k;
        }
      }
      wl.swap(merged);
    }
    for (Work& wk : wl) {
      const Region& R = lay.regions[wk.region];
      const uint32_t* src = nullptr;
      const uint16_t* src16 = nullptr;
      if (R.kind == RK_SHA_BLOCK) src = lay.sha_prog.data() + wk.start;
      else if (R.kind == RK_POSEIDON) src16 = lay.pos_prog.data() + lay.pos_prog_off[lay.pos[R.a[0]].n + 1] + wk.start;
      else if (R.kind == RK_ECT) src = lay.ec_prog.data() + lay.ec_prog_off[R.a[1]] + wk.start;
      else continue;
      wk.pad = (uint32_t)out.mprog.size();
      for (uint32_t q = 0; q < wk.count; q++)
        if (kept(R.off + wk.start + q)) {
          out.mprog.push_back(src ? src[q] : src16[q]);
          if (src16) mix_t[lay.pos[R.a[0]].n + 1] |= (pos_img_need_t(lay.pos[R.a[0]].n + 1, src16[q]) & PI_MIX) != 0;
        }
    }
  }
  for (int t = 2; t <= POS_MAX_T; t++)
    if (!mix_t[t]) out.pos_nomix |= 1u << t;
  if (out.mprog.empty()) out.mprog.push_back(0);
}

}  // namespace pzk

using namespace pzk;

extern "C" {

static int sym_check_impl(const pzk_params* params, const char* sym, size_t sym_len, uint64_t* witness_size) {
  if (!params || !sym) return api_fail(PZK_E_ARG, "null argument");
  Layout L;
  std::string why;
  if (!build_layout(*params, L, why)) return api_fail(PZK_E_PARAMS, why);
  std::vector<uint32_t> inv;
  if (!parse_sym(sym, sym_len, L.wit_size, inv, why)) return api_fail(PZK_E_ARG, why);
  if (witness_size) *witness_size = inv.size();
  return 0;
}

static int layout_query_impl(const pzk_params* params, pzk_info* info, uint32_t* n_regions) {
  if (!params || !info) return api_fail(PZK_E_ARG, "null argument");
  Layout L;
  std::string why;
  if (!build_layout(*params, L, why)) return api_fail(PZK_E_PARAMS, why);
  memset(info, 0, sizeof *info);
  info->witness_size = L.wit_size;
  info->n_inputs = L.n_inputs;
  info->n_outputs = L.n_outputs;
  info->n_public_inputs = L.n_public;
  info->n_input_groups = (uint32_t)L.inputs.size();
  info->pipeline_depth = nsets_env(params->circuit == PZK_CIRCUIT_QUERY);
  if (n_regions) *n_regions = (uint32_t)L.regions.size();
  return 0;
}

static int layout_region_impl(const pzk_params* params, uint32_t i, uint64_t* off, uint32_t* len, uint32_t* kind) {
  if (!params) return api_fail(PZK_E_ARG, "null argument");
  Layout L;
  std::string why;
  if (!build_layout(*params, L, why)) return api_fail(PZK_E_PARAMS, why);
  if (i >= L.regions.size()) return api_fail(PZK_E_ARG, "region index out of range");
  if (off) *off = L.regions[i].off;
  if (len) *len = L.regions[i].len;
  if (kind) *kind = L.regions[i].kind;
  return 0;
}

int pzk_sym_check(const pzk_params* params, const char* sym, size_t sym_len, uint64_t* witness_size) {
  return guarded([&] { return sym_check_impl(params, sym, sym_len, witness_size); });
}

int pzk_layout_query(const pzk_params* params, pzk_info* info, uint32_t* n_regions) {
  return guarded([&] { return layout_query_impl(params, info, n_regions); });
}

int pzk_layout_region(const pzk_params* params, uint32_t i, uint64_t* off, uint32_t* len, uint32_t* kind) {
  return guarded([&] { return layout_region_impl(params, i, off, len, kind); });
}

}  // extern "C"
