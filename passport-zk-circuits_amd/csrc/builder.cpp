// Layout builder (see builder.hpp). Template sizes follow the circom sources cited inline;
// every offset here is re-derived independently of the CPU oracle, and the parity tests
// compare the two layouts element by element.
#include "builder.hpp"

#include <algorithm>
#include <map>

namespace pzk {

namespace {

constexpr uint32_t SHA_BLOCK_LEN = 150762;  // Sha2_224_256Shedule (36,048) + Sha2_224_256Rounds(64) (114,714)

struct Builder {
  Layout& L;
  uint64_t cur = 0;
  explicit Builder(Layout& l) : L(l) {}

  int value() { return (int)L.n_values++; }

  uint32_t region(uint32_t kind, uint64_t len, std::initializer_list<int32_t> a = {}) {
    Region r{};
    r.off = cur;
    r.len = (uint32_t)len;
    r.kind = kind;
    int i = 0;
    for (int32_t x : a) r.a[i++] = x;
    L.regions.push_back(r);
    cur += len;
    return (uint32_t)L.regions.size() - 1;
  }

  int sha_job(int in_off, int blocks) {
    ShaJob j{};
    j.in_off = in_off;
    j.blocks = blocks;
    j.core_off = (int)L.sha_core_words;
    j.digest_slot = -1;
    L.sha_core_words += blocks * SHA_BLOCK_CORE + 8;
    L.sha.push_back(j);
    return (int)L.sha.size() - 1;
  }

  // Sha256HashChunks(B) (sha256HashChunks.circom:8-48), optionally inside ShaHashChunks(B,256)
  // (hash.circom:32-68): own/wrapper signals as one RK_SHA_OWN region, then (sch, rds) per block.
  int sha256(int in_off, int blocks, bool wrapper) {
    int job = sha_job(in_off, blocks);
    uint64_t own = (wrapper ? 256 + 512ull * blocks : 0) + 256 + 512ull * blocks + 256ull * (blocks + 1) + 256;
    region(RK_SHA_OWN, own, {job, blocks, in_off, wrapper ? 1 : 0});
    for (int m = 0; m < blocks; m++) region(RK_SHA_BLOCK, SHA_BLOCK_LEN, {job, m});
    return job;
  }

  // PoseidonHash(n) (poseidon.circom:214-226) as one RK_POSEIDON region; returns output slot
  int poseidon(int n, const std::vector<int>& in_slots, int level) {
    PosTask t{};
    t.n = n;
    int i = 0;
    for (int s : in_slots) t.in_slot[i++] = s;
    t.out_slot = value();
    t.core_off = (int)L.pos_core_elems;
    t.level = level;
    L.pos_core_elems += pos_core_len(n + 1);
    L.max_t = std::max(L.max_t, n + 1);
    L.pos.push_back(t);
    region(RK_POSEIDON, pos_hash_size(n), {(int32_t)L.pos.size() - 1, n});
    return t.out_slot;
  }

  void finalize() {
    L.wit_size = cur;
    // Poseidon tasks: launch order = (level, t); remap region references
    std::vector<int> order(L.pos.size());
    for (size_t i = 0; i < order.size(); i++) order[i] = (int)i;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
      if (L.pos[a].level != L.pos[b].level) return L.pos[a].level < L.pos[b].level;
      return L.pos[a].n < L.pos[b].n;
    });
    std::vector<int> inv(order.size());
    std::vector<PosTask> sorted;
    for (size_t i = 0; i < order.size(); i++) { inv[order[i]] = (int)i; sorted.push_back(L.pos[order[i]]); }
    L.pos = sorted;
    int max_level = -1;
    for (auto& t : L.pos) max_level = std::max(max_level, t.level);
    L.pos_level_start.assign(1, 0);
    for (int lv = 0; lv <= max_level; lv++) {
      uint32_t e = L.pos_level_start.back();
      while (e < L.pos.size() && L.pos[e].level == lv) e++;
      L.pos_level_start.push_back(e);
    }
    for (uint32_t ri = 0; ri < L.regions.size(); ri++) {
      Region& r = L.regions[ri];
      if (r.kind == RK_POSEIDON) r.a[0] = inv[r.a[0]];
      std::vector<Work>* wl = r.kind == RK_SHA_BLOCK || r.kind == RK_SHA_OWN ? &L.work_sha
                              : r.kind == RK_POSEIDON                       ? &L.work_pos
                                                                            : &L.work_gen;
      uint32_t chunk = r.kind == RK_POSEIDON ? r.len : EMIT_CHUNK;
      for (uint32_t s = 0; s < r.len; s += chunk) wl->push_back(Work{ri, s, std::min(chunk, r.len - s), 0});
    }
  }
};

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
