// Builder shared by the layout translation units (builder.cpp, builder_register.cpp).
#pragma once
#include <algorithm>

#include "builder.hpp"

namespace pzk {

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

  int sha_job(int in_off, int blocks, int src = 0) {
    ShaJob j{};
    j.in_off = in_off;
    j.src = src;
    j.blocks = blocks;
    j.core_off = (int)L.sha_core_words;
    j.digest_slot = -1;
    j.hout = j.core_off + blocks * SHA_BLOCK_CORE;
    L.sha_core_words += blocks * SHA_BLOCK_CORE + 8;
    L.sha.push_back(j);
    return (int)L.sha.size() - 1;
  }

  // Sha256HashChunks(B) (sha256HashChunks.circom:8-48), optionally inside ShaHashChunks(B,256)
  // (hash.circom:32-68): own/wrapper signals as one RK_SHA_OWN region, then (sch, rds) per block.
  int sha256(int in_off, int blocks, bool wrapper, int src = 0) {
    int job = sha_job(in_off, blocks, src);
    uint64_t own = (wrapper ? 256 + 512ull * blocks : 0) + 256 + 512ull * blocks + 256ull * (blocks + 1) + 256;
    region(RK_SHA_OWN, own, {job, blocks, in_off, wrapper ? 1 : 0});
    for (int m = 0; m < blocks; m++) region(RK_SHA_BLOCK, SHA_BLOCK_LEN, {job, m});
    return job;
  }

  // Sha1HashChunks(B) (hasher/sha1/sha1.circom:7-57): own signals + H(0..4) as one RK_SHA1_OWN
  // region, then one RK_SHA1_BLOCK per Sha1compression
  int sha1(int in_off, int blocks, int src = 0) {
    ShaJob j{};
    j.in_off = in_off;
    j.blocks = blocks;
    j.core_off = (int)L.sha_core_words;
    j.digest_slot = -1;
    j.src = src;
    j.algo = 1;
    j.hout = j.core_off + blocks * SHA1_BLOCK_CORE;
    L.sha_core_words += blocks * SHA1_BLOCK_CORE + 8;
    L.sha.push_back(j);
    const int job = (int)L.sha.size() - 1;
    sha1_regions(job, in_off, blocks, false);
    return job;
  }
  // Sha1HashChunks regions of job (optionally inside ShaHashChunks(B,160): wrapper out[160] | in[512B] first)
  void sha1_regions(int job, int in_off, int blocks, bool wrapper) {
    region(RK_SHA1_OWN, (wrapper ? 160 + 512ull * blocks : 0) + 160 + 512ull * blocks + 5 * SHA1_CONST_SIGS,
           {job, blocks, in_off, wrapper ? 1 : 0});
    for (int m = 0; m < blocks; m++) region(RK_SHA1_BLOCK, SHA1_BLOCK_SIGS, {job, m});
  }
  // Sha384HashChunks / Sha512HashChunks(B) (hasher/sha2/sha384/sha384HashChunks.circom:8-48): own signals as
  // one RK_SHA5_OWN region, then one RK_SHA5_BLOCK (schedule + rounds) per 1024-bit block
  int sha512(int in_off, int blocks, int O, int src = 0, bool wrapper = false) {
    const int job = sha512_job(in_off, blocks, O, src);
    sha512_regions(job, in_off, blocks, wrapper);
    return job;
  }
  // the job alone: core = per block Hin, W, A, E (SHA5_BLOCK_CORE u32), then Hout as 8 u64 and as 16 big-endian
  // u32 words (hout: the form every digest consumer reads, bit i = word i / 32, bit 31 - i % 32)
  int sha512_job(int in_off, int blocks, int O, int src = 0) {
    ShaJob j{};
    j.in_off = in_off;
    j.blocks = blocks;
    j.digest_slot = -1;
    j.src = src;
    j.algo = O == 384 ? 3 : 4;
    L.sha_core_words += L.sha_core_words & 1;  // 64-bit words: 8-byte aligned within the row
    j.core_off = (int)L.sha_core_words;
    j.hout = j.core_off + blocks * SHA5_BLOCK_CORE + 16;
    L.sha_core_words += blocks * SHA5_BLOCK_CORE + 32;
    L.sha.push_back(j);
    return (int)L.sha.size() - 1;
  }
  // regions of a SHA-384/512 job, optionally inside ShaHashChunks(B, O) (hash.circom:32-68: out[O] | in[1024B] first)
  void sha512_regions(int job, int in_off, int blocks, bool wrapper) {
    const uint64_t O = L.sha[job].algo == 3 ? 384 : 512;
    region(RK_SHA5_OWN, (wrapper ? O + 1024ull * blocks : 0) + O + 1024ull * blocks + 512ull * (blocks + 1) + 512,
           {job, blocks, in_off, (int32_t)O, wrapper ? 1 : 0});
    for (int m = 0; m < blocks; m++) region(RK_SHA5_BLOCK, SHA5_BLOCK_SIGS, {job, m});
  }
  // a SHA job of either algorithm whose regions are placed later (sha_regions)
  int hash_job(int algo, int in_off, int blocks) {
    if (algo > 256) return sha512_job(in_off, blocks, algo);
    if (algo == 224) { const int j = sha_job(in_off, blocks); L.sha[j].algo = 2; return j; }
    if (algo != 160) return sha_job(in_off, blocks);
    ShaJob j{};
    j.in_off = in_off;
    j.blocks = blocks;
    j.core_off = (int)L.sha_core_words;
    j.digest_slot = -1;
    j.algo = 1;
    j.hout = j.core_off + blocks * SHA1_BLOCK_CORE;
    L.sha_core_words += blocks * SHA1_BLOCK_CORE + 8;
    L.sha.push_back(j);
    return (int)L.sha.size() - 1;
  }

  // PoseidonHash(n) (poseidon.circom:214-226) as one RK_POSEIDON region; returns output slot
  int poseidon(int n, const std::vector<int>& in_slots, int level, int out_slot = -1) {
    PosTask t{};
    t.n = n;
    int i = 0;
    for (int s : in_slots) t.in_slot[i++] = s;
    t.out_slot = out_slot >= 0 ? out_slot : value();
    t.core_off = (int)L.pos_core_elems;  // a multiple of 4 Fr: each task's slice starts on a 128-byte line
    t.level = level;
    t.smt_level = -1;
    L.pos_core_elems += (pos_core_len(n + 1) + 3) & ~3u;  // (k_pos_core1 writes whole lines, poseidon.hpp)
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
      int e = emitter_of(r.kind);
      if (emitter_packed(e)) continue;
      std::vector<Work>* wl = &L.work[e];
      if (r.kind == RK_BJJ_STEPS) {  // step-aligned: steps [k*S, (k+1)*S); step i starts at signal sig(i)
        auto sig = [](uint32_t i) -> uint32_t { return i == 0 ? 0 : 46 + 60 * (i - 1); };
        for (uint32_t i = 0; i < (uint32_t)BJJ_STEPS; i += BJJ_EMIT_STEPS) {
          uint32_t a0 = sig(i), a1 = i + BJJ_EMIT_STEPS >= (uint32_t)BJJ_STEPS ? r.len : sig(i + BJJ_EMIT_STEPS);
          wl->push_back(Work{ri, a0, a1 - a0, 0});
        }
        continue;
      }
      uint32_t chunk = emitter_whole(e) ? r.len : emit_chunk(e);
      for (uint32_t s = 0; s < r.len; s += chunk) wl->push_back(Work{ri, s, std::min(chunk, r.len - s), 0});
    }
    // SHA regions of hashers fed by derived messages are emitted after the chain that builds them
    for (auto [e, ed] : {std::pair<int, int>{E_SHA, E_SHAD}, std::pair<int, int>{E_SHA5, E_SHA5D}}) {
      std::vector<Work> keep, later;
      for (const Work& w : L.work[e]) (L.sha[L.regions[w.region].a[0]].src ? later : keep).push_back(w);
      L.work[e].swap(keep);
      L.work[ed].swap(later);
    }
    // Poseidon emission: one launch per width t, each with the LDS its image needs; the SMT level blocks (their core
    // state comes from the SMT chain) last, in groups of their own
    {
      auto t_of = [&](const Work& w) { return L.pos[L.regions[w.region].a[0]].n + 1; };
      auto chain_of = [&](const Work& w) { return L.pos[L.regions[w.region].a[0]].smt_level >= 0 ? 1 : 0; };
      std::vector<Work>& pw = L.work[E_POS];
      std::stable_sort(pw.begin(), pw.end(), [&](const Work& x, const Work& y) {
        return chain_of(x) != chain_of(y) ? chain_of(x) < chain_of(y) : t_of(x) < t_of(y);
      });
      L.pos_emit_groups.clear();
      L.pos_chain_group = ~0u;
      for (uint32_t i = 0; i < pw.size(); i++) {
        uint32_t t = (uint32_t)t_of(pw[i]);
        const bool ch = chain_of(pw[i]) != 0;
        if (ch && L.pos_chain_group == ~0u) {
          L.pos_chain_group = (uint32_t)L.pos_emit_groups.size();
          L.pos_emit_groups.push_back({t, i, 0});
        } else if (L.pos_emit_groups.empty() || L.pos_emit_groups.back()[0] != t) {
          L.pos_emit_groups.push_back({t, i, 0});
        }
        L.pos_emit_groups.back()[2]++;
      }
      if (L.pos_chain_group == ~0u) L.pos_chain_group = (uint32_t)L.pos_emit_groups.size();
    }
    // packed emitters: consecutive regions (witness order) share work items of <= GEN_PACK signals; E_GEN's regions
    // that read the SMT chain's output come after all others, from work item gen_chain_work on
    auto smt_chain_region = [](uint32_t kind) {
      return kind == RK_SMT_OWN || kind == RK_SMTHASH || kind == RK_SMT_LEVEL || kind == RK_SWITCHER ||
             kind == RK_ISEQ_ROOT;
    };
    for (int e = 0; e < E_COUNT; e++) {
      if (!emitter_packed(e)) continue;
      Work cur_w{0, 0, 0, 0};
      auto flush = [&]() { if (cur_w.count) L.work[e].push_back(cur_w); cur_w = Work{(uint32_t)L.gen_pieces.size(), 0, 0, 0}; };
      flush();
      for (int pass = 0; pass < (e == E_GEN ? 2 : 1); pass++) {
        if (pass == 1) {
          flush();
          L.gen_chain_work = (uint32_t)L.work[e].size();
        }
        for (uint32_t ri = 0; ri < L.regions.size(); ri++) {
          const Region& r = L.regions[ri];
          if (emitter_of(r.kind) != e || (e == E_GEN && smt_chain_region(r.kind) != (pass == 1))) continue;
          for (uint32_t s = 0; s < r.len;) {
            if (cur_w.count == GEN_PACK || cur_w.pad == GEN_MAX_PIECES) flush();
            uint32_t take = std::min(r.len - s, GEN_PACK - cur_w.count);
            L.gen_pieces.push_back(GenPiece{ri, s, cur_w.count, 0});
            cur_w.count += take; cur_w.pad++; s += take;
          }
        }
      }
      flush();
    }
  }
};


}  // namespace pzk
