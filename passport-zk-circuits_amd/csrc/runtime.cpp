// Host runtime + C-ABI (include/pzkwit.h): instance layout, device buffers, launch order.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/pzkwit.h"
#include "builder.hpp"
#include "kernels.hpp"
#include "bufs.hpp"
#include "ec_common.hpp"
#include "poseidon.hpp"
#include "query_layout.hpp"
#include "host_api.hpp"

using namespace pzk;

static thread_local std::string g_err;
static int fail(int code, const std::string& msg) { g_err = msg; return code; }
namespace pzk {
int api_fail(int code, const std::string& msg) { return fail(code, msg); }  // passport.cpp
}
#define HIPCHK(x)                                                                              \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) return fail(PZK_E_HIP, std::string(#x ": ") + hipGetErrorString(e_)); \
  } while (0)

// kernel phases, timed with HIP events on the launch stream when PZK_EXEC_TIMING is set
enum Phase {
  PH_LOAD, PH_SHA_CORE, PH_PREP, PH_RSA_CORE, PH_BJJ_CORE, PH_POS_CORE, PH_SMT,
  PH_EMIT_GEN, PH_EMIT_SHA, PH_EMIT_POS, PH_EMIT_BITS, PH_EMIT_FLOW, PH_EMIT_MM, PH_EMIT_BJJ,
  PH_EC_CORE, PH_EC_TABLE, PH_EMIT_ECT, PH_PSS, PH_EMIT_ECR, PH_EMIT_QRY, PH_COUNT
};
static const char* PHASE_NAMES[PH_COUNT] = {"load_values", "sha_core", "prep",     "rsa_core",  "bjj_core",
                                            "pos_core",    "smt",      "emit_gen", "emit_sha",  "emit_pos",
                                            "emit_bits",   "emit_flow", "emit_mm", "emit_bjj",
                                            "ec_core",     "ec_table",  "emit_ect", "pss",       "emit_ecr",
                                            "emit_qry"};
static const char* PHASE_KERNELS[PH_COUNT] = {"k_load_values", "k_sha_core",  "k_prep",      "k_rsa_core",
                                              "k_bjj_core",    "k_pos_core",  "k_smt_prep+k_smt_chain",
                                              "k_emit_gen",    "k_emit_sha",  "k_emit_pos",  "k_emit_bits",
                                              "k_emit_flow",   "k_emit_mm",   "k_emit_bjj",
                                              "k_ec_core",     "k_ec_table",  "k_emit_ect",
                                              "k_pss_mgf+k_sha_core+k_pss_mdash", "k_emit_ecr", "k_emit_qry"};
static const int EMIT_PHASE[E_COUNT] = {PH_EMIT_GEN, PH_EMIT_SHA, PH_EMIT_POS, PH_EMIT_BITS,
                                        PH_EMIT_FLOW, PH_EMIT_MM, PH_EMIT_BJJ, PH_EMIT_GEN, PH_EMIT_ECT,
                                        PH_EMIT_SHA, PH_EMIT_SHA, PH_EMIT_SHA, PH_EMIT_SHA, PH_EMIT_ECR,
                                        PH_EMIT_QRY};

// Per-phase HIP-event timing. A phase may be bracketed several times per batch (e.g. Poseidon
// levels before and after the SMT prep); its time is the sum of its brackets, each bracket
// recorded on the stream the phase's kernels run on.
struct Timing {
  static constexpr int RING = 8, OCC = 4;
  hipEvent_t ev[RING][PH_COUNT][OCC][2] = {};
  int used[RING][PH_COUNT] = {};
  bool pending[RING] = {};
  int head = 0;
  double ms[PH_COUNT] = {};
  uint64_t n[PH_COUNT] = {};
  void collect(int slot) {
    if (!pending[slot]) return;
    for (int p = 0; p < PH_COUNT; p++) {
      if (!used[slot][p]) continue;
      double sum = 0;
      bool ok = true;
      for (int k = 0; k < used[slot][p]; k++) {
        float t = 0;
        (void)hipEventSynchronize(ev[slot][p][k][1]);
        if (hipEventElapsedTime(&t, ev[slot][p][k][0], ev[slot][p][k][1]) == hipSuccess) sum += t; else ok = false;
      }
      if (ok) { ms[p] += sum; n[p]++; }
      used[slot][p] = 0;
    }
    pending[slot] = false;
  }
  void destroy() {
    for (auto& a : ev)
      for (auto& b : a)
        for (auto& c : b)
          for (auto& e : c)
            if (e) (void)hipEventDestroy(e);
  }
};

struct PhaseScope {
  Timing* T; int slot, ph, k = -1; hipStream_t st;
  PhaseScope(Timing* t, int s, int p, hipStream_t stream) : T(t), slot(s), ph(p), st(stream) {
    if (!T || T->used[slot][ph] >= Timing::OCC) return;
    k = T->used[slot][ph];
    for (auto& e : T->ev[slot][ph][k]) if (!e) (void)hipEventCreate(&e);
    (void)hipEventRecord(T->ev[slot][ph][k][0], st);
  }
  ~PhaseScope() {
    if (k < 0) return;
    (void)hipEventRecord(T->ev[slot][ph][k][1], st);
    T->used[slot][ph] = k + 1;
  }
};

// per-witness core state of one batch (one set per pipeline slot)
struct Scratch {
  size_t cap = 0;
  uint32_t* d_sha_core = nullptr;
  fr* d_pos_core = nullptr;
  fr* d_values = nullptr;
  uint64_t* d_rsa_core = nullptr;
  uint64_t* d_rsa_colsum = nullptr;  // RSA x*y column sums, SoA [(3 i + c)][witness]
  fr *d_bjj_core = nullptr, *d_bjj_scratch = nullptr, *d_smt_core = nullptr;
  uint64_t *d_ec_core = nullptr, *d_ec_jac = nullptr;
  fr* d_ec_inv = nullptr;
  uint8_t* d_ec_tab = nullptr;
  uint8_t* d_derived = nullptr;  // RSA-PSS derived SHA messages
  uint32_t* d_smt_order = nullptr;  // witnesses by SMT insertion level, deepest first (k_smt_order)
  void free_all() {
    void* ptrs[] = {d_sha_core, d_pos_core, d_values, d_rsa_core, d_rsa_colsum, d_bjj_core, d_bjj_scratch,
                    d_smt_core, d_ec_core, d_ec_jac, d_ec_inv, d_ec_tab, d_derived, d_smt_order};
    for (void* p : ptrs)
      if (p) (void)hipFree(p);
    *this = Scratch();
  }
};

// QueryIdentity: chain streams its calls rotate over (PZK_QRY_CHAINS = 1..4, default 4: the high-priority pool)
static int qry_chain_streams() {
  static const int v = getenv("PZK_QRY_CHAINS") ? atoi(getenv("PZK_QRY_CHAINS")) : 4;
  return v < 1 ? 1 : v > 4 ? 4 : v;
}
// QueryIdentity: emitter stream pairs its calls alternate over (PZK_QRY_EMIT = 1 | 2, default 2). With one pair the
// two emitter streams paced the line: with the quad SMT chain the Poseidon emitter stream ran 81 % and the other
// emitter stream 73 % of the timed region while the chain streams ran 48-67 % (profiles/r6d). Calls in flight never
// share output rows (pzkwit.h: a reused d_wtns needs a call index >= k + pipeline_depth), so consecutive calls'
// emitters need no ordering between them.
static int qry_emit_pairs() {
  static const int v = getenv("PZK_QRY_EMIT") ? atoi(getenv("PZK_QRY_EMIT")) : 2;
  return v < 2 ? 1 : 2;
}

// PZK_POST=0 (A/B): the register call's chain-dependent emission stays behind the chain on the emitter streams
// (rounds 1-4) instead of on its own post-chain stream
static bool post_chain_split(bool shared) {
  const char* e = getenv("PZK_POST");
  return e ? atoi(e) != 0 : !shared;
}
// live register instances per device (pzk_instance_create / destroy): an instance's stream set depends on whether
// it shares its device with other register instances (ensure_chain_streams)
static std::mutex g_reg_mu;
static std::map<int, int> g_register_instances;
static void register_count_add(int device, int d) {
  std::lock_guard<std::mutex> lk(g_reg_mu);
  g_register_instances[device] += d;
}
static int register_count(int device) {
  std::lock_guard<std::mutex> lk(g_reg_mu);
  auto it = g_register_instances.find(device);
  return it == g_register_instances.end() ? 0 : it->second;
}

// scratch sets (pipeline depth): call k uses set k % nsets and waits for call k - nsets (nsets = 3, or
// PZK_NSETS = 2..6 for A/B; nsets_env)
static constexpr int NSETS = PIPELINE_SETS_MAX;  // capacity

struct pzk_instance {
  pzk_params params;
  Timing timing;
  Layout lay;
  int device = 0;
  hipStream_t stream = nullptr;
  // side streams of the register pipeline (signature core; SHA emitters; other emitters, s_emit below). A register
  // instance has seven: main, s_rsa and the SMT chain streams s_tail / s_chain2 at high priority, s_sha, s_emit and
  // s_post at low priority (eight with PZK_SMT_CHAINS=3); HIP gives each priority GPU_MAX_HW_QUEUES (4) hardware
  // queues, so no two of them share one (pzk_instance_create)
  hipStream_t s_rsa = nullptr, s_sha = nullptr;
  hipEvent_t ev_load = nullptr, ev_sha = nullptr, ev_rsa = nullptr, ev_bjj = nullptr, ev_entry = nullptr, ev_dep = nullptr;
  // device copies of the layout
  Region* d_regions = nullptr;
  Work* d_work[E_COUNT] = {};
  GenPiece* d_gen_pieces = nullptr;
  uint32_t* d_sha_prog = nullptr;
  uint16_t* d_pos_prog = nullptr;
  ShaJob* d_sha = nullptr;
  PosTask* d_pos = nullptr;
  ValueLoad* d_loads = nullptr;
  int32_t* d_level_task = nullptr;
  fr* d_pos_consts = nullptr;
  fr* d_bjj_table = nullptr;  // fixed-base Base8 table (register circuit)
  // ECDSA (SIGNATURE_TYPE 20)
  uint64_t* d_ec_gpow = nullptr;
  uint32_t *d_ec_prog = nullptr, *d_ec_tab_off = nullptr;
  int32_t* d_ec_ops[3] = {};
  fr* d_inv_small = nullptr;
  PosParamIndex pix{};
  int pos_consts_n = 0;  // constants per copy (Montgomery copy first, then normal form)
  fr* d_pos_zimg = nullptr;  // zero-input Poseidon images + hashes (poseidon.hpp pos_zimg_off)
  fr* d_qc = nullptr;        // the quad SMT chain's constants (smt_chain4.hpp)
  PosConsts pos_consts() const {
    return PosConsts{d_pos_consts, d_pos_consts + pos_consts_n, pix, d_pos_consts + 2 * pos_consts_n, d_pos_zimg, d_qc};
  }
  // per-batch scratch, grown on demand; two sets, alternating per call, so that call k + 1's
  // cores can run while call k's emitters still read set k % 2
  Scratch scr[NSETS];
  uint64_t calls = 0;  // pzk_witness_batch calls so far (selects the scratch set)
  int nsets = 3;       // scratch sets in use (pipeline depth)
  int prio_lo = 0, prio_hi = 0;  // the device's stream priority range
  // ev_done[s][i]: end of the last call that used scratch set s, on stream i (main, rsa, sha, emit, tail, chain2)
  static constexpr int NSTREAMS = 10;  // ev_done slots (the streams list at the end of batch_locked)
  hipEvent_t ev_done[NSETS][NSTREAMS] = {};
  hipEvent_t ev_gather[2] = {};  // end of the last gather out of d_o0[slot]
  hipStream_t s_emit = nullptr;
  hipStream_t s_tail = nullptr;  // the small tail emitters (PZK_TAIL=own), so the next call's SHA emitter never queues behind them
  hipStream_t s_chain2 = nullptr, s_chain3 = nullptr;  // register calls: further SMT chain streams (PZK_SMT_CHAINS)
  // register calls: the emission that reads the SMT chain's output (the SMT level Poseidon blocks, the SMT regions),
  // one stream for every call so that a later call's writes of those regions follow an earlier call's
  hipStream_t s_post = nullptr;
  // register calls, PZK_SIGEMIT=own (A/B): the signature emitters (k_emit_mm) on a stream of their own, so the next
  // call's RSA core never queues behind them (PZK_MM_PRIO=hi|lo, default lo)
  hipStream_t s_mm = nullptr;
  // register calls with two SHA emitter streams (ensure_chain_streams): odd calls put the SHA emitters and the emission
  // behind them (the s_sha role) on s_sha2, so consecutive calls' SHA emitters do not queue behind each other on one
  // hardware queue (the O2-shaped line: that queue ran 90 % of the period and paced the pipeline, profiles/r5g)
  hipStream_t s_sha2 = nullptr;
  uint64_t chain_rr = 0;           // register calls: SMT chain stream rotation
  bool chain_set_shared = false;   // the chain stream set (s_tail ..) was made for a device shared with other register instances
  // register instances sharing a device run on that device's one stream set (ensure_chain_streams): the instance's
  // own main / rsa / sha / emit streams wait here meanwhile
  bool on_pool = false;
  hipStream_t own[4] = {};
  bool sha2_on = false;            // odd calls' SHA emission on s_sha2 (mapped layouts keeping <= 1/2 of the signals)
  hipEvent_t ev_pos = nullptr, ev_tab = nullptr, ev_smt = nullptr, ev_chain = nullptr;
  std::mutex mu;  // one in-flight call per instance (pzkwit.h): concurrent callers are serialised
  // optional signal -> witness map (circom .sym, pzk_instance_create_mapped): the emitters write the
  // --O0 witness of a chunk into d_o0[slot]; k_wtns_gather compacts it into the caller's rows
  uint64_t out_size = 0;          // elements per output witness (= lay.wit_size without a map)
  // monotone map (every .sym map circom writes): the emitters write the mapped witness directly
  // (mapsink.hpp): keep bitmap over the O0 indices + the kept count below every 64-signal boundary
  uint64_t* d_keep_bits = nullptr;
  uint32_t* d_keep_rank = nullptr;
  uint32_t* d_mprog = nullptr;  // the kept elements' descriptors of the descriptor-driven work items (Work.pad)
  uint32_t pos_nomix = 0;       // DevLayout.pos_nomix (mapped instances)
  uint32_t ect_split = ~0u;     // ECDSA: EC table work items [0, ect_split) on the signature stream, the rest on s_sha
  // any other map: O0 chunks into staging slots, then k_wtns_gather
  uint32_t* d_map = nullptr;      // out_size entries: O0 index of output element k
  std::vector<uint32_t> kept;     // mapped instances: the kept O0 indices, sorted (pzk_phase_info's bytes)
  uint64_t kept_in(uint64_t off, uint64_t len) const {  // kept signals in [off, off + len) (all without a map)
    if (kept.empty()) return len;
    return (uint64_t)(std::lower_bound(kept.begin(), kept.end(), (uint32_t)(off + len)) -
                      std::lower_bound(kept.begin(), kept.end(), (uint32_t)off));
  }
  uint8_t* d_o0[2] = {};
  size_t o0_cap = 0;
  // staging for the host-buffer path
  size_t host_cap = 0;
  uint8_t *d_in = nullptr, *d_out = nullptr;
  int32_t* d_status = nullptr;
  // streamed delivery (pzk_witness_stream): two chunk slots of device inputs / rows / statuses and
  // their pinned host copies, an input+compute stream and a device->host copy stream
  size_t st_cap = 0;
  uint8_t *st_din[2] = {}, *st_dout[2] = {}, *st_hout[2] = {};
  int32_t *st_dst[2] = {}, *st_hst[2] = {};
  hipStream_t s_in = nullptr, s_d2h = nullptr;
  hipEvent_t ev_comp[2] = {}, ev_d2h[2] = {};
  DevLayout dev_layout() const {
    DevLayout L{};
    L.wit_size = lay.wit_size;
    L.n_inputs = lay.n_inputs;
    L.n_derived = lay.n_derived;
    L.n_regions = (uint32_t)lay.regions.size();
    L.n_sha = (uint32_t)lay.sha.size();
    L.sha_core_words = (lay.sha_core_words + 1) & ~1u;  // even: SHA-512 cores are read as 64-bit words
    L.n_pos = (uint32_t)lay.pos.size();
    L.pos_core_elems = lay.pos_core_elems;
    L.n_values = lay.n_values;
    L.n_pos_levels = (uint32_t)lay.pos_level_start.size() - 1;
    L.regions = d_regions;
    L.gen_pieces = d_gen_pieces;
    L.sha_prog = d_sha_prog;
    L.pos_prog = d_pos_prog;
    for (int t = 0; t <= POS_MAX_T; t++) L.pos_prog_off[t] = lay.pos_prog_off[t];
    L.sha = d_sha;
    L.pos = d_pos;
    L.reg = lay.reg;
    L.rsa_core_words = lay.rsa_core_words;
    L.bjj_core_fr = lay.bjj_core_fr;
    L.smt_core_fr = lay.smt_core_fr;
    L.ec_gpow = d_ec_gpow;
    L.ec_prog = d_ec_prog;
    for (int t = 0; t < 3; t++) { L.ec_prog_off[t] = lay.ec_prog_off[t]; L.ec_tab_n[t] = lay.ec_tab_n[t]; }
    L.ec_tab_off = d_ec_tab_off;
    L.ec_tab_entries = lay.ec_tab_entries;
    L.keep = KeepMap{d_keep_bits, d_keep_rank};
    L.mprog = d_mprog;
    L.pos_nomix = pos_nomix;
    return L;
  }
};

static std::string data_dir() {
  const char* env = getenv("PZK_DATA_DIR");
  if (env && *env) return env;
  Dl_info info;
  if (dladdr((void*)&data_dir, &info) && info.dli_fname) {
    std::string p(info.dli_fname);
    size_t k = p.rfind('/');
    std::string dir = k == std::string::npos ? "." : p.substr(0, k);
    return dir + "/../data";
  }
  return "data";
}

__global__ void k_to_mont_inplace(fr* a, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) a[i] = fr_to_mont(a[i]);
}
// partial-round constant products for pos_core_group: sc[S index] = S[i] * C[5t + r] at i = (2t-1) r (the
// S[0] term) and i = (2t-1) r + t + k - 1 (the S'[k] updates); Montgomery in, Montgomery out
__global__ void k_pos_sc(const fr* m, fr* sc, PosParamIndex ix) {
  const int t = blockIdx.x + 2, r = threadIdx.x;
  if (t > POS_MAX_T || ix.nrp[t] == 0 || r >= ix.nrp[t]) return;
  const fr c = m[ix.c_off[t] + 5 * t + r];
  const int sb = ix.s_off[t] + (2 * t - 1) * r;
  sc[sb] = fr_mul(m[sb], c);
  for (int k = 1; k < t; k++) sc[sb + t + k - 1] = fr_mul(m[sb + t + k - 1], c);
}

static int load_poseidon(pzk_instance* I) {
  std::string path = data_dir() + "/poseidon_t2_6.bin";
  FILE* fp = fopen(path.c_str(), "rb");
  if (!fp) return fail(PZK_E_DATA, "cannot open Poseidon parameters " + path);
  std::vector<uint8_t> raw;
  uint8_t buf[65536];
  size_t k;
  while ((k = fread(buf, 1, sizeof buf, fp)) > 0) raw.insert(raw.end(), buf, buf + k);
  fclose(fp);
  if (raw.size() < 12 || memcmp(raw.data(), "PZKPOS01", 8)) return fail(PZK_E_DATA, "bad Poseidon parameter file");
  uint32_t nt;
  memcpy(&nt, raw.data() + 8, 4);
  size_t off = 12;
  std::vector<uint8_t> consts;
  memset(&I->pix, 0, sizeof I->pix);
  for (uint32_t q = 0; q < nt; q++) {
    uint32_t h[4];
    if (off + 16 > raw.size()) return fail(PZK_E_DATA, "truncated Poseidon parameter file");
    memcpy(h, raw.data() + off, 16);
    off += 16;
    int t = (int)h[0];
    if (t < 2 || t > POS_MAX_T || (int)h[1] != pos_nrp(t)) return fail(PZK_E_DATA, "unexpected Poseidon t/RP");
    size_t n_el = h[2] + 2ull * t * t + h[3];
    if (off + 32 * n_el > raw.size()) return fail(PZK_E_DATA, "truncated Poseidon parameter file");
    int base = (int)(consts.size() / 32);
    I->pix.nrp[t] = (int)h[1];
    I->pix.c_off[t] = base;
    I->pix.m_off[t] = base + (int)h[2];
    I->pix.p_off[t] = base + (int)h[2] + t * t;
    I->pix.s_off[t] = base + (int)h[2] + 2 * t * t;
    consts.insert(consts.end(), raw.begin() + off, raw.begin() + off + 32 * n_el);
    off += 32 * n_el;
  }
  int n = (int)(consts.size() / 32);
  // three copies: Montgomery form (cores), normal form (the emitters' round-constant adds), and the partial-round
  // products S * C (k_pos_sc) at S's indices
  HIPCHK(hipMalloc(&I->d_pos_consts, 3 * consts.size()));
  HIPCHK(hipMemcpy(I->d_pos_consts, consts.data(), consts.size(), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(I->d_pos_consts + n, consts.data(), consts.size(), hipMemcpyHostToDevice));
  HIPCHK(hipMemset(I->d_pos_consts + 2 * n, 0, consts.size()));
  I->pos_consts_n = n;
  hipLaunchKernelGGL(k_to_mont_inplace, dim3((n + 255) / 256), dim3(256), 0, 0, I->d_pos_consts, n);
  HIPCHK(hipGetLastError());
  hipLaunchKernelGGL(k_pos_sc, dim3(POS_MAX_T - 1), dim3(64), 0, 0, I->d_pos_consts, I->d_pos_consts + 2 * n, I->pix);
  HIPCHK(hipGetLastError());
  // the zero-input blocks (every PoseidonHash of zeros, e.g. the SMT levels below a proof's insertion level)
  fr* scratch = nullptr;
  HIPCHK(hipMalloc(&I->d_pos_zimg, sizeof(fr) * POS_ZBUF_TOTAL));
  HIPCHK(hipMalloc(&scratch, sizeof(fr) * (4 + 512)));
  HIPCHK(launch_pos_zero_img(I->pos_consts(), scratch, I->d_pos_zimg, nullptr));
  // the quad SMT chain's constant table (width 3)
  HIPCHK(hipMalloc(&I->d_qc, sizeof(fr) * QC_SIZE));
  HIPCHK(launch_qc_build(I->pos_consts(), I->d_qc, nullptr));
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipFree(scratch));
  // the zero-input blocks in O0 signal order (PosConsts::Zrow): image element pos_prog[i] at row position i
  const std::vector<uint16_t>& prog = I->lay.pos_prog;
  if (!prog.empty()) {
    std::vector<fr> buf(POS_ZBUF_TOTAL);
    HIPCHK(hipMemcpy(buf.data(), I->d_pos_zimg, sizeof(fr) * POS_ZIMG_TOTAL, hipMemcpyDeviceToHost));
    for (int t = 2; t <= POS_MAX_T; t++) {
      const uint32_t n = pos_hash_size_c(t - 1), img = (uint32_t)PosImg(t).size;
      if (I->lay.pos_prog_off[t] + n > prog.size()) return fail(PZK_E_DATA, "internal: Poseidon block program size");
      for (uint32_t i = 0; i < n; i++) {
        const uint16_t d = prog[I->lay.pos_prog_off[t] + i];
        if (d >= img) return fail(PZK_E_DATA, "internal: Poseidon block descriptor out of the image");
        buf[pos_zrow_off(t) + i] = buf[pos_zimg_off(t) + d];
      }
    }
    HIPCHK(hipMemcpy(I->d_pos_zimg + POS_ZIMG_TOTAL, buf.data() + POS_ZIMG_TOTAL,
                     sizeof(fr) * (POS_ZBUF_TOTAL - POS_ZIMG_TOTAL), hipMemcpyHostToDevice));
  }
  return 0;
}

template <typename T>
static int upload(T** dst, const std::vector<T>& v) {
  if (v.empty()) { *dst = nullptr; return 0; }
  HIPCHK(hipMalloc(dst, sizeof(T) * v.size()));
  HIPCHK(hipMemcpy(*dst, v.data(), sizeof(T) * v.size(), hipMemcpyHostToDevice));
  return 0;
}

static void free_scratch(pzk_instance* I) {
  for (Scratch& s : I->scr) s.free_all();
}

static void free_stream_bufs(pzk_instance* I) {
  for (int k = 0; k < 2; k++) {
    for (void* p : {(void*)I->st_din[k], (void*)I->st_dout[k], (void*)I->st_dst[k]})
      if (p) (void)hipFree(p);
    for (void* p : {(void*)I->st_hout[k], (void*)I->st_hst[k]})
      if (p) (void)hipHostFree(p);
    I->st_din[k] = I->st_dout[k] = I->st_hout[k] = nullptr;
    I->st_dst[k] = I->st_hst[k] = nullptr;
  }
  I->st_cap = 0;
}

// The device's register stream set (PZK_SHARED_STREAMS=0: one set per instance, the round-5 scheme): main, rsa, the two
// SMT chain streams at high priority; sha, emit, post, sha2 at low priority — GPU_MAX_HW_QUEUES (4) hardware queues per
// priority, so the set shares no queue whatever number of register instances run on the device.
struct PoolSet {
  hipStream_t s[8] = {};
  int refs = 0;
};
static std::map<int, PoolSet> g_pools;  // per device, under g_reg_mu
static bool shared_streams_on() {  // PZK_SHARED_STREAMS=1 (A/B; default off, see ensure_chain_streams)
  static const bool v = getenv("PZK_SHARED_STREAMS") && atoi(getenv("PZK_SHARED_STREAMS")) != 0;
  return v;
}
static void pool_release(int device) {
  std::lock_guard<std::mutex> lk(g_reg_mu);
  PoolSet& P = g_pools[device];
  if (--P.refs > 0) return;
  for (hipStream_t& st : P.s)
    if (st) { (void)hipStreamDestroy(st); st = nullptr; }
}
static bool pool_acquire(int device, int prio_lo, int prio_hi, hipStream_t* out) {
  std::lock_guard<std::mutex> lk(g_reg_mu);
  PoolSet& P = g_pools[device];
  if (P.refs == 0) {
    for (int k = 0; k < 8; k++)
      if (hipStreamCreateWithPriority(&P.s[k], hipStreamNonBlocking, k < 4 ? prio_hi : prio_lo) != hipSuccess) {
        for (hipStream_t& st : P.s)
          if (st) { (void)hipStreamDestroy(st); st = nullptr; }
        return false;
      }
  }
  P.refs++;
  for (int k = 0; k < 8; k++) out[k] = P.s[k];
  return true;
}
// leave the device's stream set: the instance's own main / rsa / sha / emit streams come back
static void pool_leave(pzk_instance* I) {
  if (!I->on_pool) return;
  I->stream = I->own[0];
  I->s_rsa = I->own[1];
  I->s_sha = I->own[2];
  I->s_emit = I->own[3];
  for (hipStream_t& o : I->own) o = nullptr;
  I->s_tail = I->s_chain2 = I->s_chain3 = I->s_post = I->s_mm = I->s_sha2 = nullptr;
  I->on_pool = false;
  pool_release(I->device);
}
static void release_streams(pzk_instance* I) {
  pool_leave(I);
  for (hipStream_t s : {I->stream, I->s_rsa, I->s_sha, I->s_emit, I->s_tail, I->s_chain2, I->s_chain3, I->s_post, I->s_mm,
                        I->s_sha2})
    if (s) (void)hipStreamDestroy(s);
}

static void free_all(pzk_instance* I) {
  free_scratch(I);
  void* ptrs[] = {I->d_regions, I->d_gen_pieces, I->d_sha_prog, I->d_pos_prog, I->d_sha, I->d_pos, I->d_loads, I->d_level_task,
                  I->d_pos_consts, I->d_bjj_table, I->d_in, I->d_out, I->d_status, I->d_ec_gpow, I->d_ec_prog,
                  I->d_ec_tab_off, I->d_ec_ops[0], I->d_ec_ops[1], I->d_ec_ops[2], I->d_inv_small, I->d_map,
                  I->d_o0[0], I->d_o0[1], I->d_keep_bits, I->d_keep_rank, I->d_mprog, I->d_pos_zimg, I->d_qc};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  for (auto* p : I->d_work)
    if (p) (void)hipFree(p);
  release_streams(I);
  for (hipEvent_t e : {I->ev_load, I->ev_sha, I->ev_rsa, I->ev_bjj, I->ev_entry, I->ev_dep, I->ev_pos, I->ev_tab,
                       I->ev_smt, I->ev_chain})
    if (e) (void)hipEventDestroy(e);
  for (auto& set : I->ev_done)
    for (hipEvent_t e : set)
      if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : I->ev_gather)
    if (e) (void)hipEventDestroy(e);
  free_stream_bufs(I);
  for (hipStream_t st : {I->s_in, I->s_d2h})
    if (st) (void)hipStreamDestroy(st);
  for (int k = 0; k < 2; k++)
    for (hipEvent_t e : {I->ev_comp[k], I->ev_d2h[k]})
      if (e) (void)hipEventDestroy(e);
  I->timing.destroy();
}

// The caller's current device is switched to the instance's for the duration of a call and
// restored on return (every stream, event and buffer of an instance lives on its device).
struct DeviceGuard {
  int prev = -1;
  hipError_t err = hipSuccess;
  explicit DeviceGuard(int dev) {
    err = hipGetDevice(&prev);
    if (err == hipSuccess && prev != dev) err = hipSetDevice(dev);
    else prev = -1;
  }
  ~DeviceGuard() { if (prev >= 0) (void)hipSetDevice(prev); }
};

// wait until every stream of the instance has drained (all calls issued so far are complete)
static int sync_all(pzk_instance* I) {
  for (hipStream_t s : {I->stream, I->s_rsa, I->s_sha, I->s_emit, I->s_tail, I->s_chain2, I->s_chain3, I->s_post, I->s_mm,
                        I->s_sha2})
    if (s) HIPCHK(hipStreamSynchronize(s));
  return 0;
}

extern "C" {

const char* pzk_last_error(void) { return g_err.c_str(); }
const char* pzk_version(void) { return "pzkwit 0.2.0 (gfx950)"; }

static int pzk_instance_create_impl(const pzk_params* params, pzk_instance** out) {
  if (!params || !out) return fail(PZK_E_ARG, "null argument");
  if (const char* u = getenv("PZK_SHA_U")) {  // tuning switch of the SHA emitter (kernels.hip)
    int v = atoi(u);
    if (v != 8 && v != 16 && v != 32) return fail(PZK_E_ARG, std::string("PZK_SHA_U=") + u + ": valid values are 8, 16, 32");
  }
  if (const char* u = getenv("PZK_BJJ_SEGS")) {  // tuning switch of k_bjj_core (kernels.hip)
    int v = atoi(u);
    const bool sc = bjj_uses_scratch();
    if (sc ? (v != 8 && v != 16 && v != 32) : (v != 16 && v != 32 && v != 64))
      return fail(PZK_E_ARG, std::string("PZK_BJJ_SEGS=") + u +
                                 (sc ? ": valid values are 8, 16, 32 (PZK_BJJ=scratch)" : ": valid values are 16, 32, 64"));
  }
  if (const char* u = getenv("PZK_BJJ"))
    if (strcmp(u, "scratch") && strcmp(u, "rc")) return fail(PZK_E_ARG, std::string("PZK_BJJ=") + u + ": valid values are rc, scratch");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    return fail(PZK_E_NODEVICE, "no HIP device visible: pzkwit has no CPU fallback");
  pzk_instance* I = new pzk_instance();
  I->params = *params;
  I->nsets = nsets_env(params->circuit == PZK_CIRCUIT_QUERY);
  std::string why;
  if (!build_layout(*params, I->lay, why)) { delete I; return fail(PZK_E_PARAMS, why); }
  HIPCHK(hipGetDevice(&I->device));
  int rc;
  if ((rc = load_poseidon(I)) != 0) { free_all(I); delete I; return rc; }
  std::vector<int32_t> level_task(SMT_LEVELS, -1);
  for (size_t i = 0; i < I->lay.pos.size(); i++)
    if (I->lay.pos[i].smt_level >= 0) level_task[I->lay.pos[i].smt_level] = (int32_t)i;
  rc = upload(&I->d_regions, I->lay.regions);
  for (int e = 0; e < E_COUNT && !rc; e++) rc = upload(&I->d_work[e], I->lay.work[e]);
  if (!rc) rc = upload(&I->d_gen_pieces, I->lay.gen_pieces);
  if (!rc) rc = upload(&I->d_sha_prog, I->lay.sha_prog);
  if (!rc) rc = upload(&I->d_pos_prog, I->lay.pos_prog);
  if (!rc) rc = upload(&I->d_sha, I->lay.sha);
  if (!rc) rc = upload(&I->d_pos, I->lay.pos);
  if (!rc) rc = upload(&I->d_loads, I->lay.loads);
  const bool chains = I->lay.is_register || I->lay.is_query;  // SMT / BabyJubJub chains
  if (!rc && chains) rc = upload(&I->d_level_task, level_task);
  if (!rc && chains) {
    if (hipMalloc(&I->d_bjj_table, sizeof(fr) * 3 * BJJ_TABLE_WINDOWS * 256) != hipSuccess ||
        launch_bjj_table(I->d_bjj_table, nullptr) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
      rc = fail(PZK_E_HIP, "BabyJubJub table setup failed");
  }
  if (!rc && I->lay.is_ecdsa) {
    static const char* const names[EC_N_CURVES] = {"/p256_gpow8.bin", "/bp256_gpow8.bin", "/p224_gpow8.bin", "/bp384_gpow8.bin"};
    const EcGeo& G = EC_GEO[I->lay.reg.ec_curve];
    std::string path = data_dir() + names[I->lay.reg.ec_curve];
    std::vector<uint64_t> tab((size_t)G.parts * 256 * 2 * G.nl);  // [PARTS][256][2][N] chunks
    FILE* fp = fopen(path.c_str(), "rb");
    size_t got = fp ? fread(tab.data(), 8, tab.size(), fp) : 0;
    if (fp) fclose(fp);
    if (got != tab.size()) rc = fail(PZK_E_DATA, "cannot read the EC generator table " + path);
    if (!rc) rc = upload(&I->d_ec_gpow, tab);
    if (!rc) rc = upload(&I->d_ec_prog, I->lay.ec_prog);
    if (!rc) rc = upload(&I->d_ec_tab_off, I->lay.ec_tab_off);
    for (int t = 0; t < 3 && !rc; t++) rc = upload(&I->d_ec_ops[t], I->lay.ec_ops[t]);
    if (!rc && (hipMalloc(&I->d_inv_small, sizeof(fr) * 256) != hipSuccess ||
                launch_inv_small(I->d_inv_small, nullptr) != hipSuccess || hipDeviceSynchronize() != hipSuccess))
      rc = fail(PZK_E_HIP, "ECDSA constant setup failed");
  }
  if (!rc && I->lay.is_query &&
      (hipMalloc(&I->d_inv_small, sizeof(fr) * 256) != hipSuccess ||
       launch_inv_small(I->d_inv_small, nullptr) != hipSuccess || hipDeviceSynchronize() != hipSuccess))
    rc = fail(PZK_E_HIP, "QueryIdentity constant setup failed");
  if (rc) { free_all(I); delete I; return rc; }
  // The dependency chains (main stream: Poseidon/SMT/BJJ cores; s_rsa: RSA core) get the
  // highest queue priority, the bulk SHA emitter the lowest: when the chip is full of emitter
  // workgroups, the dispatcher hands freed CU slots to the latency-bound chain kernels first.
  int prio_lo = 0, prio_hi = 0;
  (void)hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
  bool ok = hipStreamCreateWithPriority(&I->stream, hipStreamNonBlocking, prio_hi) == hipSuccess &&
            hipStreamCreateWithPriority(&I->s_rsa, hipStreamNonBlocking, prio_hi) == hipSuccess;
  I->prio_lo = prio_lo;
  I->prio_hi = prio_hi;
  // (PZK_SHA_PRIO=hi, A/B: the SHA emitter stream at high priority — give the process GPU_MAX_HW_QUEUES >= 5 then,
  // or it shares a hardware queue with a chain stream)
  static const bool sha_hi = getenv("PZK_SHA_PRIO") && !strcmp(getenv("PZK_SHA_PRIO"), "hi");
  ok = ok && hipStreamCreateWithPriority(&I->s_sha, hipStreamNonBlocking, sha_hi ? prio_hi : prio_lo) == hipSuccess &&
       hipStreamCreateWithPriority(&I->s_emit, hipStreamNonBlocking, prio_lo) == hipSuccess;
  // the chain streams: QueryIdentity's now (its third / fourth chain, high priority); the register circuit's at its
  // first call (ensure_chain_streams), when it is known whether other register instances share the process
  if (ok && !I->lay.is_register) {
    ok = hipStreamCreateWithPriority(&I->s_tail, hipStreamNonBlocking, prio_hi) == hipSuccess;
    if (ok && I->lay.is_query && qry_chain_streams() >= 4)
      ok = hipStreamCreateWithPriority(&I->s_chain2, hipStreamNonBlocking, prio_hi) == hipSuccess;
    // QueryIdentity: a second pair of emitter streams for odd calls (qry_emit_pairs): the low-priority pool's other
    // two hardware queues
    if (ok && I->lay.is_query && qry_emit_pairs() >= 2)
      ok = hipStreamCreateWithPriority(&I->s_sha2, hipStreamNonBlocking, prio_lo) == hipSuccess &&
           hipStreamCreateWithPriority(&I->s_post, hipStreamNonBlocking, prio_lo) == hipSuccess;
  }
  for (hipEvent_t* e : {&I->ev_load, &I->ev_sha, &I->ev_rsa, &I->ev_bjj, &I->ev_entry, &I->ev_dep, &I->ev_pos, &I->ev_tab,
                        &I->ev_smt, &I->ev_chain})
    ok = ok && hipEventCreateWithFlags(e, hipEventDisableTiming) == hipSuccess;
  for (hipEvent_t& e : I->ev_gather) {
    ok = ok && hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess;
    ok = ok && hipEventRecord(e, nullptr) == hipSuccess;
  }
  for (auto& set : I->ev_done)
    for (hipEvent_t& e : set) {
      ok = ok && hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess;
      // recorded once on the null stream, so the first two calls' waits are satisfied
      ok = ok && hipEventRecord(e, nullptr) == hipSuccess;
    }
  if (!ok) { free_all(I); delete I; return fail(PZK_E_HIP, "hipStreamCreate/hipEventCreate failed"); }
  I->out_size = I->lay.wit_size;
  if (I->lay.is_ecdsa) {  // PZK_ECT_SPLIT: the share of the EC table elements emitted on the SHA emitter stream
    static const double frac = getenv("PZK_ECT_SPLIT") ? atof(getenv("PZK_ECT_SPLIT")) : 0.0;
    const std::vector<Work>& wl = I->lay.work[E_ECT];
    uint64_t tot = 0, acc = 0;
    for (const Work& w : wl) tot += w.count;
    I->ect_split = (uint32_t)wl.size();
    for (uint32_t i = 0; i < wl.size() && frac > 0; i++) {
      if ((double)acc >= (1.0 - frac) * (double)tot) { I->ect_split = i; break; }
      acc += wl[i].count;
    }
  }
  if (I->lay.is_register) register_count_add(I->device, 1);
  *out = I;
  return 0;
}

static int pzk_instance_create_mapped_impl(const pzk_params* params, const char* sym, size_t sym_len, pzk_instance** out) {
  if (!params || !out) return fail(PZK_E_ARG, "null argument");
  if (!sym) return pzk_instance_create(params, out);
  pzk_instance* I = nullptr;
  int rc = pzk_instance_create(params, &I);
  if (rc) return rc;
  std::vector<uint32_t> inv;
  std::string why;
  if (!parse_sym(sym, sym_len, I->lay.wit_size, inv, why)) { pzk_instance_destroy(I); return fail(PZK_E_ARG, why); }
  MapProgram mp;
  static const bool force_gather = getenv("PZK_SYM_GATHER") != nullptr;  // A/B: the staging + gather path
  map_program(I->lay, inv, force_gather, mp);
  bool ok;
  if (mp.direct) {
    // direct emission (mapsink.hpp): keep bitmap + ranks, and the descriptor-driven work items' kept descriptors
    ok = upload(&I->d_keep_bits, mp.bits) == 0 && upload(&I->d_keep_rank, mp.rank) == 0;
    for (int e : {E_SHA, E_SHAD, E_POS, E_ECT}) {
      if (I->d_work[e]) { (void)hipFree(I->d_work[e]); I->d_work[e] = nullptr; }
      ok = ok && upload(&I->d_work[e], mp.work[e]) == 0;
      I->lay.work[e] = mp.work[e];
    }
    ok = ok && upload(&I->d_mprog, mp.mprog) == 0;
    I->pos_nomix = mp.pos_nomix;
  } else {
    ok = upload(&I->d_map, inv) == 0;
  }
  if (!ok) {
    pzk_instance_destroy(I);
    return fail(PZK_E_NOMEM, "device allocation of the signal map failed");
  }
  I->out_size = inv.size();
  I->kept = inv;
  std::sort(I->kept.begin(), I->kept.end());
  *out = I;
  return 0;
}

static void pzk_instance_destroy_impl(pzk_instance* inst) {
  if (!inst) return;
  if (inst->lay.is_register) register_count_add(inst->device, -1);
  {
    // calls are asynchronous across the instance's streams: wait for a concurrent caller to leave and
    // for every call in flight to drain, on the instance's device, before anything is freed
    std::lock_guard<std::mutex> lock(inst->mu);
    DeviceGuard dg(inst->device);
    (void)sync_all(inst);
    free_all(inst);
  }
  delete inst;
}

static int pzk_instance_info_impl(const pzk_instance* I, pzk_info* info) {
  if (!I || !info) return fail(PZK_E_ARG, "null argument");
  memset(info, 0, sizeof *info);
  info->witness_size = I->out_size;
  info->n_inputs = I->lay.n_inputs;
  info->n_outputs = I->lay.n_outputs;
  info->n_public_inputs = I->lay.n_public;
  info->n_input_groups = (uint32_t)I->lay.inputs.size();
  info->pipeline_depth = I->nsets;
  return 0;
}

static int pzk_instance_input_impl(const pzk_instance* I, uint32_t i, const char** name, uint64_t* offset, uint64_t* length) {
  if (!I || i >= I->lay.inputs.size()) return fail(PZK_E_ARG, "input index out of range");
  if (name) *name = I->lay.inputs[i].name.c_str();
  if (offset) *offset = I->lay.inputs[i].offset;
  if (length) *length = I->lay.inputs[i].length;
  return 0;
}

static int pzk_wtns_header_impl(const pzk_instance* I, uint8_t h[76]) {
  if (!I || !h) return fail(PZK_E_ARG, "null argument");
  static const uint8_t prime[32] = {0x01, 0x00, 0x00, 0xf0, 0x93, 0xf5, 0xe1, 0x43, 0x91, 0x70, 0xb9,
                                    0x79, 0x48, 0xe8, 0x33, 0x28, 0x5d, 0x58, 0x81, 0x81, 0xb6, 0x45,
                                    0x50, 0xb8, 0x29, 0xa0, 0x31, 0xe1, 0x72, 0x4e, 0x64, 0x30};
  uint8_t* p = h;
  auto u32 = [&](uint32_t v) { memcpy(p, &v, 4); p += 4; };
  auto u64 = [&](uint64_t v) { memcpy(p, &v, 8); p += 8; };
  memcpy(p, "wtns", 4); p += 4;
  u32(2); u32(2);
  u32(1); u64(40); u32(32); memcpy(p, prime, 32); p += 32; u32((uint32_t)I->out_size);
  u32(2); u64(32ull * I->out_size);
  return 0;
}

static int ensure_scratch(pzk_instance* I, Scratch& S, size_t batch) {
  if (batch <= S.cap) return 0;
  S.free_all();
  const Layout& L = I->lay;
  struct { void** p; size_t bytes; } req[] = {
      {(void**)&S.d_sha_core, 4ull * ((L.sha_core_words + 1) & ~1u) * batch},
      {(void**)&S.d_pos_core, 32ull * L.pos_core_elems * batch},
      {(void**)&S.d_values, 32ull * std::max<uint32_t>(L.n_values, 1) * batch},
      {(void**)&S.d_rsa_core, 8ull * L.rsa_core_words * batch},
      {(void**)&S.d_rsa_colsum, L.is_register ? 8ull * 3 * 2 * L.reg.K * batch : 0},
      {(void**)&S.d_bjj_core, 32ull * L.bjj_core_fr * batch},
      {(void**)&S.d_bjj_scratch, (L.is_register || L.is_query) && bjj_uses_scratch() ? 32ull * BJJ_SCRATCH_FR * batch : 0},
      {(void**)&S.d_smt_core, 32ull * L.smt_core_fr * batch},
      {(void**)&S.d_ec_core, L.is_ecdsa ? 8ull * EC_GEO[L.reg.ec_curve].core_words * batch : 0},
      {(void**)&S.d_ec_jac, L.is_ecdsa ? 8ull * EC_GEO[L.reg.ec_curve].jac_words * batch : 0},
      {(void**)&S.d_ec_inv, L.is_ecdsa ? 32ull * EC_GEO[L.reg.ec_curve].n_inv * batch : 0},
      {(void**)&S.d_ec_tab, L.is_ecdsa ? 32ull * L.ec_tab_entries * batch : 0},
      {(void**)&S.d_derived, 32ull * L.n_derived * batch},
      {(void**)&S.d_smt_order, (L.is_register || L.is_query) ? 4ull * batch : 0},
  };
  for (auto& r : req)
    if (r.bytes && hipMalloc(r.p, r.bytes) != hipSuccess) {
      S.free_all();
      return fail(PZK_E_NOMEM, "device scratch allocation failed");
    }
  S.cap = batch;
  return 0;
}

static int check_exec_device(const pzk_instance* I, const pzk_exec* exec) {
  if (exec && exec->device >= 0 && exec->device != I->device)
    return fail(PZK_E_ARG, "pzk_exec.device " + std::to_string(exec->device) + " != the instance's device " +
                               std::to_string(I->device) + " (create one instance per device)");
  return 0;
}

// A register instance's chain and post-chain streams, chosen at every call. The SMT chain streams (s_tail, s_chain2)
// are high priority: besides dispatch order this sets the hardware queues — HIP gives each stream priority a pool of
// GPU_MAX_HW_QUEUES (4 by default) queues and lets streams share one beyond that, and a shared queue runs its streams'
// packets in submission order, so a stream waiting for the chain stalls the other. One instance: high main, rsa,
// s_tail, s_chain2; low s_sha, s_emit, s_post (+ s_sha2 for sparse maps) — nothing shared (config 4 58.3k -> 71.4k
// witnesses/s, profiles/r5c). Several register instances on one device (config 5: one per flow) with a set each
// overflow the queues (round 5: with every instance's full set config 5 ran 8.5k witnesses/s, with low-priority chain
// streams and no post-chain streams 48.2k, but only at GPU_MAX_HW_QUEUES=16 — ~41k at the default 4, profiles/r4_hwq,
// r5j-r5l). So an instance that shares its device with other register instances takes the reduced set (low-priority
// chain streams, no post-chain stream): config 5 46.9k witnesses/s at the default 4 queues (profiles/r6i). One set for
// all instances of a device (PZK_SHARED_STREAMS=1: the device pool, PoolSet — their calls queue into the same eight
// streams in submission order, which fit the default queues) measured 43.2k there: a flow's long chain (the ECDSA core
// on s_rsa) then blocks the next flow's cores. The count is per device and is re-checked at every call: an instance
// whose set no longer matches (another instance appeared on its device, or went away) drains its streams and
// rebuilds, so the order in which a caller creates and first runs its instances does not matter. PZK_CHAIN_PRIO=hi|lo
// and PZK_POST=0|1 force the reduced set's choices.
// Own sets are created into locals and assigned only once all exist: a failure leaves the instance without a set
// (retried at the next call), never with half of one.
static int ensure_chain_streams(pzk_instance* I) {
  if (!I->lay.is_register) return 0;
  const bool shared = register_count(I->device) > 1;
  const bool pool = shared && shared_streams_on();
  // odd calls' SHA emission on a second stream: default for mapped layouts keeping at most half of the signals
  // (O2-shaped 206.9k -> 218.5k witnesses/s; O1-shaped, 56 % kept, 130.8k -> 130.2k: profiles/r5q); the O0 layout
  // keeps one (+1 % with two, but each k_emit_sha launch then runs beside the other call's and takes twice as long:
  // its roofline line would read 0.35 for the same HBM work, profiles/r5p). PZK_SHA_STREAMS=1|2 forces either.
  const char* ss_env = getenv("PZK_SHA_STREAMS");
  I->sha2_on = ss_env ? atoi(ss_env) >= 2 : I->d_keep_bits != nullptr && 2 * I->out_size <= I->lay.wit_size;
  if (pool ? I->on_pool : (I->s_tail && !I->on_pool && I->chain_set_shared == shared)) return 0;
  if (I->s_tail || I->on_pool) {  // the set no longer fits: drain every call in flight, then replace it
    int rc = sync_all(I);
    if (rc) return rc;
    if (I->on_pool) {
      pool_leave(I);
    } else {
      for (hipStream_t* s : {&I->s_tail, &I->s_chain2, &I->s_chain3, &I->s_post, &I->s_mm, &I->s_sha2})
        if (*s) { (void)hipStreamDestroy(*s); *s = nullptr; }
    }
  }
  if (pool) {  // the device's one set: every register instance on it queues into the same eight streams
    hipStream_t p[8];
    if (!pool_acquire(I->device, I->prio_lo, I->prio_hi, p))
      return fail(PZK_E_HIP, "hipStreamCreateWithPriority failed (the device's register stream set)");
    I->own[0] = I->stream;
    I->own[1] = I->s_rsa;
    I->own[2] = I->s_sha;
    I->own[3] = I->s_emit;
    I->stream = p[0];
    I->s_rsa = p[1];
    I->s_tail = p[2];
    I->s_chain2 = p[3];
    I->s_sha = p[4];
    I->s_emit = p[5];
    I->s_post = p[6];
    I->s_sha2 = p[7];
    I->on_pool = true;
    return 0;
  }
  hipStream_t made[6] = {};  // s_tail, s_chain2, s_chain3, s_post, s_mm, s_sha2
  auto create = [&](int k, int prio) -> bool {
    if (hipStreamCreateWithPriority(&made[k], hipStreamNonBlocking, prio) == hipSuccess) return true;
    made[k] = nullptr;
    return false;
  };
  const char* cp_env = getenv("PZK_CHAIN_PRIO");
  const bool chain_lo = cp_env ? !strcmp(cp_env, "lo") : shared;
  const int prio_chain = chain_lo ? I->prio_lo : I->prio_hi;
  bool ok = create(0, prio_chain) && create(1, prio_chain);
  // the third chain stream only when asked for (PZK_SMT_CHAINS=3)
  if (ok && getenv("PZK_SMT_CHAINS") && atoi(getenv("PZK_SMT_CHAINS")) >= 3) ok = create(2, prio_chain);
  if (ok && post_chain_split(shared)) ok = create(3, I->prio_lo);
  static const char* se_env = getenv("PZK_SIGEMIT");
  if (ok && se_env && !strcmp(se_env, "own") && !shared && !I->lay.is_ecdsa) {
    static const char* mp_env = getenv("PZK_MM_PRIO");
    const bool hi = mp_env && !strcmp(mp_env, "hi");
    ok = create(4, hi ? I->prio_hi : I->prio_lo);
  }
  if (ok && I->sha2_on && !shared) ok = create(5, I->prio_lo);
  if (!ok) {
    for (hipStream_t s : made)
      if (s) (void)hipStreamDestroy(s);
    return fail(PZK_E_HIP, "hipStreamCreateWithPriority failed (the instance's chain streams)");
  }
  I->s_tail = made[0];
  I->s_chain2 = made[1];
  I->s_chain3 = made[2];
  I->s_post = made[3];
  I->s_mm = made[4];
  I->s_sha2 = made[5];
  I->chain_set_shared = shared;
  return 0;
}

// One call, with the instance lock held and the device set.
//
// Pipelining: call k uses scratch set k % nsets and four instance streams — main (the
// Poseidon/SMT/BabyJubJub chain), rsa (the signature core), sha (the SHA emitters) and emit (the other
// emitters). Streams are not joined at the end of a call: call k + 1's cores start while call k's
// emitters still run. Before touching set k % nsets again, call k + nsets waits for the end of call k
// on all four streams (ev_done). With a caller stream the call is joined into it at exit (serialised).
// dep: an instance stream whose work so far the call must follow (the input upload of pzk_witness_batch_host,
// the staging-slot waits of batch_mapped). Every stream of the call descends from its chain stream st (the
// other streams wait for events recorded on st), so st waiting for dep orders the whole call after it — also
// when a QueryIdentity call's chain runs on s_rsa or s_tail instead of the main stream.
static int batch_locked(pzk_instance* I, const uint8_t* d_inputs, size_t batch, uint8_t* d_wtns, size_t stride,
                        int32_t* d_status, const pzk_exec* exec, hipStream_t dep = nullptr) {
  const int set = (int)(I->calls % I->nsets);
  Scratch& S = I->scr[set];
  int rc = ensure_chain_streams(I);
  if (rc) return rc;
  rc = ensure_scratch(I, S, batch);
  if (rc) return rc;
  I->calls++;
  hipStream_t user = (exec && exec->stream) ? (hipStream_t)exec->stream : nullptr;
  // PZK_SERIAL=1 (profiling): every phase on the main stream, so kernel times are standalone
  static const bool serial = getenv("PZK_SERIAL") != nullptr;
  // QueryIdentity: the whole per-call chain (prep .. SMT chain) is one latency-bound dependency chain whose
  // length is the SMT proof depth (k_smt_chain: 0.5 ms per level for 4096 witnesses, one wave per CU), so
  // consecutive calls rotate over qry_chain_streams() (1 / 2 / 3 / 4) chain streams — main, s_rsa, s_tail,
  // s_chain2, all high priority — and their chains run side by side
  const int qry_chains = qry_chain_streams();
  hipStream_t st = I->stream;
  if (I->lay.is_query && !serial && qry_chains > 1) {
    const int c = (int)((I->calls - 1) % (uint64_t)qry_chains);
    st = c == 0 ? I->stream : c == 1 ? I->s_rsa : c == 2 ? I->s_tail : I->s_chain2;
  }
  for (hipEvent_t e : I->ev_done[set]) HIPCHK(hipStreamWaitEvent(st, e, 0));
  if (user) {
    HIPCHK(hipEventRecord(I->ev_entry, user));
    HIPCHK(hipStreamWaitEvent(st, I->ev_entry, 0));
  }
  if (dep && dep != st) {
    HIPCHK(hipEventRecord(I->ev_dep, dep));
    HIPCHK(hipStreamWaitEvent(st, I->ev_dep, 0));
  }
  const uint32_t B = (uint32_t)batch;
  const Layout& lay = I->lay;
  const uint32_t ect_split = I->ect_split;
  DevLayout L = I->dev_layout();
  ValueStore vs{S.d_values, B};
  const PosConsts K = I->pos_consts();
  Bufs bufs{d_inputs, S.d_sha_core, S.d_rsa_core, S.d_pos_core, S.d_bjj_core, S.d_smt_core, vs, d_wtns, stride,
            d_status, S.d_ec_core, S.d_ec_inv, S.d_ec_tab, I->d_inv_small, S.d_derived};
  Timing* T = nullptr;
  int slot = 0;
  if (exec && (exec->flags & PZK_EXEC_TIMING)) {
    T = &I->timing;
    slot = T->head;
    T->collect(slot);
    T->head = (T->head + 1) % Timing::RING;
    T->pending[slot] = true;
  }
  // order: the SMT level hashes' witness order (k_smt_order, depth sorted), or null (witness order)
  auto pos_levels = [&](int lo, int hi, const uint32_t* order = nullptr) -> int {
    for (int l = lo; l < hi && l + 1 < (int)lay.pos_level_start.size(); l++) {
      uint32_t a = lay.pos_level_start[l], b = lay.pos_level_start[l + 1];
      HIPCHK(launch_pos_core(K, I->d_pos, lay.pos.data(), a, b - a, vs, S.d_pos_core, lay.pos_core_elems,
                             S.d_smt_core, lay.smt_core_fr, order, st));
    }
    return 0;
  };
  // one emitter's work items [a, b) (default: all) on stream s
  auto emit = [&](int e, hipStream_t s, uint32_t a = 0, uint32_t b = ~0u) -> int {
    if (e == E_POS) {
      b = std::min<uint32_t>(b, (uint32_t)lay.pos_emit_groups.size());
      if (a >= b) return 0;
    } else {
      b = std::min<uint32_t>(b, (uint32_t)lay.work[e].size());
      if (a >= b) return 0;
    }
    PhaseScope ps(lay.work[e].empty() ? nullptr : T, slot, EMIT_PHASE[e], s);
    if (e != E_POS && (a != 0 || b != lay.work[e].size())) {  // a part of the work list
      HIPCHK(launch_emit(e, L, I->d_work[e] + a, b - a, K, bufs, B, lay.max_t, s));
      return 0;
    }
    if (e == E_POS) {  // E_POS: [a, b) are pos_emit_groups
      for (uint32_t gi = a; gi < std::min<uint32_t>(b, (uint32_t)lay.pos_emit_groups.size()); gi++) {
        const auto& g = lay.pos_emit_groups[gi];
        HIPCHK(launch_emit(e, L, I->d_work[e] + g[1], g[2], K, bufs, B, (int)g[0], s));
      }
    } else {
      HIPCHK(launch_emit(e, L, I->d_work[e], (uint32_t)lay.work[e].size(), K, bufs, B, lay.max_t, s));
    }
    return 0;
  };
  hipStream_t s_rsa = serial ? st : I->s_rsa, s_emit = serial ? st : I->s_emit,
              s_sha = serial ? st : I->s_sha2 && I->sha2_on && lay.is_register && (I->calls & 1) ? I->s_sha2 : I->s_sha,
              s_own = serial ? st : I->s_tail;
  if (d_status) HIPCHK(hipMemsetAsync(d_status, 0, sizeof(int32_t) * batch, st));
  { PhaseScope ps(T, slot, PH_LOAD, st);
    HIPCHK(launch_load_values(I->d_loads, (int)lay.loads.size(), d_inputs, lay.n_inputs, S.d_values, B, st)); }
  if (lay.is_query) {
    // QueryIdentity(80) (query.hpp): one chain on the call's chain stream — prep, the BabyJubJub key, Poseidon levels
    // 0-3 (sk hashes, nullifier, dg1 commitment, pk / position / value hashes), the SMT prep (needs the tree
    // position), levels 4-5 (the new-leaf hash and the level hashes above the insertion level), the SMT chain;
    // then the emitters on the two emitter streams (odd calls: the second emitter pair, qry_emit_pairs)
    if (!serial && I->s_sha2 && I->s_post && (I->calls & 1)) {
      s_sha = I->s_sha2;
      s_emit = I->s_post;
    }
    { PhaseScope ps(T, slot, PH_PREP, st); HIPCHK(launch_qry_prep(L, d_inputs, vs, d_status, st)); }
    { PhaseScope ps(T, slot, PH_BJJ_CORE, st);
      HIPCHK(launch_bjj_core(L, vs, I->d_bjj_table, S.d_bjj_core, S.d_bjj_scratch, st)); }
    HIPCHK(hipEventRecord(I->ev_bjj, st));
    HIPCHK(hipStreamWaitEvent(s_sha, I->ev_bjj, 0));
    if ((rc = emit(E_BJJ, s_sha))) return rc;
    { PhaseScope ps(T, slot, PH_POS_CORE, st); if ((rc = pos_levels(0, 4))) return rc; }
    { PhaseScope ps(T, slot, PH_SMT, st); HIPCHK(launch_smt_prep(L, d_inputs, vs, S.d_smt_core, d_status, st));
      HIPCHK(launch_smt_order(S.d_smt_core, L.smt_core_fr, S.d_smt_order, B, st)); }
    { PhaseScope ps(T, slot, PH_POS_CORE, st); if ((rc = pos_levels(4, 6, S.d_smt_order))) return rc; }
    // PZK_QRY_EMIT1=1: every emitter on one stream (with 3 chain streams that is 4 streams in use = the
    // hardware queues a process gets by default)
    static const bool emit1 = getenv("PZK_QRY_EMIT1") != nullptr;
    hipStream_t s_pe = emit1 ? s_sha : s_emit;
    // PZK_QRY_SPLIT=0|1 (A/B): what does not read the SMT chain — the Poseidon blocks before pos_chain_group, E_GEN's
    // regions before gen_chain_work, the query checks and the bit decompositions — is emitted before the chain, the
    // rest after it, as the register circuit's post-chain split does
    static const bool split = [] { const char* e = getenv("PZK_QRY_SPLIT"); return e ? atoi(e) != 0 : true; }();
    if (split) {
      HIPCHK(hipEventRecord(I->ev_pos, st));
      HIPCHK(hipStreamWaitEvent(s_pe, I->ev_pos, 0));
      if ((rc = emit(E_POS, s_pe, 0, lay.pos_chain_group))) return rc;
      HIPCHK(hipStreamWaitEvent(s_sha, I->ev_pos, 0));
      if ((rc = emit(E_QRY, s_sha))) return rc;
      if ((rc = emit(E_BITS, s_sha))) return rc;  // Num2Bits(254) of the tree position reads level 3
      if ((rc = emit(E_GEN, s_sha, 0, lay.gen_chain_work))) return rc;
    }
    { PhaseScope ps(T, slot, PH_SMT, st);
      HIPCHK(launch_smt_chain(L, K, I->d_level_task, d_inputs, vs, S.d_pos_core, S.d_smt_core, S.d_smt_order, d_status,
                              st)); }
    HIPCHK(hipEventRecord(I->ev_chain, st));
    HIPCHK(hipStreamWaitEvent(s_pe, I->ev_chain, 0));
    if ((rc = emit(E_POS, s_pe, split ? lay.pos_chain_group : 0))) return rc;
    HIPCHK(hipStreamWaitEvent(s_sha, I->ev_chain, 0));
    if ((rc = emit(E_GEN, s_sha, split ? lay.gen_chain_work : 0))) return rc;
    if (!split) {
      if ((rc = emit(E_QRY, s_sha))) return rc;
      if ((rc = emit(E_BITS, s_sha))) return rc;
    }
  } else if (!lay.is_register) {
    // standalone circuits: the core on the main stream; PoseidonHash(n)'s emitters on the emit stream behind it, so
    // call k's emitters run beside call k + 1's core (config 1 27.2M -> 28.7M witnesses/s); the SHA hashers' stay on
    // the main stream (config 2 200k serial vs 175k overlapped: the SHA core took 4x longer beside the emitter,
    // profiles/r5j). PZK_OVERLAP=0|1 forces one (A/B).
    static const char* ov_env = getenv("PZK_OVERLAP");
    const bool overlap = ov_env ? atoi(ov_env) != 0 : L.n_sha == 0;
    if (!overlap) s_emit = st;
    { PhaseScope ps(T, slot, PH_SHA_CORE, st);
      HIPCHK(launch_sha_core(L, d_inputs, S.d_derived, 0, L.n_sha, S.d_sha_core, d_status, B, st)); }
    { PhaseScope ps(T, slot, PH_POS_CORE, st); if ((rc = pos_levels(0, 1 << 20))) return rc; }
    if (s_emit != st) {
      HIPCHK(hipEventRecord(I->ev_pos, st));
      HIPCHK(hipStreamWaitEvent(s_emit, I->ev_pos, 0));
    }
    for (int e = 0; e < E_COUNT; e++)
      if ((rc = emit(e, s_emit))) return rc;
    s_rsa = s_sha = s_own = st;
  } else {
    // Four streams. The dependency chains get the high-priority streams: the
    // signature core (rsa) depends only on the inputs; the Poseidon/SMT/BabyJubJub chain (main)
    // on the SHA core. The emitters run on the two low-priority streams: the SHA emitters
    // (bandwidth-bound) on sha, everything else (the VALU-heavy BigMultModP / Poseidon emitters,
    // the small regions and the checks) on emit.
    HIPCHK(hipEventRecord(I->ev_load, st));
    HIPCHK(hipStreamWaitEvent(s_rsa, I->ev_load, 0));
    const bool pss = lay.reg.pss_s8 != 0;
    const uint32_t n_sha_main = pss ? (uint32_t)lay.reg.j_mgf : (uint32_t)lay.sha.size();
    if (!lay.is_ecdsa) {
      PhaseScope ps(T, slot, PH_RSA_CORE, s_rsa);
      HIPCHK(launch_rsa_core(L, d_inputs, S.d_rsa_core, S.d_rsa_colsum, d_status, B, s_rsa));
    }
    { PhaseScope ps(T, slot, PH_SHA_CORE, st);
      HIPCHK(launch_sha_core(L, d_inputs, S.d_derived, 0, n_sha_main, S.d_sha_core, d_status, B, st)); }
    HIPCHK(hipEventRecord(I->ev_sha, st));
    if (pss) {
      // RSA-PSS chain (pss.hpp) behind the RSA core: MGF1 messages from EM, their hashes, M' (needs
      // the SA digest), its hash. ev_rsa marks the chain's end: the PSS checks and regions read all of it.
      HIPCHK(hipStreamWaitEvent(s_rsa, I->ev_sha, 0));
      PhaseScope ps(T, slot, PH_PSS, s_rsa);
      HIPCHK(launch_pss(L, 0, S.d_rsa_core, S.d_sha_core, S.d_derived, B, s_rsa));
      HIPCHK(launch_sha_core(L, d_inputs, S.d_derived, (uint32_t)lay.reg.j_mgf, (uint32_t)lay.reg.n_mgf,
                             S.d_sha_core, d_status, B, s_rsa));
      HIPCHK(launch_pss(L, 1, S.d_rsa_core, S.d_sha_core, S.d_derived, B, s_rsa));
      HIPCHK(launch_sha_core(L, d_inputs, S.d_derived, (uint32_t)lay.reg.j_hd, 1, S.d_sha_core, d_status, B,
                             s_rsa));
    }
    if (lay.is_ecdsa) {
      // ECDSA chain (needs the SA digest): EC core, then the value tables of the table ops
      HIPCHK(hipStreamWaitEvent(s_rsa, I->ev_sha, 0));
      { PhaseScope ps(T, slot, PH_EC_CORE, s_rsa);
        HIPCHK(launch_ec_core(L, d_inputs, S.d_sha_core, S.d_ec_core, S.d_ec_jac, S.d_ec_inv, d_status, B, s_rsa)); }
    }
    HIPCHK(hipEventRecord(I->ev_rsa, s_rsa));
    if (lay.is_ecdsa) {
      { PhaseScope ps(T, slot, PH_EC_TABLE, s_rsa);
        for (int t = 0; t < 3; t++)
          HIPCHK(launch_ec_table(L, t, I->d_ec_ops[t], (uint32_t)lay.ec_ops[t].size(), S.d_ec_core, S.d_ec_tab,
                                 d_status, B, s_rsa)); }
      HIPCHK(hipEventRecord(I->ev_tab, s_rsa));
    }
    // SHA emitters (all hashers of the main SHA core)
    HIPCHK(hipStreamWaitEvent(s_sha, I->ev_sha, 0));
    if ((rc = emit(E_SHA, s_sha))) return rc;
    if ((rc = emit(E_SHA1, s_sha))) return rc;  // SHA-1 hashers (SIGNATURE_TYPE 3, DG_HASH_TYPE 160)
    if ((rc = emit(E_SHA5, s_sha))) return rc;  // SHA-384/512 hashers (standalone circuits)
    // signature emitters: BigMultModP blocks / EC table blocks, PSS derived hashers. RSA instances: on the
    // RSA stream right behind the chain they read, so they overlap the SHA emitters instead of queueing
    // behind the previous call's Poseidon emitters (config 3: 71.21k vs 70.75k witnesses/s). ECDSA
    // instances: on the emit stream, because there the next call's EC core (a long chain) would queue
    // behind this call's EC table emitter. Tuning switch PZK_SIGEMIT=rsa|emit forces one placement.
    static const char* se_env = getenv("PZK_SIGEMIT");
    const bool sig_on_rsa = se_env ? strcmp(se_env, "emit") != 0 : !lay.is_ecdsa;
    hipStream_t s_sig = I->s_mm && !serial ? I->s_mm : sig_on_rsa ? s_rsa : s_emit;
    HIPCHK(hipStreamWaitEvent(s_sig, I->ev_rsa, 0));
    if ((rc = emit(E_MM, s_sig))) return rc;
    if ((rc = emit(E_SHAD, s_sig))) return rc;
    if ((rc = emit(E_SHA5D, s_sig))) return rc;  // SHA-384 PSS hashers (SIGNATURE_TYPE 13)
    if (lay.is_ecdsa) {
      if ((rc = emit(E_ECR, s_sig))) return rc;  // the generator multiplication's selection tables (EC core only)
      HIPCHK(hipStreamWaitEvent(s_sig, I->ev_tab, 0));
      // the EC table blocks are ~60 % of an ECDSA witness: the first part on the signature stream, the rest on the
      // SHA emitter stream after this call's SHA emitters (PZK_ECT_SPLIT: the share of the elements there)
      if ((rc = emit(E_ECT, s_sig, 0, ect_split))) return rc;
    }
    // main chain
    { PhaseScope ps(T, slot, PH_PREP, st); HIPCHK(launch_prep(L, d_inputs, S.d_sha_core, vs, d_status, st)); }
    { PhaseScope ps(T, slot, PH_POS_CORE, st); if ((rc = pos_levels(0, 2))) return rc; }
    { PhaseScope ps(T, slot, PH_SMT, st); HIPCHK(launch_smt_prep(L, d_inputs, vs, S.d_smt_core, d_status, st));
      HIPCHK(launch_smt_order(S.d_smt_core, L.smt_core_fr, S.d_smt_order, B, st)); }
    { PhaseScope ps(T, slot, PH_POS_CORE, st); if ((rc = pos_levels(2, 3, S.d_smt_order))) return rc; }
    // The SMT chain (one dependent Poseidon permutation per proof level above the insertion level: ~0.5-1 ms per
    // level per call, so 25+ ms for the proof depths of a real registration tree) runs on its own stream (the fifth,
    // otherwise idle in register calls), so the next call's SHA core / prep / Poseidon / BabyJubJub chain does not
    // queue behind it; only the emitters that read its output (the SMT level images, the small SMT regions) wait.
    static const char* tail_env = getenv("PZK_TAIL");
    static const int tail_mode = !tail_env ? 2 : !strcmp(tail_env, "emit") ? 1 : !strcmp(tail_env, "sha") ? 0
                                 : !strcmp(tail_env, "rsa") ? 3 : !strcmp(tail_env, "own") ? 4 : 2;
    // PZK_SMT (A/B, profiles/r4_smt, r4_own): main = the chain on the main stream (rounds 1-3); own (default) = on
    // the fifth stream, the tail emitters placed by PZK_TAIL (78.8k / 52.1k witnesses/s at SMT depth 0 / 40-79);
    // tail = on the fifth stream with the tail emitters behind it there (76.8k / 47.3k)
    static const char* smt_env = getenv("PZK_SMT");
    static const int smt_mode = !smt_env ? 1 : !strcmp(smt_env, "main") ? 0 : !strcmp(smt_env, "tail") ? 2 : 1;
    // PZK_SMT_CHAINS=1..3 (A/B): consecutive calls' chains rotate over that many streams, so that many chains run
    // side by side (QueryIdentity's rotation, §11); r4_ect: 64.8k (2) vs 52.3k (1) at depth 40-79
    static const int smt_chains = getenv("PZK_SMT_CHAINS") ? atoi(getenv("PZK_SMT_CHAINS")) : 2;
    const hipStream_t chain_streams[3] = {I->s_tail, I->s_chain2, I->s_chain3};
    const int n_chain = smt_chains < 1 ? 1 : smt_chains >= 3 && I->s_chain3 ? 3 : smt_chains >= 2 ? 2 : 1;
    hipStream_t s_smt = (serial || tail_mode == 4 || smt_mode == 0) ? st : chain_streams[I->chain_rr++ % n_chain];
    if (s_smt != st) {
      HIPCHK(hipEventRecord(I->ev_smt, st));
      HIPCHK(hipStreamWaitEvent(s_smt, I->ev_smt, 0));
    }
    { PhaseScope ps(T, slot, PH_SMT, s_smt);
      HIPCHK(launch_smt_chain(L, K, I->d_level_task, d_inputs, vs, S.d_pos_core, S.d_smt_core, S.d_smt_order, d_status,
                              s_smt)); }
    HIPCHK(hipEventRecord(I->ev_chain, s_smt));
    { PhaseScope ps(T, slot, PH_BJJ_CORE, st);
      HIPCHK(launch_bjj_core(L, vs, I->d_bjj_table, S.d_bjj_core, S.d_bjj_scratch, st)); }
    HIPCHK(hipEventRecord(I->ev_bjj, st));
    { PhaseScope ps(T, slot, PH_POS_CORE, st); if ((rc = pos_levels(3, 1 << 20))) return rc; }
    HIPCHK(hipEventRecord(I->ev_pos, st));
    // BabyJubJub emitter behind the SHA emitters; of the chain's tail emitters, the Poseidon blocks go
    // behind the signature emitters and the small regions / flow / checks behind the SHA emitters
    // (default, "split": 70.7k vs 68.3k / 69.0k witnesses/s for all-on-sha / all-on-emit; "rsa", the tail on
    // the RSA stream, equals split; tuning switch PZK_TAIL=sha|emit|split|rsa, profiles/README.md)
    hipStream_t s_tail = tail_mode == 1 ? s_emit : tail_mode == 3 ? s_rsa : tail_mode == 4 ? s_own : s_sha,
                s_pos = tail_mode == 0 ? s_sha : s_emit, s_bjj = tail_mode == 4 ? s_own : s_sha;
    if (s_smt != st && smt_mode == 2) s_tail = s_smt;
    HIPCHK(hipStreamWaitEvent(s_bjj, I->ev_bjj, 0));
    if ((rc = emit(E_BJJ, s_bjj))) return rc;
    // The emission that reads the chain's output — the SMT level Poseidon blocks (pos_emit_groups from
    // pos_chain_group) and the SMT regions of E_GEN (work items from gen_chain_work) — goes to the post-chain stream
    // (s_post, one for all calls, so a later call's writes of those regions follow an earlier call's). The emitter
    // streams then never wait for the chain: with proofs of depth 1-79 (config 4) the chain of a 2048-witness call
    // takes 35-48 ms beside the emitters, longer than the call period, and every emitter queued behind a wait for it
    // idled (PZK_POST=0: the rounds 1-4 placement, everything behind the chain)
    const bool post = I->s_post && !serial && s_smt != st;
    const uint32_t pos_split = post ? lay.pos_chain_group : ~0u, gen_split = post ? lay.gen_chain_work : ~0u;
    HIPCHK(hipStreamWaitEvent(s_pos, I->ev_pos, 0));
    if (!post && s_smt != st && s_pos != s_smt) HIPCHK(hipStreamWaitEvent(s_pos, I->ev_chain, 0));  // SMT level images
    if ((rc = emit(E_POS, s_pos, 0, pos_split))) return rc;
    HIPCHK(hipStreamWaitEvent(s_tail, I->ev_pos, 0));
    HIPCHK(hipStreamWaitEvent(s_tail, I->ev_rsa, 0));
    if (!post && s_smt != st && s_tail != s_smt) HIPCHK(hipStreamWaitEvent(s_tail, I->ev_chain, 0));  // SMT regions
    if ((rc = emit(E_GEN, s_tail, 0, gen_split))) return rc;
    if (post) {
      HIPCHK(hipStreamWaitEvent(I->s_post, I->ev_pos, 0));
      HIPCHK(hipStreamWaitEvent(I->s_post, I->ev_chain, 0));
      if ((rc = emit(E_POS, I->s_post, pos_split))) return rc;
      if ((rc = emit(E_GEN, I->s_post, gen_split))) return rc;
    }
    if ((rc = emit(E_FLOW, s_tail))) return rc;
    if (!lay.is_ecdsa) {
      PhaseScope ps(T, slot, PH_PREP, s_tail);
      HIPCHK(launch_rsa_check(L, d_inputs, S.d_sha_core, S.d_rsa_core, d_status, B, s_tail));
    }
    if ((rc = emit(E_BITS, s_tail))) return rc;
    if ((rc = emit(E_GENR, s_tail))) return rc;
    if (lay.is_ecdsa && ect_split < lay.work[E_ECT].size()) {
      HIPCHK(hipStreamWaitEvent(s_sha, I->ev_tab, 0));
      if ((rc = emit(E_ECT, s_sha, ect_split))) return rc;
    }
  }
  auto or_st = [&](hipStream_t s) { return serial || !s ? st : s; };  // streams an instance does not have: st
  hipStream_t streams[pzk_instance::NSTREAMS] = {st, s_rsa, s_sha, s_emit, s_own, or_st(I->s_chain2),
                                                 or_st(I->s_chain3), or_st(I->s_post), or_st(I->s_mm), st};  // (s_sha2: in slot 2 when used)
  for (int i = 0; i < pzk_instance::NSTREAMS; i++) HIPCHK(hipEventRecord(I->ev_done[set][i], streams[i]));
  if (user) {
    for (hipEvent_t e : I->ev_done[set]) HIPCHK(hipStreamWaitEvent(user, e, 0));
  }
  if (exec && (exec->flags & PZK_EXEC_SYNC)) {
    if (user) HIPCHK(hipStreamSynchronize(user));
    else if ((rc = sync_all(I))) return rc;
  }
  return 0;
}

// With a non-monotone signal map: chunks of MAP_CHUNK witnesses, each through the O0 pipeline into d_o0[slot]
// (slot = chunk index & 1), then k_wtns_gather into the caller's rows on the main stream. The only guard of a
// slot is ev_gather[slot] (the gather two chunks back that read it): the main stream waits for it, and the
// chunk's call waits for the main stream (batch_locked's dep), whichever stream its chain runs on. The caller's
// stream is joined the same way (its inputs may still be in flight there).
static constexpr size_t MAP_CHUNK = 1024, MAP_CHUNK_MIN = 64;  // witnesses per O0 chunk (halved while it does not fit)
static int batch_mapped(pzk_instance* I, const uint8_t* d_inputs, size_t batch, uint8_t* d_wtns, size_t stride,
                        int32_t* d_status, const pzk_exec* exec) {
  const size_t o0_stride = 32ull * I->lay.wit_size;
  size_t chunk = std::min(batch, MAP_CHUNK);
  if (chunk > I->o0_cap) {  // the chains cost the same for any chunk size: take the largest that fits
    int rc = sync_all(I);  // the slots may still be read by an earlier call's gather
    if (rc) return rc;
    for (auto& p : I->d_o0) { if (p) (void)hipFree(p); p = nullptr; }
    I->o0_cap = 0;
    for (;;) {
      bool ok = true;
      for (auto& p : I->d_o0) ok = ok && hipMalloc(&p, o0_stride * chunk) == hipSuccess;
      if (ok) break;
      for (auto& p : I->d_o0) { if (p) (void)hipFree(p); p = nullptr; }
      (void)hipGetLastError();
      if (chunk <= MAP_CHUNK_MIN) return fail(PZK_E_NOMEM, "device O0 staging allocation failed");
      chunk /= 2;
    }
    I->o0_cap = chunk;
  }
  chunk = std::min(chunk, I->o0_cap);
  hipStream_t user = (exec && exec->stream) ? (hipStream_t)exec->stream : nullptr;
  if (user) {  // inputs may come from the caller's stream
    HIPCHK(hipEventRecord(I->ev_entry, user));
    HIPCHK(hipStreamWaitEvent(I->stream, I->ev_entry, 0));
  }
  pzk_exec ex{I->device, exec ? (exec->flags & PZK_EXEC_TIMING) : 0, nullptr};
  for (size_t lo = 0; lo < batch; lo += chunk) {
    const size_t n = std::min(chunk, batch - lo);
    const int set = (int)(I->calls % I->nsets), slot = (int)((lo / chunk) & 1);
    HIPCHK(hipStreamWaitEvent(I->stream, I->ev_gather[slot], 0));  // the gather two chunks back read this slot
    int rc = batch_locked(I, d_inputs + 32ull * I->lay.n_inputs * lo, n, I->d_o0[slot], o0_stride,
                          d_status ? d_status + lo : nullptr, &ex, I->stream);
    if (rc) return rc;
    for (int i = 0; i < pzk_instance::NSTREAMS; i++) HIPCHK(hipStreamWaitEvent(I->stream, I->ev_done[set][i], 0));
    HIPCHK(launch_wtns_gather(I->d_o0[slot], o0_stride, I->d_map, I->out_size, d_wtns + stride * lo, stride, (uint32_t)n,
                              I->stream));
    HIPCHK(hipEventRecord(I->ev_done[set][0], I->stream));
    HIPCHK(hipEventRecord(I->ev_gather[slot], I->stream));
  }
  if (user)
    for (auto& set : I->ev_done)
      for (hipEvent_t e : set) HIPCHK(hipStreamWaitEvent(user, e, 0));
  if (exec && (exec->flags & PZK_EXEC_SYNC)) {
    if (user) HIPCHK(hipStreamSynchronize(user));
    else return sync_all(I);
  }
  return 0;
}

static int pzk_witness_batch_impl(pzk_instance* I, const uint8_t* d_inputs, size_t batch, uint8_t* d_wtns, size_t stride,
                      int32_t* d_status, const pzk_exec* exec) {
  if (!I || !d_inputs || !d_wtns) return fail(PZK_E_ARG, "null argument");
  if (batch == 0) return 0;
  if (batch > 65535) return fail(PZK_E_ARG, "batch > 65535: split it");
  if (stride < 32ull * I->out_size || stride % 16) return fail(PZK_E_ARG, "bad witness stride");
  int rc = check_exec_device(I, exec);
  if (rc) return rc;
  std::lock_guard<std::mutex> lock(I->mu);
  DeviceGuard dg(I->device);
  if (dg.err != hipSuccess) return fail(PZK_E_HIP, std::string("hipSetDevice: ") + hipGetErrorString(dg.err));
  if (I->d_map) return batch_mapped(I, d_inputs, batch, d_wtns, stride, d_status, exec);
  return batch_locked(I, d_inputs, batch, d_wtns, stride, d_status, exec);  // O0, or a monotone map emitted directly
}

static int pzk_instance_sync_impl(pzk_instance* I) {
  if (!I) return fail(PZK_E_ARG, "null argument");
  std::lock_guard<std::mutex> lock(I->mu);
  DeviceGuard dg(I->device);
  if (dg.err != hipSuccess) return fail(PZK_E_HIP, std::string("hipSetDevice: ") + hipGetErrorString(dg.err));
  return sync_all(I);
}

static int pzk_witness_batch_host_impl(pzk_instance* I, const uint8_t* h_inputs, size_t batch, uint8_t* h_wtns,
                           int32_t* h_status, const pzk_exec* exec) {
  if (!I || !h_inputs || !h_wtns) return fail(PZK_E_ARG, "null argument");
  if (batch == 0) return 0;
  if (batch > 65535) return fail(PZK_E_ARG, "batch > 65535: split it");
  int rc = check_exec_device(I, exec);
  if (rc) return rc;
  std::lock_guard<std::mutex> lock(I->mu);
  DeviceGuard dg(I->device);
  if (dg.err != hipSuccess) return fail(PZK_E_HIP, std::string("hipSetDevice: ") + hipGetErrorString(dg.err));
  size_t in_bytes = 32ull * I->lay.n_inputs * batch, out_bytes = 32ull * I->out_size * batch;
  // the staging buffers may still be read/written by an earlier device call: drain before reuse
  if ((rc = sync_all(I))) return rc;
  if (batch > I->host_cap) {
    if (I->d_in) (void)hipFree(I->d_in);
    if (I->d_out) (void)hipFree(I->d_out);
    if (I->d_status) (void)hipFree(I->d_status);
    I->d_in = I->d_out = nullptr; I->d_status = nullptr; I->host_cap = 0;
    HIPCHK(hipMalloc(&I->d_in, in_bytes));
    HIPCHK(hipMalloc(&I->d_out, out_bytes));
    HIPCHK(hipMalloc(&I->d_status, 4 * batch));
    I->host_cap = batch;
  }
  hipStream_t st = I->stream;
  HIPCHK(hipMemcpyAsync(I->d_in, h_inputs, in_bytes, hipMemcpyHostToDevice, st));
  pzk_exec ex{I->device, exec ? (exec->flags & PZK_EXEC_TIMING) : 0, nullptr};
  // the upload is on the main stream: batch_mapped orders every chunk after it, batch_locked via dep
  rc = I->d_map ? batch_mapped(I, I->d_in, batch, I->d_out, 32ull * I->out_size, I->d_status, &ex)
                : batch_locked(I, I->d_in, batch, I->d_out, 32ull * I->out_size, I->d_status, &ex, st);
  if (rc) return rc;
  if ((rc = sync_all(I))) return rc;
  HIPCHK(hipMemcpy(h_wtns, I->d_out, out_bytes, hipMemcpyDeviceToHost));
  if (h_status) HIPCHK(hipMemcpy(h_status, I->d_status, 4 * batch, hipMemcpyDeviceToHost));
  return 0;
}

// Streamed delivery: chunk c's inputs go up and its witnesses are computed on s_in (the
// call joined into it), then copied down on s_d2h into pinned slot c % 2 while chunk c + 1 computes; the
// calling thread hands chunk c - 1's pinned rows to the sink meanwhile. Chunk c + 2 reuses slot c % 2:
// its upload waits for the device->host copy of chunk c (ev_d2h), and its copy down is issued only after
// the sink of chunk c has returned.
static int pzk_witness_stream_impl(pzk_instance* I, const uint8_t* h_inputs, size_t batch, size_t chunk, pzk_sink_fn sink,
                       void* user, const pzk_exec* exec) {
  if (!I || !h_inputs || !sink) return fail(PZK_E_ARG, "null argument");
  if (batch == 0) return 0;
  int rc = check_exec_device(I, exec);
  if (rc) return rc;
  std::lock_guard<std::mutex> lock(I->mu);
  DeviceGuard dg(I->device);
  if (dg.err != hipSuccess) return fail(PZK_E_HIP, std::string("hipSetDevice: ") + hipGetErrorString(dg.err));
  const size_t in_row = 32ull * I->lay.n_inputs, out_row = 32ull * I->out_size;
  // default: ~4 GiB of rows per chunk, so a chunk's compute (whose chains cost the same for few witnesses
  // as for many) stays short against its device->host copy also for small (mapped) rows
  if (chunk == 0) chunk = std::max<size_t>(1, (size_t(4) << 30) / out_row);
  chunk = std::min({chunk, batch, size_t(65535)});
  if ((rc = sync_all(I))) return rc;
  if (!I->s_in) {
    bool ok = hipStreamCreateWithFlags(&I->s_in, hipStreamNonBlocking) == hipSuccess &&
              hipStreamCreateWithFlags(&I->s_d2h, hipStreamNonBlocking) == hipSuccess;
    for (int k = 0; k < 2 && ok; k++)
      ok = hipEventCreateWithFlags(&I->ev_comp[k], hipEventDisableTiming) == hipSuccess &&
           hipEventCreateWithFlags(&I->ev_d2h[k], hipEventDisableTiming) == hipSuccess;
    if (!ok) return fail(PZK_E_HIP, "stream / event creation failed");
  }
  if (chunk > I->st_cap) {
    free_stream_bufs(I);
    for (int k = 0; k < 2; k++) {
      if (hipMalloc(&I->st_din[k], in_row * chunk) != hipSuccess || hipMalloc(&I->st_dout[k], out_row * chunk) != hipSuccess ||
          hipMalloc(&I->st_dst[k], 4 * chunk) != hipSuccess ||
          hipHostMalloc(&I->st_hout[k], out_row * chunk, hipHostMallocDefault) != hipSuccess ||
          hipHostMalloc(&I->st_hst[k], 4 * chunk, hipHostMallocDefault) != hipSuccess) {
        free_stream_bufs(I);
        (void)hipGetLastError();
        return fail(PZK_E_NOMEM, "stream buffers (device rows or pinned host rows) could not be allocated");
      }
    }
    I->st_cap = chunk;
  }
  const size_t n_chunks = (batch + chunk - 1) / chunk;
  pzk_exec ex{I->device, exec ? (exec->flags & PZK_EXEC_TIMING) : 0, I->s_in};
  auto deliver = [&](size_t c) -> int {
    const int k = (int)(c & 1);
    const size_t first = c * chunk, n = std::min(chunk, batch - first);
    HIPCHK(hipEventSynchronize(I->ev_d2h[k]));
    if (sink(user, first, n, I->st_hout[k], out_row, I->st_hst[k]) != 0)
      return fail(PZK_E_ARG, "the sink returned non-zero for chunk at " + std::to_string(first));
    return 0;
  };
  for (size_t c = 0; c < n_chunks; c++) {
    const int k = (int)(c & 1);
    const size_t first = c * chunk, n = std::min(chunk, batch - first);
    HIPCHK(hipStreamWaitEvent(I->s_in, I->ev_d2h[k], 0));  // chunk c - 2's rows have left slot k
    HIPCHK(hipMemcpyAsync(I->st_din[k], h_inputs + in_row * first, in_row * n, hipMemcpyHostToDevice, I->s_in));
    rc = I->d_map ? batch_mapped(I, I->st_din[k], n, I->st_dout[k], out_row, I->st_dst[k], &ex)
                  : batch_locked(I, I->st_din[k], n, I->st_dout[k], out_row, I->st_dst[k], &ex);
    if (rc) return rc;
    HIPCHK(hipEventRecord(I->ev_comp[k], I->s_in));
    if (c > 0 && (rc = deliver(c - 1))) return rc;  // chunk c - 1 to the sink while chunk c computes
    HIPCHK(hipStreamWaitEvent(I->s_d2h, I->ev_comp[k], 0));
    HIPCHK(hipMemcpyAsync(I->st_hout[k], I->st_dout[k], out_row * n, hipMemcpyDeviceToHost, I->s_d2h));
    HIPCHK(hipMemcpyAsync(I->st_hst[k], I->st_dst[k], 4 * n, hipMemcpyDeviceToHost, I->s_d2h));
    HIPCHK(hipEventRecord(I->ev_d2h[k], I->s_d2h));
  }
  return deliver(n_chunks - 1);
}

static int pzk_timing_impl(pzk_instance* I, const char** names, double* ms, uint64_t* launches, uint32_t* count, int reset) {
  if (!I || !count) return fail(PZK_E_ARG, "null argument");
  for (int s = 0; s < Timing::RING; s++) I->timing.collect(s);
  uint32_t n = std::min<uint32_t>(*count, PH_COUNT);
  for (uint32_t p = 0; p < n; p++) {
    if (names) names[p] = PHASE_NAMES[p];
    if (ms) ms[p] = I->timing.ms[p];
    if (launches) launches[p] = I->timing.n[p];
  }
  *count = PH_COUNT;
  if (reset) {
    memset(I->timing.ms, 0, sizeof I->timing.ms);
    memset(I->timing.n, 0, sizeof I->timing.n);
  }
  return 0;
}

static int pzk_phase_info_impl(const pzk_instance* I, uint32_t phase, const char** name, const char** kernel,
                   uint64_t* bytes_per_witness) {
  if (!I || phase >= PH_COUNT) return fail(PZK_E_ARG, "bad phase");
  if (name) *name = PHASE_NAMES[phase];
  if (kernel) {
    *kernel = PHASE_KERNELS[phase];
    if (phase == PH_PREP && I->lay.is_query) *kernel = "k_qry_prep";
    if (phase == PH_EMIT_SHA) {  // the SHA-2 and SHA-1 emitters share the phase: name the ones this instance runs
      const bool s2 = !I->lay.work[E_SHA].empty() || !I->lay.work[E_SHAD].empty(), s1 = !I->lay.work[E_SHA1].empty();
      const bool s5 = !I->lay.work[E_SHA5].empty() || !I->lay.work[E_SHA5D].empty();
      *kernel = s5 ? (s2 ? "k_emit_sha+k_emit_sha512" : "k_emit_sha512")
                   : s1 ? (s2 ? "k_emit_sha+k_emit_sha1" : "k_emit_sha1") : "k_emit_sha";
    }
  }
  if (bytes_per_witness) {
    // ALGORITHMIC HBM bytes per witness: every witness element the phase writes (32 B) + the
    // unique bytes it must read (input elements copied, core state it expands)
    const Layout& L = I->lay;
    uint64_t b = 0;
    for (const Region& r : L.regions) {
      if (EMIT_PHASE[emitter_of(r.kind)] != (int)phase) continue;
      b += 32ull * I->kept_in(r.off, r.len);  // the elements the phase writes (a .sym map: the kept ones)
      if (r.kind == RK_SHA_OWN) b += 32ull * 512 * r.a[1] * (r.a[3] ? 2 : 1);  // message bits copied
      if (r.kind == RK_SHA_BLOCK) b += 4ull * SHA_BLOCK_CORE;
      if (r.kind == RK_SHA1_OWN) b += 32ull * 512 * r.a[1];  // message bits copied
      if (r.kind == RK_SHA1_BLOCK) b += 4ull * SHA1_BLOCK_CORE;
      if (r.kind == RK_SHA5_OWN) b += 32ull * 1024 * r.a[1] * (r.a[4] ? 2 : 1);  // message bits copied
      if (r.kind == RK_SHA5_BLOCK) b += 4ull * SHA5_BLOCK_CORE;
      if (r.kind == RK_INCOPY) b += 32ull * r.len;
      if (r.kind == RK_POSEIDON) b += 32ull * pos_core_len(r.a[1] + 1);
      if (r.kind == RK_MODMUL) b += 8ull * MM_CORE_WORDS(L.reg.K);
      if (r.kind == RK_FLOW) {  // the encapsulated content and signed attributes bits it copies (and compares)
        const ShaJob& je = L.sha[r.a[2]];
        b += 32ull * ((je.algo >= 3 ? 1024 : 512) * (uint64_t)je.blocks + 1024);
      }
    }
    if (phase == PH_SHA_CORE)
      for (const ShaJob& j : L.sha)
        b += j.algo >= 3 ? 32ull * 1024 * j.blocks + 4ull * (j.blocks * SHA5_BLOCK_CORE + 32)
                         : 32ull * 512 * j.blocks + 4ull * (j.blocks * (j.algo == 1 ? SHA1_BLOCK_CORE : SHA_BLOCK_CORE) + 8);
    if (phase == PH_POS_CORE)  // the round states written (not the line padding between task slices)
      for (const PosTask& t : L.pos) b += 32ull * pos_core_len(t.n + 1);
    if (phase == PH_PREP && L.is_register) {  // k_prep: the input elements it reads (one 32-byte
      const RegInfo& G = L.reg;                                     // element per key / DG1 bit) + the SA digest
      uint64_t el = G.ecdsa ? 2ull * G.ec_nl : 15;
      if (G.aa && G.aa_ec) el += 2ull * G.aa_hs;
      else if (G.aa) el += 4 * 200 + 224;
      b += 32ull * (el + 4ull * G.dg1_chunk) + 32;
    }
    if (phase == PH_PREP && L.is_query)  // k_qry_prep: the DG1 bits and the scalar inputs it reads (QI_EVID ..
      b += 32ull * (q_dg1_len(L.reg.q_td1) + QI_DG1) +  // QI_PKPASS) + the value slots written: DG1 fields, dg1
           32ull * (9 + 4 + 1 + 240);                   // chunks, citizenship index and its 240 IsEqual inverses
    if (phase == PH_SMT && (L.is_register || L.is_query))  // siblings, root and key read; SMT core and the
      b += 32ull * (SMT_LEVELS + 2) + 32ull * SMT_CORE_FR + 32ull * 2 * SMT_LEVELS;  // level hash inputs written
    if (phase == PH_RSA_CORE)  // core written + signature and modulus read; k_rsa_inv reads every remainder and the
      b += 8ull * L.rsa_core_words + 32ull * 2 * L.reg.K + 8ull * L.reg.n_modmul * L.reg.K + 32ull * L.reg.K;  // modulus
    if (phase == PH_BJJ_CORE) b += 32ull * L.bjj_core_fr;
    if (phase == PH_LOAD) b += 64ull * L.loads.size();
    *bytes_per_witness = b;
  }
  return 0;
}


// ------------------------------------------------------------------ C-ABI entry points (guarded)
int pzk_instance_create(const pzk_params* params, pzk_instance** out) {
  return guarded([&] { return pzk_instance_create_impl(params, out); });
}

int pzk_instance_create_mapped(const pzk_params* params, const char* sym, size_t sym_len, pzk_instance** out) {
  return guarded([&] { return pzk_instance_create_mapped_impl(params, sym, sym_len, out); });
}

void pzk_instance_destroy(pzk_instance* inst) {
  (void)guarded([&] { pzk_instance_destroy_impl(inst); return 0; });
}

int pzk_instance_info(const pzk_instance* I, pzk_info* info) {
  return guarded([&] { return pzk_instance_info_impl(I, info); });
}

int pzk_instance_input(const pzk_instance* I, uint32_t i, const char** name, uint64_t* offset, uint64_t* length) {
  return guarded([&] { return pzk_instance_input_impl(I, i, name, offset, length); });
}

int pzk_wtns_header(const pzk_instance* I, uint8_t h[76]) {
  return guarded([&] { return pzk_wtns_header_impl(I, h); });
}

int pzk_witness_batch(pzk_instance* I, const uint8_t* d_inputs, size_t batch, uint8_t* d_wtns, size_t stride,
                      int32_t* d_status, const pzk_exec* exec) {
  return guarded([&] { return pzk_witness_batch_impl(I, d_inputs, batch, d_wtns, stride, d_status, exec); });
}

int pzk_instance_sync(pzk_instance* I) {
  return guarded([&] { return pzk_instance_sync_impl(I); });
}

int pzk_witness_batch_host(pzk_instance* I, const uint8_t* h_inputs, size_t batch, uint8_t* h_wtns,
                           int32_t* h_status, const pzk_exec* exec) {
  return guarded([&] { return pzk_witness_batch_host_impl(I, h_inputs, batch, h_wtns, h_status, exec); });
}

int pzk_witness_stream(pzk_instance* I, const uint8_t* h_inputs, size_t batch, size_t chunk, pzk_sink_fn sink,
                       void* user, const pzk_exec* exec) {
  return guarded([&] { return pzk_witness_stream_impl(I, h_inputs, batch, chunk, sink, user, exec); });
}

int pzk_timing(pzk_instance* I, const char** names, double* ms, uint64_t* launches, uint32_t* count, int reset) {
  return guarded([&] { return pzk_timing_impl(I, names, ms, launches, count, reset); });
}

int pzk_phase_info(const pzk_instance* I, uint32_t phase, const char** name, const char** kernel,
                   uint64_t* bytes_per_witness) {
  return guarded([&] { return pzk_phase_info_impl(I, phase, name, kernel, bytes_per_witness); });
}

}  // extern "C"
