// Host runtime + C-ABI (include/pzkwit.h): instance layout, device buffers, launch order.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../../include/pzkwit.h"
#include "builder.hpp"
#include "kernels.hpp"
#include "poseidon.hpp"

using namespace pzk;

static thread_local std::string g_err;
static int fail(int code, const std::string& msg) { g_err = msg; return code; }
#define HIPCHK(x)                                                                              \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) return fail(PZK_E_HIP, std::string(#x ": ") + hipGetErrorString(e_)); \
  } while (0)

struct pzk_instance {
  pzk_params params;
  Layout lay;            // host layout (builder.hpp)
  int device = 0;
  hipStream_t stream = nullptr;
  // device copies of the layout
  Region* d_regions = nullptr;
  Work *d_work_sha = nullptr, *d_work_pos = nullptr, *d_work_gen = nullptr;
  ShaJob* d_sha = nullptr;
  PosTask* d_pos = nullptr;
  ValueLoad* d_loads = nullptr;
  fr* d_pos_consts = nullptr;
  PosParamIndex pix{};
  // per-batch scratch, grown on demand
  size_t cap = 0;
  uint32_t* d_sha_core = nullptr;
  fr* d_pos_core = nullptr;
  fr* d_values = nullptr;
  // staging for the host-buffer path
  size_t host_cap = 0;
  uint8_t *d_in = nullptr, *d_out = nullptr;
  int32_t* d_status = nullptr;
  DevLayout dev_layout() const {
    DevLayout L{};
    L.wit_size = lay.wit_size;
    L.n_inputs = lay.n_inputs;
    L.n_regions = (uint32_t)lay.regions.size();
    L.n_sha = (uint32_t)lay.sha.size();
    L.sha_core_words = lay.sha_core_words;
    L.n_pos = (uint32_t)lay.pos.size();
    L.pos_core_elems = lay.pos_core_elems;
    L.n_values = lay.n_values;
    L.n_pos_levels = (uint32_t)lay.pos_level_start.size() - 1;
    L.regions = d_regions;
    L.sha = d_sha;
    L.pos = d_pos;
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
  HIPCHK(hipMalloc(&I->d_pos_consts, consts.size()));
  HIPCHK(hipMemcpy(I->d_pos_consts, consts.data(), consts.size(), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_to_mont_inplace, dim3((n + 255) / 256), dim3(256), 0, 0, I->d_pos_consts, n);
  HIPCHK(hipGetLastError());
  HIPCHK(hipDeviceSynchronize());
  return 0;
}

template <typename T>
static int upload(T** dst, const std::vector<T>& v) {
  if (v.empty()) { *dst = nullptr; return 0; }
  HIPCHK(hipMalloc(dst, sizeof(T) * v.size()));
  HIPCHK(hipMemcpy(*dst, v.data(), sizeof(T) * v.size(), hipMemcpyHostToDevice));
  return 0;
}

static void free_all(pzk_instance* I) {
  void* ptrs[] = {I->d_regions, I->d_work_sha, I->d_work_pos, I->d_work_gen, I->d_sha, I->d_pos, I->d_loads,
                  I->d_pos_consts, I->d_sha_core, I->d_pos_core, I->d_values, I->d_in, I->d_out, I->d_status};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  if (I->stream) (void)hipStreamDestroy(I->stream);
}

extern "C" {

const char* pzk_last_error(void) { return g_err.c_str(); }
const char* pzk_version(void) { return "pzkwit 0.1.0 (gfx950)"; }

int pzk_instance_create(const pzk_params* params, pzk_instance** out) {
  if (!params || !out) return fail(PZK_E_ARG, "null argument");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    return fail(PZK_E_NODEVICE, "no HIP device visible: pzkwit has no CPU fallback");
  pzk_instance* I = new pzk_instance();
  I->params = *params;
  std::string why;
  if (!build_layout(*params, I->lay, why)) { delete I; return fail(PZK_E_PARAMS, why); }
  HIPCHK(hipGetDevice(&I->device));
  int rc;
  if ((rc = load_poseidon(I)) != 0) { free_all(I); delete I; return rc; }
  if ((rc = upload(&I->d_regions, I->lay.regions)) || (rc = upload(&I->d_work_sha, I->lay.work_sha)) ||
      (rc = upload(&I->d_work_pos, I->lay.work_pos)) || (rc = upload(&I->d_work_gen, I->lay.work_gen)) ||
      (rc = upload(&I->d_sha, I->lay.sha)) || (rc = upload(&I->d_pos, I->lay.pos)) ||
      (rc = upload(&I->d_loads, I->lay.loads))) {
    free_all(I); delete I; return rc;
  }
  if (hipStreamCreateWithFlags(&I->stream, hipStreamNonBlocking) != hipSuccess) {
    free_all(I); delete I; return fail(PZK_E_HIP, "hipStreamCreate failed");
  }
  *out = I;
  return 0;
}

void pzk_instance_destroy(pzk_instance* inst) {
  if (!inst) return;
  free_all(inst);
  delete inst;
}

int pzk_instance_info(const pzk_instance* I, pzk_info* info) {
  if (!I || !info) return fail(PZK_E_ARG, "null argument");
  memset(info, 0, sizeof *info);
  info->witness_size = I->lay.wit_size;
  info->n_inputs = I->lay.n_inputs;
  info->n_outputs = I->lay.n_outputs;
  info->n_public_inputs = I->lay.n_public;
  info->n_input_groups = (uint32_t)I->lay.inputs.size();
  return 0;
}

int pzk_instance_input(const pzk_instance* I, uint32_t i, const char** name, uint64_t* offset, uint64_t* length) {
  if (!I || i >= I->lay.inputs.size()) return fail(PZK_E_ARG, "input index out of range");
  if (name) *name = I->lay.inputs[i].name.c_str();
  if (offset) *offset = I->lay.inputs[i].offset;
  if (length) *length = I->lay.inputs[i].length;
  return 0;
}

int pzk_wtns_header(const pzk_instance* I, uint8_t h[76]) {
  if (!I || !h) return fail(PZK_E_ARG, "null argument");
  static const uint8_t prime[32] = {0x01, 0x00, 0x00, 0xf0, 0x93, 0xf5, 0xe1, 0x43, 0x91, 0x70, 0xb9,
                                    0x79, 0x48, 0xe8, 0x33, 0x28, 0x5d, 0x58, 0x81, 0x81, 0xb6, 0x45,
                                    0x50, 0xb8, 0x29, 0xa0, 0x31, 0xe1, 0x72, 0x4e, 0x64, 0x30};
  uint8_t* p = h;
  auto u32 = [&](uint32_t v) { memcpy(p, &v, 4); p += 4; };
  auto u64 = [&](uint64_t v) { memcpy(p, &v, 8); p += 8; };
  memcpy(p, "wtns", 4); p += 4;
  u32(2); u32(2);
  u32(1); u64(40); u32(32); memcpy(p, prime, 32); p += 32; u32((uint32_t)I->lay.wit_size);
  u32(2); u64(32ull * I->lay.wit_size);
  return 0;
}

static int ensure_scratch(pzk_instance* I, size_t batch) {
  if (batch <= I->cap) return 0;
  if (I->d_sha_core) (void)hipFree(I->d_sha_core);
  if (I->d_pos_core) (void)hipFree(I->d_pos_core);
  if (I->d_values) (void)hipFree(I->d_values);
  I->d_sha_core = nullptr; I->d_pos_core = nullptr; I->d_values = nullptr;
  size_t sha = 4ull * I->lay.sha_core_words * batch, pos = 32ull * I->lay.pos_core_elems * batch,
         val = 32ull * std::max<uint32_t>(I->lay.n_values, 1) * batch;
  if ((sha && hipMalloc(&I->d_sha_core, sha) != hipSuccess) || (pos && hipMalloc(&I->d_pos_core, pos) != hipSuccess) ||
      hipMalloc(&I->d_values, val) != hipSuccess) {
    I->cap = 0;
    return fail(PZK_E_NOMEM, "device scratch allocation failed");
  }
  I->cap = batch;
  return 0;
}

int pzk_witness_batch(pzk_instance* I, const uint8_t* d_inputs, size_t batch, uint8_t* d_wtns, size_t stride,
                      int32_t* d_status, const pzk_exec* exec) {
  if (!I || !d_inputs || !d_wtns) return fail(PZK_E_ARG, "null argument");
  if (batch == 0) return 0;
  if (batch > 65535) return fail(PZK_E_ARG, "batch > 65535: split it");
  if (stride < 32ull * I->lay.wit_size || stride % 16) return fail(PZK_E_ARG, "bad witness stride");
  if (exec && exec->device != I->device) HIPCHK(hipSetDevice(exec->device));
  int rc = ensure_scratch(I, batch);
  if (rc) return rc;
  hipStream_t st = (exec && exec->stream) ? (hipStream_t)exec->stream : I->stream;
  const uint32_t B = (uint32_t)batch;
  DevLayout L = I->dev_layout();
  ValueStore vs{I->d_values, B};
  PosConsts K{I->d_pos_consts, I->pix};
  if (d_status) HIPCHK(hipMemsetAsync(d_status, 0, sizeof(int32_t) * batch, st));
  HIPCHK(launch_load_values(I->d_loads, (int)I->lay.loads.size(), d_inputs, I->lay.n_inputs, I->d_values, B, st));
  HIPCHK(launch_sha_core(L, d_inputs, I->d_sha_core, d_status, B, st));
  for (size_t l = 0; l + 1 < I->lay.pos_level_start.size(); l++) {
    uint32_t a = I->lay.pos_level_start[l], b = I->lay.pos_level_start[l + 1];
    HIPCHK(launch_pos_core(K, I->d_pos, I->lay.pos.data(), a, b - a, vs, I->d_pos_core, I->lay.pos_core_elems, st));
  }
  HIPCHK(launch_emit_gen(L, I->d_work_gen, (uint32_t)I->lay.work_gen.size(), d_inputs, vs, d_wtns, stride, B, st));
  HIPCHK(launch_emit_sha(L, I->d_work_sha, (uint32_t)I->lay.work_sha.size(), d_inputs, I->d_sha_core, d_wtns, stride,
                         B, st));
  HIPCHK(launch_emit_pos(L, I->d_work_pos, (uint32_t)I->lay.work_pos.size(), K, vs, I->d_pos_core, d_wtns, stride, B,
                         I->lay.max_t, st));
  if (exec && (exec->flags & PZK_EXEC_SYNC)) HIPCHK(hipStreamSynchronize(st));
  return 0;
}

int pzk_witness_batch_host(pzk_instance* I, const uint8_t* h_inputs, size_t batch, uint8_t* h_wtns,
                           int32_t* h_status, const pzk_exec* exec) {
  if (!I || !h_inputs || !h_wtns) return fail(PZK_E_ARG, "null argument");
  if (batch == 0) return 0;
  size_t in_bytes = 32ull * I->lay.n_inputs * batch, out_bytes = 32ull * I->lay.wit_size * batch;
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
  hipStream_t st = (exec && exec->stream) ? (hipStream_t)exec->stream : I->stream;
  HIPCHK(hipMemcpyAsync(I->d_in, h_inputs, in_bytes, hipMemcpyHostToDevice, st));
  pzk_exec ex{I->device, 0, st};
  int rc = pzk_witness_batch(I, I->d_in, batch, I->d_out, 32ull * I->lay.wit_size, I->d_status, &ex);
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(h_wtns, I->d_out, out_bytes, hipMemcpyDeviceToHost, st));
  if (h_status) HIPCHK(hipMemcpyAsync(h_status, I->d_status, 4 * batch, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  return 0;
}

}  // extern "C"
