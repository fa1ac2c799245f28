/* pzkwit_napi.c — Node N-API addon over the libpzkwit C-ABI (include/pzkwit.h).
 *
 * The JS host the reference's callers use (test/automatisationTest.js:37-51 via circom_tester,
 * circuits/scripts/gen-witness.sh:25 via generate_witness.js) talks to a witness calculator
 * object; witness_calculator.js in this directory rebuilds that object on top of these
 * primitives:
 *
 *   version()                              -> string
 *   createInstance(params)                 -> handle (napi external; destroyed by the GC)
 *   instanceInfo(handle)                   -> { witnessSize, nInputs, nOutputs, nPublicInputs,
 *                                               inputs: [{ name, offset, length }] }
 *   wtnsHeader(handle)                     -> Buffer(76)
 *   witnessBatch(handle, inputs, batch)    -> Promise<{ witness: Buffer, status: Int32Array }>
 *        inputs: Buffer of batch x nInputs x 32 B (LE normal form); runs pzk_witness_batch_host
 *        on a libuv worker thread (napi_create_async_work), so the event loop stays free.
 *
 * Errors: a failing pzk_* call throws (or rejects with) an Error carrying pzk_last_error().
 * N-API version 4 features only (Node >= 10.16 / 12.x).
 */
#define NAPI_VERSION 4
#include <node_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/pzkwit.h"

#define CHECK(call)                                                         \
  do {                                                                      \
    if ((call) != napi_ok) {                                                \
      napi_throw_error(env, NULL, "pzkwit N-API call failed: " #call);      \
      return NULL;                                                          \
    }                                                                       \
  } while (0)

static napi_value throw_pzk(napi_env env, const char* what) {
  char msg[512];
  snprintf(msg, sizeof msg, "%s: %s", what, pzk_last_error());
  napi_throw_error(env, NULL, msg);
  return NULL;
}

static void finalize_instance(napi_env env, void* data, void* hint) {
  (void)env; (void)hint;
  pzk_instance_destroy((pzk_instance*)data);
}

static pzk_instance* get_instance(napi_env env, napi_value v) {
  void* p = NULL;
  if (napi_get_value_external(env, v, &p) != napi_ok || !p) {
    napi_throw_type_error(env, NULL, "expected a pzkwit instance handle");
    return NULL;
  }
  return (pzk_instance*)p;
}

static int32_t get_i32_prop(napi_env env, napi_value obj, const char* key, int32_t dflt) {
  bool has = false;
  napi_value v;
  int32_t out = dflt;
  if (napi_has_named_property(env, obj, key, &has) != napi_ok || !has) return dflt;
  if (napi_get_named_property(env, obj, key, &v) != napi_ok) return dflt;
  if (napi_get_value_int32(env, v, &out) != napi_ok) return dflt;
  return out;
}

static napi_value js_version(napi_env env, napi_callback_info info) {
  (void)info;
  napi_value s;
  CHECK(napi_create_string_utf8(env, pzk_version(), NAPI_AUTO_LENGTH, &s));
  return s;
}

/* params: { circuit, sizeArg, SIGNATURE_TYPE, DG_HASH_TYPE, DOCUMENT_TYPE, EC_BLOCK_NUMBER, EC_SHIFT,
 *           DG1_SHIFT, AA_SIGNATURE_ALGO, DG15_SHIFT, DG15_BLOCK_NUMBER, AA_SHIFT } — the template
 * parameter names of registerIdentityBuilder.circom:41-52 */
static napi_value js_create_instance(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1], ext;
  CHECK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  if (argc < 1) { napi_throw_type_error(env, NULL, "createInstance(params)"); return NULL; }
  pzk_params p;
  p.circuit = get_i32_prop(env, argv[0], "circuit", PZK_CIRCUIT_REGISTER);
  p.size_arg = get_i32_prop(env, argv[0], "sizeArg", 0);
  p.signature_type = get_i32_prop(env, argv[0], "SIGNATURE_TYPE", 1);
  p.dg_hash_type = get_i32_prop(env, argv[0], "DG_HASH_TYPE", 256);
  p.document_type = get_i32_prop(env, argv[0], "DOCUMENT_TYPE", 3);
  p.ec_block_number = get_i32_prop(env, argv[0], "EC_BLOCK_NUMBER", 4);
  p.ec_shift = get_i32_prop(env, argv[0], "EC_SHIFT", 600);
  p.dg1_shift = get_i32_prop(env, argv[0], "DG1_SHIFT", 248);
  p.aa_signature_algo = get_i32_prop(env, argv[0], "AA_SIGNATURE_ALGO", 1);
  p.dg15_shift = get_i32_prop(env, argv[0], "DG15_SHIFT", 1496);
  p.dg15_block_number = get_i32_prop(env, argv[0], "DG15_BLOCK_NUMBER", 3);
  p.aa_shift = get_i32_prop(env, argv[0], "AA_SHIFT", 256);
  pzk_instance* inst = NULL;
  if (pzk_instance_create(&p, &inst) != 0) return throw_pzk(env, "pzk_instance_create");
  CHECK(napi_create_external(env, inst, finalize_instance, NULL, &ext));
  return ext;
}

static napi_value js_instance_info(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1], obj, v, arr;
  CHECK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  pzk_instance* inst = get_instance(env, argv[0]);
  if (!inst) return NULL;
  pzk_info pi;
  if (pzk_instance_info(inst, &pi) != 0) return throw_pzk(env, "pzk_instance_info");
  CHECK(napi_create_object(env, &obj));
  CHECK(napi_create_double(env, (double)pi.witness_size, &v));
  CHECK(napi_set_named_property(env, obj, "witnessSize", v));
  CHECK(napi_create_double(env, (double)pi.n_inputs, &v));
  CHECK(napi_set_named_property(env, obj, "nInputs", v));
  CHECK(napi_create_uint32(env, pi.n_outputs, &v));
  CHECK(napi_set_named_property(env, obj, "nOutputs", v));
  CHECK(napi_create_uint32(env, pi.n_public_inputs, &v));
  CHECK(napi_set_named_property(env, obj, "nPublicInputs", v));
  CHECK(napi_create_array_with_length(env, pi.n_input_groups, &arr));
  for (uint32_t i = 0; i < pi.n_input_groups; i++) {
    const char* name = NULL;
    uint64_t off = 0, len = 0;
    if (pzk_instance_input(inst, i, &name, &off, &len) != 0) return throw_pzk(env, "pzk_instance_input");
    napi_value g, s, o, l;
    CHECK(napi_create_object(env, &g));
    CHECK(napi_create_string_utf8(env, name, NAPI_AUTO_LENGTH, &s));
    CHECK(napi_create_double(env, (double)off, &o));
    CHECK(napi_create_double(env, (double)len, &l));
    CHECK(napi_set_named_property(env, g, "name", s));
    CHECK(napi_set_named_property(env, g, "offset", o));
    CHECK(napi_set_named_property(env, g, "length", l));
    CHECK(napi_set_element(env, arr, i, g));
  }
  CHECK(napi_set_named_property(env, obj, "inputs", arr));
  return obj;
}

static napi_value js_wtns_header(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1], buf;
  CHECK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  pzk_instance* inst = get_instance(env, argv[0]);
  if (!inst) return NULL;
  void* data = NULL;
  CHECK(napi_create_buffer(env, 76, &data, &buf));
  if (pzk_wtns_header(inst, (uint8_t*)data) != 0) return throw_pzk(env, "pzk_wtns_header");
  return buf;
}

/* ---------------------------------------------------------------- async batch */
typedef struct {
  napi_async_work work;
  napi_deferred deferred;
  napi_ref inputs_ref;
  pzk_instance* inst;
  const uint8_t* inputs;
  size_t batch;
  uint8_t* wtns;     /* malloc'd, handed to a Buffer on completion */
  int32_t* status;
  size_t wtns_bytes;
  int rc;
  char err[512];
} batch_job;

static void batch_execute(napi_env env, void* data) {
  (void)env;
  batch_job* j = (batch_job*)data;
  j->rc = pzk_witness_batch_host(j->inst, j->inputs, j->batch, j->wtns, j->status, NULL);
  if (j->rc) snprintf(j->err, sizeof j->err, "pzk_witness_batch_host: %s", pzk_last_error());
}

static void free_cb(napi_env env, void* data, void* hint) { (void)env; (void)hint; free(data); }

static void batch_complete(napi_env env, napi_status st, void* data) {
  batch_job* j = (batch_job*)data;
  napi_value result = NULL, err_msg, err;
  napi_delete_reference(env, j->inputs_ref);
  if (st != napi_ok || j->rc != 0) {
    napi_create_string_utf8(env, j->rc ? j->err : "pzkwit: async work cancelled", NAPI_AUTO_LENGTH, &err_msg);
    napi_create_error(env, NULL, err_msg, &err);
    napi_reject_deferred(env, j->deferred, err);
    free(j->wtns);
    free(j->status);
  } else {
    napi_value wbuf, sab, sarr;
    napi_create_object(env, &result);
    napi_create_external_buffer(env, j->wtns_bytes, j->wtns, free_cb, NULL, &wbuf);
    napi_create_external_arraybuffer(env, j->status, j->batch * sizeof(int32_t), free_cb, NULL, &sab);
    napi_create_typedarray(env, napi_int32_array, j->batch, sab, 0, &sarr);
    napi_set_named_property(env, result, "witness", wbuf);
    napi_set_named_property(env, result, "status", sarr);
    napi_resolve_deferred(env, j->deferred, result);
  }
  napi_delete_async_work(env, j->work);
  free(j);
}

static napi_value js_witness_batch(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3], promise, name;
  CHECK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  if (argc < 3) { napi_throw_type_error(env, NULL, "witnessBatch(handle, inputs, batch)"); return NULL; }
  pzk_instance* inst = get_instance(env, argv[0]);
  if (!inst) return NULL;
  void* in_data = NULL;
  size_t in_len = 0;
  if (napi_get_buffer_info(env, argv[1], &in_data, &in_len) != napi_ok) {
    napi_throw_type_error(env, NULL, "inputs must be a Buffer");
    return NULL;
  }
  uint32_t batch = 0;
  CHECK(napi_get_value_uint32(env, argv[2], &batch));
  pzk_info pi;
  if (pzk_instance_info(inst, &pi) != 0) return throw_pzk(env, "pzk_instance_info");
  if ((uint64_t)in_len != (uint64_t)batch * pi.n_inputs * 32) {
    napi_throw_range_error(env, NULL, "inputs length != batch * nInputs * 32");
    return NULL;
  }
  batch_job* j = (batch_job*)calloc(1, sizeof(batch_job));
  j->inst = inst;
  j->inputs = (const uint8_t*)in_data;
  j->batch = batch;
  j->wtns_bytes = (size_t)batch * pi.witness_size * 32;
  j->wtns = (uint8_t*)malloc(j->wtns_bytes ? j->wtns_bytes : 1);
  j->status = (int32_t*)calloc(batch ? batch : 1, sizeof(int32_t));
  if (!j->wtns || !j->status) {
    free(j->wtns); free(j->status); free(j);
    napi_throw_error(env, NULL, "pzkwit: host allocation failed");
    return NULL;
  }
  CHECK(napi_create_reference(env, argv[1], 1, &j->inputs_ref));  /* keep the input Buffer alive */
  CHECK(napi_create_promise(env, &j->deferred, &promise));
  CHECK(napi_create_string_utf8(env, "pzkwit.witnessBatch", NAPI_AUTO_LENGTH, &name));
  CHECK(napi_create_async_work(env, NULL, name, batch_execute, batch_complete, j, &j->work));
  CHECK(napi_queue_async_work(env, j->work));
  return promise;
}

static napi_value init(napi_env env, napi_value exports) {
  napi_property_descriptor props[] = {
      {"version", NULL, js_version, NULL, NULL, NULL, napi_enumerable, NULL},
      {"createInstance", NULL, js_create_instance, NULL, NULL, NULL, napi_enumerable, NULL},
      {"instanceInfo", NULL, js_instance_info, NULL, NULL, NULL, napi_enumerable, NULL},
      {"wtnsHeader", NULL, js_wtns_header, NULL, NULL, NULL, napi_enumerable, NULL},
      {"witnessBatch", NULL, js_witness_batch, NULL, NULL, NULL, napi_enumerable, NULL},
  };
  CHECK(napi_define_properties(env, exports, sizeof props / sizeof props[0], props));
  return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, init)
