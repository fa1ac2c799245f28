/* pzkwit_napi.c — Node N-API addon over the libpzkwit C-ABI (include/pzkwit.h).
 *
 * The JS host the reference's callers use (test/automatisationTest.js:37-51 via circom_tester,
 * circuits/scripts/gen-witness.sh:25 via generate_witness.js) talks to a witness calculator
 * object; witness_calculator.js in this directory rebuilds that object on top of these
 * primitives:
 *
 *   version()                              -> string
 *   createInstance(params [, sym])         -> handle (napi external; destroyed by the GC); sym: the circuit's
 *                                             .sym text (string or Buffer) -> pzk_instance_create_mapped, the
 *                                             witness in the layout circom --O1/--O2 writes (compile-circuit.sh:34)
 *   instanceInfo(handle)                   -> { witnessSize, nInputs, nOutputs, nPublicInputs,
 *                                               inputs: [{ name, offset, length }] }
 *   wtnsHeader(handle)                     -> Buffer(76)
 *   witnessBatch(handle, inputs, batch)    -> Promise<{ witness: Buffer, status: Int32Array }>
 *        inputs: Buffer of batch x nInputs x 32 B (LE normal form); runs pzk_witness_batch_host
 *        on a libuv worker thread (napi_create_async_work), so the event loop stays free.
 *
 *   witnessBatchWtns(handle, inputs, batch) -> Promise<{ wtns: Buffer, status: Int32Array }>: the same batch as
 *        ONE Buffer of batch .wtns images back to back (76-byte header + witness each), so a caller takes
 *        per-input .wtns as views (subarray) instead of copies; rows arrive through pzk_witness_stream (pinned
 *        chunks, device->host copy beside compute) and are copied once into their image.
 *   witnessStream(handle, inputs, batch, chunk, onChunk) -> Promise<void>: pzk_witness_stream, the streamed
 *        form of gen-witness.sh:25's one-.wtns-per-input loop. onChunk(first, rows, status) runs on the JS
 *        thread for each chunk in order: rows is an ArrayBuffer over the library's PINNED chunk slot (n x
 *        witnessSize x 32 B, no copy), valid until onChunk returns or the promise it returns settles: it is then
 *        DETACHED (every view of it reads as empty) before the slot is reused — a JS-owned copy where the runtime
 *        refuses external buffers; status is an Int32Array copy. A truthy result (or promise value) or a throw stops the stream and
 *        rejects the call (a throw with its own error). Host memory stays at two chunks whatever the batch.
 *
 *   passportParse({ dg1, dg15, sod })       -> { params, name, refAaShift, ... } (pzk_passport_parse)
 *   passportInputs(params, passports, identity, threads)
 *                                           -> Promise<{ rows: Buffer, status: Int32Array }>: the bulk SOD
 *        preprocessor (include/pzkpassport.h, pzk_passport_inputs) on a libuv worker thread: replaces one
 *        processPassport (test/process_passport.js:674-816) per passport with one call for the batch.
 *        passports: [{ dg1: Buffer, dg15: Buffer | null, sod: Buffer }]; identity: Buffer of
 *        n x 82 x 32 B (slaveMerkleRoot, skIdentity, 80 branches) or null.
 *
 * Errors: a failing pzk_* call throws (or rejects with) an Error carrying pzk_last_error().
 * N-API version 7 (Node >= 12.19 / 14.x): napi_detach_arraybuffer invalidates a streamed chunk's view when the
 * chunk is done with.
 */
#define NAPI_VERSION 7
#define _POSIX_C_SOURCE 200809L
#include <node_api.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/pzkpassport.h"
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
static void read_params(napi_env env, napi_value obj, pzk_params* pp) {
  pzk_params p;
  p.circuit = get_i32_prop(env, obj, "circuit", PZK_CIRCUIT_REGISTER);
  p.size_arg = get_i32_prop(env, obj, "sizeArg", 0);
  p.signature_type = get_i32_prop(env, obj, "SIGNATURE_TYPE", 1);
  p.dg_hash_type = get_i32_prop(env, obj, "DG_HASH_TYPE", 256);
  p.document_type = get_i32_prop(env, obj, "DOCUMENT_TYPE", 3);
  p.ec_block_number = get_i32_prop(env, obj, "EC_BLOCK_NUMBER", 4);
  p.ec_shift = get_i32_prop(env, obj, "EC_SHIFT", 600);
  p.dg1_shift = get_i32_prop(env, obj, "DG1_SHIFT", 248);
  p.aa_signature_algo = get_i32_prop(env, obj, "AA_SIGNATURE_ALGO", 1);
  p.dg15_shift = get_i32_prop(env, obj, "DG15_SHIFT", 1496);
  p.dg15_block_number = get_i32_prop(env, obj, "DG15_BLOCK_NUMBER", 3);
  p.aa_shift = get_i32_prop(env, obj, "AA_SHIFT", 256);
  *pp = p;
}

/* a string or Buffer argument as bytes (strings copied into malloc'd memory: *owned = 1) */
static int get_bytes(napi_env env, napi_value v, const char** data, size_t* len, int* owned) {
  napi_valuetype t;
  bool is_buf = false;
  *owned = 0;
  if (napi_typeof(env, v, &t) != napi_ok) return -1;
  if (t == napi_string) {
    size_t n = 0;
    if (napi_get_value_string_utf8(env, v, NULL, 0, &n) != napi_ok) return -1;
    char* b = (char*)malloc(n + 1);
    if (!b || napi_get_value_string_utf8(env, v, b, n + 1, &n) != napi_ok) { free(b); return -1; }
    *data = b; *len = n; *owned = 1;
    return 0;
  }
  if (napi_is_buffer(env, v, &is_buf) != napi_ok || !is_buf) return -1;
  void* d = NULL;
  if (napi_get_buffer_info(env, v, &d, len) != napi_ok) return -1;
  *data = (const char*)d;
  return 0;
}

static napi_value js_create_instance(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2], ext;
  CHECK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  if (argc < 1) { napi_throw_type_error(env, NULL, "createInstance(params [, sym])"); return NULL; }
  pzk_params p;
  read_params(env, argv[0], &p);
  const char* sym = NULL;
  size_t sym_len = 0;
  int owned = 0;
  if (argc >= 2) {
    napi_valuetype t;
    CHECK(napi_typeof(env, argv[1], &t));
    if (t != napi_undefined && t != napi_null && get_bytes(env, argv[1], &sym, &sym_len, &owned) != 0) {
      napi_throw_type_error(env, NULL, "createInstance: sym must be a string or a Buffer");
      return NULL;
    }
  }
  pzk_instance* inst = NULL;
  const int rc = sym ? pzk_instance_create_mapped(&p, sym, sym_len, &inst) : pzk_instance_create(&p, &inst);
  if (owned) free((void*)sym);
  if (rc != 0) return throw_pzk(env, sym ? "pzk_instance_create_mapped" : "pzk_instance_create");
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


/* ---------------------------------------------------------------- streamed delivery (pzk_witness_stream) */
typedef struct {
  napi_async_work work;
  napi_deferred deferred;
  napi_ref inputs_ref;
  napi_ref error_ref;           /* the exception onChunk threw, to reject with */
  napi_threadsafe_function tsfn;
  pzk_instance* inst;
  const uint8_t* inputs;
  size_t batch, chunk;
  /* the chunk being handed over (set on the worker thread, read on the JS thread) */
  size_t first, n, stride;
  const uint8_t* rows;
  const int32_t* status;
  napi_ref rows_ref;            /* the ArrayBuffer over the pinned chunk handed to onChunk (JS thread only) */
  int rows_external;            /* 1: it views the library's pinned slot (detached when the chunk is done) */
  pthread_mutex_t mu;
  pthread_cond_t cv;
  int handed, sink_rc;
  /* witnessBatchWtns: the sink copies rows into batch .wtns images instead of calling JS */
  uint8_t* images;
  int32_t* img_status;
  size_t img_bytes;
  uint8_t header[76];
  int rc;
  char err[512];
} stream_job;

static void stream_release(stream_job* j, int rc) {
  pthread_mutex_lock(&j->mu);
  j->sink_rc = rc;
  j->handed = 1;
  pthread_cond_signal(&j->cv);
  pthread_mutex_unlock(&j->mu);
}

static stream_job* cb_job(napi_env env, napi_callback_info info, napi_value* arg) {
  size_t argc = 1;
  void* data = NULL;
  if (napi_get_cb_info(env, info, &argc, arg, NULL, &data) != napi_ok) return NULL;
  if (argc < 1) napi_get_undefined(env, arg);
  return (stream_job*)data;
}

static int truthy(napi_env env, napi_value v) {
  napi_value b;
  bool r = false;
  if (napi_coerce_to_bool(env, v, &b) != napi_ok || napi_get_value_bool(env, b, &r) != napi_ok) return 1;
  return r ? 1 : 0;
}

/* JS thread: onChunk is done with the chunk (returned, threw, or its promise settled). The pinned slot its rows
 * live in is reused two chunks later and freed with the instance, so the ArrayBuffer over it is detached first:
 * any view of it a callback kept (an un-awaited write, a stored subarray) then reads as empty instead of reading
 * recycled or freed memory. A copied chunk (rows_external = 0) stays valid and is left to the GC. */
static void chunk_done(napi_env env, stream_job* j, int rc) {
  if (j->rows_ref) {
    napi_value ab;
    if (j->rows_external && napi_get_reference_value(env, j->rows_ref, &ab) == napi_ok && ab)
      napi_detach_arraybuffer(env, ab);
    napi_delete_reference(env, j->rows_ref);
    j->rows_ref = NULL;
  }
  stream_release(j, rc);
}

/* the promise onChunk returned settled */
static napi_value chunk_fulfilled(napi_env env, napi_callback_info info) {
  napi_value v;
  stream_job* j = cb_job(env, info, &v);
  if (j) chunk_done(env, j, truthy(env, v));
  return NULL;
}
static napi_value chunk_rejected(napi_env env, napi_callback_info info) {
  napi_value v;
  stream_job* j = cb_job(env, info, &v);
  if (j) {
    if (!j->error_ref) napi_create_reference(env, v, 1, &j->error_ref);
    chunk_done(env, j, 1);
  }
  return NULL;
}

static void noop_finalize(napi_env env, void* data, void* hint) { (void)env; (void)data; (void)hint; }

/* the chunk's rows as an ArrayBuffer: external over the pinned slot (zero copy, detached in chunk_done), or —
 * where the runtime refuses external buffers (V8 sandbox) — a JS-owned copy */
static int chunk_arraybuffer(napi_env env, stream_job* j, napi_value* ab) {
  const size_t bytes = j->n * j->stride;
  j->rows_external = napi_create_external_arraybuffer(env, (void*)j->rows, bytes, noop_finalize, NULL, ab) == napi_ok;
  if (!j->rows_external) {
    void* copy = NULL;
    if (napi_create_arraybuffer(env, bytes, &copy, ab) != napi_ok) return 0;
    memcpy(copy, j->rows, bytes);
  }
  return napi_create_reference(env, *ab, 1, &j->rows_ref) == napi_ok;
}

/* JS thread: onChunk(first, rows, status) for the chunk the worker is blocked on */
static void stream_call_js(napi_env env, napi_value js_cb, void* context, void* data) {
  stream_job* j = (stream_job*)data;
  (void)context;
  if (!env) { stream_release(j, 1); return; }  /* the environment is shutting down: nothing was handed to JS */
  napi_value argv[3], undef, ret, sab;
  void* st_copy = NULL;
  int ok = napi_create_double(env, (double)j->first, &argv[0]) == napi_ok && chunk_arraybuffer(env, j, &argv[1]) &&
           napi_create_arraybuffer(env, j->n * sizeof(int32_t), &st_copy, &sab) == napi_ok;
  if (ok) {
    memcpy(st_copy, j->status, j->n * sizeof(int32_t));
    ok = napi_create_typedarray(env, napi_int32_array, j->n, sab, 0, &argv[2]) == napi_ok &&
         napi_get_undefined(env, &undef) == napi_ok;
  }
  if (!ok) { chunk_done(env, j, 1); return; }
  if (napi_call_function(env, undef, js_cb, 3, argv, &ret) != napi_ok) {
    napi_value exc;
    if (napi_get_and_clear_last_exception(env, &exc) == napi_ok && !j->error_ref)
      napi_create_reference(env, exc, 1, &j->error_ref);
    chunk_done(env, j, 1);
    return;
  }
  /* a thenable: wait for it to settle (e.g. an fs.promises write of the chunk's .wtns files) */
  napi_valuetype t;
  bool has_then = false;
  napi_value then_fn;
  if (napi_typeof(env, ret, &t) == napi_ok && t == napi_object &&
      napi_has_named_property(env, ret, "then", &has_then) == napi_ok && has_then &&
      napi_get_named_property(env, ret, "then", &then_fn) == napi_ok) {
    napi_value fns[2];
    if (napi_create_function(env, "fulfilled", NAPI_AUTO_LENGTH, chunk_fulfilled, j, &fns[0]) == napi_ok &&
        napi_create_function(env, "rejected", NAPI_AUTO_LENGTH, chunk_rejected, j, &fns[1]) == napi_ok &&
        napi_call_function(env, ret, then_fn, 2, fns, NULL) == napi_ok)
      return;
    chunk_done(env, j, 1);
    return;
  }
  chunk_done(env, j, truthy(env, ret));
}

/* worker thread (inside pzk_witness_stream): hand the chunk to JS and wait until it is done with the rows */
static int stream_sink(void* user, size_t first, size_t n, const uint8_t* rows, size_t stride, const int32_t* status) {
  stream_job* j = (stream_job*)user;
  if (j->images) {  /* witnessBatchWtns: one copy into the chunk's .wtns images */
    const size_t img = 76 + stride;
    for (size_t i = 0; i < n; i++) {
      memcpy(j->images + (first + i) * img, j->header, 76);
      memcpy(j->images + (first + i) * img + 76, rows + i * stride, stride);
    }
    memcpy(j->img_status + first, status, n * sizeof(int32_t));
    return 0;
  }
  pthread_mutex_lock(&j->mu);
  j->first = first; j->n = n; j->rows = rows; j->stride = stride; j->status = status; j->handed = 0;
  pthread_mutex_unlock(&j->mu);
  if (napi_call_threadsafe_function(j->tsfn, j, napi_tsfn_blocking) != napi_ok) return 1;
  pthread_mutex_lock(&j->mu);
  while (!j->handed) pthread_cond_wait(&j->cv, &j->mu);
  const int rc = j->sink_rc;
  pthread_mutex_unlock(&j->mu);
  return rc;
}

static void stream_execute(napi_env env, void* data) {
  (void)env;
  stream_job* j = (stream_job*)data;
  j->rc = pzk_witness_stream(j->inst, j->inputs, j->batch, j->chunk, stream_sink, j, NULL);
  if (j->rc) snprintf(j->err, sizeof j->err, "pzk_witness_stream: %s", pzk_last_error());
}

static void stream_complete(napi_env env, napi_status st, void* data) {
  stream_job* j = (stream_job*)data;
  napi_value err_msg, err, result;
  napi_delete_reference(env, j->inputs_ref);
  if (j->tsfn) napi_release_threadsafe_function(j->tsfn, napi_tsfn_release);
  if (st != napi_ok || j->rc != 0) {
    if (j->error_ref && napi_get_reference_value(env, j->error_ref, &err) == napi_ok && err) {
      napi_reject_deferred(env, j->deferred, err);
    } else {
      napi_create_string_utf8(env, j->rc ? j->err : "pzkwit: async work cancelled", NAPI_AUTO_LENGTH, &err_msg);
      napi_create_error(env, NULL, err_msg, &err);
      napi_reject_deferred(env, j->deferred, err);
    }
    free(j->images);
    free(j->img_status);
  } else if (j->images) {
    napi_value wbuf, sab, sarr;
    napi_create_object(env, &result);
    napi_create_external_buffer(env, j->img_bytes, j->images, free_cb, NULL, &wbuf);
    napi_create_external_arraybuffer(env, j->img_status, j->batch * sizeof(int32_t), free_cb, NULL, &sab);
    napi_create_typedarray(env, napi_int32_array, j->batch, sab, 0, &sarr);
    napi_set_named_property(env, result, "wtns", wbuf);
    napi_set_named_property(env, result, "status", sarr);
    napi_resolve_deferred(env, j->deferred, result);
  } else {
    napi_get_undefined(env, &result);
    napi_resolve_deferred(env, j->deferred, result);
  }
  if (j->error_ref) napi_delete_reference(env, j->error_ref);
  pthread_mutex_destroy(&j->mu);
  pthread_cond_destroy(&j->cv);
  napi_delete_async_work(env, j->work);
  free(j);
}

/* shared argument handling of witnessStream / witnessBatchWtns: (handle, inputs, batch, ...) */
static stream_job* stream_job_new(napi_env env, napi_value* argv, pzk_info* pi) {
  pzk_instance* inst = get_instance(env, argv[0]);
  if (!inst) return NULL;
  void* in_data = NULL;
  size_t in_len = 0;
  if (napi_get_buffer_info(env, argv[1], &in_data, &in_len) != napi_ok) {
    napi_throw_type_error(env, NULL, "inputs must be a Buffer");
    return NULL;
  }
  uint32_t batch = 0;
  if (napi_get_value_uint32(env, argv[2], &batch) != napi_ok) { napi_throw_type_error(env, NULL, "batch"); return NULL; }
  if (pzk_instance_info(inst, pi) != 0) { throw_pzk(env, "pzk_instance_info"); return NULL; }
  if ((uint64_t)in_len != (uint64_t)batch * pi->n_inputs * 32) {
    napi_throw_range_error(env, NULL, "inputs length != batch * nInputs * 32");
    return NULL;
  }
  stream_job* j = (stream_job*)calloc(1, sizeof(stream_job));
  if (!j) { napi_throw_error(env, NULL, "pzkwit: host allocation failed"); return NULL; }
  j->inst = inst;
  j->inputs = (const uint8_t*)in_data;
  j->batch = batch;
  pthread_mutex_init(&j->mu, NULL);
  pthread_cond_init(&j->cv, NULL);
  if (napi_create_reference(env, argv[1], 1, &j->inputs_ref) != napi_ok) {
    free(j);
    napi_throw_error(env, NULL, "pzkwit: reference");
    return NULL;
  }
  return j;
}

static napi_value stream_start(napi_env env, stream_job* j, const char* what) {
  napi_value promise, name;
  CHECK(napi_create_promise(env, &j->deferred, &promise));
  CHECK(napi_create_string_utf8(env, what, NAPI_AUTO_LENGTH, &name));
  CHECK(napi_create_async_work(env, NULL, name, stream_execute, stream_complete, j, &j->work));
  CHECK(napi_queue_async_work(env, j->work));
  return promise;
}

static napi_value js_witness_stream(napi_env env, napi_callback_info info) {
  size_t argc = 5;
  napi_value argv[5], name;
  CHECK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  if (argc < 5) { napi_throw_type_error(env, NULL, "witnessStream(handle, inputs, batch, chunk, onChunk)"); return NULL; }
  napi_valuetype t;
  CHECK(napi_typeof(env, argv[4], &t));
  if (t != napi_function) { napi_throw_type_error(env, NULL, "onChunk must be a function"); return NULL; }
  uint32_t chunk = 0;
  CHECK(napi_get_value_uint32(env, argv[3], &chunk));
  pzk_info pi;
  stream_job* j = stream_job_new(env, argv, &pi);
  if (!j) return NULL;
  j->chunk = chunk;
  CHECK(napi_create_string_utf8(env, "pzkwit.witnessStream", NAPI_AUTO_LENGTH, &name));
  CHECK(napi_create_threadsafe_function(env, argv[4], NULL, name, 0, 1, NULL, NULL, NULL, stream_call_js, &j->tsfn));
  return stream_start(env, j, "pzkwit.witnessStream");
}

static napi_value js_witness_batch_wtns(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  CHECK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  if (argc < 3) { napi_throw_type_error(env, NULL, "witnessBatchWtns(handle, inputs, batch)"); return NULL; }
  pzk_info pi;
  stream_job* j = stream_job_new(env, argv, &pi);
  if (!j) return NULL;
  j->img_bytes = j->batch * (76 + (size_t)pi.witness_size * 32);
  j->images = (uint8_t*)malloc(j->img_bytes ? j->img_bytes : 1);
  j->img_status = (int32_t*)calloc(j->batch ? j->batch : 1, sizeof(int32_t));
  if (!j->images || !j->img_status || pzk_wtns_header(j->inst, j->header) != 0) {
    napi_delete_reference(env, j->inputs_ref);
    free(j->images); free(j->img_status); free(j);
    napi_throw_error(env, NULL, "pzkwit: host allocation failed");
    return NULL;
  }
  return stream_start(env, j, "pzkwit.witnessBatchWtns");
}

/* ---------------------------------------------------------------- SOD preprocessor (pzkpassport.h) */
static napi_value params_object(napi_env env, const pzk_params* p) {
  napi_value o, v;
  if (napi_create_object(env, &o) != napi_ok) return NULL;
  const struct { const char* k; int32_t v; } f[] = {
      {"circuit", p->circuit}, {"SIGNATURE_TYPE", p->signature_type}, {"DG_HASH_TYPE", p->dg_hash_type},
      {"DOCUMENT_TYPE", p->document_type}, {"EC_BLOCK_NUMBER", p->ec_block_number}, {"EC_SHIFT", p->ec_shift},
      {"DG1_SHIFT", p->dg1_shift}, {"AA_SIGNATURE_ALGO", p->aa_signature_algo}, {"DG15_SHIFT", p->dg15_shift},
      {"DG15_BLOCK_NUMBER", p->dg15_block_number}, {"AA_SHIFT", p->aa_shift}};
  for (size_t i = 0; i < sizeof f / sizeof f[0]; i++) {
    if (napi_create_int32(env, f[i].v, &v) != napi_ok || napi_set_named_property(env, o, f[i].k, v) != napi_ok)
      return NULL;
  }
  return o;
}

/* passport object { dg1, dg15, sod } of Buffers (dg15 may be null / absent) -> source */
static int get_passport(napi_env env, napi_value obj, pzk_passport_src* src) {
  const char* keys[3] = {"dg1", "dg15", "sod"};
  const uint8_t** ptr[3] = {&src->dg1, &src->dg15, &src->sod};
  size_t* len[3] = {&src->dg1_len, &src->dg15_len, &src->sod_len};
  for (int i = 0; i < 3; i++) {
    bool has = false, is_buf = false;
    napi_value v;
    *ptr[i] = NULL; *len[i] = 0;
    if (napi_has_named_property(env, obj, keys[i], &has) != napi_ok) return -1;
    if (!has) { if (i == 1) continue; return -1; }
    if (napi_get_named_property(env, obj, keys[i], &v) != napi_ok) return -1;
    napi_valuetype t;
    if (napi_typeof(env, v, &t) != napi_ok) return -1;
    if (i == 1 && (t == napi_null || t == napi_undefined)) continue;
    if (napi_is_buffer(env, v, &is_buf) != napi_ok || !is_buf) return -1;
    void* d = NULL;
    if (napi_get_buffer_info(env, v, &d, len[i]) != napi_ok) return -1;
    *ptr[i] = (const uint8_t*)d;
  }
  return 0;
}

static napi_value js_passport_parse(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1], obj, v;
  CHECK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  pzk_passport_src src;
  if (argc < 1 || get_passport(env, argv[0], &src) != 0) {
    napi_throw_type_error(env, NULL, "passportParse({ dg1: Buffer, dg15: Buffer | null, sod: Buffer })");
    return NULL;
  }
  pzk_passport_info pi;
  if (pzk_passport_parse(&src, &pi) != 0) return throw_pzk(env, "pzk_passport_parse");
  CHECK(napi_create_object(env, &obj));
  napi_value po = params_object(env, &pi.params);
  if (!po) { napi_throw_error(env, NULL, "pzkwit: params object"); return NULL; }
  CHECK(napi_set_named_property(env, obj, "params", po));
  CHECK(napi_create_string_utf8(env, pi.name, NAPI_AUTO_LENGTH, &v));
  CHECK(napi_set_named_property(env, obj, "name", v));
  const struct { const char* k; int32_t v; } f[] = {
      {"refAaShift", pi.ref_aa_shift}, {"dgHashBytes", pi.dg_hash_bytes}, {"hashBytes", pi.hash_bytes},
      {"dg1Len", pi.dg1_len}, {"dg15Len", pi.dg15_len}, {"ecLen", pi.ec_len}, {"saLen", pi.sa_len},
      {"chunkNumber", pi.chunk_number}, {"chunkBits", pi.chunk_bits}, {"salt", pi.salt}};
  for (size_t i = 0; i < sizeof f / sizeof f[0]; i++) {
    CHECK(napi_create_int32(env, f[i].v, &v));
    CHECK(napi_set_named_property(env, obj, f[i].k, v));
  }
  return obj;
}

typedef struct {
  napi_async_work work;
  napi_deferred deferred;
  napi_ref args_ref;  /* keeps the passports array and the identity Buffer alive */
  pzk_params params;
  pzk_passport_src* srcs;
  size_t n;
  const uint8_t* identity;
  uint8_t* rows;
  int32_t* status;
  size_t row_bytes;
  int threads, rc;
  char err[512];
} pp_job;

static void pp_execute(napi_env env, void* data) {
  (void)env;
  pp_job* j = (pp_job*)data;
  j->rc = pzk_passport_inputs(&j->params, j->srcs, j->n, j->identity, j->rows, j->status, j->threads);
  if (j->rc) snprintf(j->err, sizeof j->err, "pzk_passport_inputs: %s", pzk_last_error());
}

static void pp_complete(napi_env env, napi_status st, void* data) {
  pp_job* j = (pp_job*)data;
  napi_value result, err_msg, err;
  napi_delete_reference(env, j->args_ref);
  free(j->srcs);
  if (st != napi_ok || j->rc != 0) {
    napi_create_string_utf8(env, j->rc ? j->err : "pzkwit: async work cancelled", NAPI_AUTO_LENGTH, &err_msg);
    napi_create_error(env, NULL, err_msg, &err);
    napi_reject_deferred(env, j->deferred, err);
    free(j->rows);
    free(j->status);
  } else {
    napi_value rbuf, sab, sarr;
    napi_create_object(env, &result);
    napi_create_external_buffer(env, j->n * j->row_bytes, j->rows, free_cb, NULL, &rbuf);
    napi_create_external_arraybuffer(env, j->status, j->n * sizeof(int32_t), free_cb, NULL, &sab);
    napi_create_typedarray(env, napi_int32_array, j->n, sab, 0, &sarr);
    napi_set_named_property(env, result, "rows", rbuf);
    napi_set_named_property(env, result, "status", sarr);
    napi_resolve_deferred(env, j->deferred, result);
  }
  napi_delete_async_work(env, j->work);
  free(j);
}

static napi_value js_passport_inputs(napi_env env, napi_callback_info info) {
  size_t argc = 4;
  napi_value argv[4], promise, name, holder;
  CHECK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  if (argc < 2) { napi_throw_type_error(env, NULL, "passportInputs(params, passports [, identity, threads])"); return NULL; }
  pzk_params p;
  read_params(env, argv[0], &p);
  bool is_arr = false;
  CHECK(napi_is_array(env, argv[1], &is_arr));
  if (!is_arr) { napi_throw_type_error(env, NULL, "passports must be an array"); return NULL; }
  uint32_t n = 0;
  CHECK(napi_get_array_length(env, argv[1], &n));
  pzk_info li;
  if (pzk_layout_query(&p, &li, NULL) != 0) return throw_pzk(env, "pzk_layout_query");
  const uint8_t* ident = NULL;
  if (argc >= 3) {
    napi_valuetype t;
    CHECK(napi_typeof(env, argv[2], &t));
    if (t != napi_null && t != napi_undefined) {
      void* d = NULL;
      size_t len = 0;
      if (napi_get_buffer_info(env, argv[2], &d, &len) != napi_ok || len != (size_t)n * 82 * 32) {
        napi_throw_range_error(env, NULL, "identity must be a Buffer of n x 82 x 32 bytes");
        return NULL;
      }
      ident = (const uint8_t*)d;
    }
  }
  int32_t threads = 0;
  if (argc >= 4) {
    napi_valuetype t;
    CHECK(napi_typeof(env, argv[3], &t));
    if (t == napi_number) CHECK(napi_get_value_int32(env, argv[3], &threads));
  }
  pp_job* j = (pp_job*)calloc(1, sizeof(pp_job));
  if (!j) { napi_throw_error(env, NULL, "pzkwit: host allocation failed"); return NULL; }
  j->params = p;
  j->n = n;
  j->identity = ident;
  j->threads = threads;
  j->row_bytes = (size_t)li.n_inputs * 32;
  j->srcs = (pzk_passport_src*)calloc(n ? n : 1, sizeof(pzk_passport_src));
  j->rows = (uint8_t*)malloc(n ? (size_t)n * j->row_bytes : 1);
  j->status = (int32_t*)calloc(n ? n : 1, sizeof(int32_t));
  if (!j->srcs || !j->rows || !j->status) {
    free(j->srcs); free(j->rows); free(j->status); free(j);
    napi_throw_error(env, NULL, "pzkwit: host allocation failed");
    return NULL;
  }
  for (uint32_t i = 0; i < n; i++) {
    napi_value e;
    if (napi_get_element(env, argv[1], i, &e) != napi_ok || get_passport(env, e, &j->srcs[i]) != 0) {
      char msg[128];
      snprintf(msg, sizeof msg, "passports[%u] must be { dg1: Buffer, dg15: Buffer | null, sod: Buffer }", i);
      free(j->srcs); free(j->rows); free(j->status); free(j);
      napi_throw_type_error(env, NULL, msg);
      return NULL;
    }
  }
  CHECK(napi_create_array_with_length(env, 2, &holder));  /* the job reads the Buffers on a worker thread */
  CHECK(napi_set_element(env, holder, 0, argv[1]));
  if (ident) CHECK(napi_set_element(env, holder, 1, argv[2]));
  CHECK(napi_create_reference(env, holder, 1, &j->args_ref));
  CHECK(napi_create_promise(env, &j->deferred, &promise));
  CHECK(napi_create_string_utf8(env, "pzkwit.passportInputs", NAPI_AUTO_LENGTH, &name));
  CHECK(napi_create_async_work(env, NULL, name, pp_execute, pp_complete, j, &j->work));
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
      {"witnessBatchWtns", NULL, js_witness_batch_wtns, NULL, NULL, NULL, napi_enumerable, NULL},
      {"witnessStream", NULL, js_witness_stream, NULL, NULL, NULL, napi_enumerable, NULL},
      {"passportParse", NULL, js_passport_parse, NULL, NULL, NULL, napi_enumerable, NULL},
      {"passportInputs", NULL, js_passport_inputs, NULL, NULL, NULL, napi_enumerable, NULL},
  };
  CHECK(napi_define_properties(env, exports, sizeof props / sizeof props[0], props));
  return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, init)
