// N-API addon: the Node.js side of the drop-in boundary.
//
// The reference's host is Node.js: its proofs come from snarkjs.plonk.prove /
// plonk.fullProve [EXT] (snarkjs 0.4.12, /root/reference/package.json:18). This
// addon binds the C-ABI in include/nzcb.h one-to-one; index.js wraps it in the
// snarkjs-compatible Promise API. Every prove / fullProveDevice call runs on a thread of
// its own and takes a free lane of the context (nzcb_prove_logged), so concurrent promises
// on one context are proved at the same time, up to the context's lanes (setLanes); the
// result and the optional logger come back to the main thread through thread-safe
// functions, and the event loop is never blocked.
#define NAPI_VERSION 6
#include <node_api.h>

#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/nzcb.h"

#define CHECK(call)                                                    \
  do {                                                                 \
    if ((call) != napi_ok) {                                           \
      napi_throw_error(env, nullptr, "nzcb addon: N-API call failed"); \
      return nullptr;                                                  \
    }                                                                  \
  } while (0)

namespace {

struct Ctx {
  nzcb_ctx* ctx = nullptr;
};

void ctx_finalize(napi_env, void* data, void*) {
  Ctx* c = static_cast<Ctx*>(data);
  if (c->ctx) nzcb_ctx_destroy(c->ctx);
  delete c;
}

napi_value make_error(napi_env env, int code, const char* msg) {
  napi_value m, err, c;
  napi_create_string_utf8(env, msg, NAPI_AUTO_LENGTH, &m);
  napi_create_error(env, nullptr, m, &err);
  napi_create_int32(env, code, &c);
  napi_set_named_property(env, err, "code", c);
  return err;
}

// createContext(zkey: Buffer, device: number) -> external
napi_value CreateContext(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  CHECK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  void* data = nullptr;
  size_t len = 0;
  CHECK(napi_get_buffer_info(env, argv[0], &data, &len));
  int32_t device = 0;
  if (argc > 1) napi_get_value_int32(env, argv[1], &device);
  nzcb_err err{};
  nzcb_ctx* ctx = nzcb_ctx_create(static_cast<const uint8_t*>(data), len, device, &err);
  if (!ctx) {
    napi_throw(env, make_error(env, err.code, err.msg));
    return nullptr;
  }
  Ctx* c = new Ctx();
  c->ctx = ctx;
  napi_value ext;
  CHECK(napi_create_external(env, c, ctx_finalize, nullptr, &ext));
  return ext;
}

// releaseContext(ctx): frees the context's HBM now instead of at garbage collection (a
// context whose lane setup failed is dropped this way; the external must not be used after)
napi_value ReleaseContext(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  CHECK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  Ctx* c = nullptr;
  CHECK(napi_get_value_external(env, argv[0], reinterpret_cast<void**>(&c)));
  if (c && c->ctx) {
    nzcb_ctx_destroy(c->ctx);
    c->ctx = nullptr;
  }
  return nullptr;
}

// a JS string argument as UTF-8 (false if it is not a string)
bool str_arg(napi_env env, napi_value v, std::string* out) {
  napi_valuetype t;
  if (napi_typeof(env, v, &t) != napi_ok || t != napi_string) return false;
  size_t plen = 0;
  if (napi_get_value_string_utf8(env, v, nullptr, 0, &plen) != napi_ok) return false;
  out->assign(plen + 1, '\0');
  if (napi_get_value_string_utf8(env, v, &(*out)[0], out->size(), &plen) != napi_ok) return false;
  out->resize(plen);
  return true;
}

// createContextFile(path: string, device: number) -> external (zkeys larger than a Buffer)
napi_value CreateContextFile(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  CHECK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  std::string path;
  if (argc < 1 || !str_arg(env, argv[0], &path)) {
    napi_throw_type_error(env, nullptr, "createContextFile(path: string, device?: number)");
    return nullptr;
  }
  int32_t device = 0;
  if (argc > 1) napi_get_value_int32(env, argv[1], &device);
  nzcb_err err{};
  const int devs[1] = {device};
  nzcb_ctx* ctx = nzcb_ctx_create_file(path.c_str(), devs, 1, &err);
  if (!ctx) {
    napi_throw(env, make_error(env, err.code, err.msg));
    return nullptr;
  }
  Ctx* c = new Ctx();
  c->ctx = ctx;
  napi_value ext;
  CHECK(napi_create_external(env, c, ctx_finalize, nullptr, &ext));
  return ext;
}

struct Wprog;

// one prove / fullProveDevice call: runs on its own thread, completes on the main thread
struct ProveWork {
  napi_deferred deferred = nullptr;
  napi_ref ctx_ref = nullptr, in_ref = nullptr, prog_ref = nullptr;
  napi_threadsafe_function done = nullptr;  // completion (no JS function: prove_complete)
  napi_threadsafe_function tsfn = nullptr;  // the logger, if any
  Ctx* c = nullptr;
  Wprog* prog = nullptr;                    // fullProveDevice: the witness program
  const uint8_t* in = nullptr;              // .wtns bytes (prove) or input signals (fullProveDevice)
  size_t in_len = 0;
  bool has_blinding = false;
  uint8_t blinding[NZCB_BLINDING_BYTES];
  uint8_t proof[NZCB_PROOF_BYTES];
  uint8_t pub[32 * 64];
  uint32_t npub = 0;
  int rc = 0;
  int32_t status = 0;  // fullProveDevice: the witness program's failed check, if any
  nzcb_err err{};
};

void log_trampoline(void* user, const char* msg) {
  ProveWork* w = static_cast<ProveWork*>(user);
  if (!w->tsfn) return;
  char* copy = strdup(msg);
  if (napi_call_threadsafe_function(w->tsfn, copy, napi_tsfn_blocking) != napi_ok) free(copy);
}

void call_logger(napi_env env, napi_value fn, void*, void* data) {
  char* msg = static_cast<char*>(data);
  if (env && fn) {
    napi_value s, undef;
    napi_create_string_utf8(env, msg, NAPI_AUTO_LENGTH, &s);
    napi_get_undefined(env, &undef);
    napi_call_function(env, undef, fn, 1, &s, nullptr);
  }
  free(msg);
}

void prove_complete(napi_env env, napi_value, void*, void* data) {
  ProveWork* w = static_cast<ProveWork*>(data);
  if (env) {
    if (w->rc) {
      napi_reject_deferred(env, w->deferred, make_error(env, w->rc, w->err.msg));
    } else if (w->status) {
      napi_reject_deferred(env, w->deferred, make_error(env, w->status, "Assert Failed (witness calculation)"));
    } else {
      std::string pj(8192, '\0'), uj(96 * 64 + 8, '\0');
      nzcb_proof_to_json(w->proof, &pj[0], pj.size());
      nzcb_public_to_json(w->pub, (int)w->npub, &uj[0], uj.size());
      napi_value obj, a, b;
      napi_create_object(env, &obj);
      napi_create_string_utf8(env, pj.c_str(), NAPI_AUTO_LENGTH, &a);
      napi_create_string_utf8(env, uj.c_str(), NAPI_AUTO_LENGTH, &b);
      napi_set_named_property(env, obj, "proof", a);
      napi_set_named_property(env, obj, "publicSignals", b);
      napi_resolve_deferred(env, w->deferred, obj);
    }
    napi_delete_reference(env, w->ctx_ref);
    napi_delete_reference(env, w->in_ref);
    if (w->prog_ref) napi_delete_reference(env, w->prog_ref);
  }
  if (w->tsfn) napi_release_threadsafe_function(w->tsfn, napi_tsfn_release);
  napi_release_threadsafe_function(w->done, napi_tsfn_release);
  delete w;
}

void run_fullprove_device(ProveWork* w);

void prove_thread(ProveWork* w) {
  uint32_t info[5];
  nzcb_ctx_info(w->c->ctx, info);
  w->npub = info[1];
  if (w->npub > 64) {
    w->rc = NZCB_ERR_ARG;
    std::snprintf(w->err.msg, sizeof(w->err.msg), "too many public signals for the addon buffer");
  } else if (w->prog) {
    run_fullprove_device(w);
  } else {
    w->rc = nzcb_prove_logged(w->c->ctx, w->in, w->in_len, NZCB_WITNESS_WTNS, w->has_blinding ? w->blinding : nullptr,
                              w->proof, w->pub, sizeof(w->pub), w->tsfn ? log_trampoline : nullptr, w, &w->err);
  }
  napi_call_threadsafe_function(w->done, w, napi_tsfn_blocking);
}

// the common argument handling of prove / fullProveDevice: blinding (argv[bi]), logger
// (argv[bi + 1]); creates the promise and starts the thread
napi_value start_prove(napi_env env, ProveWork* w, napi_value* argv, size_t argc, size_t bi) {
  napi_valuetype t;
  if (argc > bi && napi_typeof(env, argv[bi], &t) == napi_ok && t == napi_object) {
    void* bd = nullptr;
    size_t bl = 0;
    if (napi_get_buffer_info(env, argv[bi], &bd, &bl) == napi_ok && bl == NZCB_BLINDING_BYTES) {
      std::memcpy(w->blinding, bd, bl);
      w->has_blinding = true;
    }
  }
  napi_value name;
  if (argc > bi + 1 && napi_typeof(env, argv[bi + 1], &t) == napi_ok && t == napi_function) {
    napi_create_string_utf8(env, "nzcb-logger", NAPI_AUTO_LENGTH, &name);
    CHECK(napi_create_threadsafe_function(env, argv[bi + 1], nullptr, name, 0, 1, nullptr, nullptr, nullptr,
                                          call_logger, &w->tsfn));
  }
  napi_value promise;
  CHECK(napi_create_promise(env, &w->deferred, &promise));
  napi_create_string_utf8(env, "nzcb-prove", NAPI_AUTO_LENGTH, &name);
  CHECK(napi_create_threadsafe_function(env, nullptr, nullptr, name, 0, 1, nullptr, nullptr, nullptr, prove_complete,
                                        &w->done));
  std::thread(prove_thread, w).detach();
  return promise;
}

// prove(ctx, wtns: Buffer, blinding: Buffer|null, logger: Function|null) -> Promise<{proof, publicSignals}> (JSON strings)
napi_value Prove(napi_env env, napi_callback_info info) {
  size_t argc = 4;
  napi_value argv[4];
  CHECK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  ProveWork* w = new ProveWork();
  CHECK(napi_get_value_external(env, argv[0], reinterpret_cast<void**>(&w->c)));
  void* wd = nullptr;
  CHECK(napi_get_buffer_info(env, argv[1], &wd, &w->in_len));
  w->in = static_cast<const uint8_t*>(wd);
  CHECK(napi_create_reference(env, argv[0], 1, &w->ctx_ref));
  CHECK(napi_create_reference(env, argv[1], 1, &w->in_ref));
  return start_prove(env, w, argv, argc, 2);
}

// setLanes(ctx, lanes) -> lanes: proofs in flight on the context (nzcb_ctx_set_lanes)
napi_value SetLanes(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  CHECK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  Ctx* c = nullptr;
  CHECK(napi_get_value_external(env, argv[0], reinterpret_cast<void**>(&c)));
  int32_t lanes = 1;
  CHECK(napi_get_value_int32(env, argv[1], &lanes));
  nzcb_err err{};
  if (nzcb_ctx_set_lanes(c->ctx, lanes, &err)) {
    napi_throw(env, make_error(env, err.code, err.msg));
    return nullptr;
  }
  napi_value v;
  napi_create_int32(env, nzcb_ctx_lanes(c->ctx), &v);
  return v;
}

// ---- witness programs (nzcb_wprog_*): circom's witness calculator on the GPU ----------
struct Wprog {
  nzcb_wprog* p = nullptr;
  int device = 0;  // the program's GPU: its witness buffers live there
};

// HBM buffers reused across fullProveDevice calls (a witness of nzcp_live is 19.2 MB; a
// hipMalloc per proof would cost more than the witness program's run), keyed by (device,
// bytes): a call's buffers are on its witness program's device (the per-call
// threads never selected a device, so every buffer was on device 0)
std::mutex g_pool_mu;
std::multimap<std::pair<int, size_t>, void*> g_pool;
void* pool_get(int device, size_t bytes) {
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    auto it = g_pool.find({device, bytes});
    if (it != g_pool.end()) {
      void* p = it->second;
      g_pool.erase(it);
      return p;
    }
  }
  return nzcb_dev_alloc_on(device, bytes);
}
void pool_put(int device, size_t bytes, void* p) {
  if (!p) return;
  std::lock_guard<std::mutex> lk(g_pool_mu);
  g_pool.emplace(std::make_pair(device, bytes), p);
}

// plonk.fullProve with a witness program, everything in HBM: the input signals go up
// (a few KB), the witness program writes the witness into a device buffer, and the proof
// reads it there (nzcb_wprog_run_dev + nzcb_prove_logged NZCB_WITNESS_DEVICE); only the
// proof and the public signals come back
void run_fullprove_device(ProveWork* w) {
  uint32_t pi[5];
  nzcb_wprog_info(w->prog->p, pi);
  const size_t nwires = pi[0], nin = (size_t)pi[2] + pi[3];
  if (w->in_len != nin * 32) {
    w->rc = NZCB_ERR_ARG;
    std::snprintf(w->err.msg, sizeof(w->err.msg), "expected %zu input signals", nin);
    return;
  }
  const int dev = w->prog->device;
  void* din = pool_get(dev, nin * 32 ? nin * 32 : 32);
  void* dw = pool_get(dev, nwires * 32);
  if (!din || !dw || nzcb_memcpy_h2d(din, w->in, w->in_len) != 0) {
    w->rc = NZCB_ERR_HIP;
    std::snprintf(w->err.msg, sizeof(w->err.msg), "device buffers for the witness failed");
  } else {
    w->rc = nzcb_wprog_run_dev(w->prog->p, din, 1, dw, nwires * 32, &w->status, nullptr, &w->err);
    if (!w->rc && !w->status)
      w->rc = nzcb_prove_logged(w->c->ctx, dw, nwires, NZCB_WITNESS_DEVICE, w->has_blinding ? w->blinding : nullptr,
                                w->proof, w->pub, sizeof(w->pub), w->tsfn ? log_trampoline : nullptr, w, &w->err);
  }
  pool_put(dev, nin * 32 ? nin * 32 : 32, din);
  pool_put(dev, nwires * 32, dw);
}

void wprog_finalize(napi_env, void* data, void*) {
  Wprog* w = static_cast<Wprog*>(data);
  if (w->p) nzcb_wprog_destroy(w->p);
  delete w;
}

// createWitnessProgram(program: Buffer, device: number) -> external
napi_value CreateWitnessProgram(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  CHECK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  void* data = nullptr;
  size_t len = 0;
  CHECK(napi_get_buffer_info(env, argv[0], &data, &len));
  int32_t device = 0;
  if (argc > 1) napi_get_value_int32(env, argv[1], &device);
  nzcb_err err{};
  nzcb_wprog* p = nzcb_wprog_create(static_cast<const uint8_t*>(data), len, device, &err);
  if (!p) {
    napi_throw(env, make_error(env, err.code, err.msg));
    return nullptr;
  }
  Wprog* w = new Wprog();
  w->p = p;
  w->device = device;
  napi_value ext;
  CHECK(napi_create_external(env, w, wprog_finalize, nullptr, &ext));
  return ext;
}

struct WitnessWork {
  napi_async_work work = nullptr;
  napi_deferred deferred = nullptr;
  napi_ref prog_ref = nullptr, in_ref = nullptr;
  Wprog* w = nullptr;
  const uint8_t* inputs = nullptr;
  size_t in_len = 0;
  std::vector<uint8_t> out;
  int32_t status = 0;
  int rc = 0;
  nzcb_err err{};
};

void witness_execute(napi_env, void* data) {
  WitnessWork* k = static_cast<WitnessWork*>(data);
  uint32_t info[5];
  nzcb_wprog_info(k->w->p, info);
  const size_t nin = (size_t)info[2] + info[3];
  if (k->in_len != nin * 32) {
    k->rc = NZCB_ERR_ARG;
    std::snprintf(k->err.msg, sizeof(k->err.msg), "expected %zu input signals", nin);
    return;
  }
  k->out.resize((size_t)info[0] * 32);
  k->rc = nzcb_wprog_run(k->w->p, k->inputs, 1, k->out.data(), &k->status, &k->err);
}

void witness_complete(napi_env env, napi_status, void* data) {
  WitnessWork* k = static_cast<WitnessWork*>(data);
  if (k->rc) {
    napi_reject_deferred(env, k->deferred, make_error(env, k->rc, k->err.msg));
  } else if (k->status) {
    napi_reject_deferred(env, k->deferred, make_error(env, k->status, "Assert Failed (witness calculation)"));
  } else {
    napi_value buf;
    void* dst = nullptr;
    if (napi_create_buffer_copy(env, k->out.size(), k->out.data(), &dst, &buf) == napi_ok)
      napi_resolve_deferred(env, k->deferred, buf);
    else
      napi_reject_deferred(env, k->deferred, make_error(env, NZCB_ERR_INTERNAL, "buffer allocation failed"));
  }
  napi_delete_reference(env, k->prog_ref);
  napi_delete_reference(env, k->in_ref);
  napi_delete_async_work(env, k->work);
  delete k;
}

// calculateWitness(prog, inputs: Buffer (n_inputs x 32 B LE)) -> Promise<Buffer (n_wires x 32 B LE)>
napi_value CalculateWitness(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  CHECK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  WitnessWork* k = new WitnessWork();
  CHECK(napi_get_value_external(env, argv[0], reinterpret_cast<void**>(&k->w)));
  void* d = nullptr;
  CHECK(napi_get_buffer_info(env, argv[1], &d, &k->in_len));
  k->inputs = static_cast<const uint8_t*>(d);
  CHECK(napi_create_reference(env, argv[0], 1, &k->prog_ref));
  CHECK(napi_create_reference(env, argv[1], 1, &k->in_ref));
  napi_value promise, rname;
  CHECK(napi_create_promise(env, &k->deferred, &promise));
  napi_create_string_utf8(env, "nzcb-witness", NAPI_AUTO_LENGTH, &rname);
  CHECK(napi_create_async_work(env, nullptr, rname, witness_execute, witness_complete, k, &k->work));
  CHECK(napi_queue_async_work(env, k->work));
  return promise;
}

// fullProveDevice(ctx, prog, inputs: Buffer (n_inputs x 32 B LE), blinding, logger)
//   -> Promise<{proof, publicSignals}>
napi_value FullProveDevice(napi_env env, napi_callback_info info) {
  size_t argc = 5;
  napi_value argv[5];
  CHECK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  ProveWork* w = new ProveWork();
  CHECK(napi_get_value_external(env, argv[0], reinterpret_cast<void**>(&w->c)));
  CHECK(napi_get_value_external(env, argv[1], reinterpret_cast<void**>(&w->prog)));
  void* d = nullptr;
  CHECK(napi_get_buffer_info(env, argv[2], &d, &w->in_len));
  w->in = static_cast<const uint8_t*>(d);
  CHECK(napi_create_reference(env, argv[0], 1, &w->ctx_ref));
  CHECK(napi_create_reference(env, argv[1], 1, &w->prog_ref));
  CHECK(napi_create_reference(env, argv[2], 1, &w->in_ref));
  return start_prove(env, w, argv, argc, 3);
}

napi_value Info(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  CHECK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  Ctx* c = nullptr;
  CHECK(napi_get_value_external(env, argv[0], reinterpret_cast<void**>(&c)));
  uint32_t v[5];
  nzcb_ctx_info(c->ctx, v);
  napi_value obj;
  napi_create_object(env, &obj);
  const char* names[5] = {"domainSize", "nPublic", "nVars", "nAdditions", "nConstraints"};
  for (int i = 0; i < 5; i++) {
    napi_value x;
    napi_create_uint32(env, v[i], &x);
    napi_set_named_property(env, obj, names[i], x);
  }
  return obj;
}

napi_value Version(napi_env env, napi_callback_info) {
  napi_value s;
  napi_create_string_utf8(env, nzcb_version(), NAPI_AUTO_LENGTH, &s);
  return s;
}

napi_value DeviceCount(napi_env env, napi_callback_info) {
  napi_value s;
  napi_create_int32(env, nzcb_device_count(), &s);
  return s;
}

// buffer argument i -> (data, len); false if not a Buffer
bool buf_arg(napi_env env, napi_value v, const uint8_t** data, size_t* len) {
  void* d = nullptr;
  if (napi_get_buffer_info(env, v, &d, len) != napi_ok) return false;
  *data = static_cast<const uint8_t*>(d);
  return true;
}

napi_value json_string(napi_env env, const std::string& s) {
  napi_value v;
  napi_create_string_utf8(env, s.c_str(), s.size(), &v);
  return v;
}

// vkFromZkey(zkey: Buffer) -> Buffer (NZCB_VK_BYTES); snarkjs `zkey export verificationkey`
napi_value VkFromZkey(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  CHECK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  const uint8_t* z;
  size_t zl;
  if (argc < 1 || !buf_arg(env, argv[0], &z, &zl)) {
    napi_throw_type_error(env, nullptr, "vkFromZkey(zkey: Buffer)");
    return nullptr;
  }
  void* out = nullptr;
  napi_value res;
  CHECK(napi_create_buffer(env, NZCB_VK_BYTES, &out, &res));
  nzcb_err err{};
  if (nzcb_vk_from_zkey(z, zl, static_cast<uint8_t*>(out), &err) != 0) {
    napi_throw(env, make_error(env, err.code, err.msg));
    return nullptr;
  }
  return res;
}

// vkFromZkeyFile(path: string) -> Buffer (NZCB_VK_BYTES): the zkey is memory-mapped by the
// library, so files past a Buffer's 2 GiB limit (nzcp_live_final.zkey) work
napi_value VkFromZkeyFile(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  CHECK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  std::string path;
  if (argc < 1 || !str_arg(env, argv[0], &path)) {
    napi_throw_type_error(env, nullptr, "vkFromZkeyFile(path: string)");
    return nullptr;
  }
  void* out = nullptr;
  napi_value res;
  CHECK(napi_create_buffer(env, NZCB_VK_BYTES, &out, &res));
  nzcb_err err{};
  if (nzcb_vk_from_zkey_file(path.c_str(), static_cast<uint8_t*>(out), &err) != 0) {
    napi_throw(env, make_error(env, err.code, err.msg));
    return nullptr;
  }
  return res;
}

// remapWitnessProgram(program: Buffer, ownSym: Buffer, targetSym: Buffer) -> Buffer
// (nzcb_wprog_remap); throws with .unmatched when target signals have no counterpart
napi_value RemapWitnessProgram(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  CHECK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  const uint8_t *prog, *own, *tgt;
  size_t pl, ol, tl;
  if (argc < 3 || !buf_arg(env, argv[0], &prog, &pl) || !buf_arg(env, argv[1], &own, &ol) ||
      !buf_arg(env, argv[2], &tgt, &tl)) {
    napi_throw_type_error(env, nullptr, "remapWitnessProgram(program: Buffer, ownSym: Buffer, targetSym: Buffer)");
    return nullptr;
  }
  uint8_t* out = nullptr;
  size_t out_len = 0;
  uint32_t miss = 0;
  nzcb_err err{};
  if (nzcb_wprog_remap(prog, pl, reinterpret_cast<const char*>(own), ol, reinterpret_cast<const char*>(tgt), tl, &out,
                       &out_len, &miss, &err) != 0) {
    napi_value e = make_error(env, err.code, err.msg);
    napi_value m;
    napi_create_uint32(env, miss, &m);
    napi_set_named_property(env, e, "unmatched", m);
    napi_throw(env, e);
    return nullptr;
  }
  void* dst = nullptr;
  napi_value res;
  const napi_status stc = napi_create_buffer_copy(env, out_len, out, &dst, &res);
  nzcb_free(out);
  CHECK(stc);
  return res;
}

// vkToJson(vk: Buffer) -> string (verification_key.json)
napi_value VkToJson(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  CHECK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  const uint8_t* vk;
  size_t vl;
  if (argc < 1 || !buf_arg(env, argv[0], &vk, &vl) || vl != NZCB_VK_BYTES) {
    napi_throw_type_error(env, nullptr, "vkToJson(vk: Buffer)");
    return nullptr;
  }
  std::string s((size_t)nzcb_vk_to_json(vk, nullptr, 0), '\0');
  nzcb_vk_to_json(vk, &s[0], s.size());
  s.resize(std::strlen(s.c_str()));
  return json_string(env, s);
}

// verify(vk: Buffer, proof: Buffer, pub: Buffer, transcriptPublic: bool) -> bool (snarkjs plonk.verify)
napi_value Verify(napi_env env, napi_callback_info info) {
  size_t argc = 4;
  napi_value argv[4];
  CHECK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  const uint8_t *vk, *proof, *pub;
  size_t vl, pl, ul;
  if (argc < 3 || !buf_arg(env, argv[0], &vk, &vl) || !buf_arg(env, argv[1], &proof, &pl) ||
      !buf_arg(env, argv[2], &pub, &ul) || vl != NZCB_VK_BYTES || pl != NZCB_PROOF_BYTES || ul % 32) {
    napi_throw_type_error(env, nullptr, "verify(vk: Buffer, proof: Buffer, pub: Buffer, transcriptPublic)");
    return nullptr;
  }
  bool tp = true;
  if (argc > 3) napi_get_value_bool(env, argv[3], &tp);
  int valid = 0;
  nzcb_err err{};
  if (nzcb_verify(vk, proof, pub, (int)(ul / 32), tp ? 1 : 0, &valid, &err) != 0) {
    napi_throw(env, make_error(env, err.code, err.msg));
    return nullptr;
  }
  napi_value r;
  napi_get_boolean(env, valid != 0, &r);
  return r;
}

// calldata(proof: Buffer, pub: Buffer) -> string (snarkjs `zkey export soliditycalldata`)
napi_value Calldata(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  CHECK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  const uint8_t *proof, *pub;
  size_t pl, ul;
  if (argc < 2 || !buf_arg(env, argv[0], &proof, &pl) || !buf_arg(env, argv[1], &pub, &ul) ||
      pl != NZCB_PROOF_BYTES || ul % 32) {
    napi_throw_type_error(env, nullptr, "calldata(proof: Buffer, pub: Buffer)");
    return nullptr;
  }
  std::string s((size_t)nzcb_proof_to_calldata(proof, pub, (int)(ul / 32), nullptr, 0), '\0');
  nzcb_proof_to_calldata(proof, pub, (int)(ul / 32), &s[0], s.size());
  s.resize(std::strlen(s.c_str()));
  return json_string(env, s);
}

// vkToSolidity(vk: Buffer, name: string, transcriptPublic: bool) -> string
// (snarkjs `zkey export solidityverifier`)
napi_value VkToSolidity(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  CHECK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  const uint8_t* vk;
  size_t vl;
  char name[80] = {0};
  size_t nl = 0;
  bool tp = true;
  if (argc < 3 || !buf_arg(env, argv[0], &vk, &vl) || vl != NZCB_VK_BYTES ||
      napi_get_value_string_utf8(env, argv[1], name, sizeof(name), &nl) != napi_ok ||
      napi_get_value_bool(env, argv[2], &tp) != napi_ok) {
    napi_throw_type_error(env, nullptr, "vkToSolidity(vk: Buffer, name: string, transcriptPublic: boolean)");
    return nullptr;
  }
  const int need = nzcb_vk_to_solidity(vk, name, tp ? 1 : 0, nullptr, 0);
  if (need < 0) {
    napi_throw_error(env, nullptr, "solidity verifier: bad verification key or contract name");
    return nullptr;
  }
  std::string s((size_t)need, '\0');
  nzcb_vk_to_solidity(vk, name, tp ? 1 : 0, &s[0], s.size());
  s.resize(std::strlen(s.c_str()));
  return json_string(env, s);
}

// nzcpWitness(inputs: Buffer, count: number, params: [isLive, maxTbsBytes, maxArrayLenVC,
// maxMapLenVC], device: number) -> Buffer of count nzcb_nzcp_record (include/nzcb.h).
// Synchronous: one launch of the nzcp witness kernel, well under a millisecond.
napi_value NzcpWitness(napi_env env, napi_callback_info info) {
  size_t argc = 4;
  napi_value argv[4];
  CHECK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  void* data = nullptr;
  size_t len = 0;
  CHECK(napi_get_buffer_info(env, argv[0], &data, &len));
  int32_t count = 0, device = 0;
  CHECK(napi_get_value_int32(env, argv[1], &count));
  nzcb_nzcp_params prm{};
  int32_t* fields[4] = {&prm.is_live, &prm.max_tbs_bytes, &prm.max_array_len_vc, &prm.max_map_len_vc};
  for (uint32_t i = 0; i < 4; i++) {
    napi_value v;
    CHECK(napi_get_element(env, argv[2], i, &v));
    CHECK(napi_get_value_int32(env, v, fields[i]));
  }
  if (argc > 3) napi_get_value_int32(env, argv[3], &device);
  if (count < 0 || len != nzcb_nzcp_input_signals(&prm) * 32 * (size_t)count) {
    napi_throw_error(env, nullptr, "nzcpWitness: inputs must be count x input signals x 32 bytes");
    return nullptr;
  }
  void* out_data = nullptr;
  napi_value out;
  CHECK(napi_create_buffer(env, sizeof(nzcb_nzcp_record) * (size_t)(count ? count : 1), &out_data, &out));
  nzcb_err err{};
  int rc = nzcb_nzcp_witness(device, &prm, static_cast<const uint8_t*>(data), count,
                             static_cast<nzcb_nzcp_record*>(out_data), &err);
  if (rc) {
    napi_throw(env, make_error(env, err.code, err.msg));
    return nullptr;
  }
  return out;
}

// plonkSetup(r1cs: Buffer, ptau: Buffer, device: number) -> Buffer (the zkey):
// snarkjs `plonk setup` (nzcb_plonk_setup). Synchronous: a one-off key generation.
napi_value PlonkSetup(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  CHECK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  const uint8_t *r1cs, *ptau;
  size_t rl, pl;
  int32_t device = 0;
  if (argc < 2 || !buf_arg(env, argv[0], &r1cs, &rl) || !buf_arg(env, argv[1], &ptau, &pl)) {
    napi_throw_type_error(env, nullptr, "plonkSetup(r1cs: Buffer, ptau: Buffer, device?: number)");
    return nullptr;
  }
  if (argc > 2) napi_get_value_int32(env, argv[2], &device);
  uint8_t* zk = nullptr;
  size_t zl = 0;
  nzcb_err err{};
  if (nzcb_plonk_setup(r1cs, rl, ptau, pl, device, &zk, &zl, &err)) {
    napi_throw(env, make_error(env, err.code, err.msg));
    return nullptr;
  }
  void* out_data = nullptr;
  napi_value out;
  napi_status stc = napi_create_buffer_copy(env, zl, zk, &out_data, &out);
  nzcb_free(zk);
  CHECK(stc);
  return out;
}

napi_value Init(napi_env env, napi_value exports) {
  napi_property_descriptor props[] = {
      {"createContext", nullptr, CreateContext, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"prove", nullptr, Prove, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"info", nullptr, Info, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"version", nullptr, Version, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"deviceCount", nullptr, DeviceCount, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"vkFromZkey", nullptr, VkFromZkey, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"vkFromZkeyFile", nullptr, VkFromZkeyFile, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"remapWitnessProgram", nullptr, RemapWitnessProgram, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"vkToJson", nullptr, VkToJson, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"verify", nullptr, Verify, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"calldata", nullptr, Calldata, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"vkToSolidity", nullptr, VkToSolidity, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"nzcpWitness", nullptr, NzcpWitness, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"plonkSetup", nullptr, PlonkSetup, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"createContextFile", nullptr, CreateContextFile, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"createWitnessProgram", nullptr, CreateWitnessProgram, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"calculateWitness", nullptr, CalculateWitness, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"fullProveDevice", nullptr, FullProveDevice, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"setLanes", nullptr, SetLanes, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"releaseContext", nullptr, ReleaseContext, nullptr, nullptr, nullptr, napi_default, nullptr},
  };
  napi_define_properties(env, exports, sizeof(props) / sizeof(props[0]), props);
  return exports;
}

}  // namespace

NAPI_MODULE(NODE_GYP_MODULE_NAME, Init)
