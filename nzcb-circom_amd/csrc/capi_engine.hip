// C-ABI: engine, device memory and kernel-level entry points (include/nzcb.h).
#include <chrono>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

#include "../../include/nzcb_internal.h"
#include "engine.h"
#include "lagrange.h"

namespace nzcb {

Engine::Engine(int dev, int max_log_ntt, size_t max_msm_points) : device(dev) {
  NZ_HIP(hipSetDevice(dev));
  NZ_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
  if (max_log_ntt >= 0) ntt_tables.init(max_log_ntt, stream);
  if (max_msm_points) msm_scratch.init(max_msm_points);
}

Engine::~Engine() {
  if (stream) (void)hipStreamDestroy(stream);
}

void set_err(nzcb_err* err, int code, const char* msg) {
  if (!err) return;
  err->code = code;
  std::snprintf(err->msg, sizeof(err->msg), "%s", msg);
}

// ---- guard words past device buffers (common.h GuardScope) ---------------------------
thread_local int g_guard_scope = 0;
namespace {
struct GuardRec {
  size_t bytes;
  int device;
};
std::mutex g_guard_mu;
std::map<void*, GuardRec>& guard_map() {
  static std::map<void*, GuardRec> m;
  return m;
}
}  // namespace

void guard_register(void* base, size_t bytes) {
  NZ_HIP(hipMemset((uint8_t*)base + bytes, kGuardByte, kGuardBytes));
  int dev = 0;
  NZ_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(g_guard_mu);
  guard_map()[base] = GuardRec{bytes, dev};
}

void guard_unregister(void* base) {
  std::lock_guard<std::mutex> lk(g_guard_mu);
  guard_map().erase(base);
}

int guard_check(int device, size_t* checked, std::string* report) {
  std::vector<std::pair<void*, GuardRec>> recs;
  {
    std::lock_guard<std::mutex> lk(g_guard_mu);
    for (auto& kv : guard_map())
      if (device < 0 || kv.second.device == device) recs.push_back(kv);
  }
  std::vector<uint8_t> h(kGuardBytes);
  int bad = 0;
  for (auto& r : recs) {
    NZ_HIP(hipMemcpy(h.data(), (uint8_t*)r.first + r.second.bytes, kGuardBytes, hipMemcpyDeviceToHost));
    size_t k = 0;
    while (k < kGuardBytes && h[k] == kGuardByte) k++;
    if (k == kGuardBytes) continue;
    bad++;
    if (report && bad <= 8) {
      char line[160];
      std::snprintf(line, sizeof(line), "%sbuffer %p (%zu bytes, device %d): guard byte %zu overwritten",
                    report->empty() ? "" : "; ", r.first, r.second.bytes, r.second.device, k);
      *report += line;
    }
  }
  if (checked) *checked = recs.size();
  return bad;
}

__global__ void k_guard_poke(uint32_t* p, size_t at) {
  if (threadIdx.x == 0) p[at] = 0;
}

}  // namespace nzcb

using namespace nzcb;

struct nzcb_engine {
  Engine eng;
  nzcb_engine(int d, int l, size_t m) : eng(d, l, m) {}
};

#define NZ_GUARD_BEGIN try {
#define NZ_GUARD_END(err)                                   \
  }                                                         \
  catch (const nzcb::Error& e) {                            \
    set_err(err, e.code, e.what());                         \
    return e.code;                                          \
  }                                                         \
  catch (const std::exception& e) {                         \
    set_err(err, NZCB_ERR_INTERNAL, e.what());              \
    return NZCB_ERR_INTERNAL;                               \
  }

__global__ void fe_mul_kernel_r(const Fr* a, const Fr* b, Fr* o, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) o[i] = a[i] * b[i];
}
__global__ void fe_mul_kernel_q(const Fq* a, const Fq* b, Fq* o, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) o[i] = a[i] * b[i];
}

// uniform-ish Fr in Montgomery form: 253 random bits (< r) from a splitmix64 stream per element
__global__ void random_fr_kernel(Fr* out, size_t n, uint64_t seed) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t x = seed ^ (0x9E3779B97F4A7C15ULL * (i + 1));
  Fr v;
  for (int k = 0; k < 4; k++) {
    x += 0x9E3779B97F4A7C15ULL;
    uint64_t z = x;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    z ^= z >> 31;
    v.v[2 * k] = (uint32_t)z;
    v.v[2 * k + 1] = (uint32_t)(z >> 32);
  }
  v.v[7] &= 0x1fffffffu;
  out[i] = to_mont(v);
}

static void affine_out(const G1xyzz& r, uint8_t* out) {
  G1Affine a = xyzz_to_affine(r);
  Fq x = a.is_inf() ? Fq::zero() : from_mont(a.x);
  Fq y = a.is_inf() ? Fq::zero() : from_mont(a.y);
  std::memcpy(out, x.v, 32);
  std::memcpy(out + 32, y.v, 32);
}

extern "C" {

const char* nzcb_version(void) { return "nzcb-mi355x 0.1.0 (gfx950)"; }

int nzcb_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

void nzcb_free(void* p) { std::free(p); }

nzcb_engine* nzcb_engine_create(int device, int max_log_ntt, size_t max_msm_points, nzcb_err* err) {
  try {
    return new nzcb_engine(device, max_log_ntt, max_msm_points);
  } catch (const nzcb::Error& e) {
    set_err(err, e.code, e.what());
  } catch (const std::exception& e) {
    set_err(err, NZCB_ERR_INTERNAL, e.what());
  }
  return nullptr;
}

void nzcb_engine_destroy(nzcb_engine* e) { delete e; }

void* nzcb_dev_alloc(size_t bytes) {
  void* p = nullptr;
  if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
  return p;
}
void* nzcb_dev_alloc_on(int device, size_t bytes) {
  int cur = 0;
  if (hipGetDevice(&cur) != hipSuccess || hipSetDevice(device) != hipSuccess) return nullptr;
  void* p = nullptr;
  if (hipMalloc(&p, bytes) != hipSuccess) p = nullptr;
  (void)hipSetDevice(cur);
  return p;
}
void nzcb_dev_free(void* p) {
  if (p) (void)hipFree(p);
}
int nzcb_memcpy_h2d(void* dst, const void* src, size_t bytes) {
  return hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice) == hipSuccess ? 0 : NZCB_ERR_HIP;
}
int nzcb_memcpy_d2h(void* dst, const void* src, size_t bytes) {
  return hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost) == hipSuccess ? 0 : NZCB_ERR_HIP;
}
// Complete on return: a device-to-device hipMemcpy may return before the copy is done,
// and callers hand the destination to work on non-blocking streams next (msmsplit).
int nzcb_memcpy_d2d(void* dst, const void* src, size_t bytes) {
  if (hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, nullptr) != hipSuccess) return NZCB_ERR_HIP;
  return hipStreamSynchronize(nullptr) == hipSuccess ? 0 : NZCB_ERR_HIP;
}
// Ordered on `stream` (a hipStream_t, e.g. torch.cuda.current_stream().cuda_stream): work
// enqueued on that stream afterwards (a collective reading dst) sees the copy; no host wait.
int nzcb_memcpy_d2d_async(void* dst, const void* src, size_t bytes, void* stream) {
  return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream) == hipSuccess ? 0
                                                                                              : NZCB_ERR_HIP;
}

int nzcb_engine_ntt_dev(nzcb_engine* e, const void* in, void* out, int log_n, int inverse, nzcb_err* err) {
  NZ_GUARD_BEGIN
  Engine& g = e->eng;
  NZ_HIP(hipSetDevice(g.device));
  ntt(g.ntt_tables, (const Fr*)in, (Fr*)out, log_n, inverse != 0, g.stream);
  NZ_HIP(hipStreamSynchronize(g.stream));
  return 0;
  NZ_GUARD_END(err)
}

int nzcb_engine_ntt(nzcb_engine* e, const uint8_t* in_lem, uint8_t* out_lem, int log_n, int inverse, nzcb_err* err) {
  NZ_GUARD_BEGIN
  Engine& g = e->eng;
  NZ_HIP(hipSetDevice(g.device));
  size_t n = size_t(1) << log_n;
  DevBuf<Fr> a(n), b(n);
  NZ_HIP(hipMemcpyAsync(a.p, in_lem, n * 32, hipMemcpyHostToDevice, g.stream));
  ntt(g.ntt_tables, a.p, b.p, log_n, inverse != 0, g.stream);
  NZ_HIP(hipMemcpyAsync(out_lem, b.p, n * 32, hipMemcpyDeviceToHost, g.stream));
  NZ_HIP(hipStreamSynchronize(g.stream));
  return 0;
  NZ_GUARD_END(err)
}

int nzcb_engine_time_ntt(nzcb_engine* e, const void* in, void* out, int log_n, int inverse, int reps, double* ms,
                         nzcb_err* err) {
  NZ_GUARD_BEGIN
  Engine& g = e->eng;
  NZ_HIP(hipSetDevice(g.device));
  hipEvent_t e0, e1;
  NZ_HIP(hipEventCreate(&e0));
  NZ_HIP(hipEventCreate(&e1));
  NZ_HIP(hipEventRecord(e0, g.stream));
  for (int i = 0; i < reps; i++) ntt(g.ntt_tables, (const Fr*)in, (Fr*)out, log_n, inverse != 0, g.stream);
  NZ_HIP(hipEventRecord(e1, g.stream));
  NZ_HIP(hipEventSynchronize(e1));
  float t = 0;
  NZ_HIP(hipEventElapsedTime(&t, e0, e1));
  *ms = t / (reps > 0 ? reps : 1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return 0;
  NZ_GUARD_END(err)
}

int nzcb_engine_msm_dev(nzcb_engine* e, const void* bases, const void* scalars, size_t n, int scalars_mont,
                        uint8_t* out_affine, nzcb_err* err) {
  NZ_GUARD_BEGIN
  Engine& g = e->eng;
  NZ_HIP(hipSetDevice(g.device));
  G1xyzz r = msm(g.msm_scratch, (const G1Affine*)bases, (const Fr*)scalars, n, scalars_mont != 0, g.stream);
  affine_out(r, out_affine);
  return 0;
  NZ_GUARD_END(err)
}

int nzcb_engine_msm(nzcb_engine* e, const uint8_t* bases_lem, const uint8_t* scalars, size_t n, int scalars_mont,
                    uint8_t* out_affine, nzcb_err* err) {
  NZ_GUARD_BEGIN
  Engine& g = e->eng;
  NZ_HIP(hipSetDevice(g.device));
  DevBuf<G1Affine> b(n ? n : 1);
  DevBuf<Fr> s(n ? n : 1);
  NZ_HIP(hipMemcpyAsync(b.p, bases_lem, n * 64, hipMemcpyHostToDevice, g.stream));
  NZ_HIP(hipMemcpyAsync(s.p, scalars, n * 32, hipMemcpyHostToDevice, g.stream));
  G1xyzz r = msm(g.msm_scratch, b.p, s.p, n, scalars_mont != 0, g.stream);
  affine_out(r, out_affine);
  return 0;
  NZ_GUARD_END(err)
}

int nzcb_engine_random_fr(nzcb_engine* e, void* dev_out, size_t n, uint64_t seed, nzcb_err* err) {
  NZ_GUARD_BEGIN
  Engine& g = e->eng;
  NZ_HIP(hipSetDevice(g.device));
  hipLaunchKernelGGL(random_fr_kernel, dim3(grid_for(n, 256, 1u << 30)), dim3(256), 0, g.stream, (Fr*)dev_out, n,
                     seed);
  NZ_HIP(hipGetLastError());
  NZ_HIP(hipStreamSynchronize(g.stream));
  return 0;
  NZ_GUARD_END(err)
}

int nzcb_engine_fixed_base(nzcb_engine* e, const void* dev_scalars_mont, size_t n, void* dev_out, nzcb_err* err) {
  NZ_GUARD_BEGIN
  Engine& g = e->eng;
  NZ_HIP(hipSetDevice(g.device));
  launch_fixed_base((const Fr*)dev_scalars_mont, n, (G1Affine*)dev_out, g.stream);
  NZ_HIP(hipStreamSynchronize(g.stream));
  return 0;
  NZ_GUARD_END(err)
}

int nzcb_engine_lagrange_basis(nzcb_engine* e, const void* dev_ptau, size_t ptau_n, int log_n, void* dev_out,
                               nzcb_err* err) {
  NZ_GUARD_BEGIN
  Engine& g = e->eng;
  NZ_HIP(hipSetDevice(g.device));
  lagrange_basis((const G1Affine*)dev_ptau, ptau_n, log_n, (G1Affine*)dev_out, g.stream);
  return 0;
  NZ_GUARD_END(err)
}

int nzcb_engine_time_msm(nzcb_engine* e, const void* bases, const void* scalars, size_t n, int scalars_mont, int reps,
                         double* ms, double* acc_ms, nzcb_err* err) {
  NZ_GUARD_BEGIN
  Engine& g = e->eng;
  NZ_HIP(hipSetDevice(g.device));
  MsmScratch& sc = g.msm_scratch;
  sc.prof = true;
  sc.prof_ms = 0;
  sc.prof_launches = 0;
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < reps; i++) (void)msm(sc, (const G1Affine*)bases, (const Fr*)scalars, n, scalars_mont != 0, g.stream);
  *ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() / (reps ? reps : 1);
  *acc_ms = sc.prof_ms / (sc.prof_launches ? sc.prof_launches : 1);
  sc.prof = false;
  return 0;
  NZ_GUARD_END(err)
}

int nzcb_engine_msm_fixed_dev(nzcb_engine* e, const void* bases, size_t n_table, const void* scalars, size_t n,
                              int scalars_mont, uint8_t* out_affine, nzcb_err* err) {
  return nzcb_engine_msm_table_dev(e, bases, n_table, scalars, n, scalars_mont, 0, 0, out_affine, err);
}

int nzcb_engine_msm_table_dev(nzcb_engine* e, const void* bases, size_t n_table, const void* scalars, size_t n,
                              int scalars_mont, int window, int sparse, uint8_t* out_affine, nzcb_err* err) {
  NZ_GUARD_BEGIN
  Engine& g = e->eng;
  NZ_HIP(hipSetDevice(g.device));
  if (n > n_table) throw Error(NZCB_ERR_ARG, "msm larger than its base table");
  if (window && (window < 16 || window > 20)) throw Error(NZCB_ERR_ARG, "msm table window: 16..20");
  MsmBaseTable t;
  t.build((const G1Affine*)bases, n_table, window ? window : fixed_base_window(), g.stream);
  t.sparse = sparse != 0;
  MsmScratch sc;
  sc.init(n ? n : 1, true);
  G1xyzz r = msm(sc, (const G1Affine*)bases, (const Fr*)scalars, n, scalars_mont != 0, g.stream, &t);
  affine_out(r, out_affine);
  return 0;
  NZ_GUARD_END(err)
}

int nzcb_engine_msm_sets_dev(nzcb_engine* e, const void* bases, size_t n_table, const void* const* scalars, int sets,
                             size_t n, int scalars_mont, uint8_t* out_affine, nzcb_err* err) {
  NZ_GUARD_BEGIN
  Engine& g = e->eng;
  NZ_HIP(hipSetDevice(g.device));
  if (n > n_table) throw Error(NZCB_ERR_ARG, "msm larger than its base table");
  if (sets < 1 || sets > 3 || !scalars) throw Error(NZCB_ERR_ARG, "msm sets: 1..3 scalar vectors");
  MsmBaseTable t;
  t.build((const G1Affine*)bases, n_table, lagrange_window(), g.stream);
  t.sparse = true;
  MsmScratch sc;
  sc.init(n ? n : 1, true, 3, false);
  G1xyzz r[3];
  msm_enqueue_sets(sc, (const Fr* const*)scalars, sets, n, scalars_mont != 0, g.stream, &t);
  msm_finish_sets(sc, g.stream, r);
  for (int k = 0; k < sets; k++) affine_out(r[k], out_affine + 64 * k);
  return 0;
  NZ_GUARD_END(err)
}

int nzcb_engine_time_msm2(nzcb_engine* e, const void* bases, const void* scalars, size_t n, int scalars_mont,
                          int fixed_base, int reps, double* out, nzcb_err* err) {
  NZ_GUARD_BEGIN
  Engine& g = e->eng;
  NZ_HIP(hipSetDevice(g.device));
  std::unique_ptr<MsmBaseTable> t;
  std::unique_ptr<MsmScratch> own;
  MsmScratch* sc = &g.msm_scratch;
  double table_ms = 0;
  if (fixed_base) {  // 2: the Lagrange table's schedule (window 17, sparse); 3: window 17, dense schedule
    auto t0 = std::chrono::steady_clock::now();
    t.reset(new MsmBaseTable());
    t->build((const G1Affine*)bases, n, fixed_base >= 2 ? lagrange_window() : fixed_base_window(), g.stream);
    t->sparse = fixed_base == 2;
    NZ_HIP(hipStreamSynchronize(g.stream));
    table_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    own.reset(new MsmScratch());
    own->init(n, true);
    sc = own.get();
  }
  // warm-up: three untimed runs in the timed mode (the first MSM of a process also pays lazy
  // code-object loads and the clock ramp after the NTT rows, and the first profiled one
  // creates the phase events: ~8 ms of host time that put round 3's and round 4's first 2^18
  // row 36-100 % above its phase sum)
  sc->prof = true;
  sc->prof_phases = true;
  for (int w = 0; w < 3; w++)
    (void)msm(*sc, (const G1Affine*)bases, (const Fr*)scalars, n, scalars_mont != 0, g.stream, t.get());
  sc->prof_ms = 0;
  sc->prof_launches = 0;
  sc->prof_entries = 0;
  for (double& x : sc->phase_ms) x = 0;
  sc->host_ms = sc->enqueue_ms = sc->sort_host_ms = 0;
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < reps; i++)
    (void)msm(*sc, (const G1Affine*)bases, (const Fr*)scalars, n, scalars_mont != 0, g.stream, t.get());
  const double r = reps > 0 ? reps : 1;
  out[0] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() / r;
  for (int i = 0; i < 7; i++) out[1 + i] = sc->phase_ms[i] / r;
  out[8] = table_ms;
  out[9] = (double)sc->prof_entries / r;
  out[10] = sc->host_ms / r;
  out[11] = sc->enqueue_ms / r;
  out[12] = sc->sort_host_ms / r;
  sc->prof = sc->prof_phases = false;
  return 0;
  NZ_GUARD_END(err)
}

int nzcb_engine_fr_mul(nzcb_engine* e, const uint8_t* a_lem, const uint8_t* b_lem, uint8_t* out_lem, size_t n,
                       int field_q, nzcb_err* err) {
  NZ_GUARD_BEGIN
  Engine& g = e->eng;
  NZ_HIP(hipSetDevice(g.device));
  DevBuf<Fr> a(n), b(n), o(n);
  NZ_HIP(hipMemcpyAsync(a.p, a_lem, n * 32, hipMemcpyHostToDevice, g.stream));
  NZ_HIP(hipMemcpyAsync(b.p, b_lem, n * 32, hipMemcpyHostToDevice, g.stream));
  if (field_q)
    hipLaunchKernelGGL(fe_mul_kernel_q, dim3(grid_for(n, 256)), dim3(256), 0, g.stream, (const Fq*)a.p,
                       (const Fq*)b.p, (Fq*)o.p, n);
  else
    hipLaunchKernelGGL(fe_mul_kernel_r, dim3(grid_for(n, 256)), dim3(256), 0, g.stream, a.p, b.p, o.p, n);
  NZ_HIP(hipGetLastError());
  NZ_HIP(hipMemcpyAsync(out_lem, o.p, n * 32, hipMemcpyDeviceToHost, g.stream));
  NZ_HIP(hipStreamSynchronize(g.stream));
  return 0;
  NZ_GUARD_END(err)
}

// ---- resident fixed-base MSM tables (the serving ranks of nzcb_ctx_set_msm_split) ----
struct nzcb_msm_table {
  int device = 0;
  size_t n = 0;
  MsmBaseTable table;
  MsmScratch sc;
  hipStream_t st = nullptr;
  ~nzcb_msm_table() {
    (void)hipSetDevice(device);
    if (st) (void)hipStreamDestroy(st);
  }
};

nzcb_msm_table* nzcb_msm_table_create(int device, const void* dev_bases, size_t n, nzcb_err* err) {
  try {
    if (!dev_bases || n == 0) throw Error(NZCB_ERR_ARG, "msm table: no bases");
    NZ_HIP(hipSetDevice(device));
    auto t = new nzcb_msm_table();
    try {
      t->device = device;
      t->n = n;
      NZ_HIP(hipStreamCreateWithFlags(&t->st, hipStreamNonBlocking));
      t->table.build((const G1Affine*)dev_bases, n, fixed_base_window(), t->st);
      t->sc.init(n, true, 1, false);
      NZ_HIP(hipStreamSynchronize(t->st));
    } catch (...) {
      delete t;
      throw;
    }
    return t;
  } catch (const Error& e) {
    set_err(err, e.code, e.what());
  } catch (const std::exception& e) {
    set_err(err, NZCB_ERR_INTERNAL, e.what());
  }
  return nullptr;
}

nzcb_msm_table* nzcb_msm_table_create_lagrange(int device, const void* dev_ptau, size_t ptau_n, int log_n, size_t lo,
                                               size_t hi, nzcb_err* err) {
  try {
    if (!dev_ptau || log_n < 1 || log_n > 28) throw Error(NZCB_ERR_ARG, "lagrange table: bad PTau or domain");
    const size_t nl = ((size_t)1 << log_n) + 2;
    if (ptau_n < nl) throw Error(NZCB_ERR_ARG, "lagrange table: fewer than n + 2 PTau points");
    if (lo >= hi || hi > nl) throw Error(NZCB_ERR_ARG, "lagrange table: bad point range");
    NZ_HIP(hipSetDevice(device));
    auto t = new nzcb_msm_table();
    try {
      t->device = device;
      t->n = hi - lo;
      NZ_HIP(hipStreamCreateWithFlags(&t->st, hipStreamNonBlocking));
      {  // the whole basis (the inverse NTT needs every point), then the range's table
        DevBuf<G1Affine> basis(nl);
        lagrange_basis((const G1Affine*)dev_ptau, ptau_n, log_n, basis.p, t->st);
        t->table.build(basis.p + lo, hi - lo, lagrange_window(), t->st);
        t->table.sparse = lagrange_sparse();
        NZ_HIP(hipStreamSynchronize(t->st));
      }
      t->sc.init(hi - lo, true, 1, false);
    } catch (...) {
      delete t;
      throw;
    }
    return t;
  } catch (const Error& e) {
    set_err(err, e.code, e.what());
  } catch (const std::exception& e) {
    set_err(err, NZCB_ERR_INTERNAL, e.what());
  }
  return nullptr;
}

int nzcb_msm_table_run(nzcb_msm_table* t, const void* dev_scalars, size_t count, int scalars_mont,
                       uint8_t* out_affine, nzcb_err* err) {
  NZ_GUARD_BEGIN
  if (!t || !out_affine || (count && !dev_scalars)) throw Error(NZCB_ERR_ARG, "msm table: null argument");
  if (count > t->n) throw Error(NZCB_ERR_ARG, "msm larger than its base table");
  NZ_HIP(hipSetDevice(t->device));
  G1xyzz r = count ? msm(t->sc, nullptr, (const Fr*)dev_scalars, count, scalars_mont != 0, t->st, &t->table)
                   : G1xyzz::inf();
  affine_out(r, out_affine);
  return 0;
  NZ_GUARD_END(err)
}

void nzcb_msm_table_destroy(nzcb_msm_table* t) { delete t; }

int nzcb_debug_guard_check(int device, size_t* checked, int* damaged, nzcb_err* err) {
  NZ_GUARD_BEGIN
  std::string report;
  const int bad = guard_check(device, checked, &report);
  if (damaged) *damaged = bad;
  if (bad) throw Error(NZCB_ERR_INTERNAL, std::to_string(bad) + " damaged guard(s): " + report);
  if (err) err->code = 0;
  return 0;
  NZ_GUARD_END(err)
}

int nzcb_debug_guard_selftest(int device, nzcb_err* err) {
  NZ_GUARD_BEGIN
  NZ_HIP(hipSetDevice(device));
  size_t before = 0;
  guard_check(device, &before, nullptr);
  int bad = 0;
  {
    GuardScope gs;
    DevBuf<uint32_t> b(1000);
    // one word written 7 words past the end: inside the guard, so legal memory, and found
    hipLaunchKernelGGL(k_guard_poke, dim3(1), dim3(64), 0, nullptr, b.p, (size_t)1007);
    NZ_HIP(hipGetLastError());
    NZ_HIP(hipDeviceSynchronize());
    bad = guard_check(device, nullptr, nullptr);
  }
  const int after = guard_check(device, nullptr, nullptr);
  if (bad != 1 || after != 0)
    throw Error(NZCB_ERR_INTERNAL, "guard self-test: overrun found " + std::to_string(bad) + " time(s), " +
                                       std::to_string(after) + " left after release");
  if (err) err->code = 0;
  return 0;
  NZ_GUARD_END(err)
}

}  // extern "C"
