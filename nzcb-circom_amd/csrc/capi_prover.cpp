// C-ABI: prover context, proofs and snarkjs-format JSON (include/nzcb.h).
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/nzcb_internal.h"
#include "prover.h"

namespace nzcb {

// decimal string of a 32-byte little-endian integer (snarkjs stringifyBigInts)
std::string dec_le32(const uint8_t* le32) {
  uint32_t v[8];
  std::memcpy(v, le32, 32);
  std::string s;
  bool nz = true;
  while (nz) {
    uint64_t rem = 0;
    nz = false;
    for (int i = 7; i >= 0; i--) {
      uint64_t cur = (rem << 32) | v[i];
      v[i] = (uint32_t)(cur / 10);
      rem = cur % 10;
      if (v[i]) nz = true;
    }
    s.push_back((char)('0' + rem));
  }
  return std::string(s.rbegin(), s.rend());
}

}
using namespace nzcb;

struct nzcb_ctx {
  std::unique_ptr<Prover> p;                   // device 0, lane 0: owns that device's proving key
  std::vector<std::unique_ptr<Prover>> extra;  // device 0, lanes 1..: share it (nzcb_ctx_set_lanes)
  // devices 1.. of a device-set context (nzcb_ctx_create_devices): each holds its own
  // HBM-resident copy of the proving key in its lane 0 and the same number of lanes
  std::vector<std::unique_ptr<Prover>> dev_p;
  std::vector<std::vector<std::unique_ptr<Prover>>> dev_extra;
  nzcb_log_fn log_fn = nullptr;
  void* log_user = nullptr;
  // Concurrency (SURVEY.md §8b "Threading"): proofs hold `cfg` shared and take a lane from
  // the pool for their duration, so concurrent callers (the N-API addon's in-flight
  // promises, several host threads) run on different lanes at once; configuration calls
  // (lanes, logger, splits, transcript) hold `cfg` exclusively, after in-flight proofs.
  std::shared_mutex cfg;
  std::mutex pool_mu;
  std::condition_variable pool_cv;
  std::vector<Prover*> idle;  // lanes not proving; rebuilt by reset_pool (cfg held exclusively)
  double last_tm[11] = {0};   // phases of the last finished proof (nzcb_ctx_last_timings)
  // nzcb_debug_inject_fault: armed for the context's next proof, whichever lane takes it (a
  // per-lane flag left the other lanes of a multi-lane context armed)
  std::atomic<int> pending_fault{0};
  std::atomic<int> lane_alloc_fault{0};  // NZCB_FAULT_LANE_ALLOC: the next set_lanes growth fails
  Prover* lane(size_t i) { return i == 0 ? p.get() : extra[i - 1].get(); }
  size_t lanes() const { return 1 + extra.size(); }  // per device
  // every lane of every device (batch workers), device-interleaved so that a short batch
  // spreads over the devices first
  std::vector<Prover*> all() {
    std::vector<Prover*> v;
    for (size_t l = 0; l < lanes(); l++) {
      v.push_back(lane(l));
      for (size_t d = 0; d < dev_p.size(); d++) v.push_back(l == 0 ? dev_p[d].get() : dev_extra[d][l - 1].get());
    }
    return v;
  }
  // the lanes proofs may use: lane 0 of device 0 alone while a split covers it (the split's
  // commitments are lane 0's), else all of them
  std::vector<Prover*> usable() {
    if (p->split_send || !p->shards.empty()) return {p.get()};
    return all();
  }
  void reset_pool() {
    std::lock_guard<std::mutex> lk(pool_mu);
    idle = usable();
    std::reverse(idle.begin(), idle.end());  // lane 0 of device 0 is taken first
  }
  // a lane for one proof (blocks while all are proving), logging to `fn` or the context's logger
  Prover* acquire(nzcb_log_fn fn, void* user) {
    Prover* q;
    {
      std::unique_lock<std::mutex> lk(pool_mu);
      pool_cv.wait(lk, [&] { return !idle.empty(); });
      q = idle.back();
      idle.pop_back();
    }
    if (!fn) {
      fn = log_fn;
      user = log_user;
    }
    if (fn)
      q->log = [fn, user](const std::string& m) { fn(user, m.c_str()); };
    else
      q->log = nullptr;
    q->fault = pending_fault.exchange(0);
    return q;
  }
  void release(Prover* q) {
    {
      std::lock_guard<std::mutex> lk(pool_mu);
      std::memcpy(last_tm, q->tm, sizeof(last_tm));
      idle.push_back(q);
    }
    pool_cv.notify_one();
  }
};

namespace {

int fail(nzcb_err* err, int code, const char* msg) {
  set_err(err, code, msg);
  return code;
}

bool all_zero(const uint8_t* p, size_t n) {
  for (size_t i = 0; i < n; i++)
    if (p[i]) return false;
  return true;
}

std::string g1_json(const uint8_t* p) {
  if (all_zero(p, 64)) return "[\"0\",\"1\",\"0\"]";
  return "[\"" + dec_le32(p) + "\",\"" + dec_le32(p + 32) + "\",\"1\"]";
}

int copy_out(const std::string& s, char* out, size_t cap) {
  if (!out || cap < s.size() + 1) return (int)(s.size() + 1);
  std::memcpy(out, s.c_str(), s.size() + 1);
  return 0;
}

}  // namespace

extern "C" {

nzcb_ctx* nzcb_ctx_create(const uint8_t* zkey, size_t zkey_len, int device, nzcb_err* err) {
  try {
    auto* c = new nzcb_ctx();
    c->p.reset(new Prover(zkey, zkey_len, device));
    c->reset_pool();
    if (err) err->code = 0;
    return c;
  } catch (const Error& e) {
    set_err(err, e.code, e.what());
  } catch (const std::exception& e) {
    set_err(err, NZCB_ERR_INTERNAL, e.what());
  }
  return nullptr;
}

nzcb_ctx* nzcb_ctx_create_devices(const uint8_t* zkey, size_t zkey_len, const int* devices, int ndev, nzcb_err* err) {
  if (!devices || ndev < 1 || ndev > 64) {
    set_err(err, NZCB_ERR_ARG, "devices: 1..64 ids");
    return nullptr;
  }
  for (int i = 0; i < ndev; i++)
    for (int j = 0; j < i; j++)
      if (devices[i] == devices[j]) {
        set_err(err, NZCB_ERR_ARG, "devices: an id appears twice");
        return nullptr;
      }
  nzcb_ctx* c = nzcb_ctx_create(zkey, zkey_len, devices[0], err);
  if (!c) return nullptr;
  try {
    for (int i = 1; i < ndev; i++) {
      c->dev_p.emplace_back(new Prover(zkey, zkey_len, devices[i]));
      c->dev_extra.emplace_back();
    }
    c->reset_pool();
    NZ_HIP(hipSetDevice(devices[0]));
    if (err) err->code = 0;
    return c;
  } catch (const Error& e) {
    set_err(err, e.code, e.what());
  } catch (const std::exception& e) {
    set_err(err, NZCB_ERR_INTERNAL, e.what());
  }
  delete c;
  return nullptr;
}

nzcb_ctx* nzcb_ctx_create_file(const char* zkey_path, const int* devices, int ndev, nzcb_err* err) {
  if (!zkey_path) {
    set_err(err, NZCB_ERR_ARG, "null zkey path");
    return nullptr;
  }
  const int fd = open(zkey_path, O_RDONLY);
  if (fd < 0) {
    set_err(err, NZCB_ERR_ARG, (std::string("cannot open ") + zkey_path).c_str());
    return nullptr;
  }
  struct stat st;
  if (fstat(fd, &st) != 0 || st.st_size <= 0) {
    close(fd);
    set_err(err, NZCB_ERR_FORMAT, "zkey file is empty");
    return nullptr;
  }
  void* m = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
  close(fd);
  if (m == MAP_FAILED) {
    set_err(err, NZCB_ERR_INTERNAL, "mmap of the zkey failed");
    return nullptr;
  }
  int dev0 = 0;
  nzcb_ctx* c = devices && ndev > 0
                    ? nzcb_ctx_create_devices(static_cast<const uint8_t*>(m), (size_t)st.st_size, devices, ndev, err)
                    : nzcb_ctx_create(static_cast<const uint8_t*>(m), (size_t)st.st_size, dev0, err);
  munmap(m, (size_t)st.st_size);
  return c;
}

int nzcb_ctx_devices(const nzcb_ctx* ctx) { return ctx ? 1 + (int)ctx->dev_p.size() : 0; }

void nzcb_ctx_destroy(nzcb_ctx* ctx) { delete ctx; }

void nzcb_ctx_set_logger(nzcb_ctx* ctx, nzcb_log_fn fn, void* user) {
  if (!ctx) return;
  std::unique_lock<std::shared_mutex> lk(ctx->cfg);
  ctx->log_fn = fn;
  ctx->log_user = user;
}

void nzcb_ctx_set_transcript_public(nzcb_ctx* ctx, int on) {
  if (!ctx) return;
  std::unique_lock<std::shared_mutex> lk(ctx->cfg);
  for (Prover* q : ctx->all()) q->transcript_public = on != 0;
}

int nzcb_ctx_set_lanes(nzcb_ctx* ctx, int lanes, nzcb_err* err) {
  if (!ctx || lanes < 1 || lanes > 16) return fail(err, NZCB_ERR_ARG, "lanes must be in 1..16");
  try {
    {  // unchanged: no exclusive lock, which would wait for every proof in flight
      std::shared_lock<std::shared_mutex> lk(ctx->cfg);
      if (ctx->lanes() == (size_t)lanes) {
        if (err) err->code = 0;
        return 0;
      }
    }
    std::unique_lock<std::shared_mutex> lk(ctx->cfg);
    const size_t before = ctx->lanes();
    // trim every device's lane list to `k` lanes (a failed growth can leave device 0 one
    // lane ahead of the others)
    auto trim = [&](size_t k) {
      while (ctx->extra.size() + 1 > k) ctx->extra.pop_back();
      for (auto& de : ctx->dev_extra)
        while (de.size() + 1 > k) de.pop_back();
    };
    try {
      trim((size_t)lanes);
      while (ctx->lanes() < (size_t)lanes) {
        const int l = (int)ctx->lanes();
        ctx->extra.emplace_back(new Prover(*ctx->p, l));
        for (size_t d = 0; d < ctx->dev_p.size(); d++)
          ctx->dev_extra[d].emplace_back(new Prover(*ctx->dev_p[d], l));
        if (ctx->lane_alloc_fault.exchange(0)) {  // nzcb_debug_inject_fault(NZCB_FAULT_LANE_ALLOC)
          void* big = nullptr;
          const hipError_t e = hipMalloc(&big, size_t(1) << 50);
          if (e == hipSuccess) (void)hipFree(big);
          throw Error(NZCB_ERR_HIP, std::string("injected lane allocation failure: ") + hipGetErrorString(e));
        }
      }
    } catch (...) {
      // growth failed (out of HBM): back to the previous count on every device, so the
      // pool, lanes() and the allocations agree
      trim(std::min(before, ctx->lanes()));
      ctx->reset_pool();
      (void)hipSetDevice(ctx->p->eng->device);
      // the failed hipMalloc's error stays in HIP's per-thread last error until it is read:
      // the next NZ_HIP(hipGetLastError()) on this thread (a retried growth's NTT tables, a
      // proof) would otherwise fail with it
      for (size_t d = 0; d <= ctx->dev_p.size(); d++) {
        (void)hipSetDevice(d ? ctx->dev_p[d - 1]->eng->device : ctx->p->eng->device);
        (void)hipGetLastError();
      }
      (void)hipSetDevice(ctx->p->eng->device);
      throw;
    }
    ctx->reset_pool();
    NZ_HIP(hipSetDevice(ctx->p->eng->device));
    if (err) err->code = 0;
    return 0;
  } catch (const Error& e) {
    return fail(err, e.code, e.what());
  } catch (const std::exception& e) {
    return fail(err, NZCB_ERR_INTERNAL, e.what());
  }
}

int nzcb_ctx_lanes(const nzcb_ctx* ctx) { return ctx ? (int)ctx->lanes() : 0; }

int nzcb_ctx_set_msm_devices(nzcb_ctx* ctx, const int* devices, int ndev, nzcb_err* err) {
  if (!ctx || !devices || ndev < 1 || ndev > 64) return fail(err, NZCB_ERR_ARG, "devices: 1..64 ids");
  try {
    std::unique_lock<std::shared_mutex> lk(ctx->cfg);
    ctx->p->set_msm_devices(std::vector<int>(devices, devices + ndev));
    ctx->reset_pool();
    if (err) err->code = 0;
    return 0;
  } catch (const Error& e) {
    return fail(err, e.code, e.what());
  } catch (const std::exception& e) {
    return fail(err, NZCB_ERR_INTERNAL, e.what());
  }
}

int nzcb_ctx_set_msm_split(nzcb_ctx* ctx, int world, size_t own_points, size_t own_lagrange,
                           nzcb_msm_send_fn send, nzcb_msm_gather_fn gather, void* user, nzcb_err* err) {
  if (!ctx || world < 1 || world > 1024) return fail(err, NZCB_ERR_ARG, "msm split: world must be in 1..1024");
  try {
    std::unique_lock<std::shared_mutex> lk(ctx->cfg);
    ctx->p->set_msm_split(world, own_points, own_lagrange, send, gather, user);
    ctx->reset_pool();
    if (err) err->code = 0;
    return 0;
  } catch (const Error& e) {
    return fail(err, e.code, e.what());
  } catch (const std::exception& e) {
    return fail(err, NZCB_ERR_INTERNAL, e.what());
  }
}

// keep_going: prove every item and report each one's code in status_out (SURVEY.md §5:
// a failed proof is reported per item without aborting the batch); otherwise stop
// taking items past the first failure.
static int prove_batch(nzcb_ctx* ctx, const void* const* witnesses, size_t n_witness, int count, int witness_on_device,
                       const uint8_t* blindings, uint8_t* proofs_out, uint8_t* pubs_out, size_t pub_stride,
                       bool keep_going, int* status_out, nzcb_err* err) {
  if (!ctx || count < 0 || (count && (!witnesses || !proofs_out))) return fail(err, NZCB_ERR_ARG, "null argument");
  const size_t npub = ctx->p->nPublic;
  if (npub && (!pubs_out || pub_stride < 32 * npub)) return fail(err, NZCB_ERR_ARG, "public output buffer too small");
  std::shared_lock<std::shared_mutex> lk(ctx->cfg);
  std::atomic<int> next(0);
  std::atomic<int> first_bad(count);
  std::vector<int> codes(count, 0);
  std::vector<std::string> msgs(count);
  // one worker per lane: each takes a lane from the pool (shared with concurrent single
  // proofs), proves items until the batch is drained, and returns it
  auto worker = [&]() {
    Prover* pr = nullptr;
    for (;;) {
      const int i = next.fetch_add(1);
      if (i >= count || (!keep_going && i > first_bad.load())) break;
      if (!pr) pr = ctx->acquire(nullptr, nullptr);
      try {
        pr->prove((const uint8_t*)witnesses[i], n_witness,
                  blindings ? blindings + (size_t)i * NZCB_BLINDING_BYTES : nullptr,
                  proofs_out + (size_t)i * NZCB_PROOF_BYTES, npub ? pubs_out + (size_t)i * pub_stride : nullptr,
                  witness_on_device != 0);
      } catch (const Error& e) {
        codes[i] = e.code;
        msgs[i] = e.what();
      } catch (const std::exception& e) {
        codes[i] = NZCB_ERR_INTERNAL;
        msgs[i] = e.what();
      }
      if (codes[i]) {
        if (keep_going) {  // no partial output for a failed item
          std::memset(proofs_out + (size_t)i * NZCB_PROOF_BYTES, 0, NZCB_PROOF_BYTES);
          if (npub) std::memset(pubs_out + (size_t)i * pub_stride, 0, 32 * npub);
        }
        int cur = first_bad.load();
        while (i < cur && !first_bad.compare_exchange_weak(cur, i)) {
        }
      }
    }
    if (pr) ctx->release(pr);
  };
  const size_t nl = std::min(ctx->usable().size(), (size_t)(count > 0 ? count : 1));
  std::vector<std::thread> th;
  for (size_t l = 1; l < nl; l++) th.emplace_back(worker);
  worker();
  for (auto& t : th) t.join();
  if (status_out)
    for (int i = 0; i < count; i++) status_out[i] = codes[i];
  const int bad = first_bad.load();
  if (bad < count) {
    std::string m = "proof " + std::to_string(bad) + ": " + msgs[bad];
    return fail(err, codes[bad], m.c_str());
  }
  if (err) err->code = 0;
  return 0;
}

int nzcb_prove_batch(nzcb_ctx* ctx, const void* const* witnesses, size_t n_witness, int count, int witness_on_device,
                     const uint8_t* blindings, uint8_t* proofs_out, uint8_t* pubs_out, size_t pub_stride,
                     nzcb_err* err) {
  return prove_batch(ctx, witnesses, n_witness, count, witness_on_device, blindings, proofs_out, pubs_out, pub_stride,
                     false, nullptr, err);
}

int nzcb_prove_batch_status(nzcb_ctx* ctx, const void* const* witnesses, size_t n_witness, int count,
                            int witness_on_device, const uint8_t* blindings, uint8_t* proofs_out, uint8_t* pubs_out,
                            size_t pub_stride, int* status_out, nzcb_err* err) {
  if (count > 0 && !status_out) return fail(err, NZCB_ERR_ARG, "null argument");
  return prove_batch(ctx, witnesses, n_witness, count, witness_on_device, blindings, proofs_out, pubs_out, pub_stride,
                     true, status_out, err);
}

int nzcb_ctx_info(const nzcb_ctx* ctx, uint32_t out[5]) {
  if (!ctx || !out) return NZCB_ERR_ARG;
  const Prover& p = *ctx->p;
  out[0] = p.n;
  out[1] = p.nPublic;
  out[2] = p.nVars;
  out[3] = p.nAdditions;
  out[4] = p.nConstraints;
  return 0;
}

namespace {
// one proof on a lane of the pool; kind: NZCB_WITNESS_WTNS / _HOST / _DEVICE
int prove_one(nzcb_ctx* ctx, const void* witness, size_t n, int kind, const uint8_t* blinding, uint8_t* proof_out,
              uint8_t* pub_out, size_t pub_cap, nzcb_log_fn log, void* log_user, nzcb_err* err) {
  if (!ctx || !witness || !proof_out) return fail(err, NZCB_ERR_ARG, "null argument");
  if (kind != NZCB_WITNESS_WTNS && kind != NZCB_WITNESS_HOST && kind != NZCB_WITNESS_DEVICE)
    return fail(err, NZCB_ERR_ARG, "unknown witness kind");
  if (pub_cap < 32 * (size_t)ctx->p->nPublic || (!pub_out && ctx->p->nPublic))
    return fail(err, NZCB_ERR_ARG, "public output buffer too small");
  try {
    const uint8_t* values = (const uint8_t*)witness;
    size_t nw = n;
    if (kind == NZCB_WITNESS_WTNS) {
      Wtns w = parse_wtns(values, n);
      if (!w.q_is_r)
        return fail(err, NZCB_ERR_CURVE, "Curve of the witness does not match the curve of the proving key");
      values = w.values;
      nw = w.nWitness;
    }
    std::shared_lock<std::shared_mutex> lk(ctx->cfg);
    // a lane of a device-set context may be on another GPU: Prover::prove selects its
    // device, and the caller's current device is restored here
    int caller_dev = 0;
    NZ_HIP(hipGetDevice(&caller_dev));
    Prover* pr = ctx->acquire(log, log_user);
    try {
      pr->prove(values, nw, blinding, proof_out, pub_out, kind == NZCB_WITNESS_DEVICE);
    } catch (...) {
      pr->log = nullptr;
      ctx->release(pr);
      (void)hipSetDevice(caller_dev);
      throw;
    }
    pr->log = nullptr;
    ctx->release(pr);
    NZ_HIP(hipSetDevice(caller_dev));
    if (err) err->code = 0;
    return 0;
  } catch (const Error& e) {
    return fail(err, e.code, e.what());
  } catch (const std::exception& e) {
    return fail(err, NZCB_ERR_INTERNAL, e.what());
  }
}
}  // namespace

int nzcb_prove_witness(nzcb_ctx* ctx, const uint8_t* witness, size_t n_witness, const uint8_t* blinding,
                       uint8_t* proof_out, uint8_t* pub_out, size_t pub_cap, nzcb_err* err) {
  return prove_one(ctx, witness, n_witness, NZCB_WITNESS_HOST, blinding, proof_out, pub_out, pub_cap, nullptr, nullptr,
                   err);
}

int nzcb_prove_device(nzcb_ctx* ctx, const void* dev_witness, size_t n_witness, const uint8_t* blinding,
                      uint8_t* proof_out, uint8_t* pub_out, size_t pub_cap, nzcb_err* err) {
  return prove_one(ctx, dev_witness, n_witness, NZCB_WITNESS_DEVICE, blinding, proof_out, pub_out, pub_cap, nullptr,
                   nullptr, err);
}

int nzcb_prove(nzcb_ctx* ctx, const uint8_t* wtns, size_t wtns_len, const uint8_t* blinding, uint8_t* proof_out,
               uint8_t* pub_out, size_t pub_cap, nzcb_err* err) {
  return prove_one(ctx, wtns, wtns_len, NZCB_WITNESS_WTNS, blinding, proof_out, pub_out, pub_cap, nullptr, nullptr,
                   err);
}

int nzcb_prove_logged(nzcb_ctx* ctx, const void* witness, size_t n, int kind, const uint8_t* blinding,
                      uint8_t* proof_out, uint8_t* pub_out, size_t pub_cap, nzcb_log_fn log, void* log_user,
                      nzcb_err* err) {
  return prove_one(ctx, witness, n, kind, blinding, proof_out, pub_out, pub_cap, log, log_user, err);
}

int nzcb_ctx_last_timings(const nzcb_ctx* ctx, double* ms, int cap) {
  if (!ctx || !ms) return 0;
  int k = cap < 11 ? cap : 11;
  std::lock_guard<std::mutex> lk(const_cast<nzcb_ctx*>(ctx)->pool_mu);
  for (int i = 0; i < k; i++) ms[i] = ctx->last_tm[i];
  return k;
}

int nzcb_ctx_kernel_stats(nzcb_ctx* ctx, int enable, double out[4]) {
  if (!ctx) return NZCB_ERR_ARG;
  // switching: exclusive, so no proof is between msm_enqueue and msm_finish while `prof`
  // flips (finish would time events that enqueue never recorded), and no
  // set_lanes runs. A read-only query (enable < 0) takes the lock shared: it neither waits
  // behind the proofs in flight nor deadlocks when called from a proof's log callback
  // (ADVICE r5); its totals may then include a proof still in flight.
  std::unique_lock<std::shared_mutex> ex(ctx->cfg, std::defer_lock);
  std::shared_lock<std::shared_mutex> sh(ctx->cfg, std::defer_lock);
  if (enable >= 0) ex.lock(); else sh.lock();
  if (out) {
    for (int i = 0; i < 4; i++) out[i] = 0;
    for (Prover* q : ctx->all())
      for (auto& m : q->msc) {
        out[0] += m->prof_ms;
        out[1] += (double)m->prof_launches;
        out[2] += (double)m->prof_points;
        out[3] += (double)m->prof_entries;
      }
  }
  if (enable >= 0) {
    for (Prover* q : ctx->all()) {
      q->prof_gpu = enable != 0;
      for (auto& m : q->msc) {
        m->prof = enable != 0;
        m->prof_ms = 0;
        m->prof_launches = m->prof_points = m->prof_entries = 0;
      }
    }
  }
  return 0;
}

int nzcb_debug_inject_fault(nzcb_ctx* ctx, int kind) {
  if (!ctx || (kind != 0 && kind != NZCB_FAULT_QUOTIENT && kind != NZCB_DEBUG_GENERIC_K &&
               kind != NZCB_FAULT_LANE_ALLOC))
    return NZCB_ERR_ARG;
  std::unique_lock<std::shared_mutex> lk(ctx->cfg);
  if (kind == NZCB_FAULT_LANE_ALLOC) {
    ctx->lane_alloc_fault = 1;
    return 0;
  }
  ctx->pending_fault = kind;
  if (kind == 0) ctx->lane_alloc_fault = 0;
  return 0;
}

int nzcb_proof_to_json(const uint8_t* proof, char* out, size_t cap) {
  if (!proof) return -1;
  static const char* pts[7] = {"A", "B", "C", "Z", "T1", "T2", "T3"};
  static const char* evs[7] = {"eval_a", "eval_b", "eval_c", "eval_s1", "eval_s2", "eval_zw", "eval_r"};
  std::string s = "{";
  for (int i = 0; i < 7; i++) s += std::string("\"") + pts[i] + "\":" + g1_json(proof + 64 * i) + ",";
  for (int i = 0; i < 7; i++) s += std::string("\"") + evs[i] + "\":\"" + dec_le32(proof + 9 * 64 + 32 * i) + "\",";
  s += "\"Wxi\":" + g1_json(proof + 7 * 64) + ",";
  s += "\"Wxiw\":" + g1_json(proof + 8 * 64) + ",";
  s += "\"protocol\":\"plonk\",\"curve\":\"bn128\"}";
  return copy_out(s, out, cap);
}

int nzcb_public_to_json(const uint8_t* pub, int n_public, char* out, size_t cap) {
  std::string s = "[";
  for (int i = 0; i < n_public; i++) {
    if (i) s += ",";
    s += "\"" + dec_le32(pub + 32 * i) + "\"";
  }
  s += "]";
  return copy_out(s, out, cap);
}

}  // extern "C"
