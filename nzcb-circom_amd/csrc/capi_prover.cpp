// C-ABI: prover context, proofs and snarkjs-format JSON (include/nzcb.h).
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <cstring>
#include <mutex>
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
  std::mutex mu;  // calls on one context are serialized (SURVEY.md §8b "Threading")
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
  std::lock_guard<std::mutex> lk(ctx->mu);
  ctx->log_fn = fn;
  ctx->log_user = user;
  for (Prover* q : ctx->all()) {
    if (fn)
      q->log = [ctx](const std::string& m) { ctx->log_fn(ctx->log_user, m.c_str()); };
    else
      q->log = nullptr;
  }
}

void nzcb_ctx_set_transcript_public(nzcb_ctx* ctx, int on) {
  if (!ctx) return;
  std::lock_guard<std::mutex> lk(ctx->mu);
  for (Prover* q : ctx->all()) q->transcript_public = on != 0;
}

int nzcb_ctx_set_lanes(nzcb_ctx* ctx, int lanes, nzcb_err* err) {
  if (!ctx || lanes < 1 || lanes > 16) return fail(err, NZCB_ERR_ARG, "lanes must be in 1..16");
  try {
    std::lock_guard<std::mutex> lk(ctx->mu);
    while (ctx->lanes() > (size_t)lanes) {
      ctx->extra.pop_back();
      for (auto& de : ctx->dev_extra) de.pop_back();
    }
    while (ctx->lanes() < (size_t)lanes) {
      const int l = (int)ctx->lanes();
      ctx->extra.emplace_back(new Prover(*ctx->p, l));
      ctx->extra.back()->log = ctx->p->log;
      for (size_t d = 0; d < ctx->dev_p.size(); d++) {
        ctx->dev_extra[d].emplace_back(new Prover(*ctx->dev_p[d], l));
        ctx->dev_extra[d].back()->log = ctx->p->log;
      }
    }
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
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->p->set_msm_devices(std::vector<int>(devices, devices + ndev));
    if (err) err->code = 0;
    return 0;
  } catch (const Error& e) {
    return fail(err, e.code, e.what());
  } catch (const std::exception& e) {
    return fail(err, NZCB_ERR_INTERNAL, e.what());
  }
}

int nzcb_ctx_set_msm_split(nzcb_ctx* ctx, int world, size_t own_points, nzcb_msm_send_fn send,
                           nzcb_msm_gather_fn gather, void* user, nzcb_err* err) {
  if (!ctx || world < 1 || world > 1024) return fail(err, NZCB_ERR_ARG, "msm split: world must be in 1..1024");
  try {
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->p->set_msm_split(world, own_points, send, gather, user);
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
  std::lock_guard<std::mutex> lk(ctx->mu);
  std::atomic<int> next(0);
  std::atomic<int> first_bad(count);
  std::vector<int> codes(count, 0);
  std::vector<std::string> msgs(count);
  auto worker = [&](Prover* pr) {
    for (;;) {
      const int i = next.fetch_add(1);
      if (i >= count || (!keep_going && i > first_bad.load())) return;
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
  };
  // lane 0 of device 0 is the only lane whose commitments a split (nzcb_ctx_set_msm_devices /
  // nzcb_ctx_set_msm_split) covers, so a split context proves its batch on lane 0 alone
  std::vector<Prover*> ws = ctx->p->split_send || !ctx->p->shards.empty() ? std::vector<Prover*>{ctx->p.get()}
                                                                         : ctx->all();
  const size_t nl = std::min(ws.size(), (size_t)(count > 0 ? count : 1));
  std::vector<std::thread> th;
  for (size_t l = 1; l < nl; l++) th.emplace_back(worker, ws[l]);
  worker(ws[0]);
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

int nzcb_prove_witness(nzcb_ctx* ctx, const uint8_t* witness, size_t n_witness, const uint8_t* blinding,
                       uint8_t* proof_out, uint8_t* pub_out, size_t pub_cap, nzcb_err* err) {
  if (!ctx || !witness || !proof_out) return fail(err, NZCB_ERR_ARG, "null argument");
  if (pub_cap < 32 * (size_t)ctx->p->nPublic || (!pub_out && ctx->p->nPublic))
    return fail(err, NZCB_ERR_ARG, "public output buffer too small");
  try {
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->p->prove(witness, n_witness, blinding, proof_out, pub_out);
    if (err) err->code = 0;
    return 0;
  } catch (const Error& e) {
    return fail(err, e.code, e.what());
  } catch (const std::exception& e) {
    return fail(err, NZCB_ERR_INTERNAL, e.what());
  }
}

int nzcb_prove_device(nzcb_ctx* ctx, const void* dev_witness, size_t n_witness, const uint8_t* blinding,
                      uint8_t* proof_out, uint8_t* pub_out, size_t pub_cap, nzcb_err* err) {
  if (!ctx || !dev_witness || !proof_out) return fail(err, NZCB_ERR_ARG, "null argument");
  if (pub_cap < 32 * (size_t)ctx->p->nPublic || (!pub_out && ctx->p->nPublic))
    return fail(err, NZCB_ERR_ARG, "public output buffer too small");
  try {
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->p->prove((const uint8_t*)dev_witness, n_witness, blinding, proof_out, pub_out, true);
    if (err) err->code = 0;
    return 0;
  } catch (const Error& e) {
    return fail(err, e.code, e.what());
  } catch (const std::exception& e) {
    return fail(err, NZCB_ERR_INTERNAL, e.what());
  }
}

int nzcb_prove(nzcb_ctx* ctx, const uint8_t* wtns, size_t wtns_len, const uint8_t* blinding, uint8_t* proof_out,
               uint8_t* pub_out, size_t pub_cap, nzcb_err* err) {
  if (!ctx || !wtns) return fail(err, NZCB_ERR_ARG, "null argument");
  try {
    Wtns w = parse_wtns(wtns, wtns_len);
    if (!w.q_is_r)
      return fail(err, NZCB_ERR_CURVE, "Curve of the witness does not match the curve of the proving key");
    return nzcb_prove_witness(ctx, w.values, w.nWitness, blinding, proof_out, pub_out, pub_cap, err);
  } catch (const Error& e) {
    return fail(err, e.code, e.what());
  }
}

int nzcb_ctx_last_timings(const nzcb_ctx* ctx, double* ms, int cap) {
  if (!ctx || !ms) return 0;
  int k = cap < 9 ? cap : 9;
  for (int i = 0; i < k; i++) ms[i] = ctx->p->tm[i];
  return k;
}

int nzcb_ctx_kernel_stats(nzcb_ctx* ctx, int enable, double out[4]) {
  if (!ctx) return NZCB_ERR_ARG;
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
    for (Prover* q : ctx->all())
      for (auto& m : q->msc) {
        m->prof = enable != 0;
        m->prof_ms = 0;
        m->prof_launches = m->prof_points = m->prof_entries = 0;
      }
  }
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
