// Seeded synthetic circuit + snarkjs-0.4 PLONK setup on the GPU (nzcb_synth_setup).
//
// The reference builds its proving key with `snarkjs plonk setup nzcp_live.r1cs
// powersOfTau28_hez_final_21.ptau` (/root/reference/Makefile:59-62); circom,
// snarkjs and the ptau are [EXT] and unavailable offline, so the benchmark and
// the large-size parity tests run on the synthetic circuit family that
// oracle/synth.py defines bit-exactly. This file
// implements the same generator and the same setup (snarkjs plonk_setup restated
// in oracle/plonk.py::setup), with the heavy parts on the device:
//   * Q / sigma / Lagrange columns: iNTT_n -> coefficients, NTT_4n -> evaluations
//   * PTau [tau^i]G1: one thread per power (double-and-add in XYZZ, Fermat to affine)
//   * header commitments [Qm]..[S3]: the prover's own MSM
// tests/test_gpu_synth.py checks the zkey/wtns bytes against the oracle.
#include <cstdlib>
#include <cstring>
#include <functional>
#include <vector>

#include "../../include/nzcb_internal.h"
#include "engine.h"

namespace nzcb {
void set_err(nzcb_err* err, int code, const char* msg);

namespace {

constexpr int kT = 256;
constexpr uint32_t kInternal = 1u << 31;

struct Xoshiro {
  uint64_t s[4];
  explicit Xoshiro(uint64_t seed) {
    uint64_t x = seed;
    for (int i = 0; i < 4; i++) {
      x += 0x9E3779B97F4A7C15ULL;
      uint64_t z = x;
      z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
      z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
      s[i] = z ^ (z >> 31);
    }
  }
  static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
  uint64_t next() {
    uint64_t result = rotl(s[1] * 5, 7) * 9;
    uint64_t t = s[1] << 17;
    s[2] ^= s[0];
    s[3] ^= s[1];
    s[1] ^= s[2];
    s[0] ^= s[3];
    s[2] ^= t;
    s[3] = rotl(s[3], 45);
    return result;
  }
  uint64_t below(uint64_t m) { return next() % m; }
  // uniform Fr (normal form): 4 words LE, masked to 254 bits, rejected if >= r
  Fr fr() {
    for (;;) {
      uint64_t w[4];
      for (int i = 0; i < 4; i++) w[i] = next();
      Fr x;
      std::memcpy(x.v, w, 32);
      x.v[7] &= 0x3fffffffu;
      if (reduce_once(x) == x) return x;
    }
  }
};

__global__ void k_pow_table(Fr* out, Fr base, size_t count) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < count) out[i] = pow_u64(base, i);
}

// out[i] = [s_i] G1 as LEM affine (s_i Montgomery)
__global__ void __launch_bounds__(kT) k_fixed_base(const Fr* __restrict__ s, size_t count, G1Affine* out) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  Fr k = from_mont(s[i]);
  Fq gx = Fq::one();
  Fq gy = dbl(Fq::one());
  G1xyzz acc = G1xyzz::inf();
  for (int b = 255; b >= 0; b--) {
    acc = xyzz_dbl(acc);
    if ((k.v[b >> 5] >> (b & 31)) & 1u) acc = xyzz_add_affine(acc, gx, gy);
  }
  G1Affine a;
  if (acc.is_inf()) {
    a.x = Fq::zero();
    a.y = Fq::zero();
  } else {
    a.x = acc.X * inverse(acc.ZZ);
    a.y = acc.Y * inverse(acc.ZZZ);
  }
  out[i] = a;
}

__global__ void k_pad4(const Fr* __restrict__ src, size_t n, Fr* __restrict__ dst, size_t n4) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n4) dst[i] = i < n ? src[i] : Fr::zero();
}

// --- host G2 (only X_2 = [tau]_2 for the zkey header) ------------------------
struct Fq2 {
  Fq c0, c1;
};
Fq2 f2_add(const Fq2& a, const Fq2& b) { return {a.c0 + b.c0, a.c1 + b.c1}; }
Fq2 f2_sub(const Fq2& a, const Fq2& b) { return {a.c0 - b.c0, a.c1 - b.c1}; }
Fq2 f2_mul(const Fq2& a, const Fq2& b) { return {a.c0 * b.c0 - a.c1 * b.c1, a.c0 * b.c1 + a.c1 * b.c0}; }
Fq2 f2_inv(const Fq2& a) {
  Fq d = inverse(a.c0 * a.c0 + a.c1 * a.c1);
  return {a.c0 * d, neg(a.c1) * d};
}
bool f2_eq(const Fq2& a, const Fq2& b) { return a.c0 == b.c0 && a.c1 == b.c1; }
struct G2 {
  Fq2 x, y;
  bool inf;
};
G2 g2_dbl(const G2& p) {
  if (p.inf || (p.y.c0.is_zero() && p.y.c1.is_zero())) return {{}, {}, true};
  Fq three = Fq::one() + Fq::one() + Fq::one();
  Fq2 x2 = f2_mul(p.x, p.x);
  Fq2 lam = f2_mul({x2.c0 * three, x2.c1 * three}, f2_inv(f2_add(p.y, p.y)));
  Fq2 x3 = f2_sub(f2_mul(lam, lam), f2_add(p.x, p.x));
  Fq2 y3 = f2_sub(f2_mul(lam, f2_sub(p.x, x3)), p.y);
  return {x3, y3, false};
}
G2 g2_add(const G2& a, const G2& b) {
  if (a.inf) return b;
  if (b.inf) return a;
  if (f2_eq(a.x, b.x)) return f2_eq(a.y, b.y) ? g2_dbl(a) : G2{{}, {}, true};
  Fq2 lam = f2_mul(f2_sub(b.y, a.y), f2_inv(f2_sub(b.x, a.x)));
  Fq2 x3 = f2_sub(f2_sub(f2_mul(lam, lam), a.x), b.x);
  Fq2 y3 = f2_sub(f2_mul(lam, f2_sub(a.x, x3)), a.y);
  return {x3, y3, false};
}
Fq fq_lit(const uint32_t l[8]) {
  Fq x;
  for (int i = 0; i < 8; i++) x.v[i] = l[i];
  return to_mont(x);
}
G2 g2_mul_gen(const Fr& k_normal) {
  static const uint32_t X0[8] = {0xd992f6edu, 0x46debd5cu, 0xf75edaddu, 0x674322d4u,
                                 0x5e5c4479u, 0x426a0066u, 0x121f1e76u, 0x1800deefu};
  static const uint32_t X1[8] = {0xaef312c2u, 0x97e485b7u, 0x35a9e712u, 0xf1aa4933u,
                                 0x31fb5d25u, 0x7260bfb7u, 0x920d483au, 0x198e9393u};
  static const uint32_t Y0[8] = {0x66fa7daau, 0x4ce6cc01u, 0x0c43d37bu, 0xe3d1e769u,
                                 0x8dcb408fu, 0x4aab7180u, 0xdb8c6debu, 0x12c85ea5u};
  static const uint32_t Y1[8] = {0xd122975bu, 0x55acdadcu, 0x70b38ef3u, 0xbc4b3133u,
                                 0x690c3395u, 0xec9e99adu, 0x585ff075u, 0x090689d0u};
  G2 g{{fq_lit(X0), fq_lit(X1)}, {fq_lit(Y0), fq_lit(Y1)}, false};
  G2 acc{{}, {}, true};
  for (int b = 255; b >= 0; b--) {
    acc = g2_dbl(acc);
    if ((k_normal.v[b >> 5] >> (b & 31)) & 1u) acc = g2_add(acc, g);
  }
  return acc;
}

void put_u32(std::vector<uint8_t>& o, uint32_t v) {
  uint8_t b[4];
  std::memcpy(b, &v, 4);
  o.insert(o.end(), b, b + 4);
}
void put_u64(std::vector<uint8_t>& o, uint64_t v) {
  uint8_t b[8];
  std::memcpy(b, &v, 8);
  o.insert(o.end(), b, b + 8);
}
void put_bytes(std::vector<uint8_t>& o, const void* p, size_t n) {
  const uint8_t* b = (const uint8_t*)p;
  o.insert(o.end(), b, b + n);
}

struct Circuit {
  uint32_t n = 0, n_public = 0, n_wit = 0, n_vars = 0, n_add = 0;
  std::vector<uint32_t> sa, sb, sc;  // resolved signal ids
  std::vector<Fr> q[5];              // qm ql qr qo qc (Montgomery)
  std::vector<uint32_t> ax, ay;      // additions operands
  std::vector<Fr> ac, bc;            // Montgomery
  std::vector<Fr> wit;               // file witness (Montgomery), wit[0] = 1
};

// Bit-exact restatement of oracle/synth.py::synth_circuit
Circuit build_circuit(int power, uint32_t n_public, uint32_t n_inputs, uint64_t seed, uint32_t n_cons,
                      uint32_t flags) {
  Circuit c;
  c.n = 1u << power;
  c.n_public = n_public;
  if (n_cons == 0) n_cons = c.n - std::max(1u, c.n >> 5);
  if (!(n_public + n_inputs <= n_cons && n_cons <= c.n)) throw Error(NZCB_ERR_ARG, "bad synthetic circuit size");
  Xoshiro rng(seed);
  c.wit.push_back(Fr::one());  // signal 0 (file value 1)
  std::vector<Fr> internal;
  for (uint32_t i = 0; i < n_public + n_inputs; i++) c.wit.push_back(to_mont(rng.fr()));
  std::vector<uint32_t> pool;
  // NZCB_SYNTH_FREE_PUBLIC: public signals sit on their public-input gate only, so any
  // values satisfy the circuit (the nzcp outputs computed per pass, nzcp.hip)
  for (uint32_t i = (flags & NZCB_SYNTH_FREE_PUBLIC) ? 1 + n_public : 1; i <= n_public + n_inputs; i++)
    pool.push_back(i);
  uint32_t unused_next = 1 + n_public, unused_end = 1 + n_public + n_inputs;
  auto pick = [&]() -> uint32_t {
    if (unused_next < unused_end) return unused_next++;
    return pool[rng.below(pool.size())];
  };
  auto val = [&](uint32_t ref) -> Fr {
    if (ref & kInternal) return internal[ref & ~kInternal];
    return ref == 0 ? Fr::zero() : c.wit[ref];
  };
  for (int k = 0; k < 5; k++) c.q[k].reserve(n_cons);
  c.sa.reserve(n_cons);
  c.sb.reserve(n_cons);
  c.sc.reserve(n_cons);
  Fr one = Fr::one();
  for (uint32_t s = 1; s <= n_public; s++) {
    c.sa.push_back(s);
    c.sb.push_back(0);
    c.sc.push_back(0);
    c.q[0].push_back(Fr::zero());
    c.q[1].push_back(one);
    c.q[2].push_back(Fr::zero());
    c.q[3].push_back(Fr::zero());
    c.q[4].push_back(Fr::zero());
  }
  const Fr minus_one = neg(one);
  for (uint32_t g = 0; g < n_cons - n_public; g++) {
    uint64_t kind = rng.below(8);
    if (kind == 7 && unused_next < unused_end) kind = 0;  // additions read signals already on a gate wire
    uint32_t a = pick();
    uint32_t b = pick();
    if (kind == 7) {
      uint32_t x = pick();
      uint32_t y = pick();
      Fr acv = to_mont(rng.fr());
      Fr bcv = to_mont(rng.fr());
      uint32_t t = kInternal | (uint32_t)internal.size();
      internal.push_back(acv * val(x) + bcv * val(y));
      c.ax.push_back(x);
      c.ay.push_back(y);
      c.ac.push_back(acv);
      c.bc.push_back(bcv);
      a = t;
    }
    Fr qm = to_mont(rng.fr());
    Fr ql = to_mont(rng.fr());
    Fr qr = to_mont(rng.fr());
    Fr va = val(a), vb = val(b);
    Fr qo, qc;
    uint32_t cref;
    if (kind == 5 || kind == 6) {
      cref = pick();
      qo = to_mont(rng.fr());
      qc = neg(qm * va * vb + ql * va + qr * vb + qo * val(cref));
    } else {
      qo = minus_one;
      qc = to_mont(rng.fr());
      Fr vc = qm * va * vb + ql * va + qr * vb + qc;
      cref = (uint32_t)c.wit.size();
      c.wit.push_back(vc);
      pool.push_back(cref);
    }
    c.sa.push_back(a);
    c.sb.push_back(b);
    c.sc.push_back(cref);
    c.q[0].push_back(qm);
    c.q[1].push_back(ql);
    c.q[2].push_back(qr);
    c.q[3].push_back(qo);
    c.q[4].push_back(qc);
  }
  c.n_wit = (uint32_t)c.wit.size();
  c.n_add = (uint32_t)internal.size();
  c.n_vars = c.n_wit + c.n_add;
  auto res = [&](uint32_t r) { return (r & kInternal) ? c.n_wit + (r & ~kInternal) : r; };
  for (auto* v : {&c.sa, &c.sb, &c.sc, &c.ax, &c.ay})
    for (auto& r : *v) r = res(r);
  return c;
}

}  // namespace

// [s_i] G1 as LEM affine on `st` (microbench bases; PTau generation below)
void launch_fixed_base(const Fr* scalars_mont, size_t n, G1Affine* out, hipStream_t st) {
  hipLaunchKernelGGL(k_fixed_base, dim3(grid_for(n, kT, 1u << 30)), dim3(kT), 0, st, scalars_mont, n, out);
  NZ_HIP(hipGetLastError());
}

// Source of the powers of tau: a trapdoor tau (synthetic setups, tests), or the
// tauG1 / tauG2 sections of a snarkjs .ptau file.
struct PtauSrc {
  const uint8_t* tau_le = nullptr;  // 32 B LE trapdoor
  const uint8_t* g1 = nullptr;      // >= n + 6 LEM affine [tau^i]G1 (ptau section 2)
  size_t g1_count = 0;
  const uint8_t* x2 = nullptr;      // 128 B LEM [tau]G2 (ptau section 3, point 1)
};

// snarkjs plonk_setup's zkey for a processed circuit (sections 1-14);
// malloc'ed buffer.
static void setup_zkey(const Circuit& c, int power, int n_public, const PtauSrc& src, int device, uint8_t** zk_out,
                       size_t* zk_len) {
  const uint32_t n = c.n, n4 = 4 * n;
  const uint32_t nc = (uint32_t)c.sa.size();
  if (n != (1u << power) || nc > n) throw Error(NZCB_ERR_INTERNAL, "circuit does not fit its domain");
  Engine eng(device, power + 2, n);
  hipStream_t st = eng.stream;

  // PTau: [tau^i] G1, i < n + 6
  const size_t nptau = (size_t)n + 6;
  DevBuf<G1Affine> ptau(nptau);
  Fr tau = Fr::zero();
  if (src.tau_le) {
    std::memcpy(tau.v, src.tau_le, 32);
    tau = to_mont(reduce_once(reduce_once(tau)));
    DevBuf<Fr> taupow(nptau);
    hipLaunchKernelGGL(k_pow_table, dim3(grid_for(nptau, kT, 1u << 30)), dim3(kT), 0, st, taupow.p, tau, nptau);
    hipLaunchKernelGGL(k_fixed_base, dim3(grid_for(nptau, kT, 1u << 30)), dim3(kT), 0, st, taupow.p, nptau,
                       ptau.p);
    NZ_HIP(hipGetLastError());
    NZ_HIP(hipStreamSynchronize(st));
  } else {
    if (!src.g1 || !src.x2 || src.g1_count < nptau) throw Error(NZCB_ERR_ARG, "powers of tau too small for the circuit");
    NZ_HIP(hipMemcpyAsync(ptau.p, src.g1, nptau * 64, hipMemcpyHostToDevice, st));
  }

  DevBuf<Fr> dcol(n), dcoef(n), dpad(n4), deval(n4);
  // writeP4 for one column on n points: returns [coefs | evals4] (LEM bytes) and the commitment
  auto p4 = [&](const std::vector<Fr>& col, std::vector<uint8_t>& out, G1Affine* commit) {
    NZ_HIP(hipMemcpyAsync(dcol.p, col.data(), (size_t)n * 32, hipMemcpyHostToDevice, st));
    ntt(eng.ntt_tables, dcol.p, dcoef.p, power, true, st);
    hipLaunchKernelGGL(k_pad4, dim3(grid_for(n4, kT, 1u << 30)), dim3(kT), 0, st, dcoef.p, (size_t)n, dpad.p,
                       (size_t)n4);
    ntt(eng.ntt_tables, dpad.p, deval.p, power + 2, false, st);
    size_t off = out.size();
    out.resize(off + (size_t)5 * n * 32);
    NZ_HIP(hipMemcpyAsync(out.data() + off, dcoef.p, (size_t)n * 32, hipMemcpyDeviceToHost, st));
    NZ_HIP(hipMemcpyAsync(out.data() + off + (size_t)n * 32, deval.p, (size_t)n4 * 32, hipMemcpyDeviceToHost, st));
    NZ_HIP(hipStreamSynchronize(st));
    if (commit) *commit = xyzz_to_affine(msm(eng.msm_scratch, ptau.p, dcoef.p, n, true, st));
  };

  std::vector<uint8_t> secQ[5], secS, secL;
  G1Affine com[8];
  for (int k = 0; k < 5; k++) {
    std::vector<Fr> col(n, Fr::zero());
    for (uint32_t i = 0; i < nc; i++) col[i] = c.q[k][i];
    p4(col, secQ[k], &com[k]);
  }
  // buildSigma
  {
    std::vector<Fr> sigma((size_t)3 * n, Fr::zero());
    std::vector<Fr> last(c.n_vars);
    std::vector<uint8_t> seen(c.n_vars, 0);
    std::vector<uint64_t> first(c.n_vars, 0);
    Fr w = Fr::one();
    const Fr wn = fr_root_of_unity(power);
    Fr kk[3];
    kk[0] = Fr::one();
    kk[1] = kk[0] + kk[0];
    kk[2] = kk[1] + kk[0];
    for (uint32_t i = 0; i < n; i++) {
      uint32_t sig[3] = {0, 0, 0};
      if (i < nc) {
        sig[0] = c.sa[i];
        sig[1] = c.sb[i];
        sig[2] = c.sc[i];
      }
      for (int k = 0; k < 3; k++) {
        uint32_t s = sig[k];
        if (s >= c.n_vars) throw Error(NZCB_ERR_INTERNAL, "signal out of range");
        uint64_t p = (uint64_t)k * n + i;
        if (!seen[s]) {
          first[s] = p;
          seen[s] = 1;
        } else {
          sigma[p] = last[s];
        }
        last[s] = k ? w * kk[k] : w;
      }
      w = w * wn;
    }
    for (uint32_t s = 0; s < c.n_vars; s++) {
      if (!seen[s]) throw Error(NZCB_ERR_INTERNAL, "Variable not used");
      sigma[first[s]] = last[s];
    }
    for (int k = 0; k < 3; k++) {
      std::vector<Fr> col(sigma.begin() + (size_t)k * n, sigma.begin() + (size_t)(k + 1) * n);
      p4(col, secS, &com[5 + k]);
    }
  }
  for (int j = 0; j < std::max(n_public, 1); j++) {
    std::vector<Fr> col(n, Fr::zero());
    col[j] = Fr::one();
    p4(col, secL, nullptr);
  }
  std::vector<uint8_t> ptau_bytes(nptau * 64);
  NZ_HIP(hipMemcpyAsync(ptau_bytes.data(), ptau.p, nptau * 64, hipMemcpyDeviceToHost, st));
  NZ_HIP(hipStreamSynchronize(st));
  G2 x2{};
  if (src.tau_le) x2 = g2_mul_gen(from_mont(tau));

  // ---- assemble the zkey ----
  static const uint32_t kQ[8] = {0xd87cfd47u, 0x3c208c16u, 0x6871ca8du, 0x97816a91u,
                                 0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
  std::vector<uint8_t> s2;
  put_u32(s2, 32);
  put_bytes(s2, kQ, 32);
  put_u32(s2, 32);
  put_bytes(s2, FrParams::P, 32);
  put_u32(s2, c.n_vars);
  put_u32(s2, (uint32_t)n_public);
  put_u32(s2, n);
  put_u32(s2, c.n_add);
  put_u32(s2, nc);
  Fr k1 = Fr::one() + Fr::one();
  Fr k2 = k1 + Fr::one();
  put_bytes(s2, k1.v, 32);
  put_bytes(s2, k2.v, 32);
  for (int k = 0; k < 8; k++) put_bytes(s2, &com[k], 64);
  if (!src.tau_le) {
    put_bytes(s2, src.x2, 128);
  } else if (x2.inf) {
    std::vector<uint8_t> z(128, 0);
    put_bytes(s2, z.data(), 128);
  } else {
    put_bytes(s2, x2.x.c0.v, 32);
    put_bytes(s2, x2.x.c1.v, 32);
    put_bytes(s2, x2.y.c0.v, 32);
    put_bytes(s2, x2.y.c1.v, 32);
  }
  std::vector<uint8_t> s3;
  for (uint32_t k = 0; k < c.n_add; k++) {
    put_u32(s3, c.ax[k]);
    put_u32(s3, c.ay[k]);
    put_bytes(s3, c.ac[k].v, 32);
    put_bytes(s3, c.bc[k].v, 32);
  }
  std::vector<const std::vector<uint8_t>*> secs;
  std::vector<uint8_t> s1;
  put_u32(s1, 2);
  std::vector<uint8_t> s4(c.sa.size() * 4), s5(c.sb.size() * 4), s6(c.sc.size() * 4);
  if (nc) {
    std::memcpy(s4.data(), c.sa.data(), s4.size());
    std::memcpy(s5.data(), c.sb.data(), s5.size());
    std::memcpy(s6.data(), c.sc.data(), s6.size());
  }
  secs = {&s1, &s2, &s3, &s4, &s5, &s6, &secQ[0], &secQ[1], &secQ[2], &secQ[3], &secQ[4], &secS, &secL, &ptau_bytes};
  size_t total = 12;
  for (auto* s : secs) total += 12 + s->size();
  uint8_t* zk = (uint8_t*)std::malloc(total);
  if (!zk) throw Error(NZCB_ERR_INTERNAL, "out of host memory");
  size_t off = 0;
  auto w32 = [&](uint32_t v) { std::memcpy(zk + off, &v, 4); off += 4; };
  auto w64 = [&](uint64_t v) { std::memcpy(zk + off, &v, 8); off += 8; };
  std::memcpy(zk, "zkey", 4);
  off = 4;
  w32(1);
  w32((uint32_t)secs.size());
  for (size_t i = 0; i < secs.size(); i++) {
    w32((uint32_t)(i + 1));
    w64(secs[i]->size());
    if (!secs[i]->empty()) std::memcpy(zk + off, secs[i]->data(), secs[i]->size());
    off += secs[i]->size();
  }
  *zk_out = zk;
  *zk_len = total;
}

// The whole synthetic setup; returns (zkey, wtns) as malloc'ed buffers.
static void synth_setup(int power, int n_public, int n_inputs, uint64_t seed, uint32_t n_cons, uint32_t flags,
                        const uint8_t* tau_le, int device, uint8_t** zk_out, size_t* zk_len, uint8_t** wt_out, size_t* wt_len) {
  if (power < 1 || power > 24 || n_public < 0 || n_inputs < 0) throw Error(NZCB_ERR_ARG, "bad setup arguments");
  if (flags & ~(uint32_t)NZCB_SYNTH_FREE_PUBLIC) throw Error(NZCB_ERR_ARG, "unknown synth flags");
  Circuit c = build_circuit(power, (uint32_t)n_public, (uint32_t)n_inputs, seed, n_cons, flags);
  PtauSrc src;
  src.tau_le = tau_le;
  uint8_t* zk = nullptr;
  size_t total = 0;
  setup_zkey(c, power, n_public, src, device, &zk, &total);
  // ---- wtns ----
  size_t wtotal = 12 + 12 + 4 + 32 + 4 + 12 + (size_t)c.n_wit * 32;
  uint8_t* wt = (uint8_t*)std::malloc(wtotal);
  if (!wt) {
    std::free(zk);
    throw Error(NZCB_ERR_INTERNAL, "out of host memory");
  }
  size_t wo = 0;
  auto ww32 = [&](uint32_t v) { std::memcpy(wt + wo, &v, 4); wo += 4; };
  auto ww64 = [&](uint64_t v) { std::memcpy(wt + wo, &v, 8); wo += 8; };
  std::memcpy(wt, "wtns", 4);
  wo = 4;
  ww32(2);
  ww32(2);
  ww32(1);
  ww64(4 + 32 + 4);
  ww32(32);
  std::memcpy(wt + wo, FrParams::P, 32);
  wo += 32;
  ww32(c.n_wit);
  ww32(2);
  ww64((uint64_t)c.n_wit * 32);
  for (uint32_t i = 0; i < c.n_wit; i++) {
    Fr v = from_mont(c.wit[i]);
    std::memcpy(wt + wo, v.v, 32);
    wo += 32;
  }
  *zk_out = zk;
  *zk_len = total;
  *wt_out = wt;
  *wt_len = wtotal;
}


// ---- snarkjs `plonk setup <r1cs> <ptau> <zkey>` (/root/reference/Makefile:55,60) ------
// Restates snarkjs 0.4.12 plonk_setup.js [EXT]: processConstraints
// turns every R1CS constraint (A)(B) = (C) into one PLONK gate, after splitting each
// linear combination with more than one signal into a binary tree of addition gates
// (reduceCoef: first half, second half, then a new signal so = l1 a + l2 b, recorded as
// an "addition" for calculateAdditions); the nPublic public signals get the first
// gates. The columns, sigma, Lagrange polynomials and commitments are the synthetic
// setup's (setup_zkey). Commitments use the coefficient form against tauG1 (section 2),
// the same group elements snarkjs gets from the Lagrange points (section 12).

struct BinSections {  // iden3 binfile: magic, u32 version, u32 count, (u32 type, u64 size, data)*
  std::vector<std::pair<const uint8_t*, uint64_t>> sec[16];
};
static BinSections read_binfile(const uint8_t* d, size_t len, const char* magic, const char* what) {
  BinSections b;
  char msg[96];
  if (!d || len < 12 || std::memcmp(d, magic, 4) != 0) {
    std::snprintf(msg, sizeof msg, "%s: invalid file format", what);
    throw Error(NZCB_ERR_FORMAT, msg);
  }
  uint32_t version, nsec;
  std::memcpy(&version, d + 4, 4);
  std::memcpy(&nsec, d + 8, 4);
  size_t off = 12;
  for (uint32_t i = 0; i < nsec; i++) {
    if (off + 12 > len) throw Error(NZCB_ERR_FORMAT, "truncated section table");
    uint32_t type;
    uint64_t size;
    std::memcpy(&type, d + off, 4);
    std::memcpy(&size, d + off + 4, 8);
    off += 12;
    if (size > len - off) throw Error(NZCB_ERR_FORMAT, "truncated section");
    if (type < 16) b.sec[type].push_back({d + off, size});
    off += size;
  }
  return b;
}

struct ByteReader {
  const uint8_t* p;
  uint64_t left;
  uint32_t u32() {
    if (left < 4) throw Error(NZCB_ERR_FORMAT, "r1cs: truncated");
    uint32_t v;
    std::memcpy(&v, p, 4);
    p += 4;
    left -= 4;
    return v;
  }
  uint64_t u64() {
    const uint64_t lo = u32();
    return lo | ((uint64_t)u32() << 32);
  }
  Fr fr_normal() {  // 32 B LE normal form -> Montgomery (ffjavascript Fr.fromRprLE)
    if (left < 32) throw Error(NZCB_ERR_FORMAT, "r1cs: truncated");
    Fr v;
    std::memcpy(v.v, p, 32);
    p += 32;
    left -= 32;
    if (!(reduce_once(v) == v) || v == Fr::modulus()) throw Error(NZCB_ERR_FORMAT, "r1cs: coefficient not reduced");
    return to_mont(v);
  }
};

struct R1csCircuit {
  Circuit c;
  int power = 0;
  uint32_t n_public = 0;
};

static R1csCircuit circuit_from_r1cs(const uint8_t* d, size_t len) {
  BinSections b = read_binfile(d, len, "r1cs", "r1cs");
  if (b.sec[1].empty() || b.sec[2].empty()) throw Error(NZCB_ERR_FORMAT, "r1cs: missing header or constraints");
  ByteReader h{b.sec[1][0].first, b.sec[1][0].second};
  if (h.u32() != 32) throw Error(NZCB_ERR_FORMAT, "r1cs: field size is not 32 bytes");
  if (h.left < 32 || std::memcmp(h.p, FrParams::P, 32) != 0)
    throw Error(NZCB_ERR_CURVE, "r1cs curve does not match powers of tau ceremony curve");
  h.p += 32;
  h.left -= 32;
  const uint32_t n_wires = h.u32(), n_out = h.u32(), n_pub_in = h.u32();
  (void)h.u32();  // private inputs
  (void)h.u64();  // labels
  const uint32_t n_cons = h.u32();
  R1csCircuit r;
  Circuit& c = r.c;
  r.n_public = n_out + n_pub_in;
  if (r.n_public >= n_wires) throw Error(NZCB_ERR_FORMAT, "r1cs: more public signals than wires");
  uint32_t nvars = n_wires;
  auto gate = [&](uint32_t sl, uint32_t sr, uint32_t so, const Fr& qm, const Fr& ql, const Fr& qr, const Fr& qo,
                  const Fr& qc) {
    c.sa.push_back(sl);
    c.sb.push_back(sr);
    c.sc.push_back(so);
    c.q[0].push_back(qm);
    c.q[1].push_back(ql);
    c.q[2].push_back(qr);
    c.q[3].push_back(qo);
    c.q[4].push_back(qc);
  };
  using Term = std::pair<uint32_t, Fr>;
  std::function<Term(const std::vector<Term>&, size_t, size_t)> reduce = [&](const std::vector<Term>& v, size_t lo,
                                                                              size_t hi) -> Term {
    const size_t m = hi - lo;
    if (m == 0) return {0u, Fr::zero()};
    if (m == 1) return v[lo];
    const Term t1 = reduce(v, lo, lo + (m >> 1));
    const Term t2 = reduce(v, lo + (m >> 1), hi);
    const uint32_t so = nvars++;
    gate(t1.first, t2.first, so, Fr::zero(), neg(t1.second), neg(t2.second), Fr::one(), Fr::zero());
    c.ax.push_back(t1.first);
    c.ay.push_back(t2.first);
    c.ac.push_back(t1.second);
    c.bc.push_back(t2.second);
    return {so, Fr::one()};
  };
  struct Lc {
    uint32_t s;
    Fr coef, k;
  };
  ByteReader cr{b.sec[2][0].first, b.sec[2][0].second};
  auto read_lc = [&]() -> Lc {
    Lc lc{0u, Fr::zero(), Fr::zero()};
    std::vector<Term> terms;
    const uint32_t nt = cr.u32();
    for (uint32_t i = 0; i < nt; i++) {
      const uint32_t s = cr.u32();
      const Fr coef = cr.fr_normal();
      if (s >= n_wires) throw Error(NZCB_ERR_FORMAT, "r1cs: signal out of range");
      if (s == 0) lc.k = coef;
      else terms.push_back({s, coef});
    }
    const Term t = reduce(terms, 0, terms.size());
    lc.s = t.first;
    lc.coef = t.second;
    return lc;
  };
  for (uint32_t s = 1; s <= r.n_public; s++)
    gate(s, 0, 0, Fr::zero(), Fr::one(), Fr::zero(), Fr::zero(), Fr::zero());
  for (uint32_t i = 0; i < n_cons; i++) {
    const Lc A = read_lc();
    const Lc B = read_lc();
    const Lc C = read_lc();
    gate(A.s, B.s, C.s, A.coef * B.coef, A.coef * B.k, A.k * B.coef, neg(C.coef), A.k * B.k - C.k);
  }
  const size_t nc = c.sa.size();
  int p = 0;  // snarkjs: cirPower = log2(nConstraints - 1) + 1, at least 3
  for (size_t v = nc ? nc - 1 : 0; v > 1; v >>= 1) p++;
  p += 1;
  if (p < 3) p = 3;
  r.power = p;
  c.n = 1u << p;
  c.n_public = r.n_public;
  c.n_vars = nvars;
  c.n_add = (uint32_t)c.ax.size();
  c.n_wit = n_wires;
  return r;
}

static void plonk_setup(const uint8_t* r1cs, size_t r1cs_len, const uint8_t* ptau, size_t ptau_len, int device,
                        uint8_t** zk_out, size_t* zk_len) {
  BinSections pt = read_binfile(ptau, ptau_len, "ptau", "ptau");
  if (pt.sec[1].empty() || pt.sec[2].empty() || pt.sec[3].empty())
    throw Error(NZCB_ERR_FORMAT, "ptau: missing header, tauG1 or tauG2");
  ByteReader h{pt.sec[1][0].first, pt.sec[1][0].second};
  if (h.u32() != 32 || h.left < 40 || std::memcmp(h.p, FqParams::P, 32) != 0)
    throw Error(NZCB_ERR_FORMAT, "ptau: not a bn128 powers of tau file");
  h.p += 32;
  h.left -= 32;
  const uint32_t ptau_power = h.u32();
  R1csCircuit rc = circuit_from_r1cs(r1cs, r1cs_len);
  if (rc.power > (int)ptau_power || rc.power > 24) {
    char msg[128];
    std::snprintf(msg, sizeof msg, "circuit too big for this power of tau ceremony. %zu > 2**%u", rc.c.sa.size(),
                  ptau_power);
    throw Error(NZCB_ERR_ARG, msg);
  }
  if (pt.sec[3][0].second < 256) throw Error(NZCB_ERR_FORMAT, "ptau: tauG2 section too small");
  PtauSrc src;
  src.g1 = pt.sec[2][0].first;
  src.g1_count = pt.sec[2][0].second / 64;
  src.x2 = pt.sec[3][0].first + 128;
  setup_zkey(rc.c, rc.power, (int)rc.n_public, src, device, zk_out, zk_len);
}

// A powers-of-tau file for a trapdoor tau (the layout `snarkjs powersoftau` writes,
// sections 1-3, which is all `plonk setup` reads): header (n8, q, power, ceremonyPower),
// tauG1 = [tau^i]G1 for i < 2^(power+1) - 1 (LEM affine, from the GPU fixed-base kernel)
// and tauG2 = [1]G2, [tau]G2. Stands in for powersOfTau28_hez_final_21.ptau
// (/root/reference/README.md:40), which is not on disk.
static void ptau_synth(int power, const uint8_t* tau_le, int device, uint8_t** out, size_t* out_len) {
  if (power < 1 || power > 24) throw Error(NZCB_ERR_ARG, "ptau: power must be in 1..24");
  const size_t ng1 = ((size_t)2 << power) - 1;
  Fr tau = Fr::zero();
  std::memcpy(tau.v, tau_le, 32);
  tau = reduce_once(reduce_once(tau));
  const Fr tau_m = to_mont(tau);
  hipStream_t st;
  NZ_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  std::vector<uint8_t> g1(ng1 * 64);
  try {
    DevBuf<Fr> taupow(ng1);
    DevBuf<G1Affine> pts(ng1);
    hipLaunchKernelGGL(k_pow_table, dim3(grid_for(ng1, kT, 1u << 30)), dim3(kT), 0, st, taupow.p, tau_m, ng1);
    hipLaunchKernelGGL(k_fixed_base, dim3(grid_for(ng1, kT, 1u << 30)), dim3(kT), 0, st, taupow.p, ng1, pts.p);
    NZ_HIP(hipGetLastError());
    NZ_HIP(hipMemcpyAsync(g1.data(), pts.p, ng1 * 64, hipMemcpyDeviceToHost, st));
    NZ_HIP(hipStreamSynchronize(st));
  } catch (...) {
    (void)hipStreamDestroy(st);
    throw;
  }
  (void)hipStreamDestroy(st);
  std::vector<uint8_t> s1, s3;
  put_u32(s1, 32);
  put_bytes(s1, FqParams::P, 32);
  put_u32(s1, (uint32_t)power);
  put_u32(s1, (uint32_t)power);
  Fr one_n = Fr::zero();
  one_n.v[0] = 1;
  for (const G2& q : {g2_mul_gen(one_n), g2_mul_gen(tau)}) {
    put_bytes(s3, q.x.c0.v, 32);
    put_bytes(s3, q.x.c1.v, 32);
    put_bytes(s3, q.y.c0.v, 32);
    put_bytes(s3, q.y.c1.v, 32);
  }
  const size_t total = 12 + 3 * 12 + s1.size() + g1.size() + s3.size();
  uint8_t* buf = (uint8_t*)std::malloc(total);
  if (!buf) throw Error(NZCB_ERR_INTERNAL, "out of host memory");
  size_t o = 0;
  auto w32 = [&](uint32_t v) { std::memcpy(buf + o, &v, 4); o += 4; };
  auto w64 = [&](uint64_t v) { std::memcpy(buf + o, &v, 8); o += 8; };
  std::memcpy(buf, "ptau", 4);
  o = 4;
  w32(1);
  w32(3);
  const std::vector<uint8_t>* secs[3] = {&s1, &g1, &s3};
  for (int i = 0; i < 3; i++) {
    w32((uint32_t)(i + 1));
    w64(secs[i]->size());
    std::memcpy(buf + o, secs[i]->data(), secs[i]->size());
    o += secs[i]->size();
  }
  *out = buf;
  *out_len = total;
}

}  // namespace nzcb

extern "C" int nzcb_ptau_synth(int power, const uint8_t* tau, int device, uint8_t** ptau_out, size_t* ptau_len,
                               nzcb_err* err) {
  using namespace nzcb;
  if (!tau || !ptau_out || !ptau_len) {
    set_err(err, NZCB_ERR_ARG, "null argument");
    return NZCB_ERR_ARG;
  }
  try {
    NZ_HIP(hipSetDevice(device));
    ptau_synth(power, tau, device, ptau_out, ptau_len);
    return 0;
  } catch (const Error& e) {
    set_err(err, e.code, e.what());
    return e.code;
  } catch (const std::exception& e) {
    set_err(err, NZCB_ERR_INTERNAL, e.what());
    return NZCB_ERR_INTERNAL;
  }
}

extern "C" int nzcb_synth_setup_ex(int power, int n_public, int n_inputs, uint64_t seed, uint32_t n_constraints,
                                   uint32_t flags, const uint8_t* tau, int device, uint8_t** zkey_out,
                                   size_t* zkey_len, uint8_t** wtns_out, size_t* wtns_len, nzcb_err* err) {
  using namespace nzcb;
  if (!tau || !zkey_out || !zkey_len || !wtns_out || !wtns_len) {
    set_err(err, NZCB_ERR_ARG, "null argument");
    return NZCB_ERR_ARG;
  }
  try {
    NZ_HIP(hipSetDevice(device));
    synth_setup(power, n_public, n_inputs, seed, n_constraints, flags, tau, device, zkey_out, zkey_len, wtns_out,
                wtns_len);
    return 0;
  } catch (const Error& e) {
    set_err(err, e.code, e.what());
    return e.code;
  } catch (const std::exception& e) {
    set_err(err, NZCB_ERR_INTERNAL, e.what());
    return NZCB_ERR_INTERNAL;
  }
}

extern "C" int nzcb_synth_setup(int power, int n_public, int n_inputs, uint64_t seed, uint32_t n_constraints,
                                const uint8_t* tau, int device, uint8_t** zkey_out, size_t* zkey_len,
                                uint8_t** wtns_out, size_t* wtns_len, nzcb_err* err) {
  return nzcb_synth_setup_ex(power, n_public, n_inputs, seed, n_constraints, 0, tau, device, zkey_out, zkey_len,
                             wtns_out, wtns_len, err);
}

extern "C" int nzcb_plonk_setup(const uint8_t* r1cs, size_t r1cs_len, const uint8_t* ptau, size_t ptau_len,
                                int device, uint8_t** zkey_out, size_t* zkey_len, nzcb_err* err) {
  using namespace nzcb;
  if (!r1cs || !ptau || !zkey_out || !zkey_len) {
    set_err(err, NZCB_ERR_ARG, "null argument");
    return NZCB_ERR_ARG;
  }
  try {
    NZ_HIP(hipSetDevice(device));
    plonk_setup(r1cs, r1cs_len, ptau, ptau_len, device, zkey_out, zkey_len);
    return 0;
  } catch (const Error& e) {
    set_err(err, e.code, e.what());
    return e.code;
  } catch (const std::exception& e) {
    set_err(err, NZCB_ERR_INTERNAL, e.what());
    return NZCB_ERR_INTERNAL;
  }
}
