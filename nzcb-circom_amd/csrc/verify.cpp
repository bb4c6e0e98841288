// PLONK verification key, pairing verifier and Solidity calldata (host code;
// SURVEY.md §8f ranks 1 and 4).
//
// Replaces, next to the prover:
//   snarkjs zkey export verificationkey   (zkey_export_verificationkey.js [EXT];
//                                           /root/reference/Makefile:56,61)
//   snarkjs plonk verify / plonk.verify    (plonk_verify.js [EXT])
//   snarkjs zkey export soliditycalldata   (plonk_exportsoliditycalldata.js [EXT];
//                                           consumer of /root/reference/Makefile:57,62)
// The verifier recomputes the Fiat-Shamir challenges with the prover's transcript
// (transcript.h), the linearisation commitment D, F and E, and checks
// e(-(Wxi + u Wxiw), X_2) * e(xi Wxi + u xi w Wxiw + F - E, [1]_2) == 1 with a BN254
// optimal-ate pairing: Fq12 = Fq[w]/(w^12 - 18 w^6 + 82) (Fq2 embedded by u = w^6 - 9),
// D-type twist (x, y) -> (x w^2, y w^3), Miller loop over 6x + 2 with affine Fq2 steps
// and sparse lines, Frobenius corrections, and the exponent (p^12 - 1)/r. The CPU
// oracle oracle/pairing.py states the same algorithm; tests/test_verify.py pins both.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstring>
#include <string>
#include <vector>

#include "../../include/nzcb.h"
#include "common.h"
#include "ec.h"
#include "msm.h"
#include "ntt.h"
#include "transcript.h"
#include "zkey.h"

namespace nzcb {

namespace {

Fq fq_small(uint32_t k) {
  Fq x = Fq::zero();
  x.v[0] = k;
  return to_mont(x);
}
Fq fq_from_normal(const uint32_t (&v)[8]) {
  Fq x;
  for (int i = 0; i < 8; i++) x.v[i] = v[i];
  return to_mont(x);
}

// ---------------------------------------------------------------- Fq2 = Fq[u]/(u^2+1)
struct F2 {
  Fq a, b;
};
F2 f2_add(const F2& x, const F2& y) { return {x.a + y.a, x.b + y.b}; }
F2 f2_sub(const F2& x, const F2& y) { return {x.a - y.a, x.b - y.b}; }
F2 f2_neg(const F2& x) { return {neg(x.a), neg(x.b)}; }
F2 f2_conj(const F2& x) { return {x.a, neg(x.b)}; }
F2 f2_mul(const F2& x, const F2& y) {
  const Fq aa = x.a * y.a, bb = x.b * y.b;
  return {aa - bb, (x.a + x.b) * (y.a + y.b) - aa - bb};
}
F2 f2_scale(const F2& x, const Fq& k) { return {x.a * k, x.b * k}; }
F2 f2_inv(const F2& x) {
  const Fq d = inverse(x.a * x.a + x.b * x.b);
  return {x.a * d, neg(x.b) * d};
}
bool f2_eq(const F2& x, const F2& y) { return x.a == y.a && x.b == y.b; }
bool f2_zero(const F2& x) { return x.a.is_zero() && x.b.is_zero(); }

// ---------------------------------------------------------------- Fq12 (w^12 = 18 w^6 - 82)
struct F12 {
  Fq c[12];
};
F12 f12_one() {
  F12 r;
  for (auto& x : r.c) x = Fq::zero();
  r.c[0] = Fq::one();
  return r;
}
bool f12_eq(const F12& x, const F12& y) {
  for (int i = 0; i < 12; i++)
    if (!(x.c[i] == y.c[i])) return false;
  return true;
}
F12 f12_mul(const F12& x, const F12& y) {
  static const Fq k18 = fq_small(18), k82 = fq_small(82);
  Fq t[23];
  for (auto& v : t) v = Fq::zero();
  for (int i = 0; i < 12; i++) {
    if (x.c[i].is_zero()) continue;
    for (int j = 0; j < 12; j++) t[i + j] = t[i + j] + x.c[i] * y.c[j];
  }
  for (int k = 22; k >= 12; k--) {
    if (t[k].is_zero()) continue;
    t[k - 6] = t[k - 6] + t[k] * k18;
    t[k - 12] = t[k - 12] - t[k] * k82;
  }
  F12 r;
  for (int i = 0; i < 12; i++) r.c[i] = t[i];
  return r;
}
// e (Fq2) times w^k, k + 6 < 12
F12 f12_from_f2(const F2& e, int k) {
  static const Fq k9 = fq_small(9);
  F12 r;
  for (auto& v : r.c) v = Fq::zero();
  r.c[k] = e.a - e.b * k9;
  r.c[k + 6] = e.b;
  return r;
}

// (p^12 - 1) / r, little-endian 64-bit limbs (2790 bits)
const uint64_t kFinalExp[44] = {
    0x86964b64ca86f120ULL, 0x40a4efb7e54523a4ULL, 0x837fa97896e84abbULL, 0x361102b6b9b2b918ULL,
    0xc0de81def35692daULL, 0xbe04c7e8a6c3c760ULL, 0xd766f9c9d570bb7fULL, 0xc230974d83561841ULL,
    0x5bba1668c3be69a3ULL, 0x7f3811c410526294ULL, 0x29baee7ddadda71cULL, 0xbf813b8d145da900ULL,
    0x641bbadf423f9a2cULL, 0xa80bb4ea44eacc5eULL, 0xcd65664814fde37cULL, 0x4a0364b9580291d2ULL,
    0xee93dfb10826f0ddULL, 0x6b42db8dc5514724ULL, 0xbb10cf430b0f3785ULL, 0x40494e406f804216ULL,
    0x55cfe107acf3aafbULL, 0x2088ec80e0ebae87ULL, 0x846a3ed011a337a0ULL, 0x48a45a4a1e3a5195ULL,
    0xe5664568dfc50e16ULL, 0xab6a41294c0cc4ebULL, 0x82d0d602d268c7daULL, 0x6668449aed3cc48aULL,
    0x5062cd0fb2015dfcULL, 0x7f2940a8b1ddb3d1ULL, 0x77f5b63a2a226448ULL, 0xfef0781361e443aeULL,
    0xf977870e88d5c6c8ULL, 0x790364a61f676baaULL, 0x5887e72eceaddea3ULL, 0x1377e563a09a1b70ULL,
    0x0c54efee1bd8c3b2ULL, 0x3ec3d15ad524d8f7ULL, 0xdaf15466b2383a5dULL, 0xe1e30a73bb94fec0ULL,
    0x6a1c71015f3f7be2ULL, 0x842d43bf6369b1ffULL, 0x20fddadf107d20bcULL, 0x0000002f4b6dc970ULL};

F12 f12_pow(F12 a, const uint64_t* e, int nlimbs) {
  // left-to-right, 4-bit fixed window
  F12 tab[16];
  tab[0] = f12_one();
  for (int i = 1; i < 16; i++) tab[i] = f12_mul(tab[i - 1], a);
  F12 r = f12_one();
  bool started = false;
  for (int l = nlimbs - 1; l >= 0; l--) {
    for (int sh = 60; sh >= 0; sh -= 4) {
      if (started)
        for (int k = 0; k < 4; k++) r = f12_mul(r, r);
      const int d = (int)((e[l] >> sh) & 15);
      if (d) {
        r = started ? f12_mul(r, tab[d]) : tab[d];
        started = true;
      }
    }
  }
  return r;
}

// ---------------------------------------------------------------- G2 (twist), affine
struct P2 {
  F2 x, y;
  bool inf = false;
};
P2 p2_add(const P2& t, const P2& s) {
  if (t.inf) return s;
  if (s.inf) return t;
  F2 lam;
  if (f2_eq(t.x, s.x)) {
    if (f2_zero(f2_add(t.y, s.y))) return P2{{}, {}, true};
    const F2 xx = f2_mul(t.x, t.x);
    lam = f2_mul(f2_add(f2_add(xx, xx), xx), f2_inv(f2_add(t.y, t.y)));
  } else {
    lam = f2_mul(f2_sub(s.y, t.y), f2_inv(f2_sub(s.x, t.x)));
  }
  P2 r;
  r.x = f2_sub(f2_sub(f2_mul(lam, lam), t.x), s.x);
  r.y = f2_sub(f2_mul(lam, f2_sub(t.x, r.x)), t.y);
  return r;
}

// line through T and S (tangent when equal) evaluated at P = (xp, yp) in G1
F12 line(const P2& t, const P2& s, const Fq& xp, const Fq& yp) {
  F12 r;
  for (auto& v : r.c) v = Fq::zero();
  if (f2_eq(t.x, s.x) && f2_zero(f2_add(t.y, s.y))) {  // vertical: xP - xT w^2
    const F12 tx = f12_from_f2(t.x, 2);
    for (int i = 0; i < 12; i++) r.c[i] = neg(tx.c[i]);
    r.c[0] = r.c[0] + xp;
    return r;
  }
  F2 lam;
  if (f2_eq(t.x, s.x) && f2_eq(t.y, s.y)) {
    const F2 xx = f2_mul(t.x, t.x);
    lam = f2_mul(f2_add(f2_add(xx, xx), xx), f2_inv(f2_add(t.y, t.y)));
  } else {
    lam = f2_mul(f2_sub(s.y, t.y), f2_inv(f2_sub(s.x, t.x)));
  }
  // yP - lam xP w + (lam xT - yT) w^3
  const F12 a = f12_from_f2(f2_scale(lam, neg(xp)), 1);
  const F12 b = f12_from_f2(f2_sub(f2_mul(lam, t.x), t.y), 3);
  for (int i = 0; i < 12; i++) r.c[i] = a.c[i] + b.c[i];
  r.c[0] = r.c[0] + yp;
  return r;
}

const uint64_t kAteLoop = 0x9d797039be763ba8ULL;  // 6x + 2 = 2^64 + this (bit 64 set)

F12 miller_loop(const P2& q, const G1Affine& p) {
  if (q.inf || p.is_inf()) return f12_one();
  static const F2 g12 = {fq_from_normal({0x176f553du, 0x99e39557u, 0xc2c3330cu, 0xb78cc310u, 0xf559b143u, 0x4c0bec3cu,
                                        0x4f7911f7u, 0x2fb34798u}),
                         fq_from_normal({0x640fcba2u, 0x1665d51cu, 0x0b7c9dceu, 0x32ae2a1du, 0xd75a0794u, 0x4ba4cc8bu,
                                         0x61ebae20u, 0x16c9e550u})};
  static const F2 g13 = {fq_from_normal({0x71a0135au, 0xdc540146u, 0xa9c95998u, 0xdbaae0edu, 0xb6e2f9b9u, 0xdc5ec698u,
                                         0x489af5dcu, 0x063cf305u}),
                         fq_from_normal({0x2623b0e3u, 0x82d37f63u, 0x8fa25bd2u, 0x21807dc9u, 0xec796f2bu, 0x0704b5a7u,
                                         0xac41049au, 0x07c03cbcu})};
  static const Fq g22 = fq_from_normal({0x607cfd48u, 0xe4bd44e5u, 0xbb966e3du, 0xc28f069fu, 0xe0acccb0u, 0x5e6dd9e7u,
                                        0xe131a029u, 0x30644e72u});
  P2 r = q;
  F12 f = f12_one();
  for (int i = 63; i >= 0; i--) {
    f = f12_mul(f12_mul(f, f), line(r, r, p.x, p.y));
    r = p2_add(r, r);
    if ((kAteLoop >> i) & 1) {
      f = f12_mul(f, line(r, q, p.x, p.y));
      r = p2_add(r, q);
    }
  }
  P2 q1;  // pi(Q)
  q1.x = f2_mul(f2_conj(q.x), g12);
  q1.y = f2_mul(f2_conj(q.y), g13);
  P2 nq2;  // -pi^2(Q): xi^((p^2-1)/2) = -1, negated back
  nq2.x = f2_scale(q.x, g22);
  nq2.y = q.y;
  f = f12_mul(f, line(r, q1, p.x, p.y));
  r = p2_add(r, q1);
  f = f12_mul(f, line(r, nq2, p.x, p.y));
  return f;
}

bool pairing_check(const std::vector<std::pair<G1Affine, P2>>& pairs) {
  F12 f = f12_one();
  for (const auto& pq : pairs) f = f12_mul(f, miller_loop(pq.second, pq.first));
  return f12_eq(f12_pow(f, kFinalExp, 44), f12_one());
}

// ---------------------------------------------------------------- G1 helpers (host)
G1xyzz g1_mul(const G1Affine& p, const Fr& k_mont) {
  const Fr k = from_mont(k_mont);
  G1xyzz acc = G1xyzz::inf();
  if (p.is_inf()) return acc;
  for (int b = 255; b >= 0; b--) {
    acc = xyzz_dbl(acc);
    if ((k.v[b >> 5] >> (b & 31)) & 1u) acc = xyzz_add_affine(acc, p.x, p.y);
  }
  return acc;
}
G1Affine g1_neg(const G1Affine& p) {
  G1Affine r = p;
  if (!p.is_inf()) r.y = neg(p.y);
  return r;
}
bool g1_on_curve(const G1Affine& p) {
  if (p.is_inf()) return true;
  return p.y * p.y == p.x * p.x * p.x + fq_small(3);
}

Fq fq_from_le_normal(const uint8_t* le, bool* ok) {
  Fq x;
  std::memcpy(x.v, le, 32);
  const Fq y = reduce_once(x);
  if (!(y == x)) *ok = false;  // not canonical (>= p)
  return to_mont(x);
}
Fr fr_from_le_checked(const uint8_t* le, bool* ok) {
  Fr x;
  std::memcpy(x.v, le, 32);
  const Fr y = reduce_once(x);
  if (!(y == x)) *ok = false;  // >= r
  return to_mont(x);
}
G1Affine g1_from_le(const uint8_t* p, bool* ok) {
  G1Affine a;
  a.x = fq_from_le_normal(p, ok);
  a.y = fq_from_le_normal(p + 32, ok);
  return a;
}
void g1_to_le(const G1Affine& a, uint8_t* out) {
  if (a.is_inf()) {
    std::memset(out, 0, 64);
    return;
  }
  const Fq x = from_mont(a.x), y = from_mont(a.y);
  std::memcpy(out, x.v, 32);
  std::memcpy(out + 32, y.v, 32);
}

// binary verification key (include/nzcb.h NZCB_VK_BYTES)
struct Vk {
  uint32_t nPublic = 0, power = 0;
  Fr k1, k2, w;
  G1Affine q[8];  // Qm, Ql, Qr, Qo, Qc, S1, S2, S3
  P2 x2;
};

void vk_write(const Zkey& z, uint8_t* out) {
  std::memcpy(out, &z.nPublic, 4);
  const uint32_t pw = (uint32_t)z.power;
  std::memcpy(out + 4, &pw, 4);
  fr_to_le_normal(z.k1, out + 8);
  fr_to_le_normal(z.k2, out + 40);
  const G1Affine* pts[8] = {&z.Qm, &z.Ql, &z.Qr, &z.Qo, &z.Qc, &z.S1, &z.S2, &z.S3};
  for (int i = 0; i < 8; i++) g1_to_le(*pts[i], out + 72 + 64 * i);
  for (int i = 0; i < 4; i++) {  // X_2: x.c0, x.c1, y.c0, y.c1 (LEM in the zkey)
    Fq v;
    std::memcpy(v.v, z.X2 + 32 * i, 32);
    const Fq nv = from_mont(v);
    std::memcpy(out + 584 + 32 * i, nv.v, 32);
  }
  fr_to_le_normal(fr_root_of_unity(z.power), out + 712);
}

Vk vk_read(const uint8_t* in, bool* ok) {
  Vk v;
  std::memcpy(&v.nPublic, in, 4);
  std::memcpy(&v.power, in + 4, 4);
  if (v.power > 28) *ok = false;
  v.k1 = fr_from_le_checked(in + 8, ok);
  v.k2 = fr_from_le_checked(in + 40, ok);
  for (int i = 0; i < 8; i++) v.q[i] = g1_from_le(in + 72 + 64 * i, ok);
  v.x2.x = {fq_from_le_normal(in + 584, ok), fq_from_le_normal(in + 616, ok)};
  v.x2.y = {fq_from_le_normal(in + 648, ok), fq_from_le_normal(in + 680, ok)};
  v.w = fr_from_le_checked(in + 712, ok);
  return v;
}

P2 g2_generator() {
  P2 g;
  g.x = {fq_from_normal({0xd992f6edu, 0x46debd5cu, 0xf75edaddu, 0x674322d4u, 0x5e5c4479u, 0x426a0066u, 0x121f1e76u,
                         0x1800deefu}),
         fq_from_normal({0xaef312c2u, 0x97e485b7u, 0x35a9e712u, 0xf1aa4933u, 0x31fb5d25u, 0x7260bfb7u, 0x920d483au,
                         0x198e9393u})};
  g.y = {fq_from_normal({0x66fa7daau, 0x4ce6cc01u, 0x0c43d37bu, 0xe3d1e769u, 0x8dcb408fu, 0x4aab7180u, 0xdb8c6debu,
                         0x12c85ea5u}),
         fq_from_normal({0xd122975bu, 0x55acdadcu, 0x70b38ef3u, 0xbc4b3133u, 0x690c3395u, 0xec9e99adu, 0x585ff075u,
                         0x090689d0u})};
  return g;
}

}  // namespace

// snarkjs plonk_verify restated (see the header comment); true = valid
bool plonk_verify(const Vk& vk, const uint8_t* proof, const uint8_t* pub, int npub, bool transcript_public) {
  bool ok = true;
  G1Affine pt[9];  // A, B, C, Z, T1, T2, T3, Wxi, Wxiw
  for (int i = 0; i < 9; i++) pt[i] = g1_from_le(proof + 64 * i, &ok);
  Fr ev[7];  // eval_a, eval_b, eval_c, eval_s1, eval_s2, eval_zw, eval_r
  for (int i = 0; i < 7; i++) ev[i] = fr_from_le_checked(proof + 576 + 32 * i, &ok);
  std::vector<Fr> pubs(npub);
  for (int i = 0; i < npub; i++) pubs[i] = fr_from_le_checked(pub + 32 * i, &ok);
  if (!ok || (uint32_t)npub != vk.nPublic) return false;
  for (const auto& p : pt)
    if (!g1_on_curve(p)) return false;
  const G1Affine &A = pt[0], &B = pt[1], &C = pt[2], &Z = pt[3], &T1 = pt[4], &T2 = pt[5], &T3 = pt[6],
                 &Wxi = pt[7], &Wxiw = pt[8];
  const Fr &ea = ev[0], &eb = ev[1], &ec = ev[2], &es1 = ev[3], &es2 = ev[4], &ezw = ev[5], &er = ev[6];
  // challenges (transcript.h, as the prover)
  std::vector<uint8_t> tr;
  auto put_fr = [&](const Fr& x) {
    uint8_t b[32];
    fr_to_be(x, b);
    tr.insert(tr.end(), b, b + 32);
  };
  auto put_g1 = [&](const G1Affine& p) {
    uint8_t b[64];
    g1_uncompressed(p, b);
    tr.insert(tr.end(), b, b + 64);
  };
  if (transcript_public)
    for (const auto& x : pubs) put_fr(x);
  put_g1(A);
  put_g1(B);
  put_g1(C);
  const Fr beta = hash_to_fr(tr);
  tr.clear();
  put_fr(beta);
  const Fr gamma = hash_to_fr(tr);
  tr.clear();
  put_g1(Z);
  const Fr alpha = hash_to_fr(tr);
  tr.clear();
  put_g1(T1);
  put_g1(T2);
  put_g1(T3);
  const Fr xi = hash_to_fr(tr);
  tr.clear();
  for (const auto& e : ev) put_fr(e);
  Fr v[7];
  v[1] = hash_to_fr(tr);
  for (int i = 2; i <= 6; i++) v[i] = v[i - 1] * v[1];
  tr.clear();
  put_g1(Wxi);
  put_g1(Wxiw);
  const Fr u = hash_to_fr(tr);
  // evaluations at xi
  const uint64_t n = uint64_t(1) << vk.power;
  const Fr one = Fr::one();
  const Fr xin = pow_u64(xi, n);
  const Fr zh = xin - one;
  Fr nfr = Fr::zero();
  nfr.v[0] = (uint32_t)n;
  nfr.v[1] = (uint32_t)(n >> 32);
  nfr = to_mont(nfr);
  const int nl = npub > 0 ? npub : 1;
  std::vector<Fr> L(nl);
  Fr wp = one;
  for (int i = 0; i < nl; i++) {
    L[i] = wp * zh * inverse(nfr * (xi - wp));
    wp = wp * vk.w;
  }
  Fr pi = Fr::zero();
  for (int i = 0; i < npub; i++) pi = pi - L[i] * pubs[i];
  const Fr alpha2 = alpha * alpha;
  const Fr f1 = (ea + beta * es1 + gamma) * (eb + beta * es2 + gamma);
  const Fr num = er + pi - f1 * (ec + gamma) * ezw * alpha - L[0] * alpha2;
  const Fr t = num * inverse(zh);
  const Fr bx = beta * xi;
  const Fr e2 = (ea + bx + gamma) * (eb + bx * vk.k1 + gamma) * (ec + bx * vk.k2 + gamma) * alpha;
  const Fr e4 = L[0] * alpha2;
  const Fr e3 = f1 * beta * ezw * alpha;
  // D, F, E and the two pairing inputs
  const G1Affine &Qm = vk.q[0], &Ql = vk.q[1], &Qr = vk.q[2], &Qo = vk.q[3], &Qc = vk.q[4], &S1 = vk.q[5],
                 &S2 = vk.q[6], &S3 = vk.q[7];
  std::vector<std::pair<const G1Affine*, Fr>> terms = {
      {&Qm, ea * eb * v[1]}, {&Ql, ea * v[1]}, {&Qr, eb * v[1]}, {&Qo, ec * v[1]}, {&Qc, v[1]},
      {&Z, (e2 + e4) * v[1] + u}, {&S3, neg(e3 * v[1])},
      {&T1, one}, {&T2, xin}, {&T3, xin * xin}, {&A, v[2]}, {&B, v[3]}, {&C, v[4]}, {&S1, v[5]}, {&S2, v[6]},
      {&Wxi, xi}, {&Wxiw, u * xi * vk.w}};
  G1xyzz rhs = G1xyzz::inf();
  for (const auto& tm : terms) rhs = xyzz_add(rhs, g1_mul(*tm.first, tm.second));
  const Fr e = t + v[1] * er + v[2] * ea + v[3] * eb + v[4] * ec + v[5] * es1 + v[6] * es2 + u * ezw;
  G1Affine gen;
  gen.x = fq_small(1);
  gen.y = fq_small(2);
  rhs = xyzz_add(rhs, g1_mul(g1_neg(gen), e));
  const G1xyzz lhs = xyzz_add(g1_mul(Wxi, one), g1_mul(Wxiw, u));
  std::vector<std::pair<G1Affine, P2>> pairs = {{g1_neg(xyzz_to_affine(lhs)), vk.x2},
                                                {xyzz_to_affine(rhs), g2_generator()}};
  return pairing_check(pairs);
}

std::string dec_le32(const uint8_t* le32);  // capi_prover.cpp

}  // namespace nzcb

using namespace nzcb;

extern "C" {

int nzcb_vk_from_zkey(const uint8_t* zkey, size_t zkey_len, uint8_t* vk_out, nzcb_err* err) {
  try {
    if (!zkey || !vk_out) throw Error(NZCB_ERR_ARG, "null argument");
    const Zkey z = parse_zkey(zkey, zkey_len);
    vk_write(z, vk_out);
    if (err) err->code = 0;
    return 0;
  } catch (const Error& e) {
    set_err(err, e.code, e.what());
    return e.code;
  } catch (const std::exception& e) {
    set_err(err, NZCB_ERR_INTERNAL, e.what());
    return NZCB_ERR_INTERNAL;
  }
}

// the same from a zkey file, memory-mapped (a nzcp_live zkey is ~3.9 GB: larger than a
// Node Buffer, so `zkey export verificationkey|solidityverifier` read it through here)
int nzcb_vk_from_zkey_file(const char* zkey_path, uint8_t* vk_out, nzcb_err* err) {
  if (!zkey_path || !vk_out) {
    set_err(err, NZCB_ERR_ARG, "null argument");
    return NZCB_ERR_ARG;
  }
  const int fd = open(zkey_path, O_RDONLY);
  if (fd < 0) {
    set_err(err, NZCB_ERR_ARG, (std::string("cannot open ") + zkey_path).c_str());
    return NZCB_ERR_ARG;
  }
  struct stat st;
  if (fstat(fd, &st) != 0 || st.st_size <= 0) {
    close(fd);
    set_err(err, NZCB_ERR_FORMAT, "zkey file is empty");
    return NZCB_ERR_FORMAT;
  }
  void* m = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
  close(fd);
  if (m == MAP_FAILED) {
    set_err(err, NZCB_ERR_INTERNAL, "mmap of the zkey failed");
    return NZCB_ERR_INTERNAL;
  }
  const int rc = nzcb_vk_from_zkey(static_cast<const uint8_t*>(m), (size_t)st.st_size, vk_out, err);
  munmap(m, (size_t)st.st_size);
  return rc;
}

int nzcb_vk_to_json(const uint8_t* vk, char* out, size_t cap) {
  if (!vk) return -1;
  uint32_t npub, power;
  std::memcpy(&npub, vk, 4);
  std::memcpy(&power, vk + 4, 4);
  auto g1 = [&](const uint8_t* p) {
    bool zero = true;
    for (int i = 0; i < 64; i++) zero = zero && !p[i];
    if (zero) return std::string("[\"0\",\"1\",\"0\"]");
    return "[\"" + dec_le32(p) + "\",\"" + dec_le32(p + 32) + "\",\"1\"]";
  };
  static const char* names[8] = {"Qm", "Ql", "Qr", "Qo", "Qc", "S1", "S2", "S3"};
  std::string s = "{\"protocol\":\"plonk\",\"curve\":\"bn128\",\"nPublic\":" + std::to_string(npub) +
                  ",\"power\":" + std::to_string(power) + ",\"k1\":\"" + dec_le32(vk + 8) + "\",\"k2\":\"" +
                  dec_le32(vk + 40) + "\"";
  for (int i = 0; i < 8; i++) s += std::string(",\"") + names[i] + "\":" + g1(vk + 72 + 64 * i);
  s += ",\"X_2\":[[\"" + dec_le32(vk + 584) + "\",\"" + dec_le32(vk + 616) + "\"],[\"" + dec_le32(vk + 648) +
       "\",\"" + dec_le32(vk + 680) + "\"],[\"1\",\"0\"]]";
  s += ",\"w\":\"" + dec_le32(vk + 712) + "\"}";
  if (!out || cap < s.size() + 1) return (int)(s.size() + 1);
  std::memcpy(out, s.c_str(), s.size() + 1);
  return 0;
}

int nzcb_verify(const uint8_t* vk, const uint8_t* proof, const uint8_t* pub, int n_public, int transcript_public,
                int* valid, nzcb_err* err) {
  try {
    if (!vk || !proof || !valid || n_public < 0 || (n_public && !pub)) throw Error(NZCB_ERR_ARG, "null argument");
    bool ok = true;
    const Vk v = vk_read(vk, &ok);
    if (!ok) throw Error(NZCB_ERR_FORMAT, "invalid verification key");
    *valid = plonk_verify(v, proof, pub, n_public, transcript_public != 0) ? 1 : 0;
    if (err) err->code = 0;
    return 0;
  } catch (const Error& e) {
    set_err(err, e.code, e.what());
    return e.code;
  } catch (const std::exception& e) {
    set_err(err, NZCB_ERR_INTERNAL, e.what());
    return NZCB_ERR_INTERNAL;
  }
}

int nzcb_proof_to_calldata(const uint8_t* proof, const uint8_t* pub, int n_public, char* out, size_t cap) {
  if (!proof || n_public < 0 || (n_public && !pub)) return -1;
  static const char* hx = "0123456789abcdef";
  std::string s = "0x";
  auto put_be = [&](const uint8_t* le32) {
    for (int i = 31; i >= 0; i--) {
      s.push_back(hx[le32[i] >> 4]);
      s.push_back(hx[le32[i] & 15]);
    }
  };
  for (int i = 0; i < 9; i++) {  // uncompressed big-endian x || y (infinity: 0x40 00..)
    const uint8_t* p = proof + 64 * i;
    bool zero = true;
    for (int k = 0; k < 64; k++) zero = zero && !p[k];
    if (zero) {
      s += "40";
      s.append(126, '0');
    } else {
      put_be(p);
      put_be(p + 32);
    }
  }
  for (int i = 0; i < 7; i++) put_be(proof + 576 + 32 * i);
  s += ",[";
  for (int i = 0; i < n_public; i++) {
    if (i) s += ",";
    s += "\"0x";
    put_be(pub + 32 * i);
    s += "\"";
  }
  s += "]";
  if (!out || cap < s.size() + 1) return (int)(s.size() + 1);
  std::memcpy(out, s.c_str(), s.size() + 1);
  return 0;
}

}  // extern "C"
