// snarkjs 0.4 .zkey / .wtns parsing (see zkey.h).
#include "zkey.h"

#include <cstring>

namespace nzcb {

static const uint32_t kRLimbs[8] = {0xf0000001u, 0x43e1f593u, 0x79b97091u, 0x2833e848u,
                                    0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
static const uint32_t kQLimbs[8] = {0xd87cfd47u, 0x3c208c16u, 0x6871ca8du, 0x97816a91u,
                                    0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};

const Section& BinFile::get(uint32_t id, const char* what) const {
  if (id >= sec.size() || !sec[id].p) throw Error(NZCB_ERR_FORMAT, std::string("missing section: ") + what);
  return sec[id];
}

BinFile parse_binfile(const uint8_t* data, size_t len, const char magic[4]) {
  if (!data || len < 12 || std::memcmp(data, magic, 4) != 0)
    throw Error(NZCB_ERR_FORMAT, std::string(magic, 4) + ": Invalid File format");
  BinFile f;
  uint32_t nsec;
  std::memcpy(&f.version, data + 4, 4);
  std::memcpy(&nsec, data + 8, 4);
  size_t off = 12;
  for (uint32_t i = 0; i < nsec; i++) {
    if (off + 12 > len) throw Error(NZCB_ERR_FORMAT, "truncated section header");
    uint32_t id;
    uint64_t sz;
    std::memcpy(&id, data + off, 4);
    std::memcpy(&sz, data + off + 4, 8);
    off += 12;
    if (sz > len - off) throw Error(NZCB_ERR_FORMAT, "truncated section");
    if (id > 64) throw Error(NZCB_ERR_FORMAT, "bad section id");
    if (f.sec.size() <= id) f.sec.resize(id + 1);
    if (f.sec[id].p) throw Error(NZCB_ERR_FORMAT, "duplicated section");
    f.sec[id].p = data + off;
    f.sec[id].len = sz;
    off += sz;
  }
  return f;
}

namespace {
struct Reader {
  const uint8_t* p;
  uint64_t left;
  void need(uint64_t n) {
    if (n > left) throw Error(NZCB_ERR_FORMAT, "zkey header truncated");
  }
  uint32_t u32() {
    need(4);
    uint32_t v;
    std::memcpy(&v, p, 4);
    p += 4;
    left -= 4;
    return v;
  }
  const uint8_t* bytes(uint64_t n) {
    need(n);
    const uint8_t* r = p;
    p += n;
    left -= n;
    return r;
  }
};

G1Affine read_g1(Reader& r) {
  G1Affine a;
  std::memcpy(&a, r.bytes(64), 64);
  return a;
}
}  // namespace

Zkey parse_zkey(const uint8_t* data, size_t len) {
  Zkey z;
  z.f = parse_binfile(data, len, "zkey");
  const Section& s1 = z.f.get(1, "header");
  if (s1.len < 4) throw Error(NZCB_ERR_FORMAT, "zkey header truncated");
  uint32_t protocol;
  std::memcpy(&protocol, s1.p, 4);
  if (protocol != 2) throw Error(NZCB_ERR_NOT_PLONK, "zkey file is not plonk");
  const Section& s2 = z.f.get(2, "plonk header");
  Reader r{s2.p, s2.len};
  z.n8q = r.u32();
  const uint8_t* q = r.bytes(z.n8q);
  z.n8r = r.u32();
  const uint8_t* rr = r.bytes(z.n8r);
  if (z.n8q != 32 || z.n8r != 32 || std::memcmp(q, kQLimbs, 32) != 0 || std::memcmp(rr, kRLimbs, 32) != 0)
    throw Error(NZCB_ERR_CURVE, "Curve not supported");
  z.nVars = r.u32();
  z.nPublic = r.u32();
  z.domainSize = r.u32();
  z.nAdditions = r.u32();
  z.nConstraints = r.u32();
  if (z.domainSize == 0 || (z.domainSize & (z.domainSize - 1)))
    throw Error(NZCB_ERR_FORMAT, "domainSize is not a power of two");
  z.power = ilog2(z.domainSize);
  if (z.power + 2 > 28) throw Error(NZCB_ERR_FORMAT, "domain too large");
  if (z.nConstraints > z.domainSize) throw Error(NZCB_ERR_FORMAT, "more constraints than domain points");
  std::memcpy(z.k1.v, r.bytes(32), 32);
  std::memcpy(z.k2.v, r.bytes(32), 32);
  z.Qm = read_g1(r);
  z.Ql = read_g1(r);
  z.Qr = read_g1(r);
  z.Qo = read_g1(r);
  z.Qc = read_g1(r);
  z.S1 = read_g1(r);
  z.S2 = read_g1(r);
  z.S3 = read_g1(r);
  std::memcpy(z.X2, r.bytes(128), 128);
  const uint64_t n = z.domainSize;
  auto sized = [&](uint32_t id, const char* what, uint64_t want) {
    const Section& s = z.f.get(id, what);
    if (s.len < want) throw Error(NZCB_ERR_FORMAT, std::string("section too short: ") + what);
    Section o = s;
    o.len = want;
    return o;
  };
  z.additions = sized(3, "additions", (uint64_t)z.nAdditions * 72);
  z.amap = sized(4, "A map", (uint64_t)z.nConstraints * 4);
  z.bmap = sized(5, "B map", (uint64_t)z.nConstraints * 4);
  z.cmap = sized(6, "C map", (uint64_t)z.nConstraints * 4);
  z.qm = sized(7, "Qm", 5 * n * 32);
  z.ql = sized(8, "Ql", 5 * n * 32);
  z.qr = sized(9, "Qr", 5 * n * 32);
  z.qo = sized(10, "Qo", 5 * n * 32);
  z.qc = sized(11, "Qc", 5 * n * 32);
  z.sigma = sized(12, "sigma", 15 * n * 32);
  const Section& lag = z.f.get(13, "lagrange");
  z.nLagrange = (uint32_t)(lag.len / (5 * n * 32));
  uint32_t need_l = z.nPublic > 0 ? z.nPublic : 1;
  if (z.nLagrange < need_l) throw Error(NZCB_ERR_FORMAT, "lagrange section too short");
  z.lagrange = lag;
  z.ptau = sized(14, "PTau", (n + 6) * 64);
  return z;
}

Wtns parse_wtns(const uint8_t* data, size_t len) {
  Wtns w;
  BinFile f = parse_binfile(data, len, "wtns");
  const Section& s1 = f.get(1, "wtns header");
  Reader r{s1.p, s1.len};
  w.n8 = r.u32();
  const uint8_t* q = r.bytes(w.n8);
  w.nWitness = r.u32();
  w.q_is_r = (w.n8 == 32 && std::memcmp(q, kRLimbs, 32) == 0);
  const Section& s2 = f.get(2, "wtns data");
  if (s2.len < (uint64_t)w.nWitness * w.n8) throw Error(NZCB_ERR_FORMAT, "wtns data truncated");
  w.values = s2.p;
  return w;
}

}  // namespace nzcb
