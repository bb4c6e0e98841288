// snarkjs 0.4 PLONK .zkey and .wtns parsing (host, zero-copy views).
//
// Layout restated in SURVEY.md §8a row a3 (snarkjs 0.4.12 zkey_utils
// readHeaderPlonk / wtns_utils, @iden3/binfileutils@0.0.10 sections;
// /root/reference/yarn.lock:843-849, 7279-7292). Sections are located, not
// copied: the prover uploads the payloads to HBM as-is (they are already the
// Montgomery "LEM" representation the kernels use).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "common.h"
#include "ec.h"

namespace nzcb {

struct Section {
  const uint8_t* p = nullptr;
  uint64_t len = 0;
};

struct BinFile {
  uint32_t version = 0;
  std::vector<Section> sec;  // indexed by section id (0 unused)
  const Section& get(uint32_t id, const char* what) const;
};

BinFile parse_binfile(const uint8_t* data, size_t len, const char magic[4]);

struct Zkey {
  BinFile f;
  uint32_t n8q = 0, n8r = 0;
  uint32_t nVars = 0, nPublic = 0, domainSize = 0, nAdditions = 0, nConstraints = 0;
  int power = 0;
  Fr k1, k2;  // Montgomery (as stored)
  G1Affine Qm, Ql, Qr, Qo, Qc, S1, S2, S3;
  uint8_t X2[128];
  Section additions, amap, bmap, cmap, qm, ql, qr, qo, qc, sigma, lagrange, ptau;
  uint32_t nLagrange = 0;
};

Zkey parse_zkey(const uint8_t* data, size_t len);

struct Wtns {
  uint32_t n8 = 0;
  uint32_t nWitness = 0;
  bool q_is_r = false;
  const uint8_t* values = nullptr;  // nWitness x n8 bytes, normal form LE
};

Wtns parse_wtns(const uint8_t* data, size_t len);

}  // namespace nzcb
