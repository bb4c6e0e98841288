// Solidity PLONK verifier for one verification key: the `snarkjs zkey export
// solidityverifier <zkey> contracts/Verifier*.sol` step of the reference's key build
// (/root/reference/Makefile:57,62), whose contract the reference deploys
// (/root/reference/deploy-script.js:4-7) and calls with the `zkey export
// soliditycalldata` arguments (nzcb_proof_to_calldata: the 800 proof bytes, then the
// public signals).
//
// The contract states the verifier of csrc/verify.cpp (snarkjs 0.4.12 plonk_verify,
// transcript.h) with the EVM's BN254 precompiles: ecAdd (0x06), ecMul (0x07), the
// pairing check (0x08) and modexp (0x05) for the Fr inversions. Every intermediate
// value lives in a memory slot, so no Yul block keeps more than a handful of stack
// variables (solc's stack limit). The proof's G1 points are hashed exactly as they
// arrive (big-endian x || y, infinity as 0x40 followed by zeros, the prover's
// transcript encoding) and decoded to the precompiles' (0, 0) infinity.
//
// Parity is unpinned: the reference holds no generated verifier (its contracts/ is
// empty) and snarkjs's template is not on disk. tests/test_solidity.py runs the
// contract's assembly on proofs of this library with a Yul interpreter (tests/yul.py).
#include <cstring>
#include <string>

#include "common.h"
#include "../../include/nzcb.h"

namespace nzcb {
std::string dec_le32(const uint8_t* le32);  // capi_prover.cpp
}

namespace {

const char* kTemplate = R"SOL(// SPDX-License-Identifier: GPL-3.0
pragma solidity >=0.7.0 <0.9.0;

// PLONK verifier (snarkjs 0.4.12 protocol, BN254) for one verification key, written by
// nzcb-mi355x (nzcb_vk_to_solidity). verifyProof takes the arguments of
// `snarkjs zkey export soliditycalldata`: the 800-byte proof (A, B, C, Z, T1, T2, T3,
// Wxi, Wxiw as big-endian x || y, then eval_a, eval_b, eval_c, eval_s1, eval_s2,
// eval_zw, eval_r) and the public signals.
contract @NAME@ {
    uint256 constant R = 21888242871839275222246405745257275088548364400416034343698204186575808495617;
    uint256 constant Q = 21888242871839275222246405745257275088696311157297823662689037894645226208583;
    uint256 constant N = @N@;
    uint256 constant LOG_N = @POWER@;
    uint256 constant N_PUBLIC = @NPUB@;
    uint256 constant N_LAGRANGE = @NLAG@;
    uint256 constant TRANSCRIPT_PUBLIC = @TPUB@;
    uint256 constant W1 = @W@;
    uint256 constant K1 = @K1@;
    uint256 constant K2 = @K2@;
    uint256 constant QM_X = @QM_X@;
    uint256 constant QM_Y = @QM_Y@;
    uint256 constant QL_X = @QL_X@;
    uint256 constant QL_Y = @QL_Y@;
    uint256 constant QR_X = @QR_X@;
    uint256 constant QR_Y = @QR_Y@;
    uint256 constant QO_X = @QO_X@;
    uint256 constant QO_Y = @QO_Y@;
    uint256 constant QC_X = @QC_X@;
    uint256 constant QC_Y = @QC_Y@;
    uint256 constant S1_X = @S1_X@;
    uint256 constant S1_Y = @S1_Y@;
    uint256 constant S2_X = @S2_X@;
    uint256 constant S2_Y = @S2_Y@;
    uint256 constant S3_X = @S3_X@;
    uint256 constant S3_Y = @S3_Y@;
    // [tau]_2 and the G2 generator in the pairing precompile's order (imaginary part first)
    uint256 constant X2_X_IM = @X2_X_IM@;
    uint256 constant X2_X_RE = @X2_X_RE@;
    uint256 constant X2_Y_IM = @X2_Y_IM@;
    uint256 constant X2_Y_RE = @X2_Y_RE@;
    uint256 constant G2_X_IM = 11559732032986387107991004021392285783925812861821192530917403151452391805634;
    uint256 constant G2_X_RE = 10857046999023057135944570762232829481370756359578518086990519993285655852781;
    uint256 constant G2_Y_IM = 4082367875863433681332203403145435568316851327593401208105741076214120093531;
    uint256 constant G2_Y_RE = 8495653923123431417604973247489272438418190587263600148770280649306958101930;

    function verifyProof(bytes memory proof, uint256[] memory pubSignals) public view returns (bool) {
        if (proof.length != 800 || pubSignals.length != N_PUBLIC) return false;
        bool ok;
        assembly {
            // memory slots (offsets from m): 0x000-0x240 the 9 decoded proof points;
            // 0x240 beta, 0x260 gamma, 0x280 alpha, 0x2a0 xi, 0x2c0 u, 0x2e0-0x380 v1..v6,
            // 0x3a0 xi^n, 0x3c0 xi^n - 1, 0x3e0 PI(xi), 0x400 L1(xi), 0x420 t(xi), 0x440 f1,
            // 0x460 valid flag, 0x480 accumulator point, 0x4c0-0x5c0 precompile scratch,
            // 0x600 transcript / pairing input
            function fr_inv(a, s) -> r {
                mstore(s, 32)
                mstore(add(s, 0x20), 32)
                mstore(add(s, 0x40), 32)
                mstore(add(s, 0x60), a)
                mstore(add(s, 0x80), sub(R, 2))
                mstore(add(s, 0xa0), R)
                if iszero(staticcall(gas(), 5, s, 0xc0, s, 0x20)) { revert(0, 0) }
                r := mload(s)
            }
            // accumulator += k * (px, py)
            function acc_mul(m, px, py, k) {
                let s := add(m, 0x4c0)
                mstore(s, px)
                mstore(add(s, 0x20), py)
                mstore(add(s, 0x40), k)
                if iszero(staticcall(gas(), 7, s, 0x60, add(s, 0x40), 0x40)) { mstore(add(m, 0x460), 0) }
                mstore(s, mload(add(m, 0x480)))
                mstore(add(s, 0x20), mload(add(m, 0x4a0)))
                if iszero(staticcall(gas(), 6, s, 0x80, add(m, 0x480), 0x40)) { mstore(add(m, 0x460), 0) }
            }
            // decode and range-check the proof and the public signals
            function check_input(m, pp, ps) {
                mstore(add(m, 0x460), 1)
                for { let i := 0 } lt(i, 7) { i := add(i, 1) } {
                    if iszero(lt(mload(add(pp, add(576, mul(i, 32)))), R)) { mstore(add(m, 0x460), 0) }
                }
                for { let i := 0 } lt(i, N_PUBLIC) { i := add(i, 1) } {
                    if iszero(lt(mload(add(ps, mul(i, 32))), R)) { mstore(add(m, 0x460), 0) }
                }
                for { let i := 0 } lt(i, 9) { i := add(i, 1) } {
                    let x := mload(add(pp, mul(i, 64)))
                    let y := mload(add(pp, add(mul(i, 64), 32)))
                    let inf := and(eq(x, 0x4000000000000000000000000000000000000000000000000000000000000000), iszero(y))
                    if inf { x := 0 }
                    if iszero(inf) {
                        if iszero(and(lt(x, Q), lt(y, Q))) { mstore(add(m, 0x460), 0) }
                    }
                    mstore(add(m, mul(i, 64)), x)
                    mstore(add(m, add(mul(i, 64), 32)), y)
                }
            }
            // Fiat-Shamir: keccak256 over the prover's transcript (csrc/transcript.h)
            function challenges(m, pp, ps) {
                let t := add(m, 0x600)
                let len := 0
                if TRANSCRIPT_PUBLIC {
                    for { let i := 0 } lt(i, N_PUBLIC) { i := add(i, 1) } {
                        mstore(add(t, mul(i, 32)), mload(add(ps, mul(i, 32))))
                    }
                    len := mul(N_PUBLIC, 32)
                }
                for { let i := 0 } lt(i, 6) { i := add(i, 1) } {
                    mstore(add(t, add(len, mul(i, 32))), mload(add(pp, mul(i, 32))))
                }
                let beta := mod(keccak256(t, add(len, 192)), R)
                mstore(add(m, 0x240), beta)
                mstore(t, beta)
                mstore(add(m, 0x260), mod(keccak256(t, 32), R))
                mstore(add(m, 0x280), mod(keccak256(add(pp, 192), 64), R))
                mstore(add(m, 0x2a0), mod(keccak256(add(pp, 256), 192), R))
                mstore(add(m, 0x2c0), mod(keccak256(add(pp, 448), 128), R))
                let v1 := mod(keccak256(add(pp, 576), 224), R)
                let v := v1
                for { let i := 0 } lt(i, 6) { i := add(i, 1) } {
                    mstore(add(m, add(0x2e0, mul(i, 32))), v)
                    v := mulmod(v, v1, R)
                }
            }
            // xi^n, Z_H(xi), the Lagrange values L_i(xi) and PI(xi) = -sum_i pub_i L_i(xi)
            function lagrange(m, ps) {
                let xi := mload(add(m, 0x2a0))
                let xn := xi
                for { let i := 0 } lt(i, LOG_N) { i := add(i, 1) } { xn := mulmod(xn, xn, R) }
                mstore(add(m, 0x3a0), xn)
                let zh := addmod(xn, sub(R, 1), R)
                mstore(add(m, 0x3c0), zh)
                let wi := 1
                let pi := 0
                for { let i := 0 } lt(i, N_LAGRANGE) { i := add(i, 1) } {
                    let d := mulmod(N, addmod(xi, sub(R, wi), R), R)
                    let li := mulmod(mulmod(wi, zh, R), fr_inv(d, add(m, 0x4c0)), R)
                    if iszero(i) { mstore(add(m, 0x400), li) }
                    if lt(i, N_PUBLIC) {
                        pi := addmod(pi, sub(R, mulmod(li, mload(add(ps, mul(i, 32))), R)), R)
                    }
                    wi := mulmod(wi, W1, R)
                }
                mstore(add(m, 0x3e0), pi)
            }
            // t(xi) = (r(xi) + PI(xi) - f1 (c + gamma) z(xi w) alpha - L1(xi) alpha^2) / Z_H(xi)
            function quotient(m, pp) {
                let beta := mload(add(m, 0x240))
                let gamma := mload(add(m, 0x260))
                let alpha := mload(add(m, 0x280))
                let f1 := mulmod(addmod(addmod(mload(add(pp, 576)), mulmod(beta, mload(add(pp, 672)), R), R), gamma, R),
                                 addmod(addmod(mload(add(pp, 608)), mulmod(beta, mload(add(pp, 704)), R), R), gamma, R), R)
                mstore(add(m, 0x440), f1)
                let x := mulmod(mulmod(mulmod(f1, addmod(mload(add(pp, 640)), gamma, R), R), mload(add(pp, 736)), R), alpha, R)
                let num := addmod(addmod(mload(add(pp, 768)), mload(add(m, 0x3e0)), R), sub(R, x), R)
                num := addmod(num, sub(R, mulmod(mload(add(m, 0x400)), mulmod(alpha, alpha, R), R)), R)
                mstore(add(m, 0x420), mulmod(num, fr_inv(mload(add(m, 0x3c0)), add(m, 0x4c0)), R))
            }
            // D: the gate and permutation terms of the linearisation
            function commit_d(m, pp) {
                mstore(add(m, 0x480), 0)
                mstore(add(m, 0x4a0), 0)
                let v1 := mload(add(m, 0x2e0))
                let ea := mload(add(pp, 576))
                let eb := mload(add(pp, 608))
                acc_mul(m, QM_X, QM_Y, mulmod(mulmod(ea, eb, R), v1, R))
                acc_mul(m, QL_X, QL_Y, mulmod(ea, v1, R))
                acc_mul(m, QR_X, QR_Y, mulmod(eb, v1, R))
                acc_mul(m, QO_X, QO_Y, mulmod(mload(add(pp, 640)), v1, R))
                acc_mul(m, QC_X, QC_Y, v1)
            }
            function commit_perm(m, pp) {
                let gamma := mload(add(m, 0x260))
                let alpha := mload(add(m, 0x280))
                let bx := mulmod(mload(add(m, 0x240)), mload(add(m, 0x2a0)), R)
                let e2 := mulmod(addmod(addmod(mload(add(pp, 576)), bx, R), gamma, R),
                                 addmod(addmod(mload(add(pp, 608)), mulmod(bx, K1, R), R), gamma, R), R)
                e2 := mulmod(mulmod(e2, addmod(addmod(mload(add(pp, 640)), mulmod(bx, K2, R), R), gamma, R), R), alpha, R)
                let e4 := mulmod(mload(add(m, 0x400)), mulmod(alpha, alpha, R), R)
                let v1 := mload(add(m, 0x2e0))
                acc_mul(m, mload(add(m, 192)), mload(add(m, 224)), addmod(mulmod(addmod(e2, e4, R), v1, R), mload(add(m, 0x2c0)), R))
                let e3 := mulmod(mulmod(mulmod(mload(add(m, 0x440)), mload(add(m, 0x240)), R), mload(add(pp, 736)), R), alpha, R)
                acc_mul(m, S3_X, S3_Y, sub(R, mulmod(e3, v1, R)))
            }
            // F - E + xi Wxi + u xi w Wxiw: the quotient pieces, the opened commitments and the
            // batched evaluation e on the generator
            function commit_f(m, pp) {
                let xn := mload(add(m, 0x3a0))
                acc_mul(m, mload(add(m, 256)), mload(add(m, 288)), 1)
                acc_mul(m, mload(add(m, 320)), mload(add(m, 352)), xn)
                acc_mul(m, mload(add(m, 384)), mload(add(m, 416)), mulmod(xn, xn, R))
                acc_mul(m, mload(m), mload(add(m, 32)), mload(add(m, 0x300)))
                acc_mul(m, mload(add(m, 64)), mload(add(m, 96)), mload(add(m, 0x320)))
                acc_mul(m, mload(add(m, 128)), mload(add(m, 160)), mload(add(m, 0x340)))
                acc_mul(m, S1_X, S1_Y, mload(add(m, 0x360)))
                acc_mul(m, S2_X, S2_Y, mload(add(m, 0x380)))
                let xi := mload(add(m, 0x2a0))
                let u := mload(add(m, 0x2c0))
                acc_mul(m, mload(add(m, 448)), mload(add(m, 480)), xi)
                acc_mul(m, mload(add(m, 512)), mload(add(m, 544)), mulmod(mulmod(u, xi, R), W1, R))
                let e := addmod(mload(add(m, 0x420)), mulmod(mload(add(m, 0x2e0)), mload(add(pp, 768)), R), R)
                e := addmod(e, mulmod(mload(add(m, 0x300)), mload(add(pp, 576)), R), R)
                e := addmod(e, mulmod(mload(add(m, 0x320)), mload(add(pp, 608)), R), R)
                e := addmod(e, mulmod(mload(add(m, 0x340)), mload(add(pp, 640)), R), R)
                e := addmod(e, mulmod(mload(add(m, 0x360)), mload(add(pp, 672)), R), R)
                e := addmod(e, mulmod(mload(add(m, 0x380)), mload(add(pp, 704)), R), R)
                e := addmod(e, mulmod(u, mload(add(pp, 736)), R), R)
                acc_mul(m, 1, 2, sub(R, e))
            }
            // e(-(Wxi + u Wxiw), [tau]_2) * e(accumulator, [1]_2) == 1
            function pairing(m) -> r {
                let s := add(m, 0x4c0)
                mstore(s, mload(add(m, 512)))
                mstore(add(s, 0x20), mload(add(m, 544)))
                mstore(add(s, 0x40), mload(add(m, 0x2c0)))
                if iszero(staticcall(gas(), 7, s, 0x60, add(s, 0x40), 0x40)) { mstore(add(m, 0x460), 0) }
                mstore(s, mload(add(m, 448)))
                mstore(add(s, 0x20), mload(add(m, 480)))
                let p := add(m, 0x600)
                if iszero(staticcall(gas(), 6, s, 0x80, p, 0x40)) { mstore(add(m, 0x460), 0) }
                let y := mload(add(p, 0x20))
                if y { mstore(add(p, 0x20), sub(Q, y)) }
                mstore(add(p, 0x40), X2_X_IM)
                mstore(add(p, 0x60), X2_X_RE)
                mstore(add(p, 0x80), X2_Y_IM)
                mstore(add(p, 0xa0), X2_Y_RE)
                mstore(add(p, 0xc0), mload(add(m, 0x480)))
                mstore(add(p, 0xe0), mload(add(m, 0x4a0)))
                mstore(add(p, 0x100), G2_X_IM)
                mstore(add(p, 0x120), G2_X_RE)
                mstore(add(p, 0x140), G2_Y_IM)
                mstore(add(p, 0x160), G2_Y_RE)
                let success := staticcall(gas(), 8, p, 0x180, s, 0x20)
                r := and(and(success, mload(s)), mload(add(m, 0x460)))
            }

            let m := mload(0x40)
            let pp := add(proof, 32)
            let ps := add(pubSignals, 32)
            check_input(m, pp, ps)
            if mload(add(m, 0x460)) {
                challenges(m, pp, ps)
                lagrange(m, ps)
                quotient(m, pp)
                commit_d(m, pp)
                commit_perm(m, pp)
                commit_f(m, pp)
                ok := pairing(m)
            }
        }
        return ok;
    }
}
)SOL";

void put(std::string& s, const std::string& key, const std::string& val) {
  const std::string k = "@" + key + "@";
  for (size_t p = s.find(k); p != std::string::npos; p = s.find(k, p + val.size())) s.replace(p, k.size(), val);
}

bool valid_name(const char* n) {
  if (!n || !*n || std::strlen(n) > 64) return false;
  if (!((*n >= 'A' && *n <= 'Z') || (*n >= 'a' && *n <= 'z') || *n == '_')) return false;
  for (const char* c = n; *c; c++)
    if (!((*c >= 'A' && *c <= 'Z') || (*c >= 'a' && *c <= 'z') || (*c >= '0' && *c <= '9') || *c == '_'))
      return false;
  return true;
}

}  // namespace

extern "C" {

int nzcb_vk_to_solidity(const uint8_t* vk, const char* contract_name, int transcript_public, char* out,
                        size_t cap) {
  if (!vk) return -1;
  const char* name = contract_name ? contract_name : "PlonkVerifier";
  if (!valid_name(name)) return -1;
  uint32_t npub, power;
  std::memcpy(&npub, vk, 4);
  std::memcpy(&power, vk + 4, 4);
  if (power > 28) return -1;
  using nzcb::dec_le32;
  std::string s = kTemplate;
  put(s, "NAME", name);
  put(s, "N", std::to_string(1ull << power));
  put(s, "POWER", std::to_string(power));
  put(s, "NPUB", std::to_string(npub));
  put(s, "NLAG", std::to_string(npub > 0 ? npub : 1));
  put(s, "TPUB", transcript_public ? "1" : "0");
  put(s, "W", dec_le32(vk + 712));
  put(s, "K1", dec_le32(vk + 8));
  put(s, "K2", dec_le32(vk + 40));
  static const char* names[8] = {"QM", "QL", "QR", "QO", "QC", "S1", "S2", "S3"};
  for (int i = 0; i < 8; i++) {  // infinity stays (0, 0), the precompiles' encoding
    put(s, std::string(names[i]) + "_X", dec_le32(vk + 72 + 64 * i));
    put(s, std::string(names[i]) + "_Y", dec_le32(vk + 72 + 64 * i + 32));
  }
  put(s, "X2_X_RE", dec_le32(vk + 584));
  put(s, "X2_X_IM", dec_le32(vk + 616));
  put(s, "X2_Y_RE", dec_le32(vk + 648));
  put(s, "X2_Y_IM", dec_le32(vk + 680));
  if (!out || cap < s.size() + 1) return (int)(s.size() + 1);
  std::memcpy(out, s.c_str(), s.size() + 1);
  return 0;
}

}  // extern "C"
