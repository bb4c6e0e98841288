"""A tiny circom-2.0.x-ABI witness .wasm, written byte by byte (test data generator).

The circuit is ``template Mul() { signal input a; signal input b; signal output c;
c <== a * b; }``: wires [1, c, a, b]. The module exports what circom_runtime 0.1.17's
WitnessCalculator calls (getFieldNumLen32, getRawPrime, read/writeSharedRWMemory,
getWitnessSize, init, getInputSignalSize, setInputSignal, getInputSize, getWitness,
getMessageChar, getVersion) and imports its ``runtime`` functions. Inputs are located by
the 64-bit FNV-1a hash of their names split into two i32 halves, as circom does. The
product is computed on the low 32-bit limbs only (inputs below 2^32): this module exists
to drive the plumbing of ``plonk.fullProve`` (nzcb-circom_amd/js/index.js wtnsCalculate),
not field arithmetic. circom itself is not on disk, so the ABI follows
nzcb-circom_amd/js/index.js's restatement (parity unpinned).
"""
from __future__ import annotations

R = 21888242871839275222246405745257275088548364400416034343698204186575808495617


def _uleb(n: int) -> bytes:
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _sleb(n: int) -> bytes:
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if (n == 0 and not b & 0x40) or (n == -1 and b & 0x40):
            out.append(b)
            return bytes(out)
        out.append(b | 0x80)


def _vec(items) -> bytes:
    items = list(items)
    return _uleb(len(items)) + b"".join(items)


def _name(s: str) -> bytes:
    return _uleb(len(s)) + s.encode()


def _section(sid: int, body: bytes) -> bytes:
    return bytes([sid]) + _uleb(len(body)) + body


def fnv_halves(name: str):
    h = 0xCBF29CE484222325
    for ch in name:
        h ^= ord(ch)
        h = (h * 0x100000001B3) % (1 << 64)
    to_i32 = lambda x: x - (1 << 32) if x >= 1 << 31 else x  # noqa: E731
    return to_i32(h >> 32), to_i32(h & 0xFFFFFFFF)


I32, I64 = 0x7F, 0x7E
SHARED, WIT, COUNT = 0, 64, 256          # memory layout: shared RW limbs, witness, set counter


def i32c(v):
    return b"\x41" + _sleb(v)


def lget(i):
    return b"\x20" + _uleb(i)


def store(off=0):
    return b"\x36\x02" + _uleb(off)


def load(off=0):
    return b"\x28\x02" + _uleb(off)


def copy_limbs(src, dst):
    """8 x i32 from address src to address dst (both i32 const)."""
    return b"".join(i32c(dst + 4 * j) + i32c(src + 4 * j) + load() + store() for j in range(8))


def build_mul_wasm() -> bytes:
    types = [
        ((), (I32,)),                 # 0: () -> i32
        ((), ()),                     # 1: () -> ()
        ((I32,), (I32,)),             # 2: (i32) -> i32
        ((I32, I32), ()),             # 3: (i32, i32) -> ()
        ((I32,), ()),                 # 4: (i32) -> ()
        ((I32, I32), (I32,)),         # 5: (i32, i32) -> i32
        ((I32, I32, I32), ()),        # 6: (i32, i32, i32) -> ()
    ]
    type_sec = _vec(b"\x60" + _vec(bytes([p]) for p in ps) + _vec(bytes([r]) for r in rs) for ps, rs in types)
    imports = [("exceptionHandler", 4), ("printErrorMessage", 1), ("writeBufferMessage", 1),
               ("showSharedRWMemory", 1)]
    import_sec = _vec(_name("runtime") + _name(n) + b"\x00" + _uleb(t) for n, t in imports)
    am, al = fnv_halves("a")
    bm, bl = fnv_halves("b")
    prime = [(R >> (32 * j)) & 0xFFFFFFFF for j in range(8)]
    to_i32 = lambda x: x - (1 << 32) if x >= 1 << 31 else x  # noqa: E731

    def is_sig(m, l):  # (hMSB, hLSB) params 0, 1 equal (m, l)
        return lget(0) + i32c(m) + b"\x46" + lget(1) + i32c(l) + b"\x46" + b"\x71"

    funcs = {
        "getVersion": (0, i32c(2)),
        "getFieldNumLen32": (0, i32c(8)),
        "getRawPrime": (1, b"".join(i32c(SHARED + 4 * j) + i32c(to_i32(prime[j])) + store() for j in range(8))),
        "readSharedRWMemory": (2, lget(0) + i32c(4) + b"\x6c" + load(SHARED)),
        "writeSharedRWMemory": (3, lget(0) + i32c(4) + b"\x6c" + lget(1) + store(SHARED)),
        "getWitnessSize": (0, i32c(4)),
        "init": (4, b"".join(i32c(WIT + 4 * j) + i32c(1 if j == 0 else 0) + store() for j in range(8))
                 + i32c(COUNT) + i32c(0) + store()),
        "getInputSignalSize": (5, is_sig(am, al) + b"\x04\x40" + i32c(1) + b"\x0f\x0b"
                               + is_sig(bm, bl) + b"\x04\x40" + i32c(1) + b"\x0f\x0b" + i32c(-1)),
        "setInputSignal": (6, (
            is_sig(am, al) + b"\x04\x40" + copy_limbs(SHARED, WIT + 64) + b"\x0b"
            + is_sig(bm, bl) + b"\x04\x40" + copy_limbs(SHARED, WIT + 96) + b"\x0b"
            + is_sig(am, al) + is_sig(bm, bl) + b"\x72" + b"\x45" + b"\x04\x40" + i32c(1) + b"\x10\x00" + b"\x0b"
            # counter += 1
            + i32c(COUNT) + i32c(COUNT) + load() + i32c(1) + b"\x6a" + store()
            # when both are set: c = a * b on the low limbs (i64 product), upper limbs 0
            + i32c(COUNT) + load() + i32c(2) + b"\x46" + b"\x04\x40"
            + i32c(WIT + 32) + i32c(WIT + 64) + load() + b"\xad" + i32c(WIT + 96) + load() + b"\xad" + b"\x7e"
            + b"\xa7" + store()
            + i32c(WIT + 36) + i32c(WIT + 64) + load() + b"\xad" + i32c(WIT + 96) + load() + b"\xad" + b"\x7e"
            + b"\x42" + _sleb(32) + b"\x88" + b"\xa7" + store()
            + b"".join(i32c(WIT + 32 + 4 * j) + i32c(0) + store() for j in range(2, 8))
            + b"\x0b")),
        "getInputSize": (0, i32c(2)),
        "getWitness": (4, b"".join(i32c(SHARED + 4 * j) + lget(0) + i32c(32) + b"\x6c" + load(WIT + 4 * j) + store()
                                   for j in range(8))),
        "getMessageChar": (0, i32c(0)),
    }
    names = list(funcs)
    func_sec = _vec(_uleb(funcs[n][0]) for n in names)
    mem_sec = _vec([b"\x00" + _uleb(1)])
    nimp = len(imports)
    exp = [_name("memory") + b"\x02" + _uleb(0)]
    exp += [_name(n) + b"\x00" + _uleb(nimp + i) for i, n in enumerate(names)]
    export_sec = _vec(exp)
    bodies = []
    for n in names:
        body = _uleb(0) + funcs[n][1] + b"\x0b"       # no locals
        bodies.append(_uleb(len(body)) + body)
    code_sec = _vec(bodies)
    return (b"\x00asm\x01\x00\x00\x00" + _section(1, type_sec) + _section(2, import_sec) + _section(3, func_sec)
            + _section(5, mem_sec) + _section(7, export_sec) + _section(10, code_sec))


def mul_circuit():
    """The same circuit through nzcb.circuit: (r1cs bytes, witness program bytes)."""
    from nzcb.circuit import Circuit, w
    c = Circuit(1, 0, 2, input_names=[("a", 1), ("b", 1)])
    c.mul(w(c.in_base), w(c.in_base + 1), dst=c.out_wires[0])
    return c.write_r1cs(), c.write_program()


if __name__ == "__main__":
    import sys
    with open(sys.argv[1] if len(sys.argv) > 1 else "mul.wasm", "wb") as f:
        f.write(build_mul_wasm())
