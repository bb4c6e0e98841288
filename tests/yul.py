"""A small interpreter for the Yul subset of the generated Solidity verifier
(csrc/solidity.cpp), so tests can execute the contract's assembly on real proofs.

Test infrastructure only. It runs the `assembly { ... }` block of `verifyProof` with
EVM semantics (256-bit wrapping words, big-endian memory words, keccak256) and the four
BN254 precompiles the contract calls (0x05 modexp, 0x06 ecAdd, 0x07 ecMul, 0x08
pairing check, as EIP-196/197/198 specify them), implemented with the CPU oracle's
curve and pairing code (oracle/bn254.py, oracle/pairing.py). The Solidity around the
block is emulated: `proof` and `pubSignals` are memory pointers laid out as the ABI
decoder lays out `bytes memory` / `uint256[] memory` (length word, then data), and the
contract's `uint256 constant` declarations are visible by name.

Supported: blocks, function definitions (hoisted; parameters and `-> r` returns),
`let`, assignment, `if`, `for`, `leave`, calls, decimal and hex literals, and the
builtins listed in `_BUILTINS`.
"""
from __future__ import annotations

import re

from oracle import bn254 as bn
from oracle import pairing as pr
from oracle.keccak import keccak256

M256 = (1 << 256) - 1
_TOK = re.compile(r"\s*(?:(//[^\n]*)|(/\*.*?\*/)|(0x[0-9a-fA-F]+|\d+)|([A-Za-z_][A-Za-z0-9_.]*)|(:=|->|[{}(),]))",
                  re.S)


class Revert(Exception):
    pass


class _Leave(Exception):
    pass


def tokenize(src: str) -> list:
    out, pos = [], 0
    while pos < len(src):
        m = _TOK.match(src, pos)
        if not m or m.end() == pos:
            if src[pos:].strip() == "":
                break
            raise SyntaxError(f"yul: cannot tokenize at {src[pos:pos + 40]!r}")
        pos = m.end()
        if m.group(1) or m.group(2):
            continue
        if m.group(3):
            out.append(("num", int(m.group(3), 0)))
        elif m.group(4):
            out.append(("id", m.group(4)))
        else:
            out.append(("p", m.group(5)))
    return out


class _Parser:
    def __init__(self, toks):
        self.t, self.i = toks, 0

    def peek(self, k=0):
        return self.t[self.i + k] if self.i + k < len(self.t) else (None, None)

    def take(self, kind=None, val=None):
        tok = self.peek()
        if (kind and tok[0] != kind) or (val is not None and tok[1] != val):
            raise SyntaxError(f"yul: expected {val or kind}, got {tok}")
        self.i += 1
        return tok

    def block(self):
        self.take("p", "{")
        stmts = []
        while self.peek() != ("p", "}"):
            stmts.append(self.stmt())
        self.take("p", "}")
        return ("block", stmts)

    def expr(self):
        kind, val = self.take()
        if kind == "num":
            return ("num", val)
        if kind != "id":
            raise SyntaxError(f"yul: bad expression token {val!r}")
        if self.peek() == ("p", "("):
            self.take("p", "(")
            args = []
            while self.peek() != ("p", ")"):
                args.append(self.expr())
                if self.peek() == ("p", ","):
                    self.take("p", ",")
            self.take("p", ")")
            return ("call", val, args)
        return ("var", val)

    def idents(self):
        names = [self.take("id")[1]]
        while self.peek() == ("p", ","):
            self.take("p", ",")
            names.append(self.take("id")[1])
        return names

    def stmt(self):
        kind, val = self.peek()
        if (kind, val) == ("p", "{"):
            return self.block()
        if val == "function":
            self.take()
            name = self.take("id")[1]
            self.take("p", "(")
            params = [] if self.peek() == ("p", ")") else self.idents()
            self.take("p", ")")
            rets = []
            if self.peek() == ("p", "->"):
                self.take()
                rets = self.idents()
            return ("func", name, params, rets, self.block())
        if val == "let":
            self.take()
            names = self.idents()
            value = None
            if self.peek() == ("p", ":="):
                self.take()
                value = self.expr()
            return ("let", names, value)
        if val == "if":
            self.take()
            return ("if", self.expr(), self.block())
        if val == "for":
            self.take()
            return ("for", self.block(), self.expr(), self.block(), self.block())
        if val == "leave":
            self.take()
            return ("leave",)
        if kind == "id" and self.peek(1) in (("p", ":="), ("p", ",")):
            names = self.idents()
            self.take("p", ":=")
            return ("assign", names, self.expr())
        return ("expr", self.expr())


class Evm:
    """Memory, the precompiles and the builtins of one call."""

    def __init__(self):
        self.mem = bytearray()
        self.calls = {5: 0, 6: 0, 7: 0, 8: 0}

    def _grow(self, end):
        if end > len(self.mem):
            self.mem.extend(bytes(end - len(self.mem)))

    def mload(self, a):
        self._grow(a + 32)
        return int.from_bytes(self.mem[a:a + 32], "big")

    def mstore(self, a, v):
        self._grow(a + 32)
        self.mem[a:a + 32] = (v & M256).to_bytes(32, "big")

    def read(self, a, n):
        self._grow(a + n)
        return bytes(self.mem[a:a + n])

    def write(self, a, data):
        self._grow(a + len(data))
        self.mem[a:a + len(data)] = data

    @staticmethod
    def _g1(x, y):
        if x >= bn.P_MOD or y >= bn.P_MOD:
            return False, None
        if x == 0 and y == 0:
            return True, None
        return bn.g1_is_on_curve((x, y)), (x, y)

    def precompile(self, addr, data):
        """(success, output bytes) as EIP-196 / 197 / 198 define them."""
        self.calls[addr] = self.calls.get(addr, 0) + 1
        word = lambda k: int.from_bytes(data[32 * k:32 * k + 32].ljust(32, b"\0"), "big")  # noqa: E731
        enc = lambda pt: bytes(64) if pt is None else pt[0].to_bytes(32, "big") + pt[1].to_bytes(32, "big")  # noqa
        if addr == 5:
            lb, le, lm = word(0), word(1), word(2)
            body = data[96:].ljust(lb + le + lm, b"\0")
            b = int.from_bytes(body[:lb], "big")
            e = int.from_bytes(body[lb:lb + le], "big")
            mo = int.from_bytes(body[lb + le:lb + le + lm], "big")
            return True, (pow(b, e, mo) if mo else 0).to_bytes(lm, "big")
        if addr == 6:
            ok1, p = self._g1(word(0), word(1))
            ok2, q = self._g1(word(2), word(3))
            if not (ok1 and ok2):
                return False, b""
            return True, enc(bn.g1_add(p, q))
        if addr == 7:
            ok1, p = self._g1(word(0), word(1))
            if not ok1:
                return False, b""
            return True, enc(bn.g1_mul(p, word(2)) if p is not None else None)
        if addr == 8:
            if len(data) % 192:
                return False, b""
            pairs = []
            for k in range(len(data) // 192):
                ok1, p = self._g1(word(6 * k), word(6 * k + 1))
                xi, xr, yi, yr = (word(6 * k + j) for j in range(2, 6))
                if not ok1 or max(xi, xr, yi, yr) >= bn.P_MOD:
                    return False, b""
                q = None if (xi | xr | yi | yr) == 0 else ((xr, xi), (yr, yi))
                if q is not None and not bn.g2_is_on_curve(q):
                    return False, b""
                if p is not None and q is not None:
                    pairs.append((p, q))
            return True, (1 if (not pairs or pr.pairing_check(pairs)) else 0).to_bytes(32, "big")
        return False, b""


def _u(x):
    return x & M256


_BUILTINS = {
    "add": lambda e, a, b: _u(a + b),
    "sub": lambda e, a, b: _u(a - b),
    "mul": lambda e, a, b: _u(a * b),
    "div": lambda e, a, b: a // b if b else 0,
    "mod": lambda e, a, b: a % b if b else 0,
    "addmod": lambda e, a, b, m: (a + b) % m if m else 0,
    "mulmod": lambda e, a, b, m: (a * b) % m if m else 0,
    "lt": lambda e, a, b: int(a < b),
    "gt": lambda e, a, b: int(a > b),
    "eq": lambda e, a, b: int(a == b),
    "iszero": lambda e, a: int(a == 0),
    "and": lambda e, a, b: a & b,
    "or": lambda e, a, b: a | b,
    "xor": lambda e, a, b: a ^ b,
    "not": lambda e, a: M256 ^ a,
    "shl": lambda e, s, v: _u(v << s) if s < 256 else 0,
    "shr": lambda e, s, v: v >> s if s < 256 else 0,
    "mload": lambda e, a: e.mload(a),
    "mstore": lambda e, a, v: e.mstore(a, v),
    "keccak256": lambda e, a, n: int.from_bytes(keccak256(e.read(a, n)), "big"),
    "gas": lambda e: 1 << 32,
    "pop": lambda e, a: None,
}


class Interp:
    def __init__(self, evm: Evm, consts: dict):
        self.evm, self.consts = evm, consts

    def call_builtin(self, name, args):
        if name == "staticcall":
            _gas, addr, i, isz, o, osz = args
            ok, out = self.evm.precompile(addr, self.evm.read(i, isz))
            if ok:
                self.evm.write(o, out[:osz].ljust(osz, b"\0") if len(out) < osz else out[:osz])
            return int(ok)
        if name == "revert":
            raise Revert("revert")
        return _BUILTINS[name](self.evm, *args)

    def eval(self, ex, env, funcs):
        if ex[0] == "num":
            return ex[1]
        if ex[0] == "var":
            name = ex[1]
            for scope in reversed(env):
                if name in scope:
                    return scope[name]
            if name in self.consts:
                return self.consts[name]
            raise NameError(f"yul: unknown identifier {name}")
        name, args = ex[1], [self.eval(a, env, funcs) for a in ex[2]]
        for fs in reversed(funcs):
            if name in fs:
                return self.call_func(fs[name], args, funcs)
        return self.call_builtin(name, args)

    def call_func(self, fn, args, funcs):
        _, _name, params, rets, body = fn
        scope = dict(zip(params, args))
        for r in rets:
            scope[r] = 0
        try:
            # a function sees only its own variables, and the functions in scope
            self.block(body, [scope], funcs)
        except _Leave:
            pass
        return scope[rets[0]] if rets else None

    def block(self, blk, env, funcs):
        fs = {s[1]: s for s in blk[1] if s[0] == "func"}
        env = env + [{}]
        funcs = funcs + [fs]
        for s in blk[1]:
            self.stmt(s, env, funcs)

    def _assign(self, name, val, env):
        for scope in reversed(env):
            if name in scope:
                scope[name] = val
                return
        raise NameError(f"yul: assignment to undeclared {name}")

    def stmt(self, s, env, funcs):
        k = s[0]
        if k == "func":
            return
        if k == "block":
            self.block(s, env, funcs)
        elif k == "let":
            val = self.eval(s[2], env, funcs) if s[2] is not None else 0
            for name in s[1]:
                env[-1][name] = val
        elif k == "assign":
            self._assign(s[1][0], self.eval(s[2], env, funcs), env)
        elif k == "if":
            if self.eval(s[1], env, funcs):
                self.block(s[2], env, funcs)
        elif k == "for":
            init, cond, post, body = s[1:]
            env2 = env + [{}]
            for st in init[1]:
                self.stmt(st, env2, funcs)
            while self.eval(cond, env2, funcs):
                self.block(body, env2, funcs)
                self.block(post, env2, funcs)
        elif k == "leave":
            raise _Leave()
        elif k == "expr":
            self.eval(s[1], env, funcs)


def contract_parts(sol: str):
    """The `uint256 constant` values and the parsed assembly block of verifyProof."""
    consts = {m.group(1): int(m.group(2), 0)
              for m in re.finditer(r"uint256\s+constant\s+(\w+)\s*=\s*(0x[0-9a-fA-F]+|\d+)\s*;", sol)}
    start = sol.index("assembly")
    i = sol.index("{", start)
    depth, j = 0, i
    while True:
        if sol[j] == "{":
            depth += 1
        elif sol[j] == "}":
            depth -= 1
            if depth == 0:
                break
        j += 1
    return consts, _Parser(tokenize(sol[i:j + 1])).block()


def run_verify_proof(sol: str, proof: bytes, pub_signals: list) -> tuple:
    """Execute the contract's verifyProof assembly; returns (ok, precompile call counts)."""
    consts, blk = contract_parts(sol)
    evm = Evm()
    evm.mstore(0x40, 0x80)
    p_proof = 0x80
    evm.mstore(p_proof, len(proof))
    evm.write(p_proof + 32, proof)
    p_pub = p_proof + 32 + ((len(proof) + 31) // 32) * 32
    evm.mstore(p_pub, len(pub_signals))
    for k, v in enumerate(pub_signals):
        evm.mstore(p_pub + 32 + 32 * k, v)
    evm.mstore(0x40, p_pub + 32 + 32 * len(pub_signals))   # the free memory pointer
    outer = {"proof": p_proof, "pubSignals": p_pub, "ok": 0}
    Interp(evm, consts).block(blk, [outer], [])
    return bool(outer["ok"]), dict(evm.calls)
