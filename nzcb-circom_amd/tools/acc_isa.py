#!/usr/bin/env python3
"""ISA census of the bucket accumulation's loop (msm_accumulate29_kernel<true>, csrc/msm.hip):
compiles msm.hip for gfx950 to assembly (device only, the Makefile's flags), takes the
kernel's outer loop (the "Loop Header: Depth=1" block to its back edge), cuts it into basic
blocks and counts every block's instructions by category. DESIGN.md §4 reads the common path
(the XYZZ mixed addition every entry runs, the run-end store most waves run, the rare
doubling) off the per-block table; PMC (SQ_INSTS_VALU per entry) says which blocks execute.
  python3 tools/acc_isa.py [--asm file.s] [--kernel <mangled name prefix>]"""
import argparse
import collections
import os
import re
import subprocess
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
KERNEL = "_ZN4nzcb23msm_accumulate29_kernelILb1E"

CATS = [
    ("v_mad_u64_u32", r"v_mad_u64_u32"),
    ("v_mul (32-bit)", r"v_mul_(lo|hi)_u32|v_mul_u32"),
    ("add/sub/carry", r"v_(add|sub|subrev)(_co|_nc)?(_ci)?_u32|v_add3_u32|v_addc|v_subb|v_lshl_add_u64|v_add_u64|v_sub_u64"),
    ("shift/bitfield", r"v_(lshrrev|lshlrev|ashrrev|alignbit|bfe|bfi|lshl_or|and_or|lshl_add|or3|alignbyte|perm)"),
    ("and/or/xor", r"v_(and|or|xor|not)_b32|v_and_or|v_xad"),
    ("mov", r"v_mov_b|v_accvgpr|v_pk_mov"),
    ("cmp/cndmask", r"v_cmp|v_cndmask|v_cmpx"),
    ("other VALU", r"v_"),
    ("LDS", r"ds_"),
    ("global/buffer", r"global_|buffer_|flat_|scratch_"),
    ("s_nop", r"s_nop"),
    ("s_waitcnt", r"s_waitcnt"),
    ("SALU/branch", r"s_"),
]


def category(op):
    for name, pat in CATS:
        if re.match(pat, op):
            return name
    return "?"


def compile_asm():
    out = os.path.join(tempfile.mkdtemp(), "msm.s")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-munsafe-fp-atomics",
                    "--cuda-device-only", "-S", os.path.join(PKG, "csrc", "msm.hip"), "-o", out],
                   check=True, capture_output=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--asm")
    ap.add_argument("--kernel", default=KERNEL)
    a = ap.parse_args()
    path = a.asm or compile_asm()
    lines = open(path).read().split("\n")
    start = next(i for i, ln in enumerate(lines) if ln.startswith(a.kernel) and ln.split(":")[0].endswith("_"))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    body = lines[start:end]
    # the outer loop: from its header label to the last branch back to it
    hdr = next(i for i, ln in enumerate(body) if "Loop Header: Depth=1" in ln and "Inner" not in ln)
    label = body[hdr].split(":")[0]
    last = max(i for i, ln in enumerate(body) if re.search(r"s_(c)?branch\S*\s+" + re.escape(label) + r"\b", ln)
               or ("in Loop: Header=" + label[len(".L"):]) in ln)
    # blocks
    blocks, cur = [], None
    for ln in body[hdr:last + 40]:
        s = ln.strip()
        if re.match(r"^\.LBB\d+_\d+:", ln):
            if cur is not None and ("Loop" not in ln) and cur["name"] != "?":
                pass
            cur = {"name": ln.split(":")[0], "ops": collections.Counter(), "n": 0, "end": ""}
            blocks.append(cur)
            if "Loop" not in ln and len(blocks) > 1:
                break
            continue
        if not s or s.startswith(";") or s.startswith(".") or cur is None:
            continue
        op = s.split()[0]
        cur["ops"][category(op)] += 1
        cur["n"] += 1
        if op.startswith("s_cbranch") or op.startswith("s_branch"):
            cur["end"] += op + " " + s.split()[1] + " "
    names = [c for c, _ in CATS]
    tot = collections.Counter()
    print(f"# {os.path.basename(path)}: {a.kernel}... outer loop {label}, {len(blocks)} blocks")
    print("%-12s %6s %6s %6s %s" % ("block", "instrs", "VALU", "mads", " ".join(f"{n[:10]:>10s}" for n in names)))
    for b in blocks:
        valu = sum(v for k, v in b["ops"].items() if k in names[:8])
        tot.update(b["ops"])
        print("%-12s %6d %6d %6d %s  %s" % (b["name"], b["n"], valu, b["ops"]["v_mad_u64_u32"],
                                          " ".join(f"{b['ops'][n]:10d}" for n in names), b["end"].strip()))
    valu = sum(v for k, v in tot.items() if k in names[:8])
    print("%-12s %6d %6d %6d %s" % ("loop total", sum(tot.values()), valu, tot["v_mad_u64_u32"],
                                    " ".join(f"{tot[n]:10d}" for n in names)))


if __name__ == "__main__":
    main()
