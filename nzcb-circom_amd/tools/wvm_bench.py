#!/usr/bin/env python3
"""Time the GPU witness VM on the nzcp_live program (batches of live-shaped passes).

--levels: also run one 40-pass batch with NZCB_WVM_LEVEL_CLOCK set and print where the
time goes by level (pass 0's wall clock after each level), grouped by the level's op mix."""
import collections
import os
import struct
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "nzcb-circom_amd")]
import bench  # noqa: E402
import nzcb  # noqa: E402
from nzcb import nzcplive  # noqa: E402

SLOTS = 37  # wvm.hip kClockSlots
OPS = ["LIN", "MUL", "INV", "BITS", "CHECK", "QUIN", "SHA256", "SHA512"]


def level_mix(prog: bytes):
    """per level: Counter of op types, from the program's op and level tables"""
    u = lambda o: struct.unpack_from("<I", prog, o)[0]  # noqa: E731
    nc, nt, no, nl = u(24), u(28), u(32), u(36)
    p = 40 + nc * 32 + nt * 8
    codes = [u(p + 32 * i) & 0xFF for i in range(no)]
    lv = p + no * 32
    starts = [u(lv + 4 * i) for i in range(nl + 1)]
    return [collections.Counter(OPS[codes[k]] for k in range(starts[i], starts[i + 1])) for i in range(nl)]


def main():
    r1cs, prog, _ = nzcplive.build()
    wp = nzcb.WitnessProgram(prog)
    print(f"program: {wp.n_wires} wires, {wp.n_levels} levels, {len(prog)} bytes", flush=True)
    for count in (1, 8, 40, 256):
        inputs = bench.pass_inputs(range(count))
        din = nzcb.dev_alloc(len(inputs))
        dw = nzcb.dev_alloc(count * wp.n_wires * 32)
        nzcb.h2d(din, inputs)
        wp.run_dev(din, count, dw, wp.n_wires * 32)
        t = time.perf_counter()
        reps = 5
        for _ in range(reps):
            st = wp.run_dev(din, count, dw, wp.n_wires * 32)
        ms = (time.perf_counter() - t) / reps * 1e3
        assert not any(st)
        print(f"passes {count:4d}: {ms:8.3f} ms per batch, {ms / count:7.3f} ms per pass", flush=True)
        if count == 40 and "--levels" in sys.argv:
            path = os.path.join(tempfile.mkdtemp(), "clk.bin")
            os.environ["NZCB_WVM_LEVEL_CLOCK"] = path
            wp.run_dev(din, count, dw, wp.n_wires * 32)
            del os.environ["NZCB_WVM_LEVEL_CLOCK"]
            raw = open(path, "rb").read()
            words = struct.unpack(f"<{len(raw) // 8}Q", raw)
            rec = [words[i:i + SLOTS] for i in range(0, len(words), SLOTS)]
            mix = level_mix(prog)
            us, seg_t, seg_w = [], [], []
            for i in range(len(rec) - 1):
                t0, r = rec[i][0], rec[i + 1]
                us.append((r[0] - t0) / 100.0)  # 100 MHz wall clock
                seg_t.append(max((x - t0 for x in r[1:17] if x), default=0) / 100.0)
                seg_w.append(max((x - t0 for x in r[17:33] if x), default=0) / 100.0)
            print(f"levels: {sum(us) / 1e3:.3f} ms total (100 MHz wall clock); per level: total, "
                  "thread segment done, wave segment done (slowest wave, from the level start)")
            by = collections.defaultdict(lambda: [0, 0.0, 0.0, 0.0])
            for m, t, a, b in zip(mix, us, seg_t, seg_w):
                key = "+".join(k for k in OPS if m.get(k)) or "-"
                e = by[key]
                e[0] += 1
                e[1] += t
                e[2] += a
                e[3] += b
            for key, (n, t, a, b) in sorted(by.items(), key=lambda kv: -kv[1][1]):
                print(f"  {key:28s} {n:4d} levels {t / 1e3:7.3f} ms  {t / n:7.2f} us/level "
                      f"(threads {a / n:6.2f}, waves {b / n:6.2f})")
            for i in range(len(rec) - 1):
                r = rec[i + 1]
                if r[33]:
                    ph = [(r[k + 1] - r[k]) / 100.0 for k in range(33, 36)]
                    print(f"  level {i:4d} SHA phases: words {(r[34] - r[33]) / 100.0:6.2f} us, compression "
                          f"{ph[1]:6.2f} us, signals {ph[2]:6.2f} us (from the block start {(r[36] - r[33]) / 100.0:6.2f})")
            top = sorted(range(len(us)), key=lambda i: -us[i])[:12]
            for i in top:
                print(f"  level {i:4d}: {us[i]:8.2f} us (threads {seg_t[i]:7.2f}, waves {seg_w[i]:7.2f})  {dict(mix[i])}")
        nzcb.dev_free(din)
        nzcb.dev_free(dw)
    wp.close()


if __name__ == "__main__":
    main()
