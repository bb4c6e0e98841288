"""One proof's MSMs split across ranks (BASELINE configs[4]):
one process per GPU under torch.distributed (backend "nccl" = RCCL over xGMI on ROCm).

Rank 0 proves. Every commitment MSM sum_i s_i [tau^i]G1 is split by PTau point range,
rank r taking [r N / W, (r+1) N / W) of N = n + 6 points; each rank holds the
shifted-base table of its range resident in HBM (nzcb_msm_table). Per commitment:

  rank 0: header (SCALARS, slot, count), then the `count` scalars      -- broadcast
  rank r: partial over its range of those scalars (GPU)
  rank 0: header (GATHER, slot), then one 64-byte affine partial per rank -- all-gather
  rank 0: adds the partials in rank order (csrc/prover.hip commit_finish)

RCCL has no elliptic-curve reduction, so the "one reduce over xGMI" of the north star is
the all-gather of W x 64 bytes plus W - 1 point additions on rank 0. The header
broadcast keeps every rank's collective sequence identical while up to three
commitments are in flight. Rounds 2-5 (Fiat-Shamir) stay on rank 0, so the split only
shortens the MSM share of a proof (Amdahl).

``SplitRoot`` installs the callbacks on rank 0's ProverContext; ``serve`` is the loop of
the other ranks. Both take a ``Comm`` (torch.distributed + the tensor device) and the
serving side a ``partial(slot, scalars, count) -> 64 bytes`` backend: ``GpuRange`` in
production, anything with the same signature in tests (the CPU port over gloo).
"""
from __future__ import annotations

import ctypes
import struct

HDR_SCALARS, HDR_GATHER, HDR_STOP = 1, 2, 3


def point_ranges(n_points: int, world: int) -> list:
    return [(r * n_points // world, (r + 1) * n_points // world) for r in range(world)]


class Comm:
    """torch.distributed collectives on byte tensors (cuda tensors for nccl, cpu for gloo)."""

    def __init__(self, dist, device: str):
        import torch
        self.torch, self.dist, self.device = torch, dist, device
        self.rank, self.world = dist.get_rank(), dist.get_world_size()

    def _sync(self):
        if self.device.startswith("cuda"):
            self.torch.cuda.current_stream().synchronize()

    def header(self, kind: int = 0, slot: int = 0, count: int = 0) -> tuple:
        t = self.torch.tensor([kind, slot, count], dtype=self.torch.int64, device=self.device)
        self.dist.broadcast(t, 0)
        self._sync()
        return tuple(int(x) for x in t.cpu().tolist())

    def bcast(self, t):
        self.dist.broadcast(t, 0)
        self._sync()
        return t

    def allgather64(self, own: bytes) -> bytes:
        src = self.torch.tensor(list(own), dtype=self.torch.uint8, device=self.device)
        out = [self.torch.empty(64, dtype=self.torch.uint8, device=self.device) for _ in range(self.world)]
        self.dist.all_gather(out, src)
        self._sync()
        return b"".join(bytes(o.cpu().tolist()) for o in out)

    def empty(self, nbytes: int):
        return self.torch.empty(max(nbytes, 1), dtype=self.torch.uint8, device=self.device)


class SplitRoot:
    """Rank 0: the send/gather callbacks of nzcb_ctx_set_msm_split over `comm`."""

    def __init__(self, comm: Comm, n_points: int, scalar_source=None):
        self.comm = comm
        self.ranges = point_ranges(n_points, comm.world)
        self.own_points = self.ranges[0][1]
        # scalar_source(dev_ptr, count, tensor): fills the broadcast tensor (device copy by
        # default; tests pass host bytes instead)
        self.scalar_source = scalar_source or self._device_copy
        self.sent = 0

    def _device_copy(self, src, count: int, t):
        import nzcb
        if self.comm.device.startswith("cuda"):
            nzcb.d2d(t.data_ptr(), src, 32 * count)
        else:
            t.copy_(self.comm.torch.frombuffer(bytearray(nzcb.d2h(src, 32 * count)), dtype=self.comm.torch.uint8))

    def send(self, slot: int, src, count: int):
        self.comm.header(HDR_SCALARS, slot, count)
        t = self.comm.empty(32 * count)
        if count:
            self.scalar_source(src, count, t)
        self.comm.bcast(t)
        self.sent += 1

    def gather(self, slot: int, own: bytes) -> bytes:
        self.comm.header(HDR_GATHER, slot, 0)
        return self.comm.allgather64(own)

    def install(self, ctx):
        ctx.set_msm_split(self.comm.world, self.own_points, self.send, self.gather)

    def stop(self):
        self.comm.header(HDR_STOP, 0, 0)


def serve(comm: Comm, partial) -> int:
    """Ranks 1..: answer rank 0's commitments until STOP. partial(slot, scalars_tensor,
    count) -> 64 bytes over this rank's point range. Returns the commitments served."""
    parts = {}
    served = 0
    while True:
        kind, slot, count = comm.header()
        if kind == HDR_STOP:
            return served
        if kind == HDR_SCALARS:
            t = comm.bcast(comm.empty(32 * count))
            parts[slot] = partial(slot, t, count)
            served += 1
        elif kind == HDR_GATHER:
            comm.allgather64(parts.pop(slot))
        else:
            raise RuntimeError(f"msm split: unknown header {kind}")


class GpuRange:
    """A serving rank's backend: the resident fixed-base table of its PTau range."""

    def __init__(self, dev_ptau: int, lo: int, hi: int, device: int):
        import nzcb
        self.nzcb = nzcb
        self.lo, self.hi = lo, hi
        self.table = nzcb.MsmTable(dev_ptau + 64 * lo, hi - lo, device)
        self.staging = None   # HBM copy of this range's scalars when they arrive in host tensors (gloo)

    def __call__(self, slot: int, t, count: int) -> bytes:
        cnt = max(0, min(count, self.hi) - self.lo)
        if not cnt:
            return bytes(64)
        src = t.data_ptr() + 32 * self.lo
        if not getattr(t, "is_cuda", True):
            if self.staging is None:
                self.staging = self.nzcb.dev_alloc(32 * (self.hi - self.lo))
            self.nzcb.memcpy_h2d_ptr(self.staging, src, 32 * cnt)
            src = self.staging
        return self.table.run(src, cnt, True)

    def close(self):
        self.table.close()
        if self.staging:
            self.nzcb.dev_free(self.staging)
            self.staging = None


def zkey_section(ptr: int, size: int, sid: int) -> tuple:
    """(address, length) of section `sid` of a snarkjs binary file held in memory (e.g. the
    PTau section 14 of a zkey buffer from nzcb.plonk_setup_raw)."""
    if ctypes.string_at(ptr, 4) not in (b"zkey", b"ptau", b"wtns", b"r1cs"):
        raise ValueError("not a snarkjs binary file")
    nsec = struct.unpack("<I", ctypes.string_at(ptr + 8, 4))[0]
    o = 12
    for _ in range(nsec):
        s, ln = struct.unpack("<IQ", ctypes.string_at(ptr + o, 12))
        if s == sid:
            return ptr + o + 12, ln
        o += 12 + ln
        if o > size:
            break
    raise ValueError(f"section {sid} not found")
