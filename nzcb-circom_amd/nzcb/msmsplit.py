"""One proof's MSMs split across ranks (BASELINE configs[4]):
one process per GPU under torch.distributed (backend "nccl" = RCCL over xGMI on ROCm).

Rank 0 proves. Every commitment MSM sum_i s_i [tau^i]G1 is split by PTau point range,
rank r taking [r N / W, (r+1) N / W) of N = n + 6 points; each rank holds the
shifted-base table of its range resident in HBM (nzcb_msm_table). A, B and C are committed
over the Lagrange basis (n + 2 points: [L_k(tau)], k < n, and the two blinding points) from
their gate values; since round 6 they are split the same way over that basis (rank r taking
[r L / W, (r+1) L / W) of L = n + 2; nzcb_msm_table_create_lagrange), their slot carrying
MSM_LAGRANGE, so all nine commitments of a proof leave rank 0. Per commitment:

  rank 0: its scalars cut into W slices (one device copy into the send rows)
  rank 0: header (SCALARS, slot, count)                                  -- broadcast, 24 B
  rank r: receives ONLY its slice [lo_r, hi_r) of the scalars            -- scatter
  rank r: partial over its range (GPU)
  rank 0: header (GATHER, slot)                                          -- broadcast, 24 B
  rank 0: one 64-byte affine partial from every rank                     -- gather to rank 0
  rank 0: adds the partials in rank order (csrc/prover.hip commit_finish)

Bytes on the wire per commitment: 32 (N - N/W) of scalars plus 64 (W - 1) of partials and
two 24-byte headers, instead of the W - 1 full copies of the scalars a broadcast moves (at
n = 2^21 and W = 8: 59 MB instead of 470 MB per commitment). Slices are
padded to the longest range so every rank's scatter buffer has one size.

RCCL has no elliptic-curve reduction, so the "one reduce over xGMI" of the north star is
the gather of W x 64 bytes plus W - 1 point additions on rank 0. The header broadcast
keeps every rank's collective sequence identical while up to three commitments are in
flight. A header is only sent once its payload is ready, so a failing scalar source
leaves the serving ranks waiting for the next header, in step with rank 0. Rounds 2-5
(Fiat-Shamir) stay on rank 0, so the split only shortens the MSM share of a proof (Amdahl).

``SplitRoot`` installs the callbacks on rank 0's ProverContext (use it as a context
manager, or call ``stop``, so the serving ranks leave their loop); ``serve`` is the loop
of the other ranks. Both take a ``Comm`` (torch.distributed + the tensor device) and the
serving side a ``partial(slot, slice_tensor, count) -> 64 bytes`` backend, where the
tensor holds this rank's ``count`` scalars starting at its range's first point:
``GpuRange`` in production, anything with the same signature in tests (the CPU port
over gloo).
"""
from __future__ import annotations

import ctypes
import struct

HDR_SCALARS, HDR_GATHER, HDR_STOP = 1, 2, 3
MSM_LAGRANGE = 0x100   # include/nzcb.h NZCB_MSM_LAGRANGE (the slot of a Lagrange-basis commitment)


def split_slot(slot: int) -> tuple:
    """(slot 0..2, over the Lagrange basis?) of a callback's slot value."""
    return slot & 0xFF, bool(slot & MSM_LAGRANGE)


def point_ranges(n_points: int, world: int) -> list:
    return [(r * n_points // world, (r + 1) * n_points // world) for r in range(world)]


def slice_counts(count: int, ranges: list) -> list:
    """Scalars of an MSM of length `count` that fall into each rank's point range."""
    return [max(0, min(count, hi) - lo) for lo, hi in ranges]


def wire_bytes(count: int, world: int, n_points: int) -> int:
    """Bytes one split commitment moves between ranks (scatter rows to ranks 1.., partials
    to rank 0, two headers to ranks 1..), for DESIGN.md §6."""
    ranges = point_ranges(n_points, world)
    row = 32 * max(hi - lo for lo, hi in ranges)
    return (world - 1) * (row + 64 + 2 * 24) if count else (world - 1) * (64 + 2 * 24)


class Comm:
    """torch.distributed collectives on byte tensors (cuda tensors for nccl, cpu for gloo)."""

    def __init__(self, dist, device: str):
        import torch
        self.torch, self.dist, self.device = torch, dist, device
        self.rank, self.world = dist.get_rank(), dist.get_world_size()

    def sync(self):
        """Host wait for torch's stream (before another stream or the host reads a result)."""
        if self.device.startswith("cuda"):
            self.torch.cuda.current_stream().synchronize()

    def send_header(self, kind: int, slot: int = 0, count: int = 0):
        """Rank 0: no read-back, no host wait (the tensor is ordered on torch's stream)."""
        t = self.torch.tensor([kind, slot, count], dtype=self.torch.int64, device=self.device)
        self.dist.broadcast(t, 0)

    def recv_header(self) -> tuple:
        t = self.torch.empty(3, dtype=self.torch.int64, device=self.device)
        self.dist.broadcast(t, 0)
        return tuple(int(x) for x in t.cpu().tolist())   # .cpu() waits for the broadcast

    def stream(self) -> int:
        """torch's current HIP stream (the one collectives are ordered after), 0 on CPU."""
        return self.torch.cuda.current_stream().cuda_stream if self.device.startswith("cuda") else 0

    def scatter_rows(self, rows, out):
        """rows: rank 0's [world, row_bytes] tensor (None elsewhere); out: this rank's row.
        Asynchronous on every backend: returns the collective's work handle, which rank 0
        waits on before it rewrites the rows (the slot's next send) and a serving rank before
        its GPU reads `out`. On RCCL the scatter is ordered after the work already on torch's
        current stream, the row copies included (SplitRoot._device_copy)."""
        return self.dist.scatter(out, list(rows.unbind(0)) if rows is not None else None, src=0, async_op=True)

    def gather64(self, own: bytes) -> bytes | None:
        """Every rank's 64-byte partial to rank 0 (None on the other ranks)."""
        src = self.torch.tensor(list(own), dtype=self.torch.uint8, device=self.device)
        if self.rank == 0:
            out = [self.torch.empty(64, dtype=self.torch.uint8, device=self.device) for _ in range(self.world)]
            self.dist.gather(src, out, dst=0)
            return bytes(self.torch.cat(out).cpu().tolist())
        self.dist.gather(src, None, dst=0)
        return None

    def empty(self, nbytes: int):
        return self.torch.empty(max(nbytes, 1), dtype=self.torch.uint8, device=self.device)


class SplitRoot:
    """Rank 0: the send/gather callbacks of nzcb_ctx_set_msm_split over `comm`."""

    SLOTS = 3   # commitments in flight (csrc/prover.hip)

    def __init__(self, comm: Comm, n_points: int, scalar_source=None, n_lagrange: int = 0):
        self.comm = comm
        self.ranges = point_ranges(n_points, comm.world)
        self.own_points = self.ranges[0][1]
        # n_lagrange = n + 2 splits A, B, C over the Lagrange basis too (0: they stay on rank 0)
        self.lranges = point_ranges(n_lagrange, comm.world) if n_lagrange else None
        self.own_lagrange = self.lranges[0][1] if self.lranges else 0
        self.row = 32 * max(hi - lo for lo, hi in self.ranges + (self.lranges or []))
        # scalar_source(src, lo, cnt, row_tensor): copies scalars [lo, lo + cnt) of the
        # commitment into a send row (device copy by default; tests pass host bytes)
        self.scalar_source = scalar_source or self._device_copy
        self._rows = {}     # slot -> [world, row] send rows (kept until the next use of the slot)
        self.sent = 0
        self.stopped = False

    def _device_copy(self, src, lo: int, cnt: int, row):
        import nzcb
        if self.comm.device.startswith("cuda"):
            # ordered on torch's current stream, which the scatter issued next waits for: the
            # rows are complete when RCCL reads them, with no host wait (the prover's scalars
            # at `src` are final: csrc/prover.hip commit_start synchronizes their event first)
            nzcb.d2d_async(row.data_ptr(), src + 32 * lo, 32 * cnt, self.comm.stream())
        else:
            row[:32 * cnt].copy_(self.comm.torch.frombuffer(bytearray(nzcb.d2h(src + 32 * lo, 32 * cnt)),
                                                            dtype=self.comm.torch.uint8))

    def send(self, slot: int, src, count: int):
        wire_slot = slot
        slot, lag = split_slot(slot)
        ranges = self.lranges if lag else self.ranges
        if ranges is None:
            raise RuntimeError("msm split: a Lagrange-basis commitment, but no Lagrange ranges (n_lagrange = 0)")
        rows, work = self._rows.get(slot, (None, None))
        if rows is None:
            rows = self.comm.torch.empty((self.comm.world, max(self.row, 1)), dtype=self.comm.torch.uint8,
                                         device=self.comm.device)
        elif work is not None:   # the slot's previous scatter must have read its rows
            work.wait()         # RCCL: torch's stream waits for it; gloo: the host does
            self.comm.sync()    # and the host waits for torch's stream before refilling
        # fill first: if the source fails, no header is out and the servers stay in step
        for r, ((lo, _), cnt) in enumerate(zip(ranges, slice_counts(count, ranges))):
            if r and cnt:
                self.scalar_source(src, lo, cnt, rows[r])
        self.comm.send_header(HDR_SCALARS, wire_slot, count)
        self.stopped = False        # a new serving session (serve() runs until the next STOP)
        out = self.comm.empty(self.row)
        self._rows[slot] = (rows, self.comm.scatter_rows(rows, out))
        self.sent += 1

    def gather(self, slot: int, own: bytes) -> bytes:
        self.comm.send_header(HDR_GATHER, split_slot(slot)[0], 0)
        return self.comm.gather64(own)

    def install(self, ctx):
        ctx.set_msm_split(self.comm.world, self.own_points, self.send, self.gather, self.own_lagrange)

    def stop(self):
        """Ends the serving ranks' serve() loop (one STOP per serve() call they make)."""
        self.stopped = True
        self.comm.send_header(HDR_STOP)
        self.comm.sync()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        if not self.stopped:     # the servers are still in serve(): release them
            self.stop()
        return False


def serve(comm: Comm, partial, n_points: int, n_lagrange: int = 0, partial_lagrange=None) -> int:
    """Ranks 1..: answer rank 0's commitments until STOP. partial(slot, slice_tensor, count)
    -> 64 bytes over this rank's PTau range; partial_lagrange the same over its range of the
    n_lagrange Lagrange-basis points (A, B, C; SplitRoot's n_lagrange). Returns the
    commitments served."""
    ranges = point_ranges(n_points, comm.world)
    lranges = point_ranges(n_lagrange, comm.world) if n_lagrange else None
    row = 32 * max(hi - lo for lo, hi in ranges + (lranges or []))
    parts = {}
    served = 0
    while True:
        kind, slot, count = comm.recv_header()
        if kind == HDR_STOP:
            return served
        if kind == HDR_SCALARS:
            slot, lag = split_slot(slot)
            if lag and (lranges is None or partial_lagrange is None):
                raise RuntimeError("msm split: a Lagrange-basis commitment, but this rank serves PTau only")
            t = comm.empty(row)
            comm.scatter_rows(None, t).wait()   # the slice has arrived (RCCL: on torch's stream) ...
            comm.sync()   # ... and the host waits for that stream: the backend reads t on its own
            cnt = slice_counts(count, lranges if lag else ranges)[comm.rank]
            parts[slot] = (partial_lagrange if lag else partial)(slot, t, cnt)
            served += 1
        elif kind == HDR_GATHER:
            comm.gather64(parts.pop(slot))
        else:
            raise RuntimeError(f"msm split: unknown header {kind}")


class GpuRange:
    """A serving rank's backend: the resident fixed-base table of its PTau range, or (lagrange)
    of its range of the Lagrange basis, computed from the whole PTau (ptau_n points, 2^log_n
    domain) on this rank's GPU."""

    def __init__(self, dev_ptau: int, lo: int, hi: int, device: int, lagrange: bool = False, ptau_n: int = 0,
                 log_n: int = 0):
        import nzcb
        self.nzcb = nzcb
        self.lo, self.hi = lo, hi
        if lagrange:
            self.table = nzcb.MsmTable.lagrange(dev_ptau, ptau_n, log_n, lo, hi, device)
        else:
            self.table = nzcb.MsmTable(dev_ptau + 64 * lo, hi - lo, device)
        self.staging = None   # HBM copy of this range's scalars when they arrive in host tensors (gloo)

    def __call__(self, slot: int, t, cnt: int) -> bytes:
        if not cnt:
            return bytes(64)
        src = t.data_ptr()
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
