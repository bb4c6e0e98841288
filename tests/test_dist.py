"""World-size-2 rehearsal of bench.py's multi-GPU batch mode on CPU (gloo): the batch
is sharded across ranks with no data-path collective, and the job time is the max
over ranks (one float all-reduce), as bench.py does over RCCL on GPUs."""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, count, out):
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    mine = list(bench.shard(count, rank, world))
    dist.barrier()
    elapsed = 0.25 * (rank + 1)
    job = bench.max_over_ranks(elapsed, dist, "cpu")
    gathered = [None] * world
    dist.all_gather_object(gathered, mine)
    out[rank] = (job, gathered)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("count", [512, 7])
def test_batch_shard_and_max_over_ranks_gloo(count):
    world = 2
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(world, _free_port(), count, out), nprocs=world, join=True)
        res = dict(out)
    for rank in range(world):
        job, gathered = res[rank]
        assert job == 0.25 * world
        flat = [i for part in gathered for i in part]
        assert flat == list(range(count))  # every proof exactly once, no overlap
        assert max(len(p) for p in gathered) - min(len(p) for p in gathered) <= 1


def _prove_worker(rank, world, port, count, out):
    """Each rank proves its shard of a batch (bench.shard) with the C port, as bench.py's
    ranks do on their GPUs; rank 0 gathers the proofs (in production they stay per rank)."""
    import json
    import torch.distributed as dist
    from oracle import cbind
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    gold = os.path.join(ROOT, "tests", "golden")
    meta = json.load(open(os.path.join(gold, "p5.json")))
    zkey = open(os.path.join(gold, "p5.zkey"), "rb").read()
    wtns = open(os.path.join(gold, "p5.wtns"), "rb").read()
    bl = bytes.fromhex(meta["proofs"]["fixed"]["blinding"])
    mine = {i: cbind.prove(zkey, wtns, bl, threads=1)[0].hex() for i in bench.shard(count, rank, world)}
    gathered = [None] * world
    dist.all_gather_object(gathered, mine)
    out[rank] = gathered
    dist.barrier()
    dist.destroy_process_group()


def test_batch_shards_prove_gloo():
    """World size 2: every proof index is proved by exactly one rank, and every proof equals
    the golden one (same witness and blinding)."""
    import json
    count, world = 5, 2
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_prove_worker, args=(world, _free_port(), count, out), nprocs=world, join=True)
        res = dict(out)
    want = json.load(open(os.path.join(ROOT, "tests", "golden", "p5.json")))["proofs"]["fixed"]["proof_bin"]
    merged = {}
    for part in res[0]:
        assert not set(part) & set(merged)
        merged.update(part)
    assert sorted(merged) == list(range(count))
    assert all(v == want for v in merged.values())


def test_launch_plan_decisions():
    """--gpus N > 1 without a launcher spawns N ranks; under a launcher
    the world must equal --gpus."""
    assert bench.launch_plan(1, {}) == "local"
    assert bench.launch_plan(8, {}) == "spawn"
    assert bench.launch_plan(8, {"WORLD_SIZE": "8"}) == "local"
    assert bench.launch_plan(1, {"WORLD_SIZE": "1"}) == "local"
    for gpus, env in ((2, {"WORLD_SIZE": "1"}), (1, {"WORLD_SIZE": "2"}), (8, {"WORLD_SIZE": "4"})):
        with pytest.raises(SystemExit) as e:
            bench.launch_plan(gpus, env)
        assert e.value.code == 2
    with pytest.raises(SystemExit):
        bench.launch_plan(0, {})


def _bench_env(**extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    env.update(NZCB_DIST_BACKEND="gloo", **extra)
    return env


@pytest.mark.parametrize("gpus", [2, 8])
def test_bench_gpus_spawns_ranks_gloo(gpus):
    """`bench.py --gpus N` with no launcher starts N fresh ranks (torch.distributed.run as a
    child) and rank 0 reports n_gpus = N from the process group, one device per rank. N = 8
    is the driver's scaling run's launch, rehearsed as 8 CPU ranks."""
    import json
    import subprocess
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--launch-check"],
                       env=_bench_env(OMP_NUM_THREADS="1"), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(s) for s in r.stdout.splitlines() if s.startswith("{")]
    assert len(lines) == 1
    assert lines[0]["n_gpus"] == gpus and lines[0]["backend"] == "gloo"
    assert sorted(x["rank"] for x in lines[0]["ranks"]) == list(range(gpus))
    assert [x["device"] for x in sorted(lines[0]["ranks"], key=lambda x: x["rank"])] == list(range(gpus))


def _build_once_worker(rank, world, port, out):
    import time
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)

    def build():
        t0 = time.time()
        time.sleep(0.4 if rank == 0 else 0.01)   # rank 0: the cold-cache generation
        return (t0, time.time())

    out[rank] = bench.build_once(dist, rank, build)
    dist.destroy_process_group()


def test_build_once_rank0_first_gloo():
    """bench.build_once: on a cold cache rank 0 builds the circuit while ranks 1..7 wait at a
    barrier, then they build (read the cache); 8 gloo ranks."""
    world = 8
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_build_once_worker, args=(world, _free_port(), out), nprocs=world, join=True)
        res = dict(out)
    end0 = res[0][1]
    assert all(res[r][0] >= end0 for r in range(1, world))


def test_bench_world_mismatch_exits_nonzero():
    """A launcher's world that differs from --gpus is refused before any work."""
    import subprocess
    env = _bench_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--launch-check"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 2
    assert "WORLD_SIZE=1" in r.stderr


def test_shard_edge_cases():
    assert [list(bench.shard(3, r, 8)) for r in range(8)] == [[0], [1], [2], [], [], [], [], []]
    assert list(bench.shard(0, 0, 1)) == []
    assert sum(len(bench.shard(512, r, 8)) for r in range(8)) == 512


# ---- single-proof MSM split across ranks (nzcb/msmsplit.py, configs[4]) ---------------
def _split_points(n, tau=0x6E7A6362746175):
    from oracle import bn254 as bn
    pts, t = [], 1
    for _ in range(n):
        pts.append(bn.g1_to_lem(bn.g1_mul(bn.G1_GEN, t)))
        t = t * tau % bn.R_MOD
    return pts


_LAG_TAU = 0x4C6167  # the CPU test's stand-in for the Lagrange basis: another point set


def _split_worker(rank, world, port, n, jobs, fail, out):
    """Rank 0 drives the protocol as the prover does (sends of up to three commitments in
    flight, then gathers); ranks 1.. serve with the CPU port's MSM over their range. A batch
    marked Lagrange (A, B, C: n - 4 = the prover's n + 2 points of another basis) travels
    with NZCB_MSM_LAGRANGE in its slot and is served from the ranks' Lagrange ranges."""
    import torch.distributed as dist
    from nzcb import msmsplit
    from oracle import cbind
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    comm = msmsplit.Comm(dist, "cpu")
    nl = n - 4
    pts, lpts = _split_points(n), _split_points(nl, _LAG_TAU)
    ranges, lranges = msmsplit.point_ranges(n, world), msmsplit.point_ranges(nl, world)

    def cpu_partial(own_slice: bytes, cnt, lag=False):
        """This rank's range partial from ITS slice of the scalars (what the scatter sends)."""
        if cnt == 0:
            return bytes(64)
        lo = (lranges if lag else ranges)[rank][0]
        return cbind.msm(b"".join((lpts if lag else pts)[lo:lo + cnt]), own_slice[:32 * cnt], threads=1)

    if rank == 0:
        def source(src, first, cnt, row):
            import torch
            row[:32 * cnt].copy_(torch.frombuffer(bytearray(src[32 * first:32 * (first + cnt)]), dtype=torch.uint8))

        with msmsplit.SplitRoot(comm, n, scalar_source=source, n_lagrange=nl) as root:
            assert root.own_points == ranges[0][1] and root.own_lagrange == lranges[0][1]
            folded = []
            for lag, batch in jobs:               # up to 3 commitments in flight, as the prover
                owns = {}
                for slot, sc in enumerate(batch):
                    count = len(sc) // 32
                    root.send(slot | (msmsplit.MSM_LAGRANGE if lag else 0), sc, count)
                    owns[slot] = cpu_partial(sc, msmsplit.slice_counts(count, lranges if lag else ranges)[0], lag)
                for slot in range(len(batch)):
                    folded.append(root.gather(slot | (msmsplit.MSM_LAGRANGE if lag else 0), owns[slot]))
            if fail:
                # a scalar source that raises sends nothing: the servers stay in step
                def bad(*_):
                    raise RuntimeError("scalar source failed")
                root.scalar_source = bad
                sc = jobs[1][1][0]
                with pytest.raises(RuntimeError):
                    root.send(0, sc, len(sc) // 32)
                root.scalar_source = source
                root.send(0, sc, len(sc) // 32)
                folded.append(root.gather(0, cpu_partial(sc, msmsplit.slice_counts(len(sc) // 32, ranges)[0])))
        out[0] = folded
    else:
        out[rank] = msmsplit.serve(comm, lambda slot, t, cnt: cpu_partial(bytes(t.tolist()), cnt), n, nl,
                                   lambda slot, t, cnt: cpu_partial(bytes(t.tolist()), cnt, True))
    dist.barrier()
    dist.destroy_process_group()


def _split_order_worker(rank, world, port, n, jobs, out):
    """Back-to-back commitments on ONE slot with a slow scalar source: every scatter is
    asynchronous (msmsplit.Comm.scatter_rows), so rank 0's next send must wait for the
    slot's previous scatter before it refills the rows, and a serving rank must wait for
    its slice before reading it; a send that skipped either wait would fold stale or torn
    scalars into the partials."""
    import time
    import torch.distributed as dist
    from nzcb import msmsplit
    from oracle import cbind
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    comm = msmsplit.Comm(dist, "cpu")
    pts = _split_points(n)
    ranges = msmsplit.point_ranges(n, world)
    lo, _ = ranges[rank]

    def cpu_partial(own_slice: bytes, cnt):
        return cbind.msm(b"".join(pts[lo:lo + cnt]), own_slice[:32 * cnt], threads=1) if cnt else bytes(64)

    if rank == 0:
        def slow_source(src, first, cnt, row):
            import torch
            time.sleep(0.05)   # a slow producer of the scalars (a long device copy)
            row[:32 * cnt].copy_(torch.frombuffer(bytearray(src[32 * first:32 * (first + cnt)]), dtype=torch.uint8))

        with msmsplit.SplitRoot(comm, n, scalar_source=slow_source) as root:
            folded = []
            for sc in jobs:                      # the same slot again and again, no gather between
                root.send(0, sc, len(sc) // 32)
                folded.append(root.gather(0, cpu_partial(sc, msmsplit.slice_counts(len(sc) // 32, ranges)[0])))
            # two sends on one slot before any gather: the second waits for the first scatter
            root.send(1, jobs[0], len(jobs[0]) // 32)
            root.send(1, jobs[1], len(jobs[1]) // 32)
            folded.append(root.gather(1, cpu_partial(jobs[1], msmsplit.slice_counts(len(jobs[1]) // 32,
                                                                                     ranges)[0])))
        out[0] = folded
    else:
        def slow_partial(slot, t, cnt):
            time.sleep(0.02)
            return cpu_partial(bytes(t.tolist()), cnt)
        out[rank] = msmsplit.serve(comm, slow_partial, n)
    dist.barrier()
    dist.destroy_process_group()


def test_msm_split_async_scatter_ordering_gloo():
    """the split's scatters are asynchronous on every backend; the waits
    that order them (rank 0 before refilling a slot's rows, serving ranks before reading a
    slice) keep every folded commitment equal to the unsplit MSM under a slow source."""
    import random
    from oracle import bn254 as bn
    from oracle import cbind
    n, world = 70, 2
    rng = random.Random(77)
    jobs = [b"".join(bn.to_lem(rng.randrange(bn.R_MOD), bn.R_MOD) for _ in range(k)) for k in (66, 70, 40, 66)]
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_split_order_worker, args=(world, _free_port(), n, jobs, out), nprocs=world, join=True)
        res = dict(out)
    pts = _split_points(n)
    want_jobs = jobs + [jobs[1]]
    assert res[1] == len(jobs) + 2   # the serving rank answered every send, the overwritten one included
    assert len(res[0]) == len(want_jobs)
    for sc, parts in zip(want_jobs, res[0]):
        count = len(sc) // 32
        acc = None
        for r in range(world):
            p = parts[64 * r:64 * r + 64]
            x, y = bn.from_le(p[:32]), bn.from_le(p[32:])
            acc = bn.g1_add(acc, None if x == 0 and y == 0 else (x, y))
        want = cbind.msm(b"".join(pts[:count]), sc, threads=1)
        assert acc == (bn.from_le(want[:32]), bn.from_le(want[32:]))


@pytest.mark.parametrize("world,fail", [(2, False), (3, False), (2, True)])
def test_msm_split_across_ranks_gloo(world, fail):
    """Every commitment's folded partials equal the unsplit MSM (C port), for MSM lengths
    shorter than, equal to and crossing the rank boundaries (the prover's n+2 .. n+6). Each
    serving rank receives only its slice of the scalars. A proof's nine commitments: A, B, C
    over the Lagrange basis (round 6, their own point ranges), Z, T1..T3, Wxi, Wxiw over PTau.
    With `fail`, a send whose scalar source raises leaves the protocol in step:
    the next commitment still folds."""
    import random
    from oracle import bn254 as bn
    from oracle import cbind
    n = 70                                    # a 2^6 domain's n + 6 PTau points
    rng = random.Random(world)

    def scal(count):
        return b"".join(bn.to_lem(rng.randrange(bn.R_MOD), bn.R_MOD) for _ in range(count))

    jobs = [(True, [scal(66), scal(66), scal(66)]), (False, [scal(67)]), (False, [scal(64), scal(64), scal(70)]),
            (False, [scal(70), scal(67)]), (False, [scal(1), scal(0)])]
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_split_worker, args=(world, _free_port(), n, jobs, fail, out), nprocs=world, join=True)
        res = dict(out)
    pts = _split_points(n)
    lpts = _split_points(n - 4, _LAG_TAU)
    flat = [(lag, sc) for lag, batch in jobs for sc in batch] + ([(False, jobs[1][1][0])] if fail else [])
    assert sum(len(b) for _, b in jobs[:4]) == 9     # one proof's commitments
    assert [res[r] for r in range(1, world)] == [len(flat)] * (world - 1)
    assert len(res[0]) == len(flat)
    for (lag, sc), parts in zip(flat, res[0]):
        count = len(sc) // 32
        acc = None
        for r in range(world):
            p = parts[64 * r:64 * r + 64]
            x, y = bn.from_le(p[:32]), bn.from_le(p[32:])
            acc = bn.g1_add(acc, None if x == 0 and y == 0 else (x, y))
        want = cbind.msm(b"".join((lpts if lag else pts)[:count]), sc, threads=1) if count else bytes(64)
        wx, wy = bn.from_le(want[:32]), bn.from_le(want[32:])
        assert acc == (None if wx == 0 and wy == 0 else (wx, wy))
