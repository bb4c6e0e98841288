#!/usr/bin/env python3
"""bench.py — PLONK proofs/s for nzcp_live (~2^21 domain) on MI355X.

Metric and config come from BASELINE.json: "PLONK proofs/sec for nzcp_live
(~2^21 constraints) at 1/2/4/8 MI355X"; workload = configs[2] (single nzcp_live
proof on one GPU), batch-sharded with no collective across ranks (configs[3]).

The statement is the reference's circuit, NZCPPubIdentity(1, 351, 0, 4, 2, 4)
(/root/reference/circuits/nzcp_live.circom), compiled by nzcb/nzcpgen.py to an r1cs
(603,800 constraints, 1.79 M PLONK gates, domain 2^21) and a witness program; the
zkey comes from nzcb_plonk_setup against a seeded-tau ptau of power 21 (the ceremony
file powersOfTau28_hez_final_21.ptau and circom are not on disk).

A "step" is one plonk.fullProve of one NZ COVID Pass: the GPU witness program
computes all 600,560 signals of the pass's witness in HBM (nzcb_wprog_run_dev, the
circom witness calculator's job), then the full proof runs (snarkjs plonk_prove rounds
1-5). The passes' input signals are resident in HBM when the timed region starts;
the 800-byte proofs and the public signals are copied back inside it. The K timed
proofs are one witness launch plus one nzcb_prove_batch call: --lanes proofs are in
flight on each GPU (lanes share the HBM-resident proving key; SURVEY.md §8e batch
mode), so one proof's latency-bound phases overlap another's compute.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...

Rank 0 prints ONE JSON line. Each rank proves K proofs on its own GPU (weak
scaling, no data-path collective); the timed region is bracketed by a barrier and
device syncs, and the max over ranks is used.
"""
import argparse
import hashlib
import json
import os
import sys
import time

# HIP maps a process's streams onto GPU_MAX_HW_QUEUES hardware queues (4 by default);
# 4 lanes x 4 streams on 4 queues falsely serialise kernels of independent proofs.
# 24 queues measured +12-16 % over 4 (DESIGN.md §4 "Concurrency"); set before HIP initialises.
if os.environ.get("GPU_MAX_HW_QUEUES", "4") == "4":  # unset or HIP's default (the box exports 4)
    os.environ["GPU_MAX_HW_QUEUES"] = "24"

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "nzcb-circom_amd"))

METRIC = "PLONK proofs/sec for nzcp_live (~2^21 constraints) at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
MSM_BYTES_PER_POINT = 96       # 64 B affine base + 32 B scalar
PROOF_BYTES_PER_N = 7104       # algorithmic bytes per proof = 7104 * n
NZCP_INPUTS = 2970             # nzcp_live input signals (toBeSigned bits + len + data)
SEED = 0x6E7A6362
TAU = 0x6E7A6362746175         # seeded ptau trapdoor
# The dominant kernel (fixed-base bucket accumulation) is bound by VALU integer
# multiply issue, not by HBM (SURVEY.md §8d "Bounding roofline"). Its algorithmic
# work is the 9x29-bit Montgomery products of one XYZZ mixed addition per bucket
# entry: 1467 v_mad_u64_u32 per entry (ISA count of the common path).
MADS_PER_ENTRY = 1467
# Peak: MI355X_MICROARCH.md chip table (256 CUs x 4 SIMDs, 2400 MHz max clock; FP32
# vector peak 157.3 TFLOPS = v_fma_f32 issuing one wave64 instruction per 2 cycles per
# SIMD). v_mad_u64_u32 issues at 5.00 / 2.60 = 1.92x the v_fma_f32 cost in the same
# harness (profiles/r1_isa_bench.txt), so the chip issues at most
# 1024 * 2.4e9 / (2 * 1.923) wave-mads/s x 64 lanes = 40.9 T lane-mads/s.
MAD_PEAK_T = 1024 * 2.4e9 / (2 * 5.00 / 2.60) * 64 / 1e12


def blinding_for(step: int) -> bytes:
    """Distinct deterministic blinding per proof (snarkjs draws Fr.random())."""
    r = 21888242871839275222246405745257275088548364400416034343698204186575808495617
    out = b""
    for i in range(11):
        h = hashlib.sha256(b"nzcb-bench" + step.to_bytes(4, "little") + bytes([i])).digest()
        out += (int.from_bytes(h, "big") % r).to_bytes(32, "little")
    return out


def shard(count: int, rank: int, world: int) -> range:
    """Proof indices of one rank in a batch of `count` (contiguous, sizes differ by <= 1)."""
    q, r = divmod(count, world)
    lo = rank * q + min(rank, r)
    return range(lo, lo + q + (1 if rank < r else 0))


def max_over_ranks(x: float, dist, device) -> float:
    """The job's time is the slowest rank's (one float all-reduce; RCCL on GPUs, gloo in tests)."""
    if dist is None:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def rank_memory(device: int, dist) -> list:
    """Per rank, after the timed region: HBM in use on its device (hipMemGetInfo, device-wide:
    ranks sharing a device in a rehearsal see each other's), i.e. the proving key, both
    fixed-base tables, every lane's working set and the witness buffers; and the process's
    peak host RSS. DESIGN.md §6 sizes an 8-rank node from these."""
    import ctypes
    import resource
    # the HIP runtime the prover library already loaded (not a second copy by name)
    with open("/proc/self/maps") as f:
        paths = [ln.split()[-1] for ln in f if "libamdhip64.so" in ln]
    hip = ctypes.CDLL(paths[0] if paths else "libamdhip64.so")
    free, total = ctypes.c_size_t(0), ctypes.c_size_t(0)
    if hip.hipSetDevice(ctypes.c_int(device)) != 0 or hip.hipMemGetInfo(ctypes.byref(free), ctypes.byref(total)) != 0:
        free.value = total.value = 0
    free, total = free.value, total.value
    me = {"rank": dist.get_rank() if dist is not None else 0, "device": device,
          "hbm_used_gib": round((total - free) / 2**30, 2), "hbm_total_gib": round(total / 2**30, 1),
          "host_peak_rss_gib": round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 2**20, 2)}
    if dist is None:
        return [me]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, me)
    return out


def pass_data(i: int) -> bytes:
    """The 20 pass-through data bytes of proof i."""
    return hashlib.sha256(b"nzcb-pass" + i.to_bytes(4, "little")).digest()[:20]


def pass_inputs(indices) -> bytes:
    """nzcp_live input signals of distinct live-shaped passes: one ToBeSigned, the 20
    pass-through data bytes derived from the proof index."""
    from nzcb import nzcp
    tbs = nzcp.pass_tbs(live=True)
    return b"".join(nzcp.input_signals(nzcp.circuit_input(tbs, pass_data(i))) for i in indices)


def accumulate_probe(n_points: int, device: int, reps: int = 10) -> dict:
    """The dominant kernel alone on the chip: `reps` fixed-base MSMs of the prover's size
    (n + 6 points, random scalars, the same c = 20 table schedule) with HIP events around
    each phase on the engine's stream (msm.hip MsmScratch::prof). Run after the timed
    region; its accumulation launches are the last `reps` of the rocprofv3 trace."""
    import nzcb
    eng = nzcb.Engine(device, max_log_ntt=-1, max_msm_points=n_points + 8)
    sc, bases = nzcb.dev_alloc(n_points * 32), nzcb.dev_alloc(n_points * 64)
    try:
        eng.random_fr(sc, n_points, 0x70726F6265)
        eng.fixed_base(sc, n_points, bases)
        eng.random_fr(sc, n_points, 0x5CA1A25)
        eng.time_msm_phases(bases, sc, n_points, True, True, 1)   # warm (table build, code load)
        ph = eng.time_msm_phases(bases, sc, n_points, True, True, reps)
    finally:
        nzcb.dev_free(sc)
        nzcb.dev_free(bases)
        eng.close()
    return ph


def cpu_model() -> str:
    """The host CPU's model name (BASELINE.md asks for it next to the core count)."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_baseline_sample(zkey_raw, wtns: bytes, n: int):
    """Time the CPU port (oracle) proving one proof of the same zkey and witness; rank 0,
    N=1 only."""
    from oracle import cbind
    out = cbind.timed_prove(zkey_raw, wtns, f"1 full proof of nzcp_live (n=2^{n.bit_length() - 1}, same zkey "
                                            f"and GPU-computed witness)")
    out["cpu_model"] = cpu_model()
    return out


def launch_plan(gpus: int, env) -> str:
    """How `bench.py --gpus N` runs:
    * "local": this process is the whole job (N = 1 without a launcher) or one rank of a
      launcher's job whose WORLD_SIZE equals N;
    * "spawn": N > 1 and no launcher; start N fresh ranks under torch.distributed.run.
    A launcher's world that differs from --gpus is an error (exit 2): the line would
    otherwise label one world with another's size."""
    if gpus < 1:
        raise SystemExit(f"bench.py: --gpus must be >= 1, got {gpus}")
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        if world != gpus:
            print(f"bench.py: --gpus {gpus} but the launcher started WORLD_SIZE={world} ranks", file=sys.stderr)
            raise SystemExit(2)
        return "local"
    return "spawn" if gpus > 1 else "local"


def spawn_ranks(gpus: int, argv) -> int:
    """Start `gpus` ranks of this script under torch.distributed.run (127.0.0.1, a free
    port) as a CHILD process and return its exit code. Called before anything in this
    process imports torch or touches HIP, so the ranks are fresh processes that each
    initialise their own GPU; rank 0's JSON line reaches stdout through the child."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)
    return subprocess.run(cmd, env=dict(os.environ)).returncode


def build_once(dist, rank: int, build):
    """The nzcp_live r1cs / witness program (nzcplive.build, cached on disk by source hash):
    rank 0 builds (or reads) it first while the other ranks wait at a barrier, so that on a
    cold cache 8 ranks do not each spend the generator's minutes and 8x its host memory; the
    others then read the cache rank 0 wrote."""
    if dist is not None and rank != 0:
        dist.barrier()
    out = build()
    if dist is not None and rank == 0:
        dist.barrier()
    return out


def launch_check(world: int, rank: int, device: int, backend: str, dist) -> None:
    """--launch-check: the launcher's decision without a proof. Every rank reports its rank
    and device to rank 0, which prints one JSON line with n_gpus = dist's world size."""
    got = [None] * world
    dist.all_gather_object(got, {"rank": rank, "device": device})
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": dist.get_world_size(), "backend": backend,
                          "ranks": got}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--lanes", type=int, default=5, help="proofs in flight per GPU")
    ap.add_argument("--batch", type=int, default=0,
                    help="fixed total batch sharded over the ranks (configs[3]: 512); default: --steps per rank")
    ap.add_argument("--msm-devices", default="",
                    help="configs[4] single-proof mode: split each MSM over these device ids, e.g. 0,1,2,3 "
                         "(one process; lanes forced to 1)")
    ap.add_argument("--msm-split", action="store_true",
                    help="configs[4] across ranks: rank 0 proves --steps proofs one at a time, every commitment "
                         "MSM split by point range over all ranks (scatter of scalar slices + gather of partials)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-probe", action="store_true", help="skip the isolated accumulation-kernel probe")
    ap.add_argument("--launch-check", action="store_true",
                    help="start the ranks, report world size and devices, and exit (no GPU work)")
    args = ap.parse_args()

    # before torch / nzcb / any HIP call: --gpus N > 1 without a launcher starts N ranks
    if launch_plan(args.gpus, os.environ) == "spawn":
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knobs (not used by the driver): gloo instead of RCCL, and every rank on
    # one device, to run the multi-rank flow on a one-GPU box
    backend = os.environ.get("NZCB_DIST_BACKEND", "nccl")
    device = int(os.environ.get("NZCB_BENCH_DEVICE", local))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        if backend == "nccl":
            # one GPU per rank: a world larger than the node's devices cannot be measured
            if torch.cuda.device_count() < world:
                print(f"bench.py: {world} ranks over RCCL need {world} GPUs, this node has "
                      f"{torch.cuda.device_count()}", file=sys.stderr)
                sys.exit(2)
            torch.cuda.set_device(device)
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            if not args.launch_check:
                torch.cuda.set_device(device)
            dist.init_process_group(backend)
        if dist.get_world_size() != args.gpus:
            print(f"bench.py: --gpus {args.gpus} but the process group has {dist.get_world_size()} ranks",
                  file=sys.stderr)
            sys.exit(2)
        world = dist.get_world_size()
    rank_devices = [device]
    if dist is not None and not args.launch_check:
        rank_devices = [None] * world
        dist.all_gather_object(rank_devices, device)
    if args.launch_check:
        if dist is not None:
            launch_check(world, rank, device, backend, dist)
            dist.destroy_process_group()
        else:
            print(json.dumps({"launch_check": True, "n_gpus": 1, "backend": None,
                              "ranks": [{"rank": 0, "device": device}]}), flush=True)
        return

    import nzcb
    from nzcb import nzcplive
    t_setup = time.time()
    # the real statement: NZCPPubIdentity(1, 351, 0, 4, 2, 4) compiled to an r1cs and a
    # witness program (nzcb/nzcpgen.py), zkey from nzcb_plonk_setup against a seeded
    # ptau of the reference's power 21 (Makefile:59-62)
    r1cs, program, _ = build_once(dist, rank, nzcplive.build)
    ctx, zkey_raw = nzcplive.context(r1cs, TAU, device)
    setup_s = time.time() - t_setup
    n = ctx.domain_size
    prover = nzcplive.NzcpLiveProver(ctx, program)

    def barrier():
        if dist is not None:
            import torch
            torch.cuda.synchronize(device)
            dist.barrier()

    # one pass's witness for the single-proof latency and the PCIe-inclusive rate
    # (neither is the reported value) and the CPU baseline's sample
    prover.upload_inputs(pass_inputs([999]))
    (w0,) = prover.witness_staged(1)
    nwit = prover.n_witness
    dev_w = nzcb.dev_alloc(nwit * 32)
    nzcb.d2d(dev_w, w0, nwit * 32)
    wit_host = nzcb.d2h(dev_w, nwit * 32)
    ctx.prove_device_raw(dev_w, nwit, blinding_for(998))
    # the latency proof runs without kernel statistics (no timing events), then one more
    # proof with them gives the per-phase GPU times and the accumulation's single-lane launch
    # (the median of 5: one proof's wall time varies by ~0.5 ms from run to run)
    lat = []
    for k in range(5):
        t_l = time.perf_counter()
        ctx.prove_device_raw(dev_w, nwit, blinding_for(997 - 10 * k))
        lat.append((time.perf_counter() - t_l) * 1e3)
    latency_ms = sorted(lat)[len(lat) // 2]
    ctx.kernel_stats(1)
    ctx.prove_device_raw(dev_w, nwit, blinding_for(996))
    lat_kms, lat_klaunch, _, _ = ctx.kernel_stats(0)  # one proof in flight: the kernel nearly alone
    single_timings = ctx.last_timings()
    t_h = time.perf_counter()
    ctx.prove_witness_raw(wit_host, blinding_for(999))
    pcie_ms = (time.perf_counter() - t_h) * 1e3
    msm_devices = [int(x) for x in args.msm_devices.split(",") if x.strip() != ""]
    if msm_devices:
        ctx.set_msm_devices(msm_devices)
        args.lanes = 1
    split = args.msm_split and world > 1
    root = backend_range = comm = None
    if split:
        # configs[4]: rank 0 proves one proof at a time, every commitment MSM split by PTau
        # range over all ranks (each rank's slice of the scalars by scatter, partials gathered to
        # rank 0; nzcb/msmsplit.py)
        from nzcb import msmsplit
        comm = msmsplit.Comm(dist, f"cuda:{device}" if backend == "nccl" else "cpu")
        args.lanes = 1
        # A, B, C too, over ranges of the n + 2-point Lagrange basis (round 6; all 9 commitments)
        n_lag = n + 2 if nzcb.lagrange_commit_enabled() else 0
        if rank == 0:
            root = msmsplit.SplitRoot(comm, n + 6, n_lagrange=n_lag)
            root.install(ctx)
        else:
            addr, size = msmsplit.zkey_section(zkey_raw[0], zkey_raw[1], 14)   # PTau [tau^i]G1
            dev_ptau = nzcb.dev_alloc(size)
            nzcb.memcpy_h2d_ptr(dev_ptau, addr, size)
            lo, hi = msmsplit.point_ranges(n + 6, world)[rank]
            lag = None
            if n_lag:   # this rank's range of the Lagrange basis, from the PTau (1.4 s at 2^21)
                llo, lhi = msmsplit.point_ranges(n_lag, world)[rank]
                lag = msmsplit.GpuRange(dev_ptau, llo, lhi, device, lagrange=True, ptau_n=size // 64,
                                        log_n=n.bit_length() - 1)
            backend_range = (msmsplit.GpuRange(dev_ptau, lo, hi, device), dev_ptau, lag)
    ctx.set_lanes(args.lanes)
    if split:
        mine = list(range(args.steps)) if rank == 0 else []
    else:
        mine = list(shard(args.batch, rank, world)) if args.batch else list(range(rank * args.steps,
                                                                                  (rank + 1) * args.steps))

    def run_proofs(count_or_none, blindings):
        """The step loop of this rank: proofs (and, in split mode, the STOP that ends the
        servers' loop), or serving rank 0's commitments."""
        if split and rank != 0:
            msmsplit.serve(comm, backend_range[0], n + 6, n_lag, backend_range[2])
            return []
        res = prover.full_prove_staged(count_or_none, blindings) if count_or_none else []
        if root is not None:
            root.stop()
        return res

    if args.warmup:
        nw = max(args.warmup, 2 * args.lanes)  # every lane proves at least once before timing
        if not split or rank == 0:
            prover.upload_inputs(pass_inputs(range(100000, 100000 + nw)))
        barrier()
        run_proofs(nw, [blinding_for(1000 + i) for i in range(nw)])
    ctx.kernel_stats(1)
    blinds = [blinding_for(i) for i in mine]
    if mine:  # a rank can hold no proofs when --batch is smaller than the world
        prover.upload_inputs(pass_inputs(mine))  # the passes' input signals, resident in HBM
        prover.witness_buffers(len(mine))
    barrier()
    t0 = time.perf_counter()
    proofs = run_proofs(len(mine), blinds)   # GPU witness program + prove_batch
    barrier()
    elapsed = time.perf_counter() - t0
    kms, klaunch, kpoints, kentries = ctx.kernel_stats(0)
    if root is not None:
        ctx.set_msm_split(1, 0, None, None)
    if backend_range is not None:
        backend_range[0].close()
        if backend_range[2] is not None:
            backend_range[2].close()
        nzcb.dev_free(backend_range[1])
    assert len({p for p, _ in proofs}) == len(mine)  # distinct passes -> distinct proofs
    # full-size checks outside the timed region: every proof's public signals equal its
    # pass's outputs from the independent nzcp kernel (csrc/nzcp.hip, bit-exact against
    # the restatement pinned by the reference's KATs), and the pairing verifier accepts
    # the first and last proof of the batch
    records = nzcb.nzcp_witness(pass_inputs(mine), len(mine), nzcb.NZCP_LIVE, device) if mine else []
    pubs_ok = all(r["status"] == 0 and [int.from_bytes(pub[32 * k:32 * k + 32], "little") for k in range(3)] == r["out"]
                  for (_, pub), r in zip(proofs, records))
    verified = pubs_ok and all(nzcb.verify(ctx.vk, proofs[i][0], proofs[i][1])
                               for i in ({0, len(proofs) - 1} if proofs else ()))
    t_w = time.perf_counter()
    prover.witness_staged(len(mine))
    witness_ms = (time.perf_counter() - t_w) * 1e3
    mem = rank_memory(device, dist)
    probe =accumulate_probe(n + 6, device) if rank == 0 and not args.no_probe else None
    elapsed = max_over_ranks(elapsed, dist, f"cuda:{device}" if backend == "nccl" else "cpu")
    total_proofs = args.steps if split else (args.batch if args.batch else args.steps * world)
    steps = len(shard(args.batch, 0, world)) if args.batch and not split else args.steps
    value = total_proofs / elapsed
    ms_step = elapsed / steps * 1e3

    if rank == 0:
        # the accumulation kernel over the timed region (HIP events on the MSM streams;
        # --lanes proofs share the chip, so these launches overlap other kernels)
        shared_ms = kms / max(klaunch, 1)
        pts_per_launch = kpoints / max(klaunch, 1)
        ent_per_launch = kentries / max(klaunch, 1)
        # the same kernel alone on the chip, same size and schedule: its duration is the
        # roofline's launch time (profiles/: the last 10 accumulation launches of the trace)
        iso_ms = probe["accumulate"] if probe else None
        launch_ms = iso_ms or shared_ms
        # the probe's launch: its own entries (random scalars: ~15 per point); the timed
        # region's average also holds the A, B, C MSMs of small witness values
        probe_entries = probe.get("entries") if probe else None
        launch_entries = probe_entries or ent_per_launch
        launch_points = (n + 6) if probe else pts_per_launch
        mads_t = MADS_PER_ENTRY * launch_entries / (launch_ms / 1e3) / 1e12 if launch_ms else 0.0
        hbm_gbs = MSM_BYTES_PER_POINT * launch_points / (launch_ms / 1e3) / 1e9 if launch_ms else 0.0
        # HBM traffic per launch is a committed PMC measurement (two separate rocprofv3 --pmc
        # passes, FETCH_SIZE and WRITE_SIZE, tools/profile_round.sh), not this run's: the line
        # names the file and the run it came from
        traffic = traffic_source = None
        tf = os.environ.get("NZCB_TRAFFIC_JSON", os.path.join(ROOT, "profiles", "accumulate_traffic.json"))
        if tf and os.path.exists(tf):
            with open(tf) as f:
                tj = json.load(f)
            traffic = tj.get("bytes_per_launch")
            traffic_source = {"file": os.path.relpath(tf, ROOT), "measured": tj.get("source", "round 5 profile set"),
                              "in_this_run": False}
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            try:
                cpu = cpu_baseline_sample(zkey_raw, nzcplive.wtns_file(wit_host), n)
            except Exception as e:  # reported, never silently replaced
                cpu = {"value": None, "unit": "proofs/s", "cores": 0, "kind": "port", "sample": f"failed: {e}"}
        proof_gbs = PROOF_BYTES_PER_N * n / (ms_step / 1e3) / 1e9
        # ranks sharing a device (the one-GPU rehearsal, NZCB_BENCH_DEVICE) are not that many
        # GPUs: n_gpus counts distinct devices and the line says it is a rehearsal
        n_devices = len(set(rank_devices))
        line = {
            "metric": METRIC,
            "value": round(value, 4),
            "unit": "proofs/s",
            "n_gpus": n_devices,
            "n_ranks": world,
            "steps": steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 3),
            "higher_is_better": True,
            "scaling": "strong" if (args.batch or split) else "weak",
            "vs_baseline": None,
            "dtype": "u32 limbs: BN254 Fr/Fq Montgomery, 8x32-bit and 9x29-bit (MSM, NTT twiddles, quotient)",
            "data": "synthetic passes: live-shaped NZ COVID Pass ToBeSigned (live key id and issuer) with 20 "
                    "pass-through data bytes that differ per proof; proving key from a seeded-tau ptau (SURVEY §8d)",
            "config": {
                "workload": f"nzcp_live fullProve: NZCPPubIdentity(1,351,0,4,2,4) witness on the GPU "
                            f"({prover.n_witness} signals) + PLONK proof, n=2^{n.bit_length() - 1}, nPublic=3, "
                            f"{NZCP_INPUTS} inputs",
                "domain_size": n,
                "n_public": 3,
                "n_constraints": ctx.n_constraints,
                "n_vars": ctx.n_vars,
                "n_additions": ctx.n_additions,
                "proofs_per_gpu": steps,
                "total_proofs": total_proofs,
                "parallelism": (f"single-proof MSM split x{world} ({backend}: each rank's scalar slice by "
                                f"scatter, 64-byte partials gathered to rank 0)" if split
                                else f"batch-shard x{world} (no collective)"),
                "proofs_in_flight_per_gpu": args.lanes,
                "msm_devices": msm_devices or None,
                "rank_devices": rank_devices,
                "dist_backend": backend if dist is not None else None,
            },
            "roofline": {
                "kernel": "msm_accumulate29_kernel (fixed-base Pippenger bucket accumulation, c=20, 2^21+6 points)",
                # VALU integer-multiply issue governs this kernel; the contract's
                # hbm/mfma vocabulary has no word for it, and there is no MFMA in modular arithmetic
                "bound": "valu",
                "achieved": round(mads_t, 3),
                "peak": round(MAD_PEAK_T, 2),
                "unit": "T v_mad_u64_u32 lane-ops/s",
                "frac": round(mads_t / MAD_PEAK_T, 4),
                "traffic": traffic,
                "traffic_source": traffic_source,
                "avg_launch_ms": round(launch_ms, 4),
                "launch_ms_basis": "isolated launches (accumulate_probe, HIP events)" if iso_ms
                                   else "timed region, shared chip (probe skipped)",
                "timed_region_avg_launch_ms": round(shared_ms, 4),
                "single_proof_avg_launch_ms": round(lat_kms / max(lat_klaunch, 1), 4),
                "launches_timed": int(klaunch),
                "points_per_launch": int(launch_points),
                "bucket_entries_per_launch": int(launch_entries),
                "timed_region_avg_entries_per_launch": int(ent_per_launch),
                "mads_per_entry": MADS_PER_ENTRY,
                "hbm": {"algorithmic_bytes_per_launch": int(MSM_BYTES_PER_POINT * launch_points),
                        "bytes_per_point": MSM_BYTES_PER_POINT, "achieved_GBs": round(hbm_gbs, 2),
                        "peak_GBs": HBM_PEAK_GBS, "frac": round(hbm_gbs / HBM_PEAK_GBS, 5)},
                "probe_phase_ms": {k: round(v, 4) for k, v in probe.items() if k != "entries"} if probe else None,
            },
            "proof_roofline": {
                "algorithmic_bytes": PROOF_BYTES_PER_N * n,
                "achieved_GBs": round(proof_gbs, 2),
                "frac": round(proof_gbs / HBM_PEAK_GBS, 5),
            },
            "rehearsal": n_devices != world,
            "proofs_verified": verified,
            "witness_program_ms_per_batch": round(witness_ms, 3),
            "single_proof_latency_ms": round(latency_ms, 3),
            "single_proof_latency_ms_runs": [round(x, 3) for x in lat],
            "phase_ms_single_proof": {k: round(v, 3) for k, v in single_timings.items()},
            "pcie_inclusive_ms": round(pcie_ms, 3),
            "setup_s": round(setup_s, 2),
            "memory_per_rank": mem,
            "cpu_baseline": cpu,
        }
        if not verified:  # never report a rate for proofs that do not verify
            line["value"] = None
            line["error"] = "proofs_verified is false: public signals differ from the nzcp records or a proof " \
                            "failed the pairing check"
        print(json.dumps(line), flush=True)
        if not verified:
            sys.exit(3)
    nzcb.dev_free(dev_w)
    prover.close()
    ctx.close()
    nzcb.free_ptr(zkey_raw[0])
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
