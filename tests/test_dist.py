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


def test_shard_edge_cases():
    assert [list(bench.shard(3, r, 8)) for r in range(8)] == [[0], [1], [2], [], [], [], [], []]
    assert list(bench.shard(0, 0, 1)) == []
    assert sum(len(bench.shard(512, r, 8)) for r in range(8)) == 512
