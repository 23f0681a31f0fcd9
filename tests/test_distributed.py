"""The N>1 bench path on CPU: world_size-2 `gloo` process group driving the
same barrier / max-over-ranks / sharding code bench.py runs over RCCL on the
MI355X node (envs shard with no data-path collective)."""
import os
import socket

import pytest
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys

    sys.path.insert(0, REPO)
    import torch
    import torch.distributed as dist

    import bench

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cpu")
    bench.barrier(world, dev)
    m = bench.max_over_ranks(1.5 + rank, world, dev)
    lo, hi = bench.shard(rank, 8192)
    bench.barrier(world, dev)
    dist.destroy_process_group()
    q.put((rank, m, lo, hi))


@pytest.mark.parametrize("world", [2, 4])
def test_bench_collectives_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # every rank sees the max elapsed time; shards are disjoint, contiguous, even
    assert all(r[1] == 1.5 + world - 1 for r in res)
    ranges = [(r[2], r[3]) for r in res]
    assert ranges == [(k * 8192, (k + 1) * 8192) for k in range(world)]


def test_shard_rejects_odd():
    import sys

    sys.path.insert(0, REPO)
    import bench

    with pytest.raises(AssertionError):
        bench.shard(0, 7)
