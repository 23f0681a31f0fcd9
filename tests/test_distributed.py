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
    per_rank = bench.gather_per_rank(1.0 + rank, 100, 10, world, dev)
    env0, game0 = bench.shard(rank, 8192, 8192, 0)
    # the staggered pre-roll: each rank resets its slice of the global plan
    plan = bench.stagger_plan(4096, 2000, game0, world * 4096)
    resets = [(t, game0 + g) for t, gs in enumerate(plan) for g in gs]
    bench.barrier(world, dev)
    dist.destroy_process_group()
    q.put((rank, m, env0, game0, resets, per_rank))


@pytest.mark.parametrize("world", [2, 4])
def test_bench_collectives_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=120) for _ in range(world)), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # every rank sees the max elapsed time; shards are disjoint, contiguous, even
    assert all(r[1] == 1.5 + world - 1 for r in res)
    # every rank gathers every rank's elapsed time / rate (bench line: window.per_rank)
    assert all(r[5] == [{"rank": k, "elapsed_s": 1.0 + k, "env_steps_per_s": round(1000 / (1.0 + k), 1)}
                        for k in range(world)] for r in res)
    assert [(r[2], r[3]) for r in res] == [(k * 8192, k * 4096) for k in range(world)]
    # the ranks' staggered resets together are exactly one unsharded run's plan
    import sys

    sys.path.insert(0, REPO)
    import bench

    union = sorted(x for r in res for x in r[4])
    glob = sorted((t, g) for t, gs in enumerate(bench.stagger_plan(world * 4096, 2000)) for g in gs)
    assert union == glob


def test_shard_rejects_odd():
    import sys

    sys.path.insert(0, REPO)
    import bench

    with pytest.raises(AssertionError):
        bench.shard(0, 7, 7, 0)


def test_stagger_plan_spreads_episode_ages():
    import sys

    sys.path.insert(0, REPO)
    import numpy as np

    import bench

    plan = bench.stagger_plan(4096, 2000)
    tick = np.empty(4096, int)
    for t, gs in enumerate(plan):
        tick[gs] = t
    ages = 2000 - tick                       # episode age of every game after the pre-roll
    assert ages.min() == 1 and ages.max() == 2000
    assert np.histogram(ages, bins=10, range=(0, 2000))[0].min() >= 400   # even spread
