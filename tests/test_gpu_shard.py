"""Multi-GPU sharding is exact ("per-shard results equal
single-GPU results for the same env indices"; §8e: envs shard with no
collective).  A shard holds global envs [env0, env0 + n) and games
[game_offset, ...): the sampler's Philox counter takes the global env index and
the random bots' streams the global game index, so each shard plays exactly its
slice of one unsharded run.

* in process: two shard engines of n envs == one engine of 2n envs, every step;
* end to end: bench.py's own sharding path with 2 ranks (gloo: both share the
  box's one GPU), under torch.distributed.run and self-launched by a plain
  `bench.py --gpus 2`, == one bench.py process of 2n envs.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]   # per-test limits below override
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W = np.array([10.0, 1.0, 1.0, 0.2, 1.0, 4.0])


def _env(nsp, nbot, bots, game_offset, max_steps):
    import torch

    from gym_microrts import microrts_ai
    from gym_microrts.envs.vec_env import MicroRTSGridModeVecEnv

    return MicroRTSGridModeVecEnv(num_selfplay_envs=nsp, num_bot_envs=nbot, max_steps=max_steps,
                                  map_paths=["maps/16x16/basesWorkers16x16.xml"], ai2s=[getattr(microrts_ai, b) for b in bots],
                                  reward_weight=W, return_tensors=True, obs_dtype=torch.int32, game_offset=game_offset)


@pytest.mark.parametrize("kind", ["selfplay", "bots"])
def test_two_shards_equal_one_run(kind):
    import ctypes

    import torch

    from gym_microrts import _native

    n, max_steps, steps = 256, 90, 200
    bots = (["randomBiasedAI", "randomAI", "coacAI", "workerRushAI"] * (2 * n))[:2 * n] if kind == "bots" else []
    nsp = 2 * n if kind == "selfplay" else 0
    g_per_env = 0.5 if kind == "selfplay" else 1
    whole = _env(nsp, len(bots), bots, 0, max_steps)
    shards = [_env(nsp // 2, len(bots) // 2, bots[r * n:(r + 1) * n] if bots else [], int(r * n * g_per_env), max_steps)
              for r in range(2)]
    envs = [whole] + shards
    for e in envs:
        e.reset()
    lib, st = _native.lib(), torch.cuda.current_stream().cuda_stream
    acts = [torch.empty((e.num_envs, 256, 7), dtype=torch.int64, device="cuda") for e in envs]
    env0s = [0, 0, n]
    resets = 0
    for s in range(steps):
        out = []
        for e, a, e0 in zip(envs, acts, env0s):
            m = e.get_action_mask()
            _native.check(lib.mrts_sample_actions_src(st, m.data_ptr(), e.source_unit_mask.data_ptr(), e.num_envs, 256, e0,
                                                      ctypes.c_uint64(77), s, a.data_ptr()))
            o, r, d, i = e.step(a)
            out.append((o.clone(), r.clone(), d.clone(), i._raw.clone(), e._mask.clone()))
        for k in range(5):
            assert torch.equal(out[0][k], torch.cat([out[1][k], out[2][k]])), f"step {s} output {k}"
        resets += int(out[0][2].sum())
    assert resets >= 2 * n
    for e in envs:
        assert e.error_flags() == 0


def test_sampler_env_offset_matches_oracle():
    import ctypes

    import torch

    from gym_microrts import _native
    from oracle_py import sample_actions

    rng = np.random.default_rng(3)
    m = (rng.random((40, 64, 78)) < 0.2).astype(np.int32)
    src = (m.sum(-1) > 0).astype(np.int32)
    md, sd = torch.from_numpy(m).cuda(), torch.from_numpy(src).cuda()
    out = torch.empty((40, 64, 7), dtype=torch.int64, device="cuda")
    for env0 in (0, 1, 4096, 123457):
        _native.check(_native.lib().mrts_sample_actions_src(torch.cuda.current_stream().cuda_stream, md.data_ptr(), sd.data_ptr(), 40,
                                                            64, env0, ctypes.c_uint64(9), 5, out.data_ptr()))
        ref = sample_actions(m, 9, 5, env0=env0)
        np.testing.assert_array_equal(out.cpu().numpy(), ref)
    # a shard's rows are the slice of the whole batch's
    np.testing.assert_array_equal(sample_actions(m[20:], 9, 5, env0=20), sample_actions(m, 9, 5)[20:])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(300)
@pytest.mark.parametrize("launcher,world", [("torchrun", 2), ("self", 2), ("self", 4)])
def test_bench_sharding_end_to_end(tmp_path, launcher, world):
    """bench.py --gpus N (N ranks, the default gloo timing group) dumps each rank's final
    outputs; they are the N slices of a 1-rank bench.py run of all the envs (same seed,
    staggered pre-roll, warmup and timed steps).  launcher = torchrun: under
    torch.distributed.run (the driver's SCALE invocation); self: a plain
    `bench.py --gpus N`, which starts its ranks itself (bench.launch_ranks).  The line
    carries one per-rank entry per rank (window.per_rank)."""
    total = 512
    common = ["--steps", "25", "--warmup", "3", "--preroll", "120", "--max-steps", "120", "--no-cpu-baseline",
              "--roofline-steps", "8", "--rank-timeout", "240"]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    bench = os.path.join(REPO, "bench.py")
    n_args = ["--gpus", str(world), "--envs-per-gpu", str(total // world), "--dump", str(tmp_path / "n")] + common
    if launcher == "torchrun":
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world), "--master-addr",
               "127.0.0.1", "--master-port", str(_free_port()), bench] + n_args
    else:
        cmd = [sys.executable, bench] + n_args
    many = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=270)
    assert many.returncode == 0, many.stderr[-3000:]
    one = subprocess.run([sys.executable, bench, "--envs-per-gpu", str(total), "--dump", str(tmp_path / "one")]
                         + common, env=env, capture_output=True, text=True, timeout=240)
    assert one.returncode == 0, one.stderr[-3000:]
    import json

    lines = [ln for ln in many.stdout.strip().splitlines() if ln.startswith("{")]
    assert len(lines) == 1, many.stdout[-3000:]   # rank 0 only
    line = json.loads(lines[0])
    assert line["n_gpus"] == world and line["window"]["auto_resets"] > 0
    assert line["process_group"]["world_size"] == world and line["process_group"]["backend"] == "gloo"
    assert ("self" in line["process_group"]["launcher"]) == (launcher == "self")
    assert line["roofline"]["samples"] == 8
    pr = line["window"]["per_rank"]
    assert [p["rank"] for p in pr] == list(range(world)) and all(p["env_steps_per_s"] > 0 for p in pr)
    assert max(p["elapsed_s"] for p in pr) * 1e3 / 25 == pytest.approx(line["ms_per_step"], abs=2e-4)   # 4-decimal line
    whole = np.load(tmp_path / "one.rank0.npz")
    parts = [np.load(tmp_path / f"n.rank{r}.npz") for r in range(world)]
    for k in ("obs", "mask", "src", "raw", "done", "stats"):
        np.testing.assert_array_equal(whole[k], np.concatenate([p[k] for p in parts]), err_msg=k)


def test_bench_world_size_mismatch_fails():
    """A launcher that started a different number of ranks than --gpus is an error."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2"], env=env, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=1" in r.stderr
