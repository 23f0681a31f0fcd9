"""Env-state checkpoint (SURVEY.md §5 "env-state checkpoint"; no reference
counterpart): get_state() after a stretch of play, more steps, set_state(), and the
same actions again must repeat the first continuation bit for bit -- obs, masks,
sources, raw rewards and dones every step -- with device bots deciding (fused and
not), partial observability, time-limit resets inside the replayed stretch, and map
cycling.  A snapshot of another configuration is refused."""
import ctypes
import os

import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]   # per-test limits below override
W = np.array([10.0, 1.0, 1.0, 0.2, 1.0, 4.0])


def _env(partial_obs=False, bot_fusion=True, cycle=False, n=32, bots=None, map_path="maps/16x16/basesWorkers16x16.xml",
         max_steps=60):
    import torch

    from gym_microrts import microrts_ai
    from gym_microrts.envs.vec_env import MicroRTSGridModeVecEnv

    bots = bots or [microrts_ai.coacAI, microrts_ai.workerRushAI, microrts_ai.randomBiasedAI, microrts_ai.lightRushAI] * (n // 8)
    kw = dict(cycle_maps=["maps/16x16/basesWorkers16x16.xml", "maps/16x16/basesWorkers16x16A.xml"]) if cycle else {}
    return MicroRTSGridModeVecEnv(num_selfplay_envs=n // 2, num_bot_envs=len(bots), max_steps=max_steps, ai2s=bots,
                                  map_paths=[map_path], partial_obs=partial_obs, reward_weight=W,
                                  return_tensors=True, obs_dtype=torch.int32, bot_fusion=bot_fusion, **kw)


def _run(env, s0, steps, act):
    import torch

    from gym_microrts import _native

    lib, out = _native.lib(), []
    hw = env.height * env.width
    for s in range(s0, s0 + steps):
        m = env.get_action_mask()
        _native.check(lib.mrts_sample_actions_src(torch.cuda.current_stream().cuda_stream, m.data_ptr(), env._src.data_ptr(),
                                                  env.num_envs, hw, 0, ctypes.c_uint64(5), s, act.data_ptr()))
        o, r, d, i = env.step(act)
        out.append((m.clone(), env._src.clone(), o.clone(), i._raw.clone(), d.clone()))
    return out


@pytest.mark.parametrize("partial_obs,bot_fusion,cycle", [(False, True, False), (False, False, False), (True, True, False),
                                                           (False, True, True)])
def test_checkpoint_replays_bit_for_bit(partial_obs, bot_fusion, cycle):
    import torch

    env = _env(partial_obs, bot_fusion, cycle)
    env.reset()
    act = torch.empty((env.num_envs, env.height * env.width, 7), dtype=torch.int64, device=env.device)
    first = _run(env, 0, 45, act)
    obs_at = first[-1][2].clone()
    state = env.get_state()
    a = _run(env, 45, 80, act)   # crosses the 60-step time limit: every game auto-resets inside
    obs_back = env.set_state(state)
    assert torch.equal(obs_back, obs_at)
    b = _run(env, 45, 80, act)
    for s, (x, y) in enumerate(zip(a, b)):
        for k in range(5):
            assert torch.equal(x[k], y[k]), f"step {45 + s} output {k}"
    assert sum(int(x[4].sum()) for x in a) > 0
    assert env.error_flags() == 0
    env.close()


def test_checkpoint_of_another_config_refused():
    import torch

    from gym_microrts import _native

    env, other = _env(n=32), _env(n=16)
    env.reset()
    other.reset()
    big, small = env.get_state(), other.get_state()
    with pytest.raises(ValueError, match="another configuration"):
        other.set_state(big)
    with pytest.raises(ValueError):
        env.set_state(object())
    # below the Python check: the C ABI reads only the fixed header of a foreign snapshot
    # (a smaller handle's snapshot is shorter than this handle's header) and refuses it
    lib, st = _native.lib(), torch.cuda.current_stream().cuda_stream
    for h, snap, obs in ((env._h, small, env._obs), (other._h, big, other._obs)):
        assert lib.mrts_load_state(h, st, snap.tensor.data_ptr(), obs.data_ptr()) == -1   # MRTS_EINVAL
    env.close()
    other.close()


@pytest.mark.parametrize("what", ["bots", "map", "partial_obs", "max_steps"])
def test_checkpoint_same_shape_other_config_refused(what):
    """a snapshot of a handle with the same shape (games, cells, map count,
    workspace size) but other bots, another map or another obs layout would copy that
    handle's device tables in; the header's configuration fingerprint refuses it.
    ADVICE r5: another time limit too (the continuation would differ from the saved run)."""
    from gym_microrts import _native, microrts_ai

    env = _env(n=32)
    if what == "bots":
        other = _env(n=32, bots=[microrts_ai.workerRushAI] * 16)
    elif what == "map":
        other = _env(n=32, map_path="maps/16x16/basesWorkers16x16B.xml")   # (16x16A is byte-identical to 16x16)
    elif what == "max_steps":
        other = _env(n=32, max_steps=61)
    else:
        other = _env(n=32, partial_obs=True)
    env.reset()
    other.reset()
    snap = env.get_state()
    if snap.tensor.numel() == int(_native.lib().mrts_state_bytes(other._h)):
        with pytest.raises(_native.MicroRTSError, match="another configuration"):
            other.set_state(snap)
    else:
        with pytest.raises(ValueError, match="another configuration"):
            other.set_state(snap)
    env.set_state(snap)   # its own snapshot still loads
    env.close()
    other.close()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("seed", range(int(os.environ.get("MRTS_FUZZ_FIRST", "0")),
                                       int(os.environ.get("MRTS_FUZZ_FIRST", "0")) + max(1, int(os.environ.get("MRTS_FUZZ_SEEDS", "12")) // 3)))
def test_fuzz_checkpoint_replays_bit_for_bit(tmp_path, seed):
    """Random maps (tests/random_maps.py, 4..32 x 4..32, walls), random device bots
    (randomBiasedAI's tick-keyed stream included), selfplay, fog, map cycling over two random
    maps of one size, short time limits: the snapshot taken at a random tick replays a random
    continuation bit for bit (MRTS_FUZZ_SEEDS // 3 cases); odd seeds on float32 obs (the bench's
    dtype), even seeds on int32."""
    import torch

    from gym_microrts import microrts_ai
    from gym_microrts.envs.vec_env import MicroRTSGridModeVecEnv
    from random_maps import write_random_map
    from test_gpu_bots import BOTS

    rng = np.random.default_rng(7000 + seed)
    w, h = int(rng.integers(4, 33)), int(rng.integers(4, 33))
    maps = [write_random_map(str(tmp_path / f"k{seed}_{j}.xml"), w, h, seed * 10 + j,
                             n_units=min(int(rng.integers(4, max(5, min(120, int(w * h * 0.5))))), w * h - 4),
                             wall_frac=float(rng.uniform(0, 0.2))) for j in range(2)]
    bots = [str(b) for b in rng.choice(BOTS + ["passiveAI"], size=int(rng.integers(0, 9)))]
    nsp = 2 * int(rng.integers(0 if bots else 1, 5))
    kw = dict(cycle_maps=maps) if rng.integers(0, 2) else {}
    env = MicroRTSGridModeVecEnv(num_selfplay_envs=nsp, num_bot_envs=len(bots), max_steps=int(rng.integers(20, 80)),
                                 ai2s=[getattr(microrts_ai, b) for b in bots], map_paths=[maps[0]],
                                 partial_obs=bool(rng.integers(0, 2)), reward_weight=W, return_tensors=True,
                                 obs_dtype=torch.float32 if seed % 2 else torch.int32, bot_fusion=bool(rng.integers(0, 4)), **kw)
    env.reset()
    act = torch.empty((env.num_envs, env.height * env.width, 7), dtype=torch.int64, device=env.device)
    t0, t1 = int(rng.integers(0, 120)), int(rng.integers(1, 120))
    first = _run(env, 0, t0, act)
    state = env.get_state()
    a = _run(env, t0, t1, act)
    obs_back = env.set_state(state)
    if first:
        assert torch.equal(obs_back, first[-1][2])
    b = _run(env, t0, t1, act)
    for s, (x, y) in enumerate(zip(a, b)):
        for k in range(5):
            assert torch.equal(x[k], y[k]), f"step {t0 + s} output {k}"
    assert env.error_flags() == 0
    env.close()


def _run_multi(env, s0, steps, acts):
    """_run for the per-bucket / per-size envs: device sampler on every engine, outputs cloned."""
    import torch

    from gym_microrts import _native

    lib, out = _native.lib(), []
    for s in range(s0, s0 + steps):
        ms = env.get_action_mask()
        for e, m, a in zip(env.envs, ms, acts):
            _native.check(lib.mrts_sample_actions_src(torch.cuda.current_stream().cuda_stream, m.data_ptr(), e._src.data_ptr(),
                                                      e.num_envs, e.height * e.width, 0, ctypes.c_uint64(9), s, a.data_ptr()))
        o, r, d, i = env.step(acts)
        rec = [x.clone() for x in ms] + [e._src.clone() for e in env.envs] + [x.clone() for x in o]
        if isinstance(r, list):
            rec += [x.clone() for x in r] + [x.clone() for x in d]
        else:
            rec += [r.clone(), d.clone(), torch.as_tensor(env.bucket.copy())]
        out.append(rec)
    return out


def _replay_check(env, first_obs_fn, t0, t1):
    import torch

    acts = [torch.empty((e.num_envs, e.height * e.width, 7), dtype=torch.int64, device=e.device) for e in env.envs]
    _run_multi(env, 0, t0, acts)
    at = [x.clone() for x in first_obs_fn()]
    state = env.get_state()
    a = _run_multi(env, t0, t1, acts)
    back = env.set_state(state)
    for x, y in zip(back, at):
        assert torch.equal(x, y)
    b = _run_multi(env, t0, t1, acts)
    for s, (x, y) in enumerate(zip(a, b)):
        for k, (u, v) in enumerate(zip(x, y)):
            assert torch.equal(u, v), f"step {t0 + s} output {k}"
    assert env.error_flags() == 0
    return a


def test_checkpoint_mixed_map_buckets_replays():
    """MicroRTSMixedMapVecEnv.get_state / set_state (configs[4]'s env: 8x8 / 16x16 / 24x24
    buckets with device bots, stepped by the grouped launch): the continuation replays bit
    for bit."""
    import torch

    from gym_microrts import microrts_ai
    from gym_microrts.envs.vec_env import MicroRTSMixedMapVecEnv

    bk = [dict(map_paths=["maps/8x8/basesWorkers8x8.xml"], num_selfplay_envs=8, ai2s=[microrts_ai.workerRushAI] * 4),
          dict(map_paths=["maps/16x16/basesWorkers16x16.xml"], num_selfplay_envs=8,
               ai2s=[microrts_ai.coacAI, microrts_ai.randomBiasedAI] * 3),
          dict(map_paths=["maps/24x24/basesWorkers24x24.xml"], num_selfplay_envs=4, ai2s=[microrts_ai.lightRushAI] * 2)]
    env = MicroRTSMixedMapVecEnv(bk, max_steps=70, reward_weight=W, return_tensors=True, obs_dtype=torch.int32)
    assert env.grouped
    env.reset()
    a = _replay_check(env, lambda: [e._obs for e in env.envs], 40, 60)
    assert sum(int(x[-1].sum()) for x in a) > 0   # games end inside the replayed stretch
    env.close()


def test_checkpoint_size_cycling_replays():
    """MicroRTSSizeCyclingVecEnv.get_state / set_state: every size engine's games, played and
    parked, the env -> size map and the cycle position come back; the continuation (games
    moving between sizes inside it) replays bit for bit and parked rows stay zero."""
    import torch

    from gym_microrts import microrts_ai
    from gym_microrts.envs.vec_env import MicroRTSSizeCyclingVecEnv

    cyc = ["maps/8x8/basesWorkers8x8.xml", "maps/16x16/basesWorkers16x16A.xml", "maps/10x10/basesTwoWorkers10x10.xml",
           "maps/24x24/basesWorkers24x24.xml", "maps/16x16/basesWorkers16x16C.xml"]
    init = ["maps/16x16/basesWorkers16x16.xml"] * 4 + ["maps/8x8/basesWorkers8x8.xml"] * 2 + \
           ["maps/10x10/basesTwoWorkers10x10.xml", "maps/16x16/basesWorkers16x16.xml", "maps/8x8/basesWorkers8x8.xml"]
    env = MicroRTSSizeCyclingVecEnv(6, 3, ai2s=[microrts_ai.coacAI, microrts_ai.workerRushAI, microrts_ai.passiveAI],
                                    map_paths=init, cycle_maps=cyc, max_steps=25, reward_weight=W, obs_dtype=torch.int32)
    obs = env.reset()
    moved = env.bucket.copy()
    a = _replay_check(env, lambda: env_obs(env), 30, 70)
    assert (np.stack([x[-1].numpy() for x in a]) != moved).any()   # envs changed size inside the replay
    for rec in a:
        bucket = rec[-1].numpy()
        for i, o in enumerate(rec[2 * len(env.envs):3 * len(env.envs)]):
            assert not o[torch.from_numpy(bucket != i).to(o.device)].any()
    env.close()


def env_obs(env):
    return [e._obs for e in env.envs]


def test_checkpoint_mixed_map_refuses_before_overwriting():
    """A bucket list in the wrong order (or of the wrong length) is refused before any bucket
    is overwritten: the env keeps stepping as if set_state had not been called."""
    import torch

    from gym_microrts.envs.vec_env import MicroRTSMixedMapVecEnv

    bk = [dict(map_paths=["maps/8x8/basesWorkers8x8.xml"], num_selfplay_envs=4),
          dict(map_paths=["maps/16x16/basesWorkers16x16.xml"], num_selfplay_envs=4)]
    env = MicroRTSMixedMapVecEnv(bk, max_steps=70, reward_weight=W, return_tensors=True, obs_dtype=torch.int32)
    env.reset()
    acts = [torch.empty((e.num_envs, e.height * e.width, 7), dtype=torch.int64, device=e.device) for e in env.envs]
    _run_multi(env, 0, 10, acts)
    st = env.get_state()
    a = _run_multi(env, 10, 5, acts)
    env.set_state(st)
    with pytest.raises(ValueError):
        env.set_state(st[::-1])
    with pytest.raises(ValueError):
        env.set_state(st[:1])
    b = _run_multi(env, 10, 5, acts)
    for x, y in zip(a, b):
        for u, v in zip(x, y):
            assert torch.equal(u, v)
    env.close()


def test_checkpoint_mixed_map_rolls_back_on_refusal():
    """Snapshots of a same-shape mixed env whose second bucket plays other bots: the first
    bucket's snapshot fits and loads, the second is refused by the engine's configuration
    fingerprint, and the first bucket is rolled back -- the env continues as if set_state had
    not been called."""
    import torch

    from gym_microrts import _native, microrts_ai
    from gym_microrts.envs.vec_env import MicroRTSMixedMapVecEnv

    def make(bot):
        bk = [dict(map_paths=["maps/8x8/basesWorkers8x8.xml"], num_selfplay_envs=4),
              dict(map_paths=["maps/16x16/basesWorkers16x16.xml"], num_selfplay_envs=2, ai2s=[bot] * 2)]
        return MicroRTSMixedMapVecEnv(bk, max_steps=70, reward_weight=W, return_tensors=True, obs_dtype=torch.int32)

    env, other = make(microrts_ai.workerRushAI), make(microrts_ai.lightRushAI)
    for e in (env, other):
        e.reset()
    for e, o in zip(env.envs, other.envs):   # same shapes: only the engine's fingerprint tells them apart
        assert int(_native.lib().mrts_state_bytes(e._h)) == int(_native.lib().mrts_state_bytes(o._h))
    acts = [torch.empty((e.num_envs, e.height * e.width, 7), dtype=torch.int64, device=e.device) for e in env.envs]
    _run_multi(other, 0, 7, acts)
    foreign = other.get_state()
    _run_multi(env, 0, 10, acts)
    st = env.get_state()
    a = _run_multi(env, 10, 5, acts)
    env.set_state(st)
    with pytest.raises(_native.MicroRTSError):
        env.set_state(foreign)
    b = _run_multi(env, 10, 5, acts)
    for x, y in zip(a, b):
        for u, v in zip(x, y):
            assert torch.equal(u, v)
    env.close()
    other.close()
