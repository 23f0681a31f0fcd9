"""Parity at BASELINE.json's full sizes: the product path (MicroRTSGridModeVecEnv ->
libmicrorts_amd.so, device tensors as bench.py uses them) against the oracle
(oracle/libmrts_oracle.so, OpenMP over games) over every env of the configuration
the headline metric is quoted on and of configs[1] / configs[3] / 24x24.

Every step compares the whole (N, HW, 78) mask, source mask, (N, H, W, P) obs (float32 --
the bench's dtype -- bit for bit as 1.0f / +0.0f, unless a test says int32), the
raw (N, 6) rewards, the weighted reward and done, on the device.  Actions are the
Philox masked sampler's (oracle_py.sample_actions == mrts_sample_actions, pinned by
test_gpu_parity.py::test_device_sampler_matches_oracle_sampler).  Small `max_steps`
put the auto-reset of every game inside the window.
"""
import os

import numpy as np
import pytest

from conftest import MAPS, OBS_DTYPES, obs_bits_equal

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]   # per-test limits below override

W = np.array([10.0, 1.0, 1.0, 0.2, 1.0, 4.0])


def _full_rollout(map_path, nsp, nbot, bot, steps, max_steps, partial_obs=False, seed=2024, obs_dtype="float32"):
    import torch

    from gym_microrts import microrts_ai
    from gym_microrts.envs.vec_env import MicroRTSGridModeVecEnv
    from oracle_py import OracleVecEnv, sample_actions

    g = MicroRTSGridModeVecEnv(num_selfplay_envs=nsp, num_bot_envs=nbot, max_steps=max_steps, map_paths=[map_path],
                               ai2s=[getattr(microrts_ai, bot)] * nbot, partial_obs=partial_obs, reward_weight=W,
                               return_tensors=True, obs_dtype=getattr(torch, obs_dtype))
    o = OracleVecEnv(nsp, nbot, [os.path.join(MAPS, map_path)], max_steps=max_steps, ai2s=[bot] * nbot,
                     partial_obs=partial_obs, reward_weight=W)
    dev = g.device

    def same(gpu, host, what, s):
        assert torch.equal(gpu, torch.from_numpy(np.ascontiguousarray(host)).to(dev)), f"{what} differs at step {s}"

    assert obs_bits_equal(g.reset(), o.reset()), "reset obs differs"
    resets = 0
    for s in range(steps):
        if s % 500 == 0:
            print(f"{map_path} {nsp}+{nbot} {bot}: step {s} / {steps}", flush=True)
        mg, mo = g.get_action_mask(), o.get_action_mask()
        same(mg, mo, "mask", s)
        same(g.source_unit_mask, o.source_unit_mask, "source mask", s)
        a = sample_actions(mo, seed, s)
        og, rg, dg, ig = g.step(torch.from_numpy(a).to(dev))
        oo, ro, do, io = o.step(a)
        assert obs_bits_equal(og, oo), f"obs differs at step {s}"
        same(ig._raw, np.array([i["raw_rewards"] for i in io]), "raw rewards", s)
        assert np.allclose(rg.cpu().numpy(), ro, rtol=0, atol=1e-12), f"weighted reward differs at step {s}"
        same(dg, np.asarray(do, bool), "done", s)
        resets += int(np.asarray(do).sum())
    assert g.error_flags() == 0
    g.close()
    o.close()
    return resets


@pytest.mark.timeout(900)
def test_fullsize_selfplay_8192_basesWorkers16x16():
    """The headline configuration: 8192 selfplay envs (4096 games), 16x16 basesWorkers."""
    resets = _full_rollout("maps/16x16/basesWorkers16x16.xml", 8192, 0, "passiveAI", steps=120, max_steps=100)
    assert resets >= 8192   # every env passed through the time-limit reset


@pytest.mark.timeout(900)
def test_fullsize_coacai_1024():
    """configs[1]: 1024 envs vs device coacAI (MRTS_SOAK_TICKS: a longer soak run)."""
    _full_rollout("maps/16x16/basesWorkers16x16.xml", 0, 1024, "coacAI", steps=int(os.environ.get("MRTS_SOAK_TICKS", "500")),
                  max_steps=400)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("obs_dtype", OBS_DTYPES)
def test_fullsize_partial_obs_4096(obs_dtype):
    """configs[3]'s env: partial_obs (31 planes), 4096 envs (MRTS_SOAK_TICKS: a longer soak run).
    float32 is the dtype configs[3]'s PPO loop consumes (k_step<.., 31, float, ..>); int32 too."""
    _full_rollout("maps/16x16/basesWorkers16x16.xml", 4096, 0, "passiveAI", steps=int(os.environ.get("MRTS_SOAK_TICKS", "120")),
                  max_steps=100, partial_obs=True, obs_dtype=obs_dtype)


@pytest.mark.timeout(900)
def test_fullsize_24x24_4096():
    """configs[4]'s largest bucket map at 4096 envs, with workerRush bot envs."""
    _full_rollout("maps/24x24/basesWorkers24x24.xml", 2048, 2048, "workerRushAI", steps=100, max_steps=80)


@pytest.mark.timeout(1000)
def test_fullsize_2000_tick_episode_1024():
    """A whole 2000-tick episode (max_steps 2000) at 1024 envs vs the
    oracle, through the bench's staggered pre-roll: games 0..255 run from reset to
    the time-limit reset at tick 2000, games 256..511 are reset at staggered ticks
    (bench.stagger_plan) so every phase of an episode -- mid-game fights, gameovers,
    auto-resets at every tick -- is stepped too.  Rewards / dones every step, the
    whole obs / mask / source tensors every 10th step and at the end."""
    import sys

    import torch

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from gym_microrts.envs.vec_env import MicroRTSGridModeVecEnv
    from oracle_py import OracleVecEnv, sample_actions

    m = "maps/16x16/basesWorkers16x16.xml"
    g = MicroRTSGridModeVecEnv(num_selfplay_envs=1024, num_bot_envs=0, max_steps=2000, map_paths=[m], reward_weight=W,
                               return_tensors=True, obs_dtype=torch.int32)
    o = OracleVecEnv(1024, 0, [os.path.join(MAPS, m)], max_steps=2000, reward_weight=W)
    dev = g.device

    def same(gpu, host, what, s):
        assert torch.equal(gpu, torch.from_numpy(np.ascontiguousarray(host)).to(dev)), f"{what} differs at step {s}"

    same(g.reset(), o.reset(), "reset obs", -1)
    plan = bench.stagger_plan(256, 1000)
    ends = 0
    for s in range(2100):
        mo = o.get_action_mask()
        a = sample_actions(mo, 31, s)
        og, rg, dg, ig = g.step(torch.from_numpy(a).to(dev))
        oo, ro, do, io = o.step(a)
        same(ig._raw, np.array([i["raw_rewards"] for i in io]), "raw rewards", s)
        same(dg, np.asarray(do, bool), "done", s)
        ends += int(np.asarray(do).sum())
        if s < 1000 and plan[s]:
            games = [256 + k for k in plan[s]]
            g.reset_games(games)
            for k in games:
                o.reset_game(k, 0)
            oo = o.encode(o.raw_obs())
        if s % 10 == 0 or s == 2099:
            same(og, oo, "obs", s)
            same(g.get_action_mask(), o.get_action_mask(), "mask", s)
            same(g.source_unit_mask, o.source_unit_mask, "source", s)
    st = g.game_stats()
    assert (st[:256, 5] >= 1).all()            # every unstaggered game finished an episode
    assert ends >= 512                         # games 0..255 (both views) reset at tick 2000
    assert g.error_flags() == 0


@pytest.mark.timeout(1200)
@pytest.mark.parametrize("obs_dtype", OBS_DTYPES)
def test_fullsize_headline_8192_staggered_2000_ticks(obs_dtype):
    """The headline configuration itself (8192 selfplay envs, 16x16 basesWorkers,
    max_steps 2000) through the bench's own loop for 2100 ticks: the device sampler
    (mrts_sample_actions_src, Philox) on the GPU and the oracle's identical C sampler
    (ovec_bench_steps) on the host, every game reset at its staggered pre-roll tick
    (bench.stagger_plan) -- so over the run every game goes through a whole 2000-tick
    episode and the window after tick 2000 holds games at every phase, as in the
    timed bench window.  Raw rewards and dones are compared every tick; the whole
    obs, mask and source tensors every 50 ticks and at the end.
    float32 obs is the bench's own kernel, k_step<256, 29, float, false> (VERDICT r5
    item 1): its obs are compared bit for bit with the oracle's one-hot as 1.0f / +0.0f.
    The int32 arm runs the same engine with int32 stores, for 300 ticks."""
    import sys

    import torch

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from gym_microrts import _native
    from gym_microrts.envs.vec_env import MicroRTSGridModeVecEnv
    from oracle_py import OracleVecEnv

    n, m, seed = 8192, "maps/16x16/basesWorkers16x16.xml", 1
    g = MicroRTSGridModeVecEnv(num_selfplay_envs=n, num_bot_envs=0, max_steps=2000, map_paths=[m], reward_weight=W,
                               return_tensors=True, obs_dtype=getattr(torch, obs_dtype))
    o = OracleVecEnv(n, 0, [os.path.join(MAPS, m)], max_steps=2000, reward_weight=W)
    dev, hw, lib = g.device, 256, _native.lib()
    act = torch.empty((n, hw, 7), dtype=torch.int64, device=dev)

    def same(gpu, host, what, s):
        assert torch.equal(gpu, torch.from_numpy(np.ascontiguousarray(host)).to(dev)), f"{what} differs at tick {s}"

    assert obs_bits_equal(g.reset(), o.reset()), "reset obs differs"
    plan = bench.stagger_plan(n // 2, 2000)
    ends = 0
    full = obs_dtype == "float32"
    ticks = int(os.environ.get("MRTS_SOAK_TICKS", "2100" if full else "300"))   # a soak run: more episodes back to back
    for s in range(ticks):
        if s % 500 == 0:
            print(f"headline lock-step: tick {s} / {ticks}", flush=True)
        g.get_action_mask()
        _native.check(bench.sample(lib, "src", g._mask, g._src, n, hw, 0, seed, s, act), None, "sample")
        og, _, dg, ig = g.step(act)
        _, ro, do = o.bench_steps(1, seed, s)
        same(ig._raw, ro, "raw rewards", s)
        same(g._done, do.astype(np.uint8), "dones", s)
        ends += int(do[:, 0].sum())
        if s < 2000 and plan[s]:
            g.reset_games(plan[s])
            for k in plan[s]:
                o.reset_game(k, 0)
        if s % 50 == 0 or s == ticks - 1:
            assert obs_bits_equal(og, o.encode(o.raw_obs())), f"obs differs at tick {s}"
            full = o.get_action_mask_full()
            same(g.get_action_mask(), full[:, :, 1:], "mask", s)
            same(g.source_unit_mask, full[:, :, 0], "source", s)
            del full
    st = g.game_stats()
    if ticks >= 2100:
        # games 0..204 restarted at pre-roll ticks <= 99 (floor(g * 2000 / 4096)): each then played a whole
        # 2000-tick episode to its time limit within the run (or ended earlier by gameover)
        assert (st[:205, 5] >= 1).all()
        assert ends >= 2 * 205
    assert g.error_flags() == 0
    g.close()
    o.close()


@pytest.mark.timeout(1200)
@pytest.mark.parametrize("obs_dtype", OBS_DTYPES)
def test_fullsize_mixed_buckets_bench_split_8192(obs_dtype):
    """configs[4] at the bench's own size and launch plan: bench.py's
    mixed workload exactly -- 8192 envs split 2048 / 4096 / 2048 over 8x8 / 16x16 /
    24x24 basesWorkers (bench.MIXED), each bucket half selfplay, a quarter vs device
    workerRushAI, a quarter vs device coacAI -- stepped by one mrts_step_group call with
    the default merge-fit | bots-first policy (8x8 and 16x16 share one 256-lane launch
    with a segment table, 24x24 keeps its own), the device Philox sampler on every
    bucket's eager masks in one grouped launch (as the bench samples), and bench.preroll's
    staggered restarts over the first 100 ticks.
    max_steps 100 over 210 ticks, so every game also reaches its time-limit auto-reset.  One oracle per
    bucket (ovec_bench_steps: the oracle's identical C sampler + step): raw rewards and
    dones every tick, the whole obs / mask / source tensors every 10 ticks.  float32 obs are
    the bench's (bit-compared as 1.0f / +0.0f); the int32 arm runs 110 ticks."""
    import sys

    import torch

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from gym_microrts import _native, microrts_ai
    from gym_microrts.envs.vec_env import MicroRTSMixedMapVecEnv
    from oracle_py import OracleVecEnv

    n, seed, max_steps = 8192, 5, 100
    ticks = int(os.environ.get("MRTS_SOAK_TICKS", "210" if obs_dtype == "float32" else "110"))   # soak: more episodes
    buckets, spec = [], []
    for m, frac in bench.MIXED:
        nb = int(n * frac) // 4 * 4
        ais = ["workerRushAI"] * (nb // 4) + ["coacAI"] * (nb // 4)
        buckets.append(dict(map_paths=[m], num_selfplay_envs=nb // 2, num_bot_envs=len(ais),
                            ai2s=[getattr(microrts_ai, a) for a in ais]))
        spec.append((m, nb // 2, ais))
    assert [b["num_selfplay_envs"] + b["num_bot_envs"] for b in buckets] == [2048, 4096, 2048]
    env = MicroRTSMixedMapVecEnv(buckets, max_steps=max_steps, return_tensors=True, reward_weight=W,
                                 obs_dtype=getattr(torch, obs_dtype))
    assert env.grouped and env.launch_plan() == ([0, 0, 1], 2)
    orc = [OracleVecEnv(nsp, len(ais), [os.path.join(MAPS, m)], max_steps=max_steps, ai2s=ais, reward_weight=W)
           for m, nsp, ais in spec]
    lib = _native.lib()
    dev = env.envs[0].device
    acts = [torch.empty((e.num_envs, e.height * e.width, 7), dtype=torch.int64, device=dev) for e in env.envs]

    def same(gpu, host, what, k, s):
        assert torch.equal(gpu, torch.from_numpy(np.ascontiguousarray(host)).to(dev)), f"bucket {k}: {what} differs at tick {s}"

    for k, (og, o) in enumerate(zip(env.reset(), orc)):
        assert obs_bits_equal(og, o.reset()), f"bucket {k}: reset obs differs"
    plans = [bench.stagger_plan(e._n_games(), max_steps) for e in env.envs]
    ends = np.zeros(3, int)
    for s in range(ticks):
        if s % 500 == 0:
            print(f"configs[4] lock-step: tick {s} / {ticks}", flush=True)
        masks = env.get_action_mask()
        # the bench's stand-in policy: every bucket in one mrts_sample_actions_src_group launch
        segs = (_native.SampleSeg * 3)(*[_native.SampleSeg(mk.data_ptr(), e.source_unit_mask.data_ptr(), e.num_envs,
                                                           e.height * e.width, 0, a.data_ptr())
                                         for e, mk, a in zip(env.envs, masks, acts)])
        _native.check(lib.mrts_sample_actions_src_group(torch.cuda.current_stream().cuda_stream, segs, 3, seed, s), None,
                      "sample_group")
        obs, rew, done, infos = env.step(acts)
        for k, (e, o) in enumerate(zip(env.envs, orc)):
            _, ro, do = o.bench_steps(1, seed, s)
            same(infos[k]._raw, ro, "raw rewards", k, s)
            same(e._done, do.astype(np.uint8), "dones", k, s)
            assert np.allclose(rew[k].cpu().numpy(), ro @ W, rtol=0, atol=1e-12), f"bucket {k}: reward at tick {s}"
            ends[k] += int(do[:, 0].sum())
        if s < max_steps:   # bench.preroll's staggered restarts
            for e, o, plan in zip(env.envs, orc, plans):
                e.reset_games(plan[s])
                for g in plan[s]:
                    o.reset_game(g, 0)
        if s % 10 == 0 or s == ticks - 1:
            for k, (e, o) in enumerate(zip(env.envs, orc)):
                assert obs_bits_equal(obs[k], o.encode(o.raw_obs())), f"bucket {k}: obs differs at tick {s}"
                full = o.get_action_mask_full()
                same(e.get_action_mask(), full[:, :, 1:], "mask", k, s)
                same(e.source_unit_mask, full[:, :, 0], "source", k, s)
                del full
    for k, e in enumerate(env.envs):
        st = e.game_stats()
        if ticks >= 210:
            assert (st[:, 5] >= 1).all(), f"bucket {k}: a game never finished an episode in the window"
            assert ends[k] >= e.num_envs
    assert env.error_flags() == 0
    env.close()
    for o in orc:
        o.close()
