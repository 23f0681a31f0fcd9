"""HIP engine (libmicrorts_amd.so) == oracle, bit for bit.

Every test drives the product path (gym_microrts.envs.vec_env ->
libmicrorts_amd.so kernels) and checks it against the CPU restatement on the
same seeded inputs: the reference's known-answer tests, long random masked
rollouts, adversarial (unmasked) action streams that exercise the illegal /
conflict / inconsistent-issue paths, auto-reset and map cycling, and the
device sampler's Philox stream.
"""
import os

import numpy as np
import pytest

import kat
from conftest import MAPS, obs_bits_equal

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]   # per-test limits below override


def _torch():
    import torch

    return torch


def make_gpu_env(num_selfplay_envs, num_bot_envs, map_path, max_steps, reward_weight=None, **kw):
    from gym_microrts import microrts_ai
    from gym_microrts.envs.vec_env import MicroRTSGridModeVecEnv

    return MicroRTSGridModeVecEnv(
        num_selfplay_envs=num_selfplay_envs,
        num_bot_envs=num_bot_envs,
        max_steps=max_steps,
        ai2s=[microrts_ai.passiveAI for _ in range(num_bot_envs)],
        map_paths=[map_path],
        reward_weight=reward_weight if reward_weight is not None else np.array([10.0, 1.0, 1.0, 0.2, 1.0, 4.0]),
        **kw,
    )


def make_oracle(num_selfplay_envs, num_bot_envs, map_path, max_steps, maps=None, game_maps=None, partial_obs=False):
    from oracle_py import OracleVecEnv

    paths = maps or [os.path.join(MAPS, map_path)]
    return OracleVecEnv(num_selfplay_envs, num_bot_envs, paths, max_steps=max_steps, ai2s=["passiveAI"] * num_bot_envs,
                        game_maps=game_maps, partial_obs=partial_obs)


def test_native_library_is_the_engine():
    from gym_microrts import _native

    assert os.path.basename(_native.LIB_PATH) == "libmicrorts_amd.so"
    assert _native.lib().mrts_version().startswith(b"microrts_amd")


def test_kat_observation():
    kat.check_observation(make_gpu_env)


def test_kat_mask():
    kat.check_mask(make_gpu_env)


def test_kat_reward():
    kat.check_rewards(make_gpu_env)


def _rollout(map_path, nsp, nbot, max_steps, steps, seed, mode="masked", return_tensors=False, partial_obs=False,
             eager_masks=True, obs_dtype="int32"):
    """Lock-step GPU vs oracle rollout; compares masks, obs, rewards, dones.  With
    return_tensors, `obs_dtype` picks the device obs (float32 obs are bit-compared:
    1.0f / +0.0f against the oracle's one-hot)."""
    from oracle_py import sample_actions

    torch = _torch()
    g = make_gpu_env(nsp, nbot, map_path, max_steps, return_tensors=return_tensors,
                     obs_dtype=getattr(torch, obs_dtype) if return_tensors else None, partial_obs=partial_obs,
                     eager_masks=eager_masks)
    o = make_oracle(nsp, nbot, map_path, max_steps, partial_obs=partial_obs)
    if return_tensors:
        assert obs_bits_equal(g.reset(), o.reset()), "reset obs"
    else:
        np.testing.assert_array_equal(g.reset(), o.reset())
    rng = np.random.default_rng(seed)
    n, hw = g.num_envs, g.height * g.width
    nvec = np.array([6, 4, 4, 4, 4, 7, 49])
    episodes = 0
    for s in range(steps):
        mg = g.get_action_mask()
        mg = np.asarray(mg.cpu() if return_tensors else mg)
        mo = o.get_action_mask()
        np.testing.assert_array_equal(mg, mo, err_msg=f"mask step {s}")
        if mode == "masked":
            a = sample_actions(mo, seed, s)
        elif mode == "uniform":   # ignores the mask: illegal actions, conflicts, bad rows
            a = (rng.random((n, hw, 7)) * nvec).astype(np.int64)
        else:                     # mix per cell
            a = sample_actions(mo, seed, s)
            u = (rng.random((n, hw, 7)) * nvec).astype(np.int64)
            pick = rng.random((n, hw, 1)) < 0.3
            a = np.where(pick, u, a)
        obs_g, rew_g, done_g, info_g = g.step(torch.from_numpy(a).to(g.device) if return_tensors else a)
        obs_o, rew_o, done_o, info_o = o.step(a)
        if return_tensors:
            assert obs_bits_equal(obs_g, obs_o), f"obs step {s}"
            rew_g, done_g = rew_g.cpu().numpy(), done_g.cpu().numpy()
        else:
            np.testing.assert_array_equal(obs_g, obs_o, err_msg=f"obs step {s}")
        np.testing.assert_array_equal(np.array([i["raw_rewards"] for i in info_g]), np.array([i["raw_rewards"] for i in info_o]),
                                      err_msg=f"raw rewards step {s}")
        if return_tensors:
            # fused in-kernel dot: sequential k = 0..5, round-to-nearest, no FMA
            raw_o = np.array([i["raw_rewards"] for i in info_o])
            seq = np.zeros(n)
            for k in range(6):
                seq = seq + raw_o[:, k] * g.reward_weight[k]
            np.testing.assert_array_equal(rew_g, seq, err_msg=f"weighted reward step {s}")
            np.testing.assert_allclose(rew_g, rew_o, rtol=0, atol=1e-12)   # vs numpy `raw @ w`
        else:
            np.testing.assert_array_equal(rew_g, rew_o, err_msg=f"weighted reward step {s}")
        np.testing.assert_array_equal(done_g, done_o, err_msg=f"done step {s}")
        episodes += int(np.asarray(done_o).sum())
    assert g.error_flags() == 0
    return episodes


@pytest.mark.parametrize("map_path,nsp,nbot,max_steps,steps", [
    ("maps/16x16/basesWorkers16x16.xml", 64, 0, 400, 900),
    ("maps/8x8/basesWorkers8x8.xml", 32, 16, 250, 800),
    ("maps/10x10/basesTwoWorkers10x10.xml", 16, 8, 300, 700),
    ("maps/24x24/basesWorkers24x24.xml", 8, 4, 300, 400),
    ("maps/barricades24x24.xml", 8, 0, 200, 300),
    ("maps/4x4/baseTwoWorkers4x4.xml", 32, 32, 150, 500),
])
def test_masked_rollout_bit_exact(map_path, nsp, nbot, max_steps, steps):
    eps = _rollout(map_path, nsp, nbot, max_steps, steps, seed=11)
    assert eps > 0


@pytest.mark.parametrize("mode", ["uniform", "mixed"])
@pytest.mark.parametrize("map_path", ["maps/16x16/basesWorkers16x16.xml", "maps/4x4/baseTwoWorkers4x4.xml"])
def test_adversarial_rollout_bit_exact(map_path, mode):
    _rollout(map_path, 32, 16, 300, 400, seed=5, mode=mode)


@pytest.mark.parametrize("map_path,nsp,nbot", [
    ("maps/16x16/basesWorkers16x16.xml", 32, 8),
    ("maps/8x8/basesWorkers8x8.xml", 32, 8),
    ("maps/24x24/basesWorkers24x24.xml", 8, 4),
    ("maps/4x4/baseTwoWorkers4x4.xml", 16, 16),
])
def test_partial_obs_rollout_bit_exact(map_path, nsp, nbot):
    """partial_obs=True (31 planes, PartiallyObservableGameState)."""
    _rollout(map_path, nsp, nbot, 250, 500, seed=17, partial_obs=True)


def test_partial_obs_tensor_path():
    _rollout("maps/16x16/basesWorkers16x16.xml", 16, 0, 300, 200, seed=4, return_tensors=True, partial_obs=True)


def test_tensor_path_bit_exact():
    _rollout("maps/16x16/basesWorkers16x16.xml", 32, 0, 300, 300, seed=3, return_tensors=True)


@pytest.mark.parametrize("partial_obs", [False, True])
@pytest.mark.parametrize("map_path,nsp,nbot", [
    ("maps/16x16/basesWorkers16x16.xml", 32, 8),        # HW * P % 4 == 0: the 16-byte store path
    ("maps/4x4/baseTwoWorkers4x4.xml", 16, 16),         # the smallest map (16-byte path)
    ("maps/9x13/basesWorkersWalls9x13.xml", 16, 8),     # 117 * P odd: the unaligned per-element fallback
    ("maps/15x15/basesWorkersWalls15x15.xml", 8, 4),    # 225 * P odd, walls
])
def test_float32_obs_rollout_bit_exact(map_path, nsp, nbot, partial_obs):
    """The bench's obs dtype over a whole rollout: float32 obs
    from k_step<.., P, float, ..> -- the 16-byte stream_obs path and the unaligned
    fallback's cast (mrts_engine.hip stream_obs) -- bit-compared with the oracle's
    one-hot as 1.0f / +0.0f every step, with bot envs, auto-resets and fog."""
    _rollout(map_path, nsp, nbot, 150, 400, seed=21, return_tensors=True, partial_obs=partial_obs, obs_dtype="float32")


@pytest.mark.parametrize("partial_obs", [False, True])
def test_standalone_mask_kernel_rollout(partial_obs):
    """eager_masks=False: every get_action_mask() launches k_masks (the masks
    are not written by the step kernel)."""
    _rollout("maps/16x16/basesWorkers16x16.xml", 16, 8, 200, 300, seed=8, partial_obs=partial_obs, eager_masks=False)


@pytest.mark.parametrize("map_path", ["maps/16x16/basesWorkers16x16.xml", "maps/24x24/basesWorkers24x24.xml",
                                      "maps/4x4/baseTwoWorkers4x4.xml"])
def test_eager_masks_equal_mask_kernel(map_path):
    """The masks k_step / k_reset write for the next tick are the bytes k_masks
    writes for the same state (mask and source channel), every step."""
    import ctypes

    from gym_microrts import _native

    torch = _torch()
    g = make_gpu_env(16, 8, map_path, 150, return_tensors=True)
    g.reset()
    hw = g.height * g.width
    m2 = torch.full((g.num_envs, hw, 78), -1, dtype=torch.int32, device=g.device)
    s2 = torch.full((g.num_envs, hw), -1, dtype=torch.int32, device=g.device)
    act = torch.empty((g.num_envs, hw, 7), dtype=torch.int64, device=g.device)
    st = torch.cuda.current_stream().cuda_stream
    for s in range(300):
        m = g.get_action_mask()
        _native.check(_native.lib().mrts_get_masks(g._h, st, m2.data_ptr(), s2.data_ptr()), g._h, "get_masks")
        assert torch.equal(m, m2), f"mask step {s}"
        assert torch.equal(g.source_unit_mask, s2), f"source step {s}"
        _native.check(_native.lib().mrts_sample_actions(st, m.data_ptr(), g.num_envs, hw, 0, ctypes.c_uint64(5), s, act.data_ptr()))
        g.step(act)
    assert g.error_flags() == 0


def test_source_guided_sampler_equals_dense_sampler():
    """mrts_sample_actions_src reads only the mask rows of source cells; the
    output is the dense sampler's (and the oracle's) bit for bit."""
    import ctypes

    from gym_microrts import _native
    from oracle_py import sample_actions

    torch = _torch()
    g = make_gpu_env(256, 0, "maps/16x16/basesWorkers16x16.xml", 2000, return_tensors=True)
    g.reset()
    st = torch.cuda.current_stream().cuda_stream
    a1 = torch.empty((256, 256, 7), dtype=torch.int64, device=g.device)
    a2 = torch.full((256, 256, 7), -1, dtype=torch.int64, device=g.device)
    for s in range(60):
        m = g.get_action_mask()
        seed = ctypes.c_uint64(0x0123456789ABCDEF + s)
        _native.check(_native.lib().mrts_sample_actions(st, m.data_ptr(), 256, 256, 0, seed, s, a1.data_ptr()))
        _native.check(_native.lib().mrts_sample_actions_src(st, m.data_ptr(), g.source_unit_mask.data_ptr(), 256, 256, 0, seed, s,
                                                            a2.data_ptr()))
        assert torch.equal(a1, a2), f"step {s}"
        if s % 20 == 0:
            np.testing.assert_array_equal(a2.cpu().numpy(), sample_actions(m.cpu().numpy(), 0x0123456789ABCDEF + s, s))
        g.step(a2)


@pytest.mark.parametrize("rows", [1, 37, 63, 64, 65, 255, 256, 257, 1000])
def test_source_guided_sampler_ragged_rows(rows):
    """Waves of 64 rows: partial last wave, odd int64 tails, many source rows
    per wave (more than one round of four cooperative row loads)."""
    import ctypes

    from gym_microrts import _native
    from oracle_py import sample_actions

    torch = _torch()
    rng = np.random.default_rng(rows)
    m = (rng.random((1, rows, 78)) < 0.2).astype(np.int32)
    m[0, ::3] = 0
    src = (m.sum(-1) > 0).astype(np.int32)
    m[0, :, 0] |= src[0]   # getMasks: a source cell always has its NOOP bit
    md, sd = torch.from_numpy(m).cuda(), torch.from_numpy(src).cuda()
    out = torch.full((1, rows, 7), -1, dtype=torch.int64, device="cuda")
    _native.check(_native.lib().mrts_sample_actions_src(torch.cuda.current_stream().cuda_stream, md.data_ptr(), sd.data_ptr(), 1,
                                                        rows, 0, ctypes.c_uint64(42), 7, out.data_ptr()))
    np.testing.assert_array_equal(out.cpu().numpy(), sample_actions(m, 42, 7))


def test_float_obs_equals_int_obs():
    torch = _torch()
    gi = make_gpu_env(8, 0, "maps/16x16/basesWorkers16x16.xml", 2000)
    gf = make_gpu_env(8, 0, "maps/16x16/basesWorkers16x16.xml", 2000, return_tensors=True)
    np.testing.assert_array_equal(gi.reset(), gf.reset().cpu().numpy().astype(np.int32))
    assert gf.reset().dtype == torch.float32


def test_device_sampler_matches_oracle_sampler():
    import ctypes

    from gym_microrts import _native
    from oracle_py import sample_actions

    torch = _torch()
    g = make_gpu_env(64, 0, "maps/16x16/basesWorkers16x16.xml", 2000, return_tensors=True)
    g.reset()
    m = g.get_action_mask()
    out = torch.empty((64, 256, 7), dtype=torch.int64, device=g.device)
    for step in (0, 1, 12345):
        _native.check(_native.lib().mrts_sample_actions(torch.cuda.current_stream().cuda_stream, m.data_ptr(), 64, 256, 0,
                                                        ctypes.c_uint64(0xDEADBEEF12345678), step, out.data_ptr()))
        ref = sample_actions(m.cpu().numpy(), 0xDEADBEEF12345678, step)
        np.testing.assert_array_equal(out.cpu().numpy(), ref)


@pytest.mark.parametrize("rows", [1, 37, 255, 256, 257, 1000])
def test_device_sampler_ragged_rows(rows):
    """Blocks of 256 rows: partial last block, odd element / int64 tails."""
    import ctypes

    from gym_microrts import _native
    from oracle_py import sample_actions

    torch = _torch()
    rng = np.random.default_rng(rows)
    m = (rng.random((1, rows, 78)) < 0.2).astype(np.int32)
    m[0, ::3] = 0   # rows with no valid entry use the uniform fallback
    md = torch.from_numpy(m).cuda()
    out = torch.full((1, rows, 7), -1, dtype=torch.int64, device="cuda")
    _native.check(_native.lib().mrts_sample_actions(torch.cuda.current_stream().cuda_stream, md.data_ptr(), 1, rows, 0,
                                                    ctypes.c_uint64(42), 7, out.data_ptr()))
    np.testing.assert_array_equal(out.cpu().numpy(), sample_actions(m, 42, 7))


def _cycling(cyc, nsp, nbot, max_steps, steps):
    from gym_microrts.envs.vec_env import MicroRTSGridModeVecEnv
    from gym_microrts import microrts_ai
    from oracle_py import sample_actions

    g = MicroRTSGridModeVecEnv(num_selfplay_envs=nsp, num_bot_envs=nbot, max_steps=max_steps, ai2s=[microrts_ai.passiveAI] * nbot,
                               map_paths=[cyc[0]], cycle_maps=cyc, reward_weight=np.array([10.0, 1.0, 1.0, 0.2, 1.0, 4.0]))
    table = [os.path.join(MAPS, p) for p in dict.fromkeys(cyc)]
    o = make_oracle(nsp, nbot, None, max_steps, maps=table)
    np.testing.assert_array_equal(g.reset(), o.reset())
    from itertools import cycle

    nxt = cycle([table.index(os.path.join(MAPS, p)) for p in cyc])
    for s in range(steps):
        mo = o.get_action_mask()
        np.testing.assert_array_equal(g.get_action_mask(), mo)
        a = sample_actions(mo, 99, s)
        og, rg, dg, _ = g.step(a)
        oo, ro, do, _ = o.step(a)
        np.testing.assert_array_equal(rg, ro)
        np.testing.assert_array_equal(dg, do)
        for e in np.nonzero(do)[0]:
            if e < nsp and e % 2:
                continue
            game = e // 2 if e < nsp else nsp // 2 + (e - nsp)
            o.reset_game(game, next(nxt))
        oo = o.encode(o.raw_obs())
        np.testing.assert_array_equal(og, oo, err_msg=f"step {s}")
    assert g.error_flags() == 0


def test_map_cycling_matches_oracle():
    """cycle_maps (vec_env.py:1038-1056): finished games restart on the next map."""
    _cycling(["maps/16x16/basesWorkers16x16A.xml", "maps/16x16/basesWorkers16x16B.xml", "maps/16x16/basesWorkers16x16C.xml"],
             8, 4, 60, 200)


def test_all16x16_maps_cycling():
    """ppo_gridnet's training-map catalogue (microrts_maps.ALL16x16_MAPS, authored
    layouts incl. melee and eight-base maps) cycled through every game."""
    from gym_microrts.microrts_maps import ALL16x16_MAPS

    _cycling(ALL16x16_MAPS, 24, 6, 70, 400)


def test_no_invariant_violation_long_run():
    """2000-step random selfplay at 1024 envs: no produce/move into an occupied
    cell, no time overflow (engine invariants that would make the Java throw)."""
    torch = _torch()
    g = make_gpu_env(1024, 0, "maps/16x16/basesWorkers16x16.xml", 2000, return_tensors=True)
    g.reset()
    from gym_microrts import _native

    act = torch.empty((1024, 256, 7), dtype=torch.int64, device=g.device)
    for s in range(2000):
        m = g.get_action_mask()
        _native.lib().mrts_sample_actions(torch.cuda.current_stream().cuda_stream, m.data_ptr(), 1024, 256, 0, 77, s, act.data_ptr())
        obs, r, d, _ = g.step(act)
    torch.cuda.synchronize()
    assert g.error_flags() == 0
    assert (obs.sum(-1) == 6).all()


def test_issue_many_inconsistent_pending_produces():
    """issue()'s candidate walk with more than 16 inconsistent pending assignments
    (the walk had a 16-entry buffer).  On barracksField16x16 player 0
    queues 18 heavies (tick 0) and 20 lights (tick 1) against 40 resources -- the
    pairwise ResourceUsage test admits both batches -- the lights complete first
    (tick 81) and leave 0 resources while the 18 heavies are still pending, so from
    then on every new action of player 0 meets 18 over-budget produces.  GPU ==
    oracle every tick, with masked random actions for every other row."""
    from oracle_py import sample_actions

    m = "maps/16x16/barracksField16x16.xml"
    g = make_gpu_env(2, 0, m, 2000)
    o = make_oracle(2, 0, m, 2000)
    np.testing.assert_array_equal(g.reset(), o.reset())
    cells = [y * 16 + x for y in (1, 4, 7, 10, 13) for x in range(0, 16, 2)]
    worst = 0
    for t in range(160):
        mg, mo = g.get_action_mask(), o.get_action_mask()
        np.testing.assert_array_equal(mg, mo, err_msg=f"mask {t}")
        a = sample_actions(mo, 11, t)
        if t < 2:
            a[:] = 0
            for c in (cells[:18] if t == 0 else cells[18:38]):
                a[0, c] = [4, 0, 0, 0, 2, 5 if t == 0 else 4, 0]
        og, rg, dg, ig = g.step(a)
        oo, ro, do, io = o.step(a)
        np.testing.assert_array_equal(og, oo, err_msg=f"obs {t}")
        np.testing.assert_array_equal(rg, ro, err_msg=f"reward {t}")
        np.testing.assert_array_equal(dg, do)
        d = o.dump_cells(0)
        res0 = o.game_resources(0)[0]
        over = int(((d[:, 1] == 0) & (d[:, 4] == 4) & (res0 < 2)).sum())
        worst = max(worst, over)
    assert worst > 16, worst
    assert g.error_flags() == 0


def test_reward_weight_reassigned_mid_run():
    """vec_env.py:1057 reads self.reward_weight every step: a reassignment after
    construction reaches the tensor path's fused `raw @ w`."""
    from oracle_py import sample_actions

    torch = _torch()
    g = make_gpu_env(16, 4, "maps/16x16/basesWorkers16x16.xml", 300, return_tensors=True)
    o = make_oracle(16, 4, "maps/16x16/basesWorkers16x16.xml", 300)
    g.reset()
    o.reset()
    for s in range(120):
        if s == 40:
            g.reward_weight = o.reward_weight = np.array([1.0, 2.0, 3.0, 0.5, 7.0, 11.0])
        mo = o.get_action_mask()
        a = sample_actions(mo, 3, s)
        _, rg, _, _ = g.step(torch.from_numpy(a).to(g.device))
        _, ro, _, _ = o.step(a)
        np.testing.assert_allclose(rg.cpu().numpy(), ro, rtol=0, atol=1e-12, err_msg=f"step {s}")


@pytest.mark.parametrize("eager", [False, True])
def test_parked_games_read_zero_in_mask_and_raw_kernels(eager):
    """a parked game's envs read zero from get_action_mask() (k_masks when
    masks are not eager) and from the JNI-shaped raw observation (k_raw), whatever
    those buffers held before the park -- not only the buffers bound at park time."""
    torch = _torch()
    from gym_microrts import _native

    env = make_gpu_env(4, 2, os.path.join(MAPS, "maps/16x16/basesWorkers16x16.xml"), 2000, eager_masks=eager,
                       return_tensors=True, obs_dtype=torch.int32)
    env.reset()
    hw = env.height * env.width
    for s in range(5):
        m = env.get_action_mask()
        a = torch.zeros((env.num_envs, hw, 7), dtype=torch.int64, device=env.device)
        env.step(a)
    raw = torch.full((env.num_envs, 6, env.height, env.width), 7, dtype=torch.int32, device=env.device)
    env._mask.fill_(3)
    env._src.fill_(1)
    env._mask_fresh = False
    env.park_games([0, 3])   # envs 0, 1 (selfplay game 0) and 5 (bot game 3)
    m = env.get_action_mask()
    _native.check(_native.lib().mrts_get_raw_obs(env._h, env._stream(), raw.data_ptr()), env._h, "raw")
    torch.cuda.synchronize()
    parked, live = [0, 1, 5], [2, 3, 4]
    assert int(m[parked].abs().sum()) == 0 and int(env._src[parked].abs().sum()) == 0
    assert int(raw[parked].abs().sum()) == 0
    assert int(env._src[live].sum()) > 0 and int(raw[live].sum()) > 0
    assert int((m[live] == 3).sum()) == 0   # live rows rewritten by the mask kernel / eager masks
    env.close()


@pytest.mark.parametrize("seed", range(6))
def test_grouped_source_sampler_equals_per_batch_calls(seed):
    """mrts_sample_actions_src_group: 1-4 batches of random shapes (ragged row counts, map
    sizes 4x4..24x24, any env0) in one launch == one mrts_sample_actions_src call per batch ==
    the oracle's sampler, bit for bit."""
    import ctypes

    from gym_microrts import _native
    from oracle_py import sample_actions

    torch = _torch()
    rng = np.random.default_rng(900 + seed)
    nseg = int(rng.integers(1, 5))
    segs, outs, refs, keep = [], [], [], []
    for k in range(nseg):
        n, hw, env0 = int(rng.integers(1, 40)), int(rng.choice([16, 37, 64, 100, 256, 576])), int(rng.integers(0, 5000))
        m = (rng.random((n, hw, 78)) < 0.15).astype(np.int32)
        m[:, ::3] = 0
        src = (m.sum(-1) > 0).astype(np.int32)
        m[:, :, 0] |= src
        md, sd = torch.from_numpy(m).cuda(), torch.from_numpy(src).cuda()
        out = torch.full((n, hw, 7), -1, dtype=torch.int64, device="cuda")
        ref = torch.full((n, hw, 7), -2, dtype=torch.int64, device="cuda")
        _native.check(_native.lib().mrts_sample_actions_src(torch.cuda.current_stream().cuda_stream, md.data_ptr(), sd.data_ptr(),
                                                            n, hw, env0, ctypes.c_uint64(77 + seed), 11, ref.data_ptr()))
        segs.append(_native.SampleSeg(md.data_ptr(), sd.data_ptr(), n, hw, env0, out.data_ptr()))
        outs.append(out)
        refs.append((ref, m, env0))
        keep += [md, sd]
    arr = (_native.SampleSeg * nseg)(*segs)
    _native.check(_native.lib().mrts_sample_actions_src_group(torch.cuda.current_stream().cuda_stream, arr, nseg,
                                                              ctypes.c_uint64(77 + seed), 11))
    for out, (ref, m, env0) in zip(outs, refs):
        assert torch.equal(out, ref)
        np.testing.assert_array_equal(out.cpu().numpy(), sample_actions(m, 77 + seed, 11, env0=env0))


def test_grouped_source_sampler_refuses_bad_groups():
    from gym_microrts import _native

    torch = _torch()
    lib, st = _native.lib(), torch.cuda.current_stream().cuda_stream
    m = torch.zeros((2, 16, 78), dtype=torch.int32, device="cuda")
    s = torch.zeros((2, 16), dtype=torch.int32, device="cuda")
    a = torch.zeros((2 * 16 * 7 + 2,), dtype=torch.int64, device="cuda")
    ok = _native.SampleSeg(m.data_ptr(), s.data_ptr(), 2, 16, 0, a.data_ptr())
    assert lib.mrts_sample_actions_src_group(st, (_native.SampleSeg * 1)(ok), 0, 1, 0) == -1   # MRTS_EINVAL
    assert lib.mrts_sample_actions_src_group(st, (_native.SampleSeg * 5)(*[ok] * 5), 5, 1, 0) == -1   # MRTS_EINVAL
    bad = _native.SampleSeg(m.data_ptr(), s.data_ptr(), 2, 16, 0, a.data_ptr() + 8)   # actions not 16-byte aligned
    assert lib.mrts_sample_actions_src_group(st, (_native.SampleSeg * 2)(ok, bad), 2, 1, 0) == -1   # MRTS_EINVAL
    assert lib.mrts_sample_actions_src_group(st, (_native.SampleSeg * 1)(ok), 1, 1, 0) == 0


def test_grouped_source_sampler_empty_segment():
    """A zero-env segment between two others owns no block: the neighbours' actions are still
    their own calls' (the block -> segment scan skips it)."""
    import ctypes

    from gym_microrts import _native

    torch = _torch()
    lib, st = _native.lib(), torch.cuda.current_stream().cuda_stream
    rng = np.random.default_rng(5)
    segs, outs, refs, keep = [], [], [], []
    for n, hw in ((3, 64), (0, 256), (5, 100)):
        m = (rng.random((max(n, 1), hw, 78)) < 0.2).astype(np.int32)
        src = (m.sum(-1) > 0).astype(np.int32)
        m[:, :, 0] |= src
        md, sd = torch.from_numpy(m).cuda(), torch.from_numpy(src).cuda()
        out = torch.full((max(n, 1), hw, 7), -1, dtype=torch.int64, device="cuda")
        ref = out.clone()
        if n:
            _native.check(lib.mrts_sample_actions_src(st, md.data_ptr(), sd.data_ptr(), n, hw, 0, ctypes.c_uint64(3), 4,
                                                      ref.data_ptr()))
        segs.append(_native.SampleSeg(md.data_ptr(), sd.data_ptr(), n, hw, 0, out.data_ptr()))
        outs.append(out)
        refs.append(ref)
        keep += [md, sd]
    _native.check(lib.mrts_sample_actions_src_group(st, (_native.SampleSeg * 3)(*segs), 3, ctypes.c_uint64(3), 4))
    for out, ref in zip(outs, refs):
        assert torch.equal(out, ref)   # the empty segment's buffer untouched (-1 both)


@pytest.mark.parametrize("return_tensors", [False, True])
def test_reward_shaping_off(return_tensors):
    """reward_shaping=False (vec_env.py:1004-1005): every raw reward channel but WinLoss reads
    0 -- in infos, in `raw @ reward_weight` and in the tensor path's fused dot -- while the
    game itself runs as with shaping (obs, masks, dones == the oracle's)."""
    from oracle_py import sample_actions

    from gym_microrts import microrts_ai
    from gym_microrts.envs.vec_env import MicroRTSGridModeVecEnv
    from oracle_py import OracleVecEnv

    torch = _torch()
    m, w = "maps/8x8/basesWorkers8x8.xml", np.array([10.0, 1.0, 1.0, 0.2, 1.0, 4.0])
    g = MicroRTSGridModeVecEnv(num_selfplay_envs=16, num_bot_envs=8, max_steps=300, map_paths=[m], reward_weight=w,
                               ai2s=[microrts_ai.workerRushAI] * 8, reward_shaping=False, return_tensors=return_tensors,
                               obs_dtype=torch.int32 if return_tensors else None)
    o = OracleVecEnv(16, 8, [os.path.join(MAPS, m)], max_steps=300, ai2s=["workerRushAI"] * 8, reward_weight=w)
    cpu = (lambda t: t.cpu().numpy()) if return_tensors else np.asarray
    np.testing.assert_array_equal(cpu(g.reset()), o.reset())
    seen_win = seen_shaped = 0
    for s in range(700):
        mo = o.get_action_mask()
        np.testing.assert_array_equal(cpu(g.get_action_mask()), mo, err_msg=f"mask {s}")
        a = sample_actions(mo, 13, s)
        og, rg, dg, ig = g.step(torch.from_numpy(a).to(g.device) if return_tensors else a)
        oo, ro, do, io = o.step(a)
        raw_o = np.array([i["raw_rewards"] for i in io])
        seen_shaped += int((raw_o[:, 1:] != 0).any())
        raw_o[:, 1:] = 0
        seen_win += int((raw_o[:, 0] != 0).any())
        np.testing.assert_array_equal(cpu(og), oo, err_msg=f"obs {s}")
        np.testing.assert_array_equal(np.array([np.asarray(i["raw_rewards"]) for i in ig]), raw_o, err_msg=f"raw {s}")
        np.testing.assert_allclose(cpu(rg), raw_o @ g.reward_weight, rtol=0, atol=1e-12, err_msg=f"reward {s}")
        np.testing.assert_array_equal(cpu(dg), do)
    assert seen_shaped > 0 and seen_win > 0   # shaped channels were zeroed; WinLoss got through
    assert g.error_flags() == 0


def test_per_env_map_paths():
    """map_paths with one entry per env (vec_env.py:120-125; all of one size): every game
    starts on its own env's map -- a selfplay pair on its first env's -- and auto-resets
    onto it again.  GPU == an oracle given the same per-game map table."""
    from gym_microrts import microrts_ai
    from gym_microrts.envs.vec_env import MicroRTSGridModeVecEnv
    from gym_microrts.microrts_maps import ALL16x16_MAPS
    from oracle_py import OracleVecEnv, sample_actions

    nsp, nbot = 12, 6
    paths = [ALL16x16_MAPS[(3 * e) % len(ALL16x16_MAPS)] for e in range(nsp + nbot)]
    w = np.array([10.0, 1.0, 1.0, 0.2, 1.0, 4.0])
    bots = ["coacAI", "workerRushAI", "lightRushAI"] * 2
    g = MicroRTSGridModeVecEnv(num_selfplay_envs=nsp, num_bot_envs=nbot, max_steps=80, map_paths=paths, reward_weight=w,
                               ai2s=[getattr(microrts_ai, b) for b in bots])
    table = list(dict.fromkeys(paths))
    game_env = [2 * k for k in range(nsp // 2)] + [nsp + j for j in range(nbot)]
    o = OracleVecEnv(nsp, nbot, [os.path.join(MAPS, p) for p in table], max_steps=80, ai2s=bots, reward_weight=w,
                     game_maps=[table.index(paths[e]) for e in game_env])
    assert len(set(paths[e] for e in game_env)) > 5
    np.testing.assert_array_equal(g.reset(), o.reset())
    for s in range(250):
        mo = o.get_action_mask()
        np.testing.assert_array_equal(g.get_action_mask(), mo, err_msg=f"mask {s}")
        a = sample_actions(mo, 17, s)
        og, rg, dg, _ = g.step(a)
        oo, ro, do, _ = o.step(a)
        np.testing.assert_array_equal(og, oo, err_msg=f"obs {s}")
        np.testing.assert_array_equal(rg, ro, err_msg=f"reward {s}")
        np.testing.assert_array_equal(dg, do)
    assert g.error_flags() == 0
