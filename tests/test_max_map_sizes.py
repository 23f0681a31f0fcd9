"""The largest maps the engine accepts, and a clear refusal just past them ("maximum sizes").

mrts_create takes a map when the step kernel's workgroup LDS fits 64 KB (about 1128 cells:
47x24, 24x47, 33x33, 16x69, ...) and, with device bots, when the map is at most 32 wide and
64 high (the bots' path finding holds one bit word per row) and the bot kernel's LDS fits.
Past 1024 cells a 256-lane workgroup holds five cells per lane and the step takes its
unprefetched path (mrts_engine.hip: neither `pf_ok` nor `pf_wide`), which no other test
reaches: the fuzz campaigns stop at 32x32.

CPU: the boundary shapes load and the next ones are refused with MRTS_ENOTIMPL (no device
work).  GPU: HIP == oracle lock-steps on the boundary shapes -- selfplay, every device bot
where bots are allowed, fused and unfused, with and without fog, dense random maps.
"""
import numpy as np
import pytest

from random_maps import write_random_map

# (w, h, bots allowed): the largest accepted shapes of each kind
BOUNDARY = [(47, 24, False), (24, 47, True), (33, 33, False), (32, 35, True), (16, 69, False), (19, 59, True)]
# just past the step kernel's LDS (ENOTIMPL), and past the bots' row-word limits
REFUSED = [(48, 24, False), (24, 48, False), (34, 34, False), (33, 20, True), (16, 65, True)]


def _create(path, nsp, nbot, ai=3):
    from gym_microrts import _native

    games = nsp // 2 + nbot
    return _native.create(nsp, nbot, 100, False, [path], [0] * games, [ai] * nbot, 1)


@pytest.mark.parametrize("w,h,bots", BOUNDARY)
def test_boundary_shapes_are_accepted(tmp_path, w, h, bots):
    from gym_microrts import _native

    p = write_random_map(str(tmp_path / f"m{w}x{h}.xml"), w, h, 1, n_units=40)
    hd = _create(p, 2, 2 if bots else 0)
    i = _native.info(hd)
    assert (i.width, i.height) == (w, h)
    _native.lib().mrts_destroy(hd)


@pytest.mark.parametrize("w,h,bots", REFUSED)
def test_past_the_limit_is_refused(tmp_path, w, h, bots):
    from gym_microrts._native import MicroRTSNotImplemented

    p = write_random_map(str(tmp_path / f"m{w}x{h}.xml"), w, h, 1, n_units=40)
    with pytest.raises(MicroRTSNotImplemented, match="LDS|bots need maps"):
        _create(p, 2, 2 if bots else 0)


def test_oracle_runs_the_boundary_shapes(tmp_path):
    """The checker itself on the largest shapes (cheap: 2 envs, 30 ticks)."""
    from oracle_py import OracleVecEnv, sample_actions

    for w, h, bots in BOUNDARY:
        p = write_random_map(str(tmp_path / f"o{w}x{h}.xml"), w, h, 2, n_units=120)
        o = OracleVecEnv(2, 2 if bots else 0, [p], max_steps=50, ai2s=["coacAI", "workerRushAI"] if bots else None)
        obs = o.reset()
        assert obs.shape == (2 + (2 if bots else 0), h, w, 29)
        for s in range(30):
            o.step(sample_actions(o.get_action_mask(), 3, s))
        o.close()


@pytest.mark.gpu
@pytest.mark.timeout(300)
@pytest.mark.parametrize("partial_obs", [False, True])
@pytest.mark.parametrize("w,h,bots", BOUNDARY)
def test_gpu_lockstep_boundary_shapes(tmp_path, w, h, bots, partial_obs):
    """HIP == oracle every tick on the largest accepted shapes: 150 units on a random map,
    masked + unmasked agent actions, 200 ticks with max_steps 90 (auto-resets inside); the
    k_bot arm on the tensor path with float32 obs, compared as bits."""
    from test_gpu_bots import BOTS, lockstep

    p = write_random_map(str(tmp_path / f"g{w}x{h}.xml"), w, h, 7, n_units=150, wall_frac=0.1)
    ais = (BOTS + ["passiveAI"]) if bots else []
    lockstep(ais, p, 4, 200, partial_obs=partial_obs, seed=w * 100 + h, max_steps=90, mode="mixed")
    if bots:   # the same with the bots in their own kernel (k_bot) instead of fused into the step
        lockstep(ais, p, 2, 120, partial_obs=partial_obs, seed=h, max_steps=60, bot_fusion=False, return_tensors=True,
                 obs_dtype="float32")


@pytest.mark.gpu
@pytest.mark.timeout(300)
@pytest.mark.parametrize("w,h", [(47, 24), (24, 47)])
def test_gpu_boundary_shapes_mask_kernel_and_tensors(tmp_path, w, h):
    """The standalone mask kernel (eager_masks=False) and the tensor contract with float32
    obs on the largest shapes."""
    import torch

    from conftest import obs_bits_equal
    from gym_microrts.envs.vec_env import MicroRTSGridModeVecEnv
    from oracle_py import OracleVecEnv, sample_actions

    p = write_random_map(str(tmp_path / f"t{w}x{h}.xml"), w, h, 9, n_units=150, wall_frac=0.1)
    W = np.array([10.0, 1.0, 1.0, 0.2, 1.0, 4.0])
    g = MicroRTSGridModeVecEnv(num_selfplay_envs=6, num_bot_envs=0, max_steps=70, map_paths=[p], reward_weight=W,
                               return_tensors=True, eager_masks=False)
    o = OracleVecEnv(6, 0, [p], max_steps=70, reward_weight=W)
    assert obs_bits_equal(g.reset(), o.reset())
    for s in range(150):
        mo = o.get_action_mask()
        assert torch.equal(g.get_action_mask().cpu(), torch.from_numpy(mo)), f"mask {s}"
        a = sample_actions(mo, 4, s)
        og, rg, dg, ig = g.step(torch.from_numpy(a).to(g.device))
        oo, ro, do, io = o.step(a)
        assert obs_bits_equal(og, oo), f"obs {s}"
        np.testing.assert_array_equal(ig._raw.cpu().numpy(), np.array([i["raw_rewards"] for i in io]))
        np.testing.assert_array_equal(dg.cpu().numpy(), do)
    assert g.error_flags() == 0
    g.close()
    o.close()
