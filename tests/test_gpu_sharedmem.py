"""MicroRTSGridModeSharedMemVecEnv (vec_env.py:1238-1362): page-locked host buffers
returned by reference and overwritten in place, bit-exact vs the oracle."""
import os

import numpy as np
import pytest

from conftest import MAPS

W = np.array([10.0, 1.0, 1.0, 0.2, 1.0, 4.0])


def test_sharedmem_requires_one_map():
    """vec_env.py:1260-1261 (raised before any device work)"""
    from gym_microrts.envs.vec_env import MicroRTSGridModeSharedMemVecEnv

    with pytest.raises(ValueError, match="same map"):
        MicroRTSGridModeSharedMemVecEnv(2, 0, map_paths=["maps/16x16/basesWorkers16x16.xml", "maps/8x8/basesWorkers8x8.xml"])


@pytest.mark.gpu
@pytest.mark.timeout(300)
@pytest.mark.parametrize("map_path,nsp,bots", [("maps/16x16/basesWorkers16x16.xml", 16, ["coacAI", "workerRushAI"] * 4),
                                               ("maps/10x10/basesTwoWorkers10x10.xml", 8, ["passiveAI", "lightRushAI"])])
def test_sharedmem_lockstep_vs_oracle(map_path, nsp, bots):
    from gym_microrts import microrts_ai
    from gym_microrts.envs.vec_env import MicroRTSGridModeSharedMemVecEnv
    from oracle_py import OracleVecEnv, sample_actions

    g = MicroRTSGridModeSharedMemVecEnv(nsp, len(bots), max_steps=150, ai2s=[getattr(microrts_ai, b) for b in bots],
                                        map_paths=[map_path], reward_weight=W)
    o = OracleVecEnv(nsp, len(bots), [os.path.join(MAPS, map_path)], max_steps=150, ai2s=bots, reward_weight=W)
    obs = g.reset()
    assert obs is g.obs and obs.dtype == np.int32
    np.testing.assert_array_equal(obs, o.reset())
    for s in range(320):
        m = g.get_action_mask()
        assert m is g.action_mask and m.shape == (g.num_envs, g.height * g.width, 78)
        mo = o.get_action_mask()
        np.testing.assert_array_equal(m, mo, err_msg=f"mask step {s}")
        a = sample_actions(mo, 99, s).reshape(g.num_envs, -1)     # (N, H*W*7) int64, as ppo_gridnet passes
        og, rg, dg, ig = g.step(a)
        oo, ro, do, io = o.step(a)
        assert og is g.obs
        np.testing.assert_array_equal(og, oo, err_msg=f"obs step {s}")
        np.testing.assert_array_equal(rg, ro, err_msg=f"reward step {s}")
        np.testing.assert_array_equal(dg, do, err_msg=f"done step {s}")
        np.testing.assert_array_equal(np.array([i["raw_rewards"] for i in ig]), np.array([i["raw_rewards"] for i in io]))
    assert g.error_flags() == 0
    g.close()
    o.close()
