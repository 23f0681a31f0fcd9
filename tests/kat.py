"""Known-answer checks of the reference's JVM-backed tests, runnable against any
env exposing the MicroRTSGridModeVecEnv surface (the oracle here, the HIP
engine in the gpu tests).  Data: tests/golden/kat_fixtures.json."""
import json
import os

import numpy as np

FIX = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "kat_fixtures.json")))


def onehot(idx, n):
    v = np.zeros(n, np.int32)
    v[idx] = 1
    return v


def check_observation(make_env):
    """tests/test_observation.py:8-108"""
    f = FIX["observation"]
    envs = make_env(num_selfplay_envs=2, num_bot_envs=0, map_path=f["map"], max_steps=f["max_steps"])
    obs = np.asarray(envs.reset())
    assert obs.shape == (2, 16, 16, 29)
    for env, y, x, name in f["expect"]:
        np.testing.assert_array_equal(obs[env][y][x], onehot(f["vectors"][name], 29), err_msg=f"env {env} ({y},{x}) {name}")
    assert obs.sum() == f["total_sum"]
    envs = make_env(num_selfplay_envs=2, num_bot_envs=0, map_path=f["wall_map"], max_steps=f["max_steps"])
    obs = np.asarray(envs.reset())
    env, y, x, name = f["wall_expect"]
    np.testing.assert_array_equal(obs[env][y][x], onehot(f["vectors"][name], 29))


def check_mask(make_env):
    """tests/test_mask.py:9-84"""
    f = FIX["mask"]
    envs = make_env(num_selfplay_envs=0, num_bot_envs=1, map_path=f["map"], max_steps=2000)
    envs.reset()
    m = np.asarray(envs.get_action_mask())
    assert m.shape == (1, 16, 78)
    for cell, ones in f["cells"].items():
        np.testing.assert_array_equal(m[0, int(cell)], onehot(ones, 78), err_msg=f"cell {cell}")
    # every other cell holds no idle player-0 unit
    others = [c for c in range(16) if str(c) not in f["cells"]]
    assert m[0, others].sum() == 0


def check_rewards(make_env):
    """tests/test_reward.py:9-106"""
    f = FIX["reward"]
    for name, script in f["scenarios"].items():
        envs = make_env(num_selfplay_envs=0, num_bot_envs=1, map_path=f["map"], max_steps=2000, reward_weight=np.array(f["reward_weight"]))
        envs.reset()
        nplanes = len(envs.action_plane_space.nvec)
        nact = len(envs.action_space.nvec)
        for stepdef in script:
            if stepdef[0] == "noop":
                for _ in range(stepdef[1]):
                    np.asarray(envs.get_action_mask())
                    envs.step(np.zeros(nact, np.int32))
                continue
            cell, comps, expect = stepdef
            np.asarray(envs.get_action_mask())
            a = np.zeros(nact, np.int32)
            a[cell * nplanes:(cell + 1) * nplanes] = comps
            r = np.asarray(envs.step(a)[1]).flatten()
            assert expect == "positive" and r > 0, (name, stepdef, r)
