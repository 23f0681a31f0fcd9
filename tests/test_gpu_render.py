"""render() of the HIP engine (vec_env.py:1075-1084).

The Java PhysicalGameStatePanel the reference draws with is absent, so the
frame's drawing rules are this engine's own: parity is the
device k_render == oracle_py.render_frame (numpy restatement of the rules)
pixel for pixel, on states reached by lock-step rollouts.  Against Java:
parity unpinned (no frame fixture exists in the reference)."""
import os
import warnings

import numpy as np
import pytest

from conftest import MAPS

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]   # per-test limits below override


@pytest.mark.parametrize("map_path,nsp,nbot", [
    ("maps/16x16/basesWorkers16x16.xml", 4, 0),
    ("maps/barricades24x24.xml", 0, 2),
    ("maps/10x10/basesTwoWorkers10x10.xml", 2, 2),
])
def test_rgb_array_frame_matches_oracle(map_path, nsp, nbot):
    from gym_microrts import microrts_ai
    from gym_microrts.envs.vec_env import MicroRTSGridModeVecEnv
    from oracle_py import OracleVecEnv, parse_map, render_frame, sample_actions

    g = MicroRTSGridModeVecEnv(num_selfplay_envs=nsp, num_bot_envs=nbot, max_steps=300, ai2s=[microrts_ai.passiveAI] * nbot,
                               map_paths=[map_path], reward_weight=np.array([10.0, 1.0, 1.0, 0.2, 1.0, 4.0]))
    o = OracleVecEnv(nsp, nbot, [os.path.join(MAPS, map_path)], max_steps=300, ai2s=["passiveAI"] * nbot)
    wall = parse_map(os.path.join(MAPS, map_path))["terrain"]
    g.reset()
    o.reset()
    seen = set()
    for s in range(120):
        if s % 20 == 0:
            f = g.render("rgb_array")
            assert f.shape == (640, 640, 3) and f.dtype == np.uint8
            ref = render_frame(o.dump_cells(0), wall, g.width, g.height)
            np.testing.assert_array_equal(f, ref, err_msg=f"frame at step {s}")
            seen |= {tuple(p) for p in np.unique(f.reshape(-1, 3), axis=0)}
        m = o.get_action_mask()
        np.testing.assert_array_equal(g.get_action_mask(), m)
        a = sample_actions(m, 3, s)
        g.step(a)
        o.step(a)
    assert (0, 0, 255) in seen and (255, 255, 255) in seen   # player-0 rims, bases


def test_human_mode_warns_once_and_draws_nothing():
    from gym_microrts.envs.vec_env import MicroRTSGridModeVecEnv

    g = MicroRTSGridModeVecEnv(num_selfplay_envs=2, num_bot_envs=0, map_paths=["maps/16x16/basesWorkers16x16.xml"])
    g.reset()
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        assert g.render() is None
        assert g.render("human") is None
    assert len(w) == 1
    with pytest.raises(ValueError):
        g.render("ansi")


def test_hello_world_example_runs():
    """BASELINE configs[0]: examples/hello_world.py (the reference loop, render()
    every step, 2 selfplay + 2 envs vs device coacAI), its whole trajectory
    replayed through the oracle: masks, obs, weighted rewards and dones equal at
    every step, with the actions the script's host sampler drew."""
    import importlib.util

    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples", "hello_world.py")
    spec = importlib.util.spec_from_file_location("hello_world_example", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    trace = []
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        episodes = mod.main(steps=300, trace=trace)
    assert episodes >= 0 and len(trace) == 300
    from oracle_py import OracleVecEnv

    m = "maps/16x16/basesWorkers16x16.xml"
    o = OracleVecEnv(2, 2, [os.path.join(MAPS, m)], max_steps=2000, ai2s=["coacAI", "coacAI"],
                     reward_weight=np.array([10.0, 1.0, 1.0, 0.2, 1.0, 4.0]))
    o.reset()
    for s, (mask, action, obs, reward, done) in enumerate(trace):
        np.testing.assert_array_equal(mask, o.get_action_mask(), err_msg=f"mask at step {s}")
        oo, ro, do, _ = o.step(action)
        np.testing.assert_array_equal(obs, oo, err_msg=f"obs at step {s}")
        np.testing.assert_array_equal(reward, ro)
        np.testing.assert_array_equal(done, do)
    o.close()


@pytest.mark.parametrize("seed", range(int(os.environ.get("MRTS_FUZZ_FIRST", "0")),
                                       int(os.environ.get("MRTS_FUZZ_FIRST", "0")) + max(1, int(os.environ.get("MRTS_FUZZ_SEEDS", "12")) // 3)))
def test_fuzz_rgb_array_random_maps(tmp_path, seed):
    """Frames of random maps (tests/random_maps.py: 4..32 x 4..32, so the cell size, the
    centring margins and non-square boards vary; walls; every unit type; actions in flight)
    == oracle_py.render_frame pixel for pixel."""
    from gym_microrts.envs.vec_env import MicroRTSGridModeVecEnv
    from oracle_py import OracleVecEnv, parse_map, render_frame, sample_actions
    from random_maps import write_random_map

    rng = np.random.default_rng(11000 + seed)
    w, h = int(rng.integers(4, 33)), int(rng.integers(4, 33))
    path = write_random_map(str(tmp_path / f"r{seed}.xml"), w, h, seed,
                            n_units=min(int(rng.integers(4, max(5, min(150, int(w * h * 0.6))))), w * h - 4),
                            wall_frac=float(rng.uniform(0, 0.25)))
    g = MicroRTSGridModeVecEnv(num_selfplay_envs=2, num_bot_envs=0, max_steps=60, map_paths=[path])
    o = OracleVecEnv(2, 0, [path], max_steps=60)
    wall = parse_map(path)["terrain"]
    g.reset()
    o.reset()
    for s in range(80):
        if s % 8 == 0:
            np.testing.assert_array_equal(g.render("rgb_array"), render_frame(o.dump_cells(0), wall, g.width, g.height),
                                          err_msg=f"{w}x{h} frame at step {s}")
        m = o.get_action_mask()
        a = sample_actions(m, seed, s)
        g.step(a)
        o.step(a)
    g.close()
    o.close()
