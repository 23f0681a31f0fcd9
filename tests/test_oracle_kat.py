"""The oracle (oracle/libmrts_oracle.so) against the reference's own known-answer
tests and the golden vectors of its python encoder.  CPU only."""
import os

import numpy as np
import pytest

import kat
from conftest import MAPS
from oracle_py import OracleVecEnv, sample_actions

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "encode_obs_golden.npz")


class _Spaces:
    def __init__(self, hw):
        class S:
            pass

        self.action_plane_space = S()
        self.action_plane_space.nvec = np.array([6, 4, 4, 4, 4, 7, 49])
        self.action_space = S()
        self.action_space.nvec = np.tile(self.action_plane_space.nvec, hw)


def make_oracle_env(num_selfplay_envs, num_bot_envs, map_path, max_steps, reward_weight=None):
    e = OracleVecEnv(num_selfplay_envs, num_bot_envs, [os.path.join(MAPS, map_path)], max_steps=max_steps,
                     ai2s=["passiveAI"] * num_bot_envs, reward_weight=reward_weight)
    sp = _Spaces(e.height * e.width)
    e.action_plane_space, e.action_space = sp.action_plane_space, sp.action_space
    return e


def test_observation_kat():
    kat.check_observation(make_oracle_env)


def test_mask_kat():
    kat.check_mask(make_oracle_env)


def test_reward_kat():
    kat.check_rewards(make_oracle_env)


@pytest.mark.parametrize("case", ["16x16", "4x4", "10x10", "24x24"])
def test_encoder_matches_reference_golden(case):
    """oracle _encode_obs restatement == the reference's own _encode_obs output."""
    g = np.load(GOLDEN)
    raw, obs = g[f"{case}_raw"], g[f"{case}_obs"]
    e = make_oracle_env(2, 0, "maps/16x16/basesWorkers16x16.xml", 100)
    import ctypes

    import oracle_py

    n, P_raw, h, w = raw.shape
    out = np.zeros((n, h, w, 29), np.int32)
    oracle_py.lib().ovec_encode_obs(oracle_py.ptr(np.ascontiguousarray(raw)), n, h, w, 0, oracle_py.ptr(out))
    np.testing.assert_array_equal(out, obs)
    del e, ctypes


def test_encoder_partial_obs_golden():
    g = np.load(GOLDEN)
    raw, obs = g["16x16_po_raw"], g["16x16_po_obs"]
    import oracle_py

    n, P_raw, h, w = raw.shape
    out = np.zeros((n, h, w, 31), np.int32)
    oracle_py.lib().ovec_encode_obs(oracle_py.ptr(np.ascontiguousarray(raw)), n, h, w, 1, oracle_py.ptr(out))
    np.testing.assert_array_equal(out, obs)


def test_random_rollout_invariants():
    """Long random selfplay rollout: engine invariants the Java asserts
    (GameState.integrityCheck, one unit per cell) and episode bookkeeping."""
    e = make_oracle_env(16, 0, "maps/8x8/basesWorkers8x8.xml", 300)
    e.reset()
    dones = 0
    for s in range(900):
        m = e.get_action_mask()
        a = sample_actions(m, 7, s)
        obs, r, d, infos = e.step(a)
        dones += int(d.sum())
        # exactly 6 one-hot groups per cell
        assert obs.shape == (16, 8, 8, 29)
        assert (obs.sum(-1) == 6).all()
        for g in range(8):
            cells = e.dump_cells(g)
            live = cells[:, 0] >= 0
            # owned units never carry a negative hp
            assert (cells[live, 2] > 0).all()
    assert dones >= 16 * 2  # max_steps=300 forces at least 3 episodes per env


README_PO_WORKER = [0, 1, 0, 0, 0, 1, 0, 0, 0, 0, 0, 1, 0, 0, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0, 0, 0, 1, 0, 1, 0]
PO_EMPTY = [1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 1, 0, 0, 0, 0, 0, 0, 0, 1, 0, 0, 0, 0, 0, 1, 0, 1, 0]


def test_partial_obs_readme_vector():
    """README.md:90-92: a worker not visible to the opponent encodes as the
    29-vector + [1,0]; enemy units (and resources) outside the player's sight
    read as empty cells (PartiallyObservableGameState)."""
    e = OracleVecEnv(2, 0, [os.path.join(MAPS, "maps/16x16/basesWorkers16x16.xml")], max_steps=100, partial_obs=True)
    obs = e.reset()
    assert obs.shape == (2, 16, 16, 31)
    assert (obs.sum(-1) == 7).all()
    assert obs[0, 1, 1].tolist() == README_PO_WORKER        # own worker (1,1), opponent 13 cells away
    assert obs[1, 14, 14].tolist() == README_PO_WORKER      # p1's view of its own worker
    for y, x in [(13, 13), (14, 14), (14, 15), (15, 15)]:   # p1 units + far resources hidden from p0
        assert obs[0, y, x].tolist() == PO_EMPTY, (y, x)
    assert obs[0, 0, 0, 13 + 1] == 1                         # resource (0,0) within the worker's sight
    assert obs[0, 0, 0, 29] == 1                             # ... and not observable by p1
    # full observability still sees everything
    f = OracleVecEnv(2, 0, [os.path.join(MAPS, "maps/16x16/basesWorkers16x16.xml")], max_steps=100).reset()
    assert f[0, 14, 14, 10 + 2] == 1


def test_partial_obs_rollout_invariants():
    e = OracleVecEnv(16, 0, [os.path.join(MAPS, "maps/8x8/basesWorkers8x8.xml")], max_steps=200, partial_obs=True)
    full = OracleVecEnv(16, 0, [os.path.join(MAPS, "maps/8x8/basesWorkers8x8.xml")], max_steps=200)
    e.reset()
    full.reset()
    for s in range(300):
        m = e.get_action_mask()
        np.testing.assert_array_equal(m, full.get_action_mask())   # masks ignore fog (own units only)
        a = sample_actions(m, 3, s)
        obs, r, d, _ = e.step(a)
        fo, fr, fd, _ = full.step(a)
        np.testing.assert_array_equal(r, fr)
        np.testing.assert_array_equal(d, fd)
        assert (obs.sum(-1) == 7).all()
        # every unit the player sees is where the full observation has it
        seen = obs[..., 13] == 0
        np.testing.assert_array_equal(obs[..., :29][seen], fo[seen])
        # own units are never hidden
        own = fo[..., 11] == 1
        np.testing.assert_array_equal(obs[..., :29][own], fo[own])


def test_bench_loop_equals_python_loop():
    """ovec_bench_steps (bench.py's CPU baseline) == get_action_mask + sample_actions
    + step + encode driven from Python, step for step."""
    path = os.path.join(MAPS, "maps/16x16/basesWorkers16x16.xml")
    a, b = OracleVecEnv(16, 0, [path], max_steps=120), OracleVecEnv(16, 0, [path], max_steps=120)
    a.reset()
    b.reset()
    for s in range(300):
        obs_a, rew_a, done_a = a.bench_steps(1, 7, s)
        m = b.get_action_mask()
        obs_b, _, done_b, infos = b.step(sample_actions(m, 7, s))
        np.testing.assert_array_equal(obs_a, obs_b, err_msg=f"step {s}")
        np.testing.assert_array_equal(rew_a, np.array([i["raw_rewards"] for i in infos]))
        np.testing.assert_array_equal(done_a[:, 0], done_b)
