"""Random-map fuzzing of GPU == oracle (tests/random_maps.py): map sizes 4..32 x 4..32, wall
density 0-25 %, 4 to 200 units of every type, random starting resources, a random mix of
device bots, selfplay pairs, full or partial observability, random time limits, masked and
unmasked agent actions.  MRTS_FUZZ_SEEDS / MRTS_FUZZ_FIRST set the number of cases and the
first seed (default 12 from 0; the round-5 campaign ran seeds 0-2199 of the single-engine
cases and 0-1499 of the grouped-launch cases, profiles/r05_fuzz/).  Odd seeds run the tensor
path with float32 obs -- the bench's kernels -- compared as bits (conftest.obs_bits_equal);
even seeds the int32 numpy / tensor contracts."""
import os

import numpy as np
import pytest

from random_maps import write_random_map
from test_gpu_bots import BOTS, lockstep

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]   # per-test limits below override
SEEDS = int(os.environ.get("MRTS_FUZZ_SEEDS", "12"))
FIRST = int(os.environ.get("MRTS_FUZZ_FIRST", "0"))


def f32(seed):
    """odd seeds: the tensor path with float32 obs (the bench's dtype), compared as bits"""
    return dict(return_tensors=True, obs_dtype="float32") if seed % 2 else {}


def case(seed):
    rng = np.random.default_rng(1000 + seed)
    w, h = int(rng.integers(4, 33)), int(rng.integers(4, 33))
    n = int(rng.integers(4, max(5, min(200, int(w * h * 0.6)))))
    bots = [str(b) for b in rng.choice(BOTS + ["passiveAI"], size=int(rng.integers(0, 9)))]
    return dict(w=w, h=h, n=n, walls=float(rng.uniform(0, 0.25)), res=(int(rng.integers(0, 30)), int(rng.integers(0, 30))),
                bots=bots, nsp=2 * int(rng.integers(0 if bots else 1, 4)), partial=bool(rng.integers(0, 2)),
                max_steps=int(rng.integers(30, 200)))


@pytest.mark.timeout(600)
@pytest.mark.parametrize("seed", range(FIRST, FIRST + SEEDS))
def test_fuzz_map_lockstep(tmp_path, seed):
    c = case(seed)
    path = write_random_map(str(tmp_path / f"fuzz{seed}.xml"), c["w"], c["h"], seed, n_units=min(c["n"], c["w"] * c["h"] - 4),
                            wall_frac=c["walls"], res=c["res"])
    lockstep(c["bots"], path, c["nsp"], 160, partial_obs=c["partial"], seed=seed, max_steps=c["max_steps"], mode="mixed",
             **f32(seed))


def group_case(seed):
    rng = np.random.default_rng(5000 + seed)
    nb = int(rng.integers(2, 5))
    sizes, spec = set(), []
    while len(sizes) < nb:
        sizes.add((int(rng.integers(4, 33)), int(rng.integers(4, 33))))
    for k, (w, h) in enumerate(sorted(sizes)):
        bots = [str(b) for b in rng.choice(BOTS + ["passiveAI"], size=int(rng.integers(0, 5)))]
        spec.append(dict(w=w, h=h, n=int(rng.integers(4, max(5, min(120, int(w * h * 0.5))))), walls=float(rng.uniform(0, 0.2)),
                         bots=bots, nsp=2 * int(rng.integers(0 if bots else 1, 3))))
    policy = [0, 1, 2, 1 | 4, 2 | 4][int(rng.integers(0, 5))]
    return spec, policy, bool(rng.integers(0, 2)), int(rng.integers(30, 150))


@pytest.mark.timeout(600)
@pytest.mark.parametrize("seed", range(FIRST, FIRST + max(1, SEEDS // 3)))
def test_fuzz_step_group_lockstep(tmp_path, seed):
    """mrts_step_group over 2-4 random map sizes (each its own engine) under every grouping
    policy -- separate launches, merge-fit, merge-all, bots first -- so maps of any size share
    a workgroup width and a segment table with others: every bucket == its own oracle."""
    from test_gpu_bots import mixed_lockstep

    spec, policy, partial, max_steps = group_case(seed)
    rows = []
    for k, c in enumerate(spec):
        path = write_random_map(str(tmp_path / f"g{seed}_{k}.xml"), c["w"], c["h"], seed * 10 + k,
                                n_units=min(c["n"], c["w"] * c["h"] - 4), wall_frac=c["walls"])
        rows.append((path, c["nsp"], c["bots"]))
    env = mixed_lockstep(rows, 120, max_steps=max_steps, partial_obs=partial, group_policy=policy,
                         obs_dtype=f32(seed).get("obs_dtype", "int32"))
    assert env.grouped


@pytest.mark.timeout(600)
@pytest.mark.parametrize("seed", range(FIRST, FIRST + max(1, SEEDS // 3)))
def test_fuzz_bot_vs_bot_lockstep(tmp_path, seed):
    """MicroRTSBotVecEnv (vec_env.py:1104-1236) on random maps: random device bots on both sides
    (k_bot for player 0 and the fused bot for player 1), fog, random time limits; raw rewards,
    dones and obs == the oracle's every tick."""
    from gym_microrts import microrts_ai
    from gym_microrts.envs.vec_env import MicroRTSBotVecEnv
    from oracle_py import OracleVecEnv

    rng = np.random.default_rng(3000 + seed)
    w, h = int(rng.integers(4, 33)), int(rng.integers(4, 33))
    n = int(rng.integers(4, max(5, min(200, int(w * h * 0.6)))))
    path = write_random_map(str(tmp_path / f"b{seed}.xml"), w, h, seed, n_units=min(n, w * h - 4),
                            wall_frac=float(rng.uniform(0, 0.25)), res=(int(rng.integers(0, 30)), int(rng.integers(0, 30))))
    k = int(rng.integers(1, 9))
    ai1 = [str(b) for b in rng.choice(BOTS + ["passiveAI"], size=k)]
    ai2 = [str(b) for b in rng.choice(BOTS + ["passiveAI"], size=k)]
    partial, max_steps = bool(rng.integers(0, 2)), int(rng.integers(30, 200))
    rw = np.array([10.0, 1.0, 1.0, 0.2, 1.0, 4.0])
    g = MicroRTSBotVecEnv(ai1s=[getattr(microrts_ai, a) for a in ai1], ai2s=[getattr(microrts_ai, a) for a in ai2],
                          map_paths=[path], max_steps=max_steps, partial_obs=partial, reward_weight=rw)
    o = OracleVecEnv(0, k, [path], max_steps=max_steps, ai2s=ai2, ai1s=ai1, partial_obs=partial, reward_weight=rw)
    g.reset()
    o.reset()
    hw = g.height * g.width
    for s in range(160):
        _, rg, dg, ig = g.step(np.zeros((k, hw * 7), np.int64))
        o.source_unit_mask = np.zeros((k, hw), np.int32)
        ro, do = o.step_raw(np.zeros((k, hw, 7), np.int64))
        np.testing.assert_array_equal(np.array([i["raw_rewards"] for i in ig]), ro, err_msg=f"step {s}")
        np.testing.assert_array_equal(dg, do[:, 0])
        np.testing.assert_array_equal(rg, ro @ rw)
        np.testing.assert_array_equal(g._obs.cpu().numpy().astype(np.int32), o.encode(o.raw_obs()), err_msg=f"obs {s}")
    assert g.error_flags() == 0
    g.close()
    o.close()


def large_case(seed):
    """A random shape past 32x32 that mrts_create still accepts (1025..1128 cells: the step's
    unprefetched path, tests/test_max_map_sizes.py), bots only where they are allowed (at
    most 32 wide and 64 high)."""
    import ctypes

    from gym_microrts import _native

    f = _native.lib().mrts_engine_lds_bytes
    f.restype, f.argtypes = ctypes.c_size_t, [ctypes.c_int, ctypes.c_int]
    rng = np.random.default_rng(7000 + seed)
    while True:
        w, h = int(rng.integers(12, 72)), int(rng.integers(12, 72))
        if 1024 < w * h <= 1200 and f(w * h, w) <= 65536:
            break
    bots_ok = w <= 32 and h <= 64
    bots = [str(b) for b in rng.choice(BOTS + ["passiveAI"], size=int(rng.integers(0, 6)))] if bots_ok else []
    return dict(w=w, h=h, n=int(rng.integers(20, 260)), walls=float(rng.uniform(0, 0.2)),
                res=(int(rng.integers(0, 30)), int(rng.integers(0, 30))), bots=bots,
                nsp=2 * int(rng.integers(0 if bots else 1, 3)), partial=bool(rng.integers(0, 2)),
                max_steps=int(rng.integers(30, 150)))


@pytest.mark.timeout(600)
@pytest.mark.parametrize("seed", range(FIRST, FIRST + max(1, SEEDS // 6)))
def test_fuzz_large_map_lockstep(tmp_path, seed):
    """Random maps of the largest accepted shapes (past 1024 cells), random bots where allowed,
    fog, time limits, masked and unmasked actions: GPU == oracle every tick."""
    c = large_case(seed)
    path = write_random_map(str(tmp_path / f"L{seed}.xml"), c["w"], c["h"], seed, n_units=c["n"], wall_frac=c["walls"],
                            res=c["res"])
    lockstep(c["bots"], path, c["nsp"], 120, partial_obs=c["partial"], seed=seed, max_steps=c["max_steps"], mode="mixed",
             **f32(seed))
