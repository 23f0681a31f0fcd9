"""Device bots (mrts_bots.hip) == the oracle's restated bots
(oracle/mrts_oracle_ai.c), bit for bit, in lock-step rollouts through the
product path (MicroRTSGridModeVecEnv -> libmicrorts_amd.so).  Bot behaviour vs
Java is PARITY UNPINNED; these tests pin GPU == oracle."""
import os

import numpy as np
import pytest

from conftest import MAPS

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]   # per-test limits below override

BOTS = ["workerRushAI", "lightRushAI", "coacAI", "randomBiasedAI", "randomAI", "POWorkerRush", "POLightRush",
        "POHeavyRush", "PORangedRush"]


def lockstep(ais, map_path, nsp, steps, partial_obs=False, seed=7, max_steps=2000, mode="masked", return_tensors=False,
             bot_fusion=True, obs_dtype="int32"):
    """obs_dtype (tensor path only): "int32", or "float32" -- the bench's dtype, compared as
    bits against the oracle's one-hot (conftest.obs_bits_equal)."""
    import torch

    from conftest import obs_bits_equal

    from gym_microrts import microrts_ai
    from gym_microrts.envs.vec_env import MicroRTSGridModeVecEnv
    from oracle_py import OracleVecEnv, sample_actions

    w = np.array([10.0, 1.0, 1.0, 0.2, 1.0, 4.0])
    g = MicroRTSGridModeVecEnv(num_selfplay_envs=nsp, num_bot_envs=len(ais), max_steps=max_steps,
                               ai2s=[getattr(microrts_ai, a) for a in ais], map_paths=[map_path], reward_weight=w,
                               partial_obs=partial_obs, return_tensors=return_tensors,
                               obs_dtype=getattr(torch, obs_dtype) if return_tensors else None, bot_fusion=bot_fusion)
    o = OracleVecEnv(nsp, len(ais), [os.path.join(MAPS, map_path)], max_steps=max_steps, ai2s=ais,
                     partial_obs=partial_obs, reward_weight=w)
    cpu = (lambda t: t.cpu().numpy()) if return_tensors else np.asarray

    def check_obs(got, want, msg):
        if return_tensors and obs_dtype == "float32":
            assert obs_bits_equal(got, want), msg
        else:
            np.testing.assert_array_equal(cpu(got), want, err_msg=msg)

    check_obs(g.reset(), o.reset(), "reset")
    rng = np.random.default_rng(seed)
    n, hw = g.num_envs, g.height * g.width
    nvec = np.array([6, 4, 4, 4, 4, 7, 49])
    outcomes = np.zeros(3, int)
    for s in range(steps):
        mo = o.get_action_mask()
        np.testing.assert_array_equal(cpu(g.get_action_mask()), mo, err_msg=f"mask step {s}")
        a = sample_actions(mo, seed, s)
        if mode == "mixed":
            u = (rng.random((n, hw, 7)) * nvec).astype(np.int64)
            a = np.where(rng.random((n, hw, 1)) < 0.3, u, a)
        ga = torch.from_numpy(a).to(g.device) if return_tensors else a
        og, rg, dg, ig = g.step(ga)
        oo, ro, do, io = o.step(a)
        check_obs(og, oo, f"obs step {s}")
        raw_g = np.array([i["raw_rewards"] for i in ig])
        raw_o = np.array([i["raw_rewards"] for i in io])
        np.testing.assert_array_equal(raw_g, raw_o, err_msg=f"raw rewards step {s}")
        np.testing.assert_array_equal(cpu(dg), do, err_msg=f"done step {s}")
        for k in np.nonzero(do)[0]:
            outcomes[int(raw_o[k, 0]) + 1] += 1
    assert g.error_flags() == 0
    g.close()
    o.close()
    return outcomes


@pytest.mark.parametrize("partial_obs", [False, True])
@pytest.mark.parametrize("ai", BOTS)
def test_bot_lockstep_16x16(ai, partial_obs):
    out = lockstep([ai] * 24, "maps/16x16/basesWorkers16x16.xml", 4, 700, partial_obs=partial_obs)
    if ai in ("workerRushAI", "lightRushAI", "POWorkerRush", "POLightRush") and not partial_obs:
        assert out[0] > 0   # the faster rushes win some games against the random agent within 700 ticks


@pytest.mark.parametrize("map_path", ["maps/8x8/basesWorkers8x8.xml", "maps/10x10/basesTwoWorkers10x10.xml",
                                      "maps/24x24/basesWorkers24x24.xml", "maps/barricades24x24.xml",
                                      "maps/4x4/baseTwoWorkers4x4.xml", "maps/32x32/basesWorkers32x32.xml",
                                      "maps/15x15/basesWorkersWalls15x15.xml", "maps/9x13/basesWorkersWalls9x13.xml"])
def test_mixed_bots_lockstep_other_maps(map_path):
    """... including 32x32, whose bot-fused k_step needs > 64 KB of LDS,
    and walled maps whose cell count is not a multiple of 4 (225, 117), full
    observability and fusion on: the fused early bot reads the step's terrain in
    place while the other waves build the terrain plane and move masks from it
    (wall plane /root/reference/tests/test_observation.py:86-108)"""
    ais = (BOTS * 3)[:16] + ["passiveAI"] * 2
    lockstep(ais, map_path, 4, 500, max_steps=300)


def test_bots_adversarial_agent_actions():
    """unmasked agent actions (illegal / conflicting) against every bot"""
    lockstep(BOTS * 2, "maps/16x16/basesWorkers16x16.xml", 2, 500, mode="mixed", max_steps=400)


def test_bots_tensor_path_and_long_episodes():
    lockstep(BOTS * 2, "maps/16x16/basesWorkers16x16.xml", 0, 2100, return_tensors=True, partial_obs=True)


@pytest.mark.parametrize("partial_obs", [False, True])
def test_bot_vs_bot_env_matches_oracle(partial_obs):
    """MicroRTSBotVecEnv (vec_env.py:1104-1236): both players are device bots."""
    import torch

    from gym_microrts import microrts_ai
    from gym_microrts.envs.vec_env import MicroRTSBotVecEnv
    from oracle_py import OracleVecEnv

    ai1 = (BOTS * 2)[:12]
    ai2 = list(reversed(ai1))
    m = "maps/16x16/basesWorkers16x16A.xml"
    w = np.array([10.0, 1.0, 1.0, 0.2, 1.0, 4.0])
    g = MicroRTSBotVecEnv(ai1s=[getattr(microrts_ai, a) for a in ai1], ai2s=[getattr(microrts_ai, a) for a in ai2],
                          map_paths=[m], max_steps=700, partial_obs=partial_obs, reward_weight=w)
    o = OracleVecEnv(0, len(ai1), [os.path.join(MAPS, m)], max_steps=700, ai2s=ai2, ai1s=ai1, partial_obs=partial_obs,
                     reward_weight=w)
    assert g.reset().shape == (12, 2)
    o.reset()
    hw = g.height * g.width
    finished = 0
    for s in range(1500):
        _, rg, dg, ig = g.step(np.zeros((12, hw * 7), np.int64))
        o.source_unit_mask = np.zeros((12, hw), np.int32)
        ro, do = o.step_raw(np.zeros((12, hw, 7), np.int64))
        np.testing.assert_array_equal(np.array([i["raw_rewards"] for i in ig]), ro, err_msg=f"step {s}")
        np.testing.assert_array_equal(dg, do[:, 0])
        np.testing.assert_array_equal(rg, ro @ w)
        np.testing.assert_array_equal(g._obs.cpu().numpy().astype(np.int32), o.encode(o.raw_obs()), err_msg=f"obs {s}")
        finished += int(do[:, 0].sum())
    assert finished > 12
    assert g.error_flags() == 0


def test_league_outcomes_on_device():
    """league.db's 30 bot-vs-bot pairs (tests/golden/league_outcomes.json; 5 matches
    each, basesWorkers16x16A, max_steps 5000: league.py:236-245) played by the
    device bots through MicroRTSBotVecEnv, driven exactly as league.py's run_m2
    (vec_env.py:1104-1236): every outcome matches the reference's record
    (deterministic pairs exactly, pairs with a random bot by majority) and the
    oracle's game for game."""
    from gym_microrts import microrts_ai
    from gym_microrts.envs.vec_env import MicroRTSBotVecEnv
    from oracle_py import OracleVecEnv
    from test_bots_oracle import check_league, league_outcomes

    L = league_outcomes()
    reps = 5
    ai1 = [q["p0"] for q in L["pairs"] for _ in range(reps)]
    ai2 = [q["p1"] for q in L["pairs"] for _ in range(reps)]
    n = len(ai1)
    w = np.array([10.0, 1.0, 1.0, 0.2, 1.0, 4.0])
    g = MicroRTSBotVecEnv(ai1s=[getattr(microrts_ai, a) for a in ai1], ai2s=[getattr(microrts_ai, a) for a in ai2],
                          map_paths=[L["map"]], max_steps=L["max_steps"], reward_weight=w)
    o = OracleVecEnv(0, n, [os.path.join(MAPS, L["map"])], max_steps=L["max_steps"], ai2s=ai2, ai1s=ai1)
    g.reset()
    o.reset()
    hw = g.height * g.width
    res, ref = [None] * n, [None] * n
    for s in range(L["max_steps"]):
        _, _, dg, ig = g.step([[[0] * 8] * 2])   # run_m2's dummy actions (league.py:326-331)
        o.source_unit_mask = np.zeros((n, hw), np.int32)
        ro, do = o.step_raw(np.zeros((n, hw, 7), np.int64))
        for k in np.nonzero(dg)[0]:
            if res[k] is None:
                res[k] = int(ig[k]["raw_rewards"][0])
        for k in np.nonzero(do[:, 0])[0]:
            if ref[k] is None:
                ref[k] = int(ro[k, 0])
        if all(x is not None for x in res):
            break
    assert res == ref
    check_league(L, res, reps)
    assert g.error_flags() == 0


def mixed_lockstep(spec, steps, max_steps=300, partial_obs=False, obs_dtype="int32", **kw):
    """MicroRTSMixedMapVecEnv (kw: concurrent / group_policy) vs one oracle per bucket:
    obs (int32, or float32 compared as bits), masks, rewards and dones bit-exact every step."""
    import torch

    from conftest import obs_bits_equal

    from gym_microrts import microrts_ai
    from gym_microrts.envs.vec_env import MicroRTSMixedMapVecEnv
    from oracle_py import OracleVecEnv, sample_actions

    w = np.array([10.0, 1.0, 1.0, 0.2, 1.0, 4.0])
    env = MicroRTSMixedMapVecEnv([dict(map_paths=[m], num_selfplay_envs=nsp, ai2s=[getattr(microrts_ai, a) for a in ais])
                                  for m, nsp, ais in spec], max_steps=max_steps, return_tensors=True, partial_obs=partial_obs,
                                 reward_weight=w, obs_dtype=getattr(torch, obs_dtype), **kw)
    orc = [OracleVecEnv(nsp, len(ais), [os.path.join(MAPS, m)], max_steps=max_steps, ai2s=ais, reward_weight=w,
                        partial_obs=partial_obs) for m, nsp, ais in spec]
    for og, oo in zip(env.reset(), [o.reset() for o in orc]):
        assert obs_bits_equal(og, oo), "reset"
    for s in range(steps):
        masks = env.get_action_mask()
        acts = []
        for mg, o in zip(masks, orc):
            mo = o.get_action_mask()
            np.testing.assert_array_equal(mg.cpu().numpy(), mo)
            acts.append(sample_actions(mo, 13, s))
        obs, rew, done, infos = env.step([torch.from_numpy(a).cuda() for a in acts])
        for k, o in enumerate(orc):
            oo, ro, do, _ = o.step(acts[k])
            assert obs_bits_equal(obs[k], oo), f"obs bucket {k} step {s}"
            np.testing.assert_array_equal(rew[k].cpu().numpy(), ro, err_msg=f"bucket {k} step {s}")
            np.testing.assert_array_equal(done[k].cpu().numpy(), do)
    assert env.error_flags() == 0
    return env


# group policies: None = one step_wait per bucket; else mrts_step_group's MRTS_GROUP_* bits
# (1 merge-fit, 2 merge-all, | 4 bots first)
@pytest.mark.parametrize("concurrent,group_policy", [(False, None), (True, None), (False, 0), (False, 1 | 4), (False, 2),
                                                     (False, 2 | 4)])
def test_mixed_map_buckets_match_oracle(concurrent, group_policy):
    """BASELINE configs[4]: 8x8 / 16x16 / 24x24 buckets in one MicroRTSMixedMapVecEnv,
    selfplay + device workerRush / coacAI envs, every bucket bit-exact vs its oracle
    (buckets back to back, each on its own HIP stream, and in one mrts_step_group
    call: separate launches, 8x8 + 16x16 in one launch, all three in one)."""
    spec = [("maps/8x8/basesWorkers8x8.xml", 8, ["workerRushAI", "coacAI"] * 2),
            ("maps/16x16/basesWorkers16x16.xml", 16, ["coacAI", "workerRushAI", "randomBiasedAI", "lightRushAI"] * 2),
            ("maps/24x24/basesWorkers24x24.xml", 4, ["workerRushAI", "coacAI"])]
    env = mixed_lockstep(spec, 400, concurrent=concurrent, group_policy=group_policy)
    assert env.grouped == (group_policy is not None)
    # the launches (mrts_step_group_plan): merge-fit merges what keeps >= 6 workgroups per CU
    # (the step kernel's own occupancy), so the 24x24 bucket's 40 KB workgroups keep their own
    expect = {None: ([0, 1, 2], 3), 0: ([0, 1, 2], 3), 5: ([0, 0, 1], 2), 2: ([0, 0, 0], 1), 6: ([0, 0, 0], 1)}
    assert env.launch_plan() == expect[group_policy]


@pytest.mark.parametrize("partial_obs", [False, True])
def test_step_group_walled_odd_sizes(partial_obs):
    """mrts_step_group merging four map sizes of different cell counts into one
    256-lane launch (merge-all, bots first): 8x8 and 10x10 games run on workgroups
    wider than their maps, walled 15x15 and 9x13 maps (HW % 4 != 0) with the early
    fused bot at the launch's width, bit-exact vs the oracle per bucket."""
    spec = [("maps/8x8/basesWorkers8x8.xml", 4, ["coacAI", "lightRushAI"]),
            ("maps/10x10/basesTwoWorkers10x10.xml", 2, ["workerRushAI", "randomBiasedAI"]),
            ("maps/15x15/basesWorkersWalls15x15.xml", 4, ["coacAI", "workerRushAI", "lightRushAI"]),
            ("maps/9x13/basesWorkersWalls9x13.xml", 2, ["coacAI", "randomBiasedAI"])]
    env = mixed_lockstep(spec, 300, max_steps=200, partial_obs=partial_obs, group_policy=2 | 4)
    assert env.grouped


def test_bots_without_fusion():
    """k_bot launched at the start of every step (mrts_set_bot_fusion(h, 0)) == oracle"""
    lockstep(["coacAI", "workerRushAI", "randomBiasedAI", "lightRushAI"] * 3, "maps/16x16/basesWorkers16x16.xml", 2, 300,
             max_steps=150, bot_fusion=False)


def test_bot_fusion_with_map_cycling_and_resets():
    """Fusion on vs off through map-cycling resets (mrts_reset_games decides the reset
    games' bot actions afresh) and explicit reset() calls."""
    import torch

    from gym_microrts import microrts_ai
    from gym_microrts.envs.vec_env import MicroRTSGridModeVecEnv

    cyc = ["maps/16x16/basesWorkers16x16A.xml", "maps/16x16/basesWorkers16x16B.xml", "maps/16x16/TwoBasesBarracks16x16.xml"]
    envs = [MicroRTSGridModeVecEnv(num_selfplay_envs=2, num_bot_envs=6, max_steps=40, map_paths=[cyc[0]], cycle_maps=cyc,
                                   ai2s=[microrts_ai.coacAI, microrts_ai.workerRushAI, microrts_ai.lightRushAI] * 2,
                                   reward_weight=np.array([10.0, 1.0, 1.0, 0.2, 1.0, 4.0]), return_tensors=True,
                                   bot_fusion=fu) for fu in (True, False)]
    from oracle_py import sample_actions

    for rep in range(2):
        obs = [e.reset() for e in envs]
        torch.testing.assert_close(obs[0], obs[1], rtol=0, atol=0)
        for s in range(130):
            masks = [e.get_action_mask() for e in envs]
            assert torch.equal(masks[0], masks[1]), f"mask rep {rep} step {s}"
            a = torch.from_numpy(sample_actions(masks[0].cpu().numpy(), 3 + rep, s)).to(envs[0].device)
            outs = [e.step(a) for e in envs]
            assert torch.equal(outs[0][0], outs[1][0]), f"obs rep {rep} step {s}"
            assert torch.equal(outs[0][1], outs[1][1]) and torch.equal(outs[0][2], outs[1][2])
    for e in envs:
        assert e.error_flags() == 0
        e.close()


def test_bot_fusion_toggled_mid_game():
    """mrts_set_bot_fusion switched on <-> off between steps: the decisions already made
    by a fused step are used exactly once, so the run stays equal to the oracle."""
    import torch

    from gym_microrts import _native, microrts_ai
    from gym_microrts.envs.vec_env import MicroRTSGridModeVecEnv
    from oracle_py import OracleVecEnv, sample_actions

    ais = ["coacAI", "workerRushAI", "lightRushAI", "randomBiasedAI"]
    w = np.array([10.0, 1.0, 1.0, 0.2, 1.0, 4.0])
    m = "maps/16x16/basesWorkers16x16.xml"
    g = MicroRTSGridModeVecEnv(num_selfplay_envs=2, num_bot_envs=len(ais), max_steps=120, map_paths=[m], reward_weight=w,
                               ai2s=[getattr(microrts_ai, a) for a in ais], return_tensors=True, obs_dtype=torch.int32)
    o = OracleVecEnv(2, len(ais), [os.path.join(MAPS, m)], max_steps=120, ai2s=ais, reward_weight=w)
    np.testing.assert_array_equal(g.reset().cpu().numpy(), o.reset())
    for s in range(300):
        if s % 37 == 0:
            _native.check(_native.lib().mrts_set_bot_fusion(g._h, (s // 37) % 2), g._h, "set_bot_fusion")
        mo = o.get_action_mask()
        np.testing.assert_array_equal(g.get_action_mask().cpu().numpy(), mo, err_msg=f"mask step {s}")
        a = sample_actions(mo, 5, s)
        og, _, dg, _ = g.step(torch.from_numpy(a).to(g.device))
        oo, _, do, _ = o.step(a)
        np.testing.assert_array_equal(og.cpu().numpy(), oo, err_msg=f"obs step {s}")
        np.testing.assert_array_equal(dg.cpu().numpy(), do, err_msg=f"done step {s}")
    assert g.error_flags() == 0
    g.close()
    o.close()


def test_step_group_tiny_map_in_wide_workgroup():
    """A 4x4 bucket merged with a 16x16 one runs on 256-lane workgroups: the step's
    first compaction then needs four ballot words in L.vis (vis_bytes), more than the
    4x4 map's visibility words -- sized for both, bit-exact vs the oracle."""
    spec = [("maps/4x4/baseTwoWorkers4x4.xml", 8, ["workerRushAI", "coacAI", "randomBiasedAI", "lightRushAI"]),
            ("maps/16x16/basesWorkers16x16.xml", 4, ["coacAI", "workerRushAI"])]
    env = mixed_lockstep(spec, 300, max_steps=120, group_policy=2 | 4)
    assert env.launch_plan() == ([0, 0], 1)
