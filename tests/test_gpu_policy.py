"""GPU == oracle under the reference's trained policy.

Every other lock-step test drives the agent side with the uniform random sampler,
which rarely reaches what a trained player does: sustained economies, barracks,
combat-unit production, focused attacks, same-tick conflicts.  Here player 0 (and
player 1 of the selfplay games) is agent_sota.pt -- the GridNet policy
experiments/ppo_gridnet_eval.py:49-52, 149 loads -- through the committed fixture
tests/golden/agent_sota_policy.npz (tests/golden/make_agent_sota.py).  Its actions
are sampled once per tick on the GPU from the engine's own obs and masks
(tests/policy.py: masked categorical by Gumbel-max, seeded) and the same int64
array is fed to the HIP engine and to the oracle, so floating point never enters the
comparison.  basesWorkers16x16A (the eval script's map), 256 selfplay envs + 256
envs vs device coacAI / workerRushAI, 1100 ticks, max_steps 800 (time-limit resets
inside the window): obs (float32, as ppo_gridnet.py consumes them, compared as
bits), masks, source mask, raw rewards and dones bit-equal every tick.  The trajectories' statistics (the oracle's event counters) are recorded and
must lie clearly above the random sampler's on the same envs and ticks."""
import json
import os

import numpy as np
import pytest

from conftest import MAPS, obs_bits_equal

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]   # per-test limits below override
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W = np.array([10.0, 1.0, 1.0, 0.2, 1.0, 4.0])
MAP = "maps/16x16/basesWorkers16x16A.xml"


def _p0_envs(nsp, nbot):
    return np.r_[np.arange(0, nsp, 2), np.arange(nsp, nsp + nbot)]


def _summary(o, raw_sum, wins):
    ev = o.event_counts()
    p0 = ev["produced"][0]
    return {"p0_raw_reward_sums": dict(zip(["win_loss", "resource_gather", "produce_worker", "produce_building",
                                             "attack", "produce_combat_unit"], [float(x) for x in raw_sum])),
            "p0_wins": int(wins), "p0_barracks": p0["Barracks"],
            "p0_combat_units": {k: p0[k] for k in ("Light", "Heavy", "Ranged")},
            "p0_attack_hits": ev["hits"][0], "p0_kills": ev["kills"][0],
            "cancel_both": ev["cancel_both"], "inconsistent": ev["inconsistent"], "produced": ev["produced"]}


@pytest.mark.timeout(900)
def test_trained_policy_lockstep_matches_oracle():
    import torch

    from gym_microrts import microrts_ai
    from gym_microrts.envs.vec_env import MicroRTSGridModeVecEnv
    from oracle_py import OracleVecEnv, sample_actions
    from policy import load_policy, policy_actions

    nsp, nbot, ticks, max_steps, seed = 256, 256, 1100, 800, 11
    ais = ["coacAI", "workerRushAI"] * (nbot // 2)
    g = MicroRTSGridModeVecEnv(num_selfplay_envs=nsp, num_bot_envs=nbot, max_steps=max_steps, map_paths=[MAP],
                               ai2s=[getattr(microrts_ai, a) for a in ais], reward_weight=W, return_tensors=True,
                               obs_dtype=torch.float32)
    o = OracleVecEnv(nsp, nbot, [os.path.join(MAPS, MAP)], max_steps=max_steps, ai2s=ais, reward_weight=W)
    dev = g.device
    net = load_policy(dev)
    gen = torch.Generator(device=dev).manual_seed(seed)
    p0 = _p0_envs(nsp, nbot)

    def same(gpu, host, what, s):
        assert torch.equal(gpu, torch.from_numpy(np.ascontiguousarray(host)).to(dev)), f"{what} differs at tick {s}"

    obs = g.reset()
    assert obs_bits_equal(obs, o.reset()), "reset obs"
    raw_sum, wins = np.zeros(6), 0
    for s in range(ticks):
        mg, mo = g.get_action_mask(), o.get_action_mask()
        same(mg, mo, "mask", s)
        same(g.source_unit_mask, o.source_unit_mask, "source mask", s)
        a = policy_actions(net, obs, mg, gen)
        obs, rg, dg, ig = g.step(a)
        oo, ro, do, io = o.step(a.cpu().numpy())
        raw = np.array([i["raw_rewards"] for i in io])
        assert obs_bits_equal(obs, oo), f"obs differs at tick {s}"   # float32: ppo_gridnet's dtype
        same(ig._raw, raw, "raw rewards", s)
        same(dg, np.asarray(do, bool), "done", s)
        raw_sum += raw[p0].sum(0)
        wins += int((raw[p0, 0] > 0).sum())
    assert g.error_flags() == 0
    pol = _summary(o, raw_sum, wins)
    g.close()
    o.close()

    # the random sampler on the same envs and ticks (oracle only: its parity is covered elsewhere)
    r = OracleVecEnv(nsp, nbot, [os.path.join(MAPS, MAP)], max_steps=max_steps, ai2s=ais, reward_weight=W)
    r.reset()
    raw_sum, wins = np.zeros(6), 0
    for s in range(ticks):
        _, ro, _, io = r.step(sample_actions(r.get_action_mask(), seed, s))
        raw = np.array([i["raw_rewards"] for i in io])
        raw_sum += raw[p0].sum(0)
        wins += int((raw[p0, 0] > 0).sum())
    rnd = _summary(r, raw_sum, wins)
    r.close()
    rec = {"envs": {"selfplay": nsp, "vs_coacAI": nbot // 2, "vs_workerRushAI": nbot // 2}, "map": MAP, "ticks": ticks,
           "max_steps": max_steps, "policy": pol, "random_sampler": rnd}
    out = os.path.join(REPO, "gpurun_out")
    if os.path.isdir(out):
        with open(os.path.join(out, "policy_trajectory_stats.json"), "w") as f:
            json.dump(rec, f, indent=1)
    print(json.dumps(rec))
    # what the trained policy reaches and the random sampler does not (or far less)
    assert pol["p0_wins"] > rnd["p0_wins"] + 10
    assert sum(pol["p0_combat_units"].values()) > 4 * max(1, sum(rnd["p0_combat_units"].values()))
    assert pol["p0_barracks"] > rnd["p0_barracks"]
    assert pol["p0_raw_reward_sums"]["attack"] > 4 * rnd["p0_raw_reward_sums"]["attack"]
    assert pol["cancel_both"] > 4 * rnd["cancel_both"]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("map_path,n,ticks,max_steps,partial_obs", [("maps/8x8/basesWorkers8x8.xml", 64, 600, 300, False),
                                                                    ("maps/24x24/basesWorkers24x24.xml", 64, 800, 500, False),
                                                                    ("maps/16x16/basesWorkers16x16.xml", 64, 800, 400, False),
                                                                    ("maps/16x16/basesWorkers16x16A.xml", 128, 900, 600, True)])
def test_trained_policy_lockstep_other_maps(map_path, n, ticks, max_steps, partial_obs):
    """The same trained policy (fully convolutional encoder / actor: any map whose sides
    divide by 4) driving 8x8 / 24x24 / 16x16 games, selfplay and vs every device bot kind
    (8x8: 128-lane fused launch; 24x24: wide-map decode and the 40 KB fused layout), and
    under partial observability (the policy reads the first 29 of the 31 planes -- hidden
    units read as empty cells -- against the fogged bots): GPU == oracle every tick."""
    import torch

    from gym_microrts import microrts_ai
    from gym_microrts.envs.vec_env import MicroRTSGridModeVecEnv
    from oracle_py import OracleVecEnv
    from policy import load_policy, policy_actions

    bots = ["coacAI", "workerRushAI", "lightRushAI", "randomBiasedAI", "POWorkerRush", "passiveAI", "randomAI", "PORangedRush"]
    ais = (bots * n)[:n]
    g = MicroRTSGridModeVecEnv(num_selfplay_envs=n, num_bot_envs=n, max_steps=max_steps, map_paths=[map_path],
                               ai2s=[getattr(microrts_ai, a) for a in ais], reward_weight=W, return_tensors=True,
                               obs_dtype=torch.float32, partial_obs=partial_obs)
    o = OracleVecEnv(n, n, [os.path.join(MAPS, map_path)], max_steps=max_steps, ai2s=ais, reward_weight=W,
                     partial_obs=partial_obs)
    dev = g.device
    net = load_policy(dev, h=g.height, w=g.width)
    gen = torch.Generator(device=dev).manual_seed(5)

    def same(gpu, host, what, s):
        assert torch.equal(gpu, torch.from_numpy(np.ascontiguousarray(host)).to(dev)), f"{what} differs at tick {s}"

    obs = g.reset()
    assert obs_bits_equal(obs, o.reset()), "reset obs"
    wins = 0
    for s in range(ticks):
        mg, mo = g.get_action_mask(), o.get_action_mask()
        same(mg, mo, "mask", s)
        a = policy_actions(net, obs[..., :29], mg, gen)
        obs, _, dg, ig = g.step(a)
        oo, ro, do, io = o.step(a.cpu().numpy())
        raw = np.array([i["raw_rewards"] for i in io])
        assert obs_bits_equal(obs, oo), f"obs differs at tick {s}"   # float32: ppo_gridnet's dtype
        same(ig._raw, raw, "raw rewards", s)
        same(dg, np.asarray(do, bool), "done", s)
        wins += int((raw[_p0_envs(n, n), 0] > 0).sum())
    assert g.error_flags() == 0
    ev = o.event_counts()
    assert sum(ev["produced"][0].values()) > 0   # the policy's economy runs on these maps too
    g.close()
    o.close()
