"""Produce rows at the exact resource boundary: k_step issues a player's
produce rows lane-parallel when all of this tick's produce rows plus its dearest
pending produce fit its resources (PSUM + PMAX <= resources, mrts_engine.hip step
(2a)), else on the ordered one-lane path.  Hand-built states put PSUM + PMAX at
resources exactly and one over, with and without a pending produce, with new rows
sharing a target cell and a new row targeting a pending produce's cell -- for
player 0 and player 1 of a selfplay game (different budgets each side) and for the
agent of games against device bots -- and the HIP engine must equal the oracle
(GameState.issue's ResourceUsage checks in the Java object model) bit for bit:
masks, obs, raw rewards (ProduceWorker / ProduceBuilding / ProduceCombatUnit) and
dones every tick while the produced units come out."""
import os

import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]   # per-test limits below override
W = np.array([10.0, 1.0, 1.0, 0.2, 1.0, 4.0])
UP, RIGHT, DOWN, LEFT = 0, 1, 2, 3
WORKER, LIGHT, HEAVY, RANGED = 3, 4, 5, 6

# player 0's producers (x, y); player 1's are the point mirror (7 - x, 7 - y)
PROD = {"A": ("Barracks", 1, 1), "B": ("Barracks", 1, 3), "C": ("Barracks", 4, 1), "D": ("Base", 3, 3)}
MIRROR_DIR = {UP: DOWN, DOWN: UP, LEFT: RIGHT, RIGHT: LEFT}


def _map(path, r0, r1):
    units, uid = [], 0
    for p in (0, 1):
        for name, (t, x, y) in PROD.items():
            if p:
                x, y = 7 - x, 7 - y
            hp = 10 if t == "Base" else 4
            units.append(f'<rts.units.Unit type="{t}" ID="{uid}" player="{p}" x="{x}" y="{y}" resources="0" hitpoints="{hp}" >'
                         "</rts.units.Unit>")
            uid += 1
    xml = (f'<rts.PhysicalGameState width="8" height="8"><terrain>{"0" * 64}</terrain><players>'
           f'<rts.Player ID="0" resources="{r0}"></rts.Player><rts.Player ID="1" resources="{r1}"></rts.Player></players>'
           f'<units>{"".join(units)}</units></rts.PhysicalGameState>')
    with open(path, "w") as f:
        f.write(xml)


# scenario: (resources p0, resources p1, tick-0 orders, tick-1 orders); an order = (producer, direction, unit type)
# PSUM = tick-1 costs (light / heavy / ranged 2, worker 1), PMAX = the pending tick-0 heavy (2)
SCENARIOS = {
    "pending_exact_p0_over_p1": (7, 6, [("A", DOWN, HEAVY)], [("B", DOWN, LIGHT), ("C", RIGHT, RANGED), ("D", DOWN, WORKER)]),
    "pending_over_p0_exact_p1": (6, 7, [("A", DOWN, HEAVY)], [("B", DOWN, LIGHT), ("C", RIGHT, RANGED), ("D", DOWN, WORKER)]),
    "no_pending_exact_and_over": (5, 4, [], [("B", DOWN, LIGHT), ("C", RIGHT, RANGED), ("D", DOWN, WORKER)]),
    "two_new_one_pending_exact": (6, 5, [("A", DOWN, HEAVY)], [("C", RIGHT, RANGED), ("B", DOWN, LIGHT)]),
    "shared_target_new_rows": (7, 7, [("A", DOWN, HEAVY)], [("B", RIGHT, LIGHT), ("D", LEFT, WORKER), ("C", RIGHT, RANGED)]),
    "target_of_pending": (9, 8, [("A", DOWN, HEAVY)], [("B", UP, LIGHT), ("C", RIGHT, RANGED), ("D", DOWN, WORKER)]),
    "starved": (2, 1, [("A", DOWN, HEAVY)], [("B", DOWN, LIGHT), ("D", DOWN, WORKER)]),
}


def _orders(a, env, player, orders):
    for name, d, t in orders:
        _, x, y = PROD[name]
        if player:
            x, y, d = 7 - x, 7 - y, MIRROR_DIR[d]
        a[env, y * 8 + x] = [4, 0, 0, 0, d, t, 0]


@pytest.mark.parametrize("name", sorted(SCENARIOS))
def test_produce_budget_boundary(tmp_path, name):
    import torch

    from gym_microrts import microrts_ai
    from gym_microrts.envs.vec_env import MicroRTSGridModeVecEnv
    from oracle_py import OracleVecEnv

    r0, r1, t0, t1 = SCENARIOS[name]
    path = str(tmp_path / f"{name}.xml")
    _map(path, r0, r1)
    ais = ["workerRushAI", "coacAI", "lightRushAI", "passiveAI"]
    g = MicroRTSGridModeVecEnv(num_selfplay_envs=2, num_bot_envs=len(ais), max_steps=200, map_paths=[path],
                               ai2s=[getattr(microrts_ai, x) for x in ais], reward_weight=W, return_tensors=True,
                               obs_dtype=torch.int32)
    o = OracleVecEnv(2, len(ais), [path], max_steps=200, ai2s=ais, reward_weight=W)
    dev = g.device

    def same(gpu, host, what, s):
        assert torch.equal(gpu, torch.from_numpy(np.ascontiguousarray(host)).to(dev)), f"{name}: {what} differs at tick {s}"

    same(g.reset(), o.reset(), "reset obs", -1)
    produced = np.zeros(6)
    for s in range(40):
        mg, mo = g.get_action_mask(), o.get_action_mask()
        same(mg, mo, "mask", s)
        a = np.zeros((g.num_envs, 64, 7), np.int64)
        orders = t0 if s == 0 else t1 if s == 1 else []
        for e in range(g.num_envs):
            _orders(a, e, 1 if e == 1 else 0, orders)   # env 1 = player 1 of the selfplay game
        og, rg, dg, ig = g.step(torch.from_numpy(a).to(dev))
        oo, ro, do, io = o.step(a)
        raw = np.array([i["raw_rewards"] for i in io])
        same(og, oo, "obs", s)
        same(ig._raw, raw, "raw rewards", s)
        same(dg, np.asarray(do, bool), "done", s)
        produced += raw[:2].sum(0)
    assert g.error_flags() == 0
    # the orders did issue (produce rewards on the selfplay views): the scenario exercised the budget path
    assert produced[2] + produced[5] > 0 or name == "starved"
    g.close()
    o.close()
