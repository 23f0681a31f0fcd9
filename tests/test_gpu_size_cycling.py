"""Map cycling across map sizes (vec_env.py:1038-1056 with cycle_maps of several
sizes): MicroRTSSizeCyclingVecEnv against one oracle per
map size holding the same envs.  An env's game plays in one size engine and is
parked (mrts_park_games) in the others; when it ends it restarts on the next
cycle map, moving to that map's size engine.  Every tick: the masks, obs,
rewards and dones of every env equal the oracle of the size it plays in, and the
rows of parked envs are zero.  The oracle's copies of the parked games keep
ticking unseen (reset_game rebuilds them when the env moves in), so the bots are
the deterministic ones (no RNG counter to carry across)."""
import os

import numpy as np
import pytest

from conftest import MAPS

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]   # per-test limits below override

CYCLE = ["maps/8x8/basesWorkers8x8.xml", "maps/16x16/basesWorkers16x16A.xml", "maps/10x10/basesTwoWorkers10x10.xml",
         "maps/16x16/melee16x16Mixed8.xml", "maps/24x24/basesWorkers24x24.xml", "maps/16x16/basesWorkers16x16C.xml",
         "maps/8x8/basesWorkers8x8.xml"]   # 7 entries: games ending together get new maps every round


def test_size_cycling_matches_per_size_oracles():
    for m in CYCLE:
        assert os.path.exists(os.path.join(MAPS, m)), m
    init = ["maps/16x16/basesWorkers16x16.xml"] * 2 + ["maps/8x8/basesWorkers8x8.xml"] * 2 + \
           ["maps/10x10/basesTwoWorkers10x10.xml", "maps/16x16/basesWorkers16x16.xml", "maps/8x8/basesWorkers8x8.xml",
            "maps/16x16/basesWorkers16x16.xml"]
    g = run_size_cycling(init, CYCLE, ["coacAI", "workerRushAI", "lightRushAI", "passiveAI"], 4, 400, 50)
    assert g.sizes == [(8, 8), (10, 10), (16, 16), (24, 24)]
    assert g.moves >= 20, g.moves


def run_size_cycling(init, cycle, bots, nsp, steps, max_steps, seed=17, partial_obs=False):
    """MicroRTSSizeCyclingVecEnv (init: one map per env, pairs sharing theirs) vs one oracle per
    size, `steps` ticks; returns the env (closed) with .moves = the envs that changed size."""
    import torch

    from gym_microrts import microrts_ai
    from gym_microrts.envs.vec_env import MicroRTSSizeCyclingVecEnv
    from oracle_py import OracleVecEnv, sample_actions

    CYCLE = cycle
    nbot = len(bots)
    n = nsp + nbot
    rw = np.array([10.0, 1.0, 1.0, 0.2, 1.0, 4.0])
    g = MicroRTSSizeCyclingVecEnv(nsp, nbot, ai2s=[getattr(microrts_ai, b) for b in bots], map_paths=init, cycle_maps=CYCLE,
                                  max_steps=max_steps, reward_weight=rw, partial_obs=partial_obs)
    oracles = [OracleVecEnv(nsp, nbot, e._map_table, max_steps=max_steps, ai2s=bots, reward_weight=rw,
                            game_maps=list(e._game_map), partial_obs=partial_obs) for e in g.envs]
    obs = g.reset()
    for o in oracles:
        o.reset()

    def check_obs(obs, step):
        for i, (e, o) in enumerate(zip(g.envs, oracles)):
            here = g.bucket == i
            oo = o.encode(o.raw_obs())
            got = obs[i].cpu().numpy()
            np.testing.assert_array_equal(got[here], oo[here], err_msg=f"obs size {g.sizes[i]} step {step}")
            assert not got[~here].any()

    check_obs(obs, -1)
    moves = 0
    cyc = iter(list(CYCLE) * 1000)
    e0 = g.envs[0]
    for s in range(steps):
        masks = g.get_action_mask()
        acts = []
        for i, (e, o) in enumerate(zip(g.envs, oracles)):
            here = g.bucket == i
            mg = masks[i].cpu().numpy()
            mo = o.get_action_mask()
            np.testing.assert_array_equal(mg[here], mo[here], err_msg=f"mask size {g.sizes[i]} step {s}")
            assert not mg[~here].any()
            a = sample_actions(np.ascontiguousarray(mg), seed, s)
            acts.append(torch.from_numpy(a).to(g.device))
            o.source_unit_mask = np.ascontiguousarray(e._src.cpu().numpy())   # parked rows: no agent rows
        before = g.bucket.copy()
        obs, rew, done, infos = g.step(acts)
        rew, done, raw = rew.cpu().numpy(), done.cpu().numpy(), np.array([r["raw_rewards"] for r in infos])
        odone = np.zeros(n, bool)
        for i, o in enumerate(oracles):
            a = acts[i].cpu().numpy()
            oo, ro, do, oinf = o.step(a)
            here = before == i
            np.testing.assert_array_equal(rew[here], ro[here], err_msg=f"reward step {s}")
            np.testing.assert_array_equal(done[here], do[here])
            np.testing.assert_array_equal(raw[here], np.array([x["raw_rewards"] for x in oinf])[here])
            odone |= do & here
        # the oracle side of the cycling: next cycle map, reset there
        for e in np.nonzero(odone)[0]:
            if e < nsp and e % 2:
                continue
            gm = e0.game_of_env(e)
            m = next(cyc)
            dst = g.sizes.index(g._size_of[m])
            oracles[dst].reset_game(gm, g.envs[dst]._map_index[os.path.join(g.envs[dst].microrts_path, m)])
            moves += dst != before[e]
        check_obs(obs, s)
    assert g.error_flags() == 0
    for o in oracles:
        o.close()
    g.close()
    g.moves = moves
    return g


DET_BOTS = ["coacAI", "workerRushAI", "lightRushAI", "passiveAI", "POWorkerRush", "POLightRush", "POHeavyRush", "PORangedRush"]
SEEDS = int(os.environ.get("MRTS_FUZZ_SEEDS", "12"))
FIRST = int(os.environ.get("MRTS_FUZZ_FIRST", "0"))


@pytest.mark.timeout(600)
@pytest.mark.parametrize("seed", range(FIRST, FIRST + max(1, SEEDS // 3)))
def test_fuzz_size_cycling(tmp_path, seed):
    """Random maps (tests/random_maps.py) of 2-4 random sizes, 1-2 maps per size, a random
    cycle of 3-9 entries, random initial maps (selfplay pairs sharing theirs), random
    deterministic bots, full or partial obs and short time limits, so games end and move
    between size engines many times: every env == the oracle of the size it plays in and
    parked rows stay zero (MRTS_FUZZ_SEEDS // 3 cases, as the grouped-launch fuzz)."""
    from random_maps import write_random_map

    rng = np.random.default_rng(9000 + seed)
    sizes = set()
    while len(sizes) < int(rng.integers(2, 5)):
        sizes.add((int(rng.integers(4, 25)), int(rng.integers(4, 25))))
    maps = []
    for k, (w, h) in enumerate(sorted(sizes)):
        for j in range(int(rng.integers(1, 3))):
            n = int(rng.integers(4, max(5, min(80, int(w * h * 0.5)))))
            maps.append(write_random_map(str(tmp_path / f"c{seed}_{k}_{j}.xml"), w, h, seed * 100 + k * 10 + j,
                                         n_units=min(n, w * h - 4), wall_frac=float(rng.uniform(0, 0.2))))
    cycle = [maps[int(i)] for i in rng.integers(0, len(maps), int(rng.integers(3, 10)))]
    bots = [str(b) for b in rng.choice(DET_BOTS, size=int(rng.integers(0, 5)))]
    nsp = 2 * int(rng.integers(0 if bots else 1, 3))
    init = []
    for _ in range(nsp // 2):
        init += [maps[int(rng.integers(0, len(maps)))]] * 2
    init += [maps[int(rng.integers(0, len(maps)))] for _ in bots]
    g = run_size_cycling(init, cycle, bots, nsp, 150, int(rng.integers(15, 60)), seed=seed, partial_obs=bool(rng.integers(0, 2)))
    print(f"size-cycling fuzz {seed}: sizes {g.sizes} envs {nsp + len(bots)} moves {g.moves}")
