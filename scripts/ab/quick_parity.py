"""experiment: a narrowed (16x16, 29-plane, float obs) library vs the oracle, bit for bit."""
import os, sys
import numpy as np, torch
REPO = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
for p in (REPO, os.path.join(REPO, "microrts-py_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")):
    sys.path.insert(0, p)
from conftest import MAPS
from gym_microrts import microrts_ai
from gym_microrts.envs.vec_env import MicroRTSGridModeVecEnv
from oracle_py import OracleVecEnv, sample_actions
W = np.array([10.0, 1.0, 1.0, 0.2, 1.0, 4.0])
def run(nsp, nbot, bot, steps, max_steps, seed=2024, m="maps/16x16/basesWorkers16x16.xml"):
    g = MicroRTSGridModeVecEnv(num_selfplay_envs=nsp, num_bot_envs=nbot, max_steps=max_steps, map_paths=[m],
                               ai2s=[getattr(microrts_ai, bot)] * nbot, reward_weight=W, return_tensors=True, obs_dtype=torch.float32)
    o = OracleVecEnv(nsp, nbot, [os.path.join(MAPS, m)], max_steps=max_steps, ai2s=[bot] * nbot, reward_weight=W)
    dev = g.device
    def same(gpu, host, what, s):
        assert torch.equal(gpu.int() if gpu.dtype == torch.float32 else gpu, torch.from_numpy(np.ascontiguousarray(host)).to(dev)), f"{what} differs at step {s}"
    same(g.reset(), o.reset(), "reset obs", -1)
    for s in range(steps):
        mg, mo = g.get_action_mask(), o.get_action_mask()
        same(mg, mo, "mask", s)
        a = sample_actions(mo, seed, s)
        og, rg, dg, ig = g.step(torch.from_numpy(a).to(dev))
        oo, ro, do, io = o.step(a)
        same(og, oo, "obs", s)
        same(ig._raw, np.array([i["raw_rewards"] for i in io]), "raw", s)
        same(dg, np.asarray(do, bool), "done", s)
    assert g.error_flags() == 0
    g.close(); o.close()
    print("ok", nsp, nbot, bot, steps, flush=True)
for bot in ["coacAI", "workerRushAI", "lightRushAI", "randomBiasedAI"]:
    run(0, 256, bot, 700, 600)
run(0, 64, "coacAI", 2100, 2000, m="maps/16x16/basesWorkers16x16A.xml")
run(512, 0, "passiveAI", 150, 100)
run(128, 0, "passiveAI", 300, 250, m="maps/16x16/melee16x16Mixed12.xml")
run(0, 128, "lightRushAI", 300, 250, m="maps/16x16/melee16x16Mixed12.xml")
run(0, 128, "coacAI", 300, 250, m="maps/16x16/melee16x16Mixed8.xml")
print("quick parity passed")
