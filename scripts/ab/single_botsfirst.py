"""EXPERIMENT: one engine holding selfplay AND bot envs (16x16, 4096 selfplay + 4096 vs
coacAI / workerRushAI / lightRushAI / randomBiasedAI), stepped by mrts_step (selfplay games
dispatched first) vs mrts_step_group with one member and MRTS_GROUP_BOTS_FIRST (bot games
first); the same bench loop (source-guided sampler + step), staggered 2000-tick pre-roll,
HIP events around the step.  Prints one line per mode."""
import ctypes
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "microrts-py_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from gym_microrts import _native, microrts_ai  # noqa: E402
from gym_microrts.envs.vec_env import MicroRTSGridModeVecEnv  # noqa: E402


def run(mode, steps=200, warm=30):
    dev = torch.device("cuda", 0)
    nsp, nbot = 4096, 4096
    bots = [microrts_ai.coacAI, microrts_ai.workerRushAI, microrts_ai.lightRushAI, microrts_ai.randomBiasedAI] * (nbot // 4)
    env = MicroRTSGridModeVecEnv(num_selfplay_envs=nsp, num_bot_envs=nbot, max_steps=2000, ai2s=bots,
                                 map_paths=["maps/16x16/basesWorkers16x16.xml"], device=dev, return_tensors=True,
                                 reward_weight=np.array([10.0, 1.0, 1.0, 0.2, 1.0, 4.0]))
    lib = _native.lib()
    n, hw = env.num_envs, env.height * env.width
    act = torch.empty((n, hw, 7), dtype=torch.int64, device=dev)
    hs = (ctypes.c_void_p * 1)(env._h)
    ev = []

    def one(s, rec=False):
        m = env.get_action_mask()
        _native.check(lib.mrts_sample_actions_src(torch.cuda.current_stream().cuda_stream, m.data_ptr(), env.source_unit_mask.data_ptr(),
                                                  n, hw, 0, 7, s, act.data_ptr()), None, "sample")
        env.step_async(act)
        if rec:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
        if mode == "natural":
            env.step_wait()
        else:
            io = (_native.StepIO * 1)(env._step_io())
            _native.check(lib.mrts_step_group(hs, 1, env._stream(), io, _native.GROUP_BOTS_FIRST), env._h, "group")
            env._tensor_outputs()
        if rec:
            b.record()
            ev.append((a, b))

    env.reset()
    bench.preroll([env], one, 2000)
    for s in range(2000, 2000 + warm):
        one(s)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for s in range(2000 + warm, 2000 + warm + steps):
        one(s, rec=(s % 4 == 0))
    torch.cuda.synchronize()
    el = time.perf_counter() - t
    step_us = np.mean([a.elapsed_time(b) for a, b in ev]) * 1e3
    assert env.error_flags() == 0
    print(f"{mode}: {n * steps / el / 1e6:.2f} M env-steps/s, step {step_us:.1f} us", flush=True)
    env.close()


for r in range(2):
    for mode in ("natural", "bots_first"):
        run(mode)
