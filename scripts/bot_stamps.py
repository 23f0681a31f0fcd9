"""Per-phase cycle counts of k_bot from an MRTS_EXP_STAMPS build (experiment tooling).

  python scripts/bot_stamps.py scripts/_exp/lib_stamps.so [envs]     (on the GPU box)

Phases: 0 load, 1 visibility / hiding, 2 reservations + unit list, 3 free rows,
4 behaviours (trains, melee, workers), 5 translateActions, 6 write-back (shader-clock deltas
of the last step, median / p90 over bot games)."""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "microrts-py_amd"))


def main(lib_path, envs=1024):
    import torch

    from gym_microrts import _native, microrts_ai
    from gym_microrts.envs.vec_env import MicroRTSGridModeVecEnv

    _native.LIB_PATH = lib_path
    env = MicroRTSGridModeVecEnv(num_selfplay_envs=0, num_bot_envs=envs, max_steps=2000, ai2s=[microrts_ai.coacAI] * envs,
                                 map_paths=["maps/16x16/basesWorkers16x16.xml"], return_tensors=True)
    lib = _native.lib()
    act = torch.empty((envs, 256, 7), dtype=torch.int64, device="cuda")
    env.reset()
    st = torch.cuda.current_stream().cuda_stream
    for s in range(200):
        m = env.get_action_mask()
        lib.mrts_sample_actions_src(ctypes.c_void_p(st), ctypes.c_void_p(m.data_ptr()), ctypes.c_void_p(env.source_unit_mask.data_ptr()),
                                    envs, 256, ctypes.c_uint64(3), s, ctypes.c_void_p(act.data_ptr()))
        env.step(act)
    torch.cuda.synchronize()
    out = np.zeros((envs, 8), np.uint64)
    f = lib.mrts_exp_bot_stamps
    f.argtypes = [ctypes.c_void_p, ctypes.c_int]
    n = f(out.ctypes.data, envs)
    d = np.diff(out[:n, :7].astype(np.int64), axis=1)
    tot = out[:n, 6].astype(np.int64) - out[:n, 0].astype(np.int64)
    names = ["load", "vis", "resv+list", "frow", "behaviours", "translate"]
    for k, nm in enumerate(names):
        print(f"{nm:12s} median {int(np.median(d[:, k])):8d}  p90 {int(np.percentile(d[:, k], 90)):8d}")
    print(f"{'total':12s} median {int(np.median(tot)):8d}  p90 {int(np.percentile(tot, 90)):8d}  (s_memtime = shader clock cycles)")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 1024)
