"""experiment: headline k_step (8192 selfplay envs) per-workgroup timeline from stamps:
0 start, 11 decoded, 1 issued, 2 executed (store), 9 end (after the output stream)."""
import ctypes, os, sys, json
import numpy as np, torch
REPO = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "microrts-py_amd"))
import bench
from gym_microrts import _native
from gym_microrts.envs.vec_env import MicroRTSGridModeVecEnv
n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
dev = torch.device("cuda", 0)
env = MicroRTSGridModeVecEnv(n, 0, max_steps=2000, map_paths=[bench.MAP], reward_weight=np.array([10.0, 1.0, 1.0, 0.2, 1.0, 4.0]),
                             device=dev, return_tensors=True)
lib = _native.lib()
lib.mrts_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
act = torch.empty((n, 256, 7), dtype=torch.int64, device=dev)
def one(s):
    env.get_action_mask()
    bench.sample(lib, "src", env._mask, env._src, n, 256, 0, 1, s, act)
    env.step(act)
env.reset()
s0 = bench.preroll([env], one, 2000)
G = n // 2
buf = np.zeros((G, 12), np.uint64)
acc = []
for s in range(s0, s0 + 30):
    one(s)
    torch.cuda.synchronize()
    lib.mrts_debug_stamps(buf.ctypes.data, G)
    b = buf.astype(np.int64)
    acc.append(b - b[:, 0].min())
a = np.stack(acc) / 100.0   # us (100 MHz)
start, logic, end = a[:, :, 0], a[:, :, 2], a[:, :, 9]
span = end.max(1)
per_game_bytes = 948428800 / 4096
out = {"span_us": float(span.mean()), "game_start_us": {q: float(np.percentile(start, q)) for q in (0, 25, 50, 75, 90, 100)},
       "logic_us (start->stored)": {q: float(np.percentile(logic - start, q)) for q in (10, 50, 90, 99)},
       "stream_us (stored->end)": {q: float(np.percentile(end - logic, q)) for q in (10, 50, 90, 99)},
       "first_stream_start_us": float((logic.min(1)).mean()), "last_start_us": float(start.max(1).mean())}
# bandwidth over time: each game writes its bytes uniformly over [logic, end]
bins = np.arange(0, span.max() + 2, 2.0)
bw = np.zeros(len(bins) - 1)
for st in range(a.shape[0]):
    for lo, hi in zip(logic[st], end[st]):
        w = np.clip(np.minimum(bins[1:], hi) - np.maximum(bins[:-1], lo), 0, None)
        bw += w / max(hi - lo, 1e-3) * per_game_bytes
bw /= a.shape[0]
out["write_GBps_per_2us_bin"] = [round(x / 2e-6 / 1e9) for x in bw]
conc = []
for t in bins[:-1]:
    conc.append(float(((logic <= t) & (end > t)).sum(1).mean()))
out["games_streaming_per_bin"] = [round(c) for c in conc]
conc2 = [float(((start <= t) & (logic > t)).sum(1).mean()) for t in bins[:-1]]
out["games_in_logic_per_bin"] = [round(c) for c in conc2]
print(json.dumps(out))
