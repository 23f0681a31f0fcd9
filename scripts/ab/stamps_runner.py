import ctypes, os, sys, json
import numpy as np, torch
REPO = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "microrts-py_amd"))
import bench
from gym_microrts import _native, microrts_ai
from gym_microrts.envs.vec_env import MicroRTSGridModeVecEnv
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
bot = sys.argv[2] if len(sys.argv) > 2 else "coacAI"
dev = torch.device("cuda", 0)
env = MicroRTSGridModeVecEnv(0, n, max_steps=2000, map_paths=[bench.MAP], ai2s=[getattr(microrts_ai, bot)] * n,
                             reward_weight=np.array([10.0, 1.0, 1.0, 0.2, 1.0, 4.0]), device=dev, return_tensors=True)
lib = _native.lib()
lib.mrts_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
act = torch.empty((n, 256, 7), dtype=torch.int64, device=dev)
def one(s):
    m = env.get_action_mask()
    bench.sample(lib, "src", env._mask, env._src, n, 256, 0, 1, s, act)
    env.step(act)
env.reset()
s0 = bench.preroll([env], one, 2000)
buf = np.zeros((n, 12), np.uint64)
acc = []
for s in range(s0, s0 + 40):
    one(s)
    torch.cuda.synchronize()
    lib.mrts_debug_stamps(buf.ctypes.data, n)
    b = buf.astype(np.int64)
    t0 = b[:, 0].min()
    acc.append(b - t0)
a = np.stack(acc)  # steps, games, 8 (100 MHz ticks -> 10 ns)
names = ["start", "issued", "executed->store", "bot start", "bot setup done", "behaviours done", "translate done", "stream done"]
end = np.maximum(a[:, :, 6], a[:, :, 7])
print("kernel span us (mean over steps):", float((end.max(1)).mean()) / 100)
for k in range(8):
    print(f"{names[k]:24s} median {np.median(a[:, :, k]) / 100:7.2f} us  p90 {np.percentile(a[:, :, k], 90) / 100:7.2f}  max {a[:, :, k].max(1).mean() / 100:7.2f}")
names += ["bot: ws+reservations", "bot: unit list", "bot: free rows", "decode"]
d = lambda i, j: (a[:, :, j] - a[:, :, i]) / 100
for i, j, nm in [(0, 11, "load+decode"), (11, 1, "issue"), (3, 8, "bot ws+resv"), (8, 9, "bot unitlist"), (9, 10, "bot freerows"), (10, 4, "bot enemy table"), (0, 1, "decode+issue"), (1, 2, "cycle+rewards+reset"), (2, 3, "store+sync"), (3, 4, "bot setup"), (4, 5, "behaviours"),
                 (5, 6, "translate"), (2, 7, "store+phaseA+stream")]:
    x = d(i, j)
    print(f"{nm:22s} median {np.median(x):6.2f} us  p90 {np.percentile(x, 90):6.2f}  max {x.max():6.2f}")
# the slowest 2% games per step: mean phase durations
span = end
sel = span >= np.percentile(span, 98, axis=1, keepdims=True)
print("slowest 2% games (mean us):")
for i, j, nm in [(0, 11, "load+decode"), (11, 1, "issue"), (1, 2, "cycle.."), (2, 3, "store+sync"), (3, 4, "bot setup"), (4, 5, "behaviours"), (5, 6, "translate"), (2, 7, "stream")]:
    print(f"   {nm:16s} {float(d(i, j)[sel].mean()):6.2f}   (all games {float(d(i, j).mean()):6.2f})")
st = env.game_stats()
print("units proxy: mean game time", st[:, 0].mean())
