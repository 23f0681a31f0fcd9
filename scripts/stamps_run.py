"""Phase stamps of the step kernel (experiment builds: `bash scripts/ab/build_variant.sh
stamps WORKTREE STAMPS=1`, mrts_engine.h MRTS_STAMPS).  Runs a bench.py workload
with the stamped library after the staggered pre-roll, and for each measured step
reads every step workgroup's phase stamps (wall_clock64, 100 MHz), then prints
per (map size, game kind) the median / p98 of each phase and the spans.

  python scripts/stamps_run.py --workload coac --envs-per-gpu 1024 [--steps 40] [--lib scripts/ab/libs/stamps.so]

Columns (µs): start = workgroup start after its launch's first; commit = state in
LDS; decode = decode + parallel issue + compactions; issue = ordered issue; cycle =
cycle + execution; tail = gameover / rewards / auto-reset; setup = the early bot's
workgroup setup; phaseA = output words; stream = phase B until the last wave's
last store; bot = bot start .. behaviours .. translate .. done; end = the
workgroup's last stamp after the launch's first start.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "microrts-py_amd"))
TICK_US = 0.01   # wall_clock64: 100 MHz


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="coac")
    ap.add_argument("--envs-per-gpu", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--preroll", type=int, default=-1)
    ap.add_argument("--max-steps", type=int, default=2000)
    ap.add_argument("--lib", default=os.path.join(REPO, "scripts", "ab", "libs", "stamps.so"))
    ap.add_argument("--json", default=None)
    ap.add_argument("--dump", default=None, help="np.save the raw stamp rows of every measured step (a list) here")
    ap.add_argument("--gap-us", type=float, default=0.0,
                    help="idle time between the sampler and the step of each measured step (synchronize + sleep)")
    ap.add_argument("--read-mb", type=int, default=0,
                    help="read a clean buffer of this size between the sampler and the step (evicts dirty cache lines)")
    a = ap.parse_args()
    from gym_microrts import _native

    _native.LIB_PATH = a.lib
    L = _native.lib()
    L.mrts_debug_stamps.restype = ctypes.c_int
    L.mrts_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    import torch

    import bench

    args = bench.parse(["--workload", a.workload, "--envs-per-gpu", str(a.envs_per_gpu), "--max-steps", str(a.max_steps),
                        "--preroll", str(a.preroll), "--no-kernel-events"])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    gap = [0.0]
    envs, one_step = build(args, dev, gap)
    for e in envs:
        e.reset()
    print(f"stamps_run: {a.workload} {a.envs_per_gpu} envs, pre-roll ...", flush=True)
    s0 = bench.preroll(envs, one_step, args.max_steps if args.preroll < 0 else args.preroll)
    print(f"stamps_run: pre-roll done ({s0} ticks)", flush=True)
    for s in range(s0, s0 + 10):
        one_step(s)
    torch.cuda.synchronize()
    rows = []
    buf = np.zeros((65536, 20), np.uint64)
    gap[0] = a.gap_us * 1e-6
    if a.read_mb:
        gap.append(torch.ones(a.read_mb << 18, dtype=torch.float32, device=dev))
    for k in range(a.steps):
        L.mrts_debug_stamps(None, 0, 1)   # zero the rows
        one_step(s0 + 10 + k)
        torch.cuda.synchronize()
        n = L.mrts_debug_stamps(buf.ctypes.data_as(ctypes.c_void_p), buf.shape[0], 0)
        assert n > 0, "no stamps: is this the STAMPS=1 library?"
        rows.append(buf[:n].copy())
    if a.dump:
        np.savez_compressed(a.dump, *rows)
    report(rows, a)


def _gap(gap):
    if len(gap) > 1:
        import torch

        torch.cuda.synchronize()
        gap[1].sum()
        torch.cuda.synchronize()
    if gap[0] > 0:
        import time

        import torch

        torch.cuda.synchronize()
        time.sleep(gap[0])


def build(args, dev, gap):
    """The bench's env + loop (bench.run_gpu / run_mixed) without its timing."""
    import numpy as np
    import torch

    import bench
    from gym_microrts import _native, microrts_ai
    from gym_microrts.envs.vec_env import MicroRTSGridModeVecEnv, MicroRTSMixedMapVecEnv

    lib = _native.lib()
    n = args.envs_per_gpu
    w = np.array([10.0, 1.0, 1.0, 0.2, 1.0, 4.0])
    if args.workload == "mixed":
        buckets = []
        for m, frac in bench.MIXED:
            nb = int(n * frac) // 4 * 4
            bots = [microrts_ai.workerRushAI] * (nb // 4) + [microrts_ai.coacAI] * (nb // 4)
            buckets.append(dict(map_paths=[m], num_selfplay_envs=nb // 2, num_bot_envs=len(bots), ai2s=bots))
        env = MicroRTSMixedMapVecEnv(buckets, max_steps=args.max_steps, device=dev, return_tensors=True, reward_weight=w)
        acts = [torch.empty((e.num_envs, e.height * e.width, 7), dtype=torch.int64, device=dev) for e in env.envs]

        def one_step(s):
            masks = env.get_action_mask()
            for e, m, ac in zip(env.envs, masks, acts):
                _native.check(bench.sample(lib, "src", m, e.source_unit_mask, e.num_envs, e.height * e.width, 0, 1, s, ac))
            _gap(gap)
            return env.step(acts)
        return env.envs, one_step
    wmap, nsp, nbot, bot, po = bench.WORKLOADS[args.workload]
    nsp = n if nsp == "all" else nsp
    nbot = n if nbot == "all" else nbot
    env = MicroRTSGridModeVecEnv(num_selfplay_envs=nsp, num_bot_envs=nbot, max_steps=args.max_steps, map_paths=[wmap],
                                 ai2s=[getattr(microrts_ai, bot)] * nbot if nbot else [], partial_obs=po, reward_weight=w,
                                 device=dev, return_tensors=True)
    hw = env.height * env.width
    act = torch.empty((n, hw, 7), dtype=torch.int64, device=dev)

    def one_step(s):
        env.get_action_mask()
        _native.check(bench.sample(lib, "src", env._mask, env._src, n, hw, 0, 1, s, act))
        _gap(gap)
        return env.step(act)
    return [env], one_step


PHASES = [("pf_issue", 2, 15), ("pf_wait", 15, 3), ("commit", 2, 3), ("decode", 3, 4), ("issue", 4, 5), ("cycle", 5, 6), ("tail", 6, 7)]


def report(steps, a):
    out = {"workload": a.workload, "envs": a.envs_per_gpu, "steps": len(steps), "groups": {}}
    acc = {}
    for r in steps:
        r = r[r[:, 2] > 0]   # rows of workgroups that ran this step
        hw = (r[:, 0] >> np.uint64(32)).astype(np.int64)
        kind = r[:, 1].astype(np.int64)
        t = r.astype(np.float64)
        # launches: the step call's launches run back to back; a row belongs to the launch
        # whose members include its map size (mixed: 24x24 alone, the rest together)
        launch = (hw == 576).astype(np.int64) if a.workload == "mixed" else np.zeros_like(hw)
        for ln in np.unique(launch):
            sel = launch == ln
            t0 = t[sel, 2].min()
            for key in set(zip(hw[sel], kind[sel] & 1)):
                m = sel & (hw == key[0]) & ((kind & 1) == key[1])
                g = acc.setdefault(f"{int(key[0])}{'_bot' if key[1] else '_selfplay'}", {})
                tt = t[m]
                first = (tt[:, 2] - t0) * TICK_US < 2.0
                ok = (tt[:, 3] > 0)
                g.setdefault("commit_first_round", []).extend((tt[first & ok, 3] - tt[first & ok, 2]) * TICK_US)
                g.setdefault("commit_later", []).extend((tt[~first & ok, 3] - tt[~first & ok, 2]) * TICK_US)
                def d(i, j):
                    ok = (tt[:, i] > 0) & (tt[:, j] > 0)
                    return (tt[ok, j] - tt[ok, i]) * TICK_US
                g.setdefault("start", []).extend((tt[:, 2] - t0) * TICK_US)
                for name, i, j in PHASES:
                    g.setdefault(name, []).extend(d(i, j))
                early = tt[:, 14] > 0
                g.setdefault("setup", []).extend((tt[early, 14] - tt[early, 7]) * TICK_US)
                a_from = np.where(tt[:, 14] > 0, tt[:, 14], tt[:, 7])
                okA = tt[:, 8] > 0
                g.setdefault("phaseA", []).extend((tt[okA, 8] - a_from[okA]) * TICK_US)
                g.setdefault("stream", []).extend(d(8, 9))
                g.setdefault("bot_setup", []).extend(d(7, 10))
                g.setdefault("behaviours", []).extend(d(10, 11))
                g.setdefault("translate", []).extend(d(11, 12))
                g.setdefault("bot_total", []).extend(d(7, 13))
                last = tt[:, 2:].max(axis=1)
                g.setdefault("end", []).extend((last - t0) * TICK_US)
                g.setdefault("logic", []).extend(d(2, 7))
                # the slowest 2 % of this step's workgroups (by end): their phases, side by side
                endv = (last - t0) * TICK_US
                cut = np.percentile(endv, 98)
                sl = tt[endv >= cut]
                def ds(i, j):
                    ok = (sl[:, i] > 0) & (sl[:, j] > 0)
                    return list((sl[ok, j] - sl[ok, i]) * TICK_US)
                g.setdefault("slow2_end", []).extend(endv[endv >= cut])
                g.setdefault("slow2_start", []).extend((sl[:, 2] - t0) * TICK_US)
                g.setdefault("slow2_logic", []).extend(ds(2, 7))
                g.setdefault("slow2_bot_setup", []).extend(ds(7, 10))
                g.setdefault("slow2_behaviours", []).extend(ds(10, 11))
                g.setdefault("slow2_translate", []).extend(ds(11, 12))
                g.setdefault("slow2_bot_total", []).extend(ds(7, 13))
                g.setdefault("slow2_stream", []).extend(ds(8, 9))
                # bot counters (fused bot games): executed translate entries, path searches,
                # their summed time (us) and four-layer rounds
                if r.shape[1] >= 20:
                    bot = tt[:, 7] > 0
                    for nm, col, scale in (("entries", 16, 1), ("searches", 17, 1), ("search_us", 18, TICK_US), ("rounds", 19, 1)):
                        g.setdefault("bot_" + nm, []).extend(tt[bot, col] * scale)
                        g.setdefault("slow2_bot_" + nm, []).extend(sl[sl[:, 7] > 0, col] * scale)
    for k, g in sorted(acc.items()):
        row = {}
        for name, v in g.items():
            v = np.asarray(v)
            if v.size:
                row[name] = {"median": round(float(np.median(v)), 2), "p98": round(float(np.percentile(v, 98)), 2),
                             "max": round(float(v.max()), 2), "n": int(v.size)}
        out["groups"][k] = row
        print(f"== {k}")
        for name, s in row.items():
            print(f"  {name:11s} median {s['median']:7.2f}  p98 {s['p98']:7.2f}  max {s['max']:7.2f}  (n {s['n']})")
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
