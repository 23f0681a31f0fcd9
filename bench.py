"""Throughput benchmark of the MI355X MicroRTS engine (BASELINE.json metric).

One "step" = one env-step of every env: get_action_mask() + device random
masked-action sampler (hello_world.py:27-64 semantics) + step(), exactly the
per-step API traffic of the reference rollout loop.  Workload:
16x16 basesWorkers, 8192 envs per GPU (4096 selfplay games, random vs random),
max_steps 2000, auto-reset on, inputs already resident in HBM.

  python bench.py [--gpus N --steps K --warmup W]
  N>1: either under a launcher (python -m torch.distributed.run --nproc-per-node N
       ... bench.py --gpus N: WORLD_SIZE must equal N), or plain `bench.py --gpus N`,
       which starts the N ranks itself as child processes (launch_ranks) before
       anything in the parent touches torch or HIP, relays rank 0's line and exits
       with the worst child status.
Each rank owns an independent contiguous shard of envs (no data-path
collective: envs never interact); the only communication is the timing
barrier and the max-over-ranks of the elapsed time.

Rank 0 prints one JSON line.  The timed region carries no HIP events;
`roofline` prices the dominant kernel from a separate pass of --roofline-steps
(>= 64) steps right after it, with HIP events around every launch of every step
(`roofline.samples` launches); `cpu_baseline` times the CPU restatement
(oracle/, OpenMP over games) on a bounded sample of the same workload (rank 0,
N=1 only).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "microrts-py_amd"))

METRIC = "env-steps/sec (whole node), 16x16 basesWorkers @8192 envs; bit-exact vs Java"
MAP = "maps/16x16/basesWorkers16x16.xml"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--envs-per-gpu", type=int, default=8192)
    ap.add_argument("--max-steps", type=int, default=2000)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--seeds", type=int, default=1,
                    help="independent runs with seeds seed, seed+1, ... (fresh env, pre-roll, warmup and K timed steps "
                         "each); the line reports the median run (BASELINE.md §3: median of 3 seeds) and every seed's value")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-events", action="store_true",
                    help="skip the event-timed roofline pass (no roofline / kernels in the line)")
    ap.add_argument("--roofline-steps", type=int, default=64,
                    help="steps of the event-timed pass after the timed window (HIP events around every launch)")
    ap.add_argument("--bot-fusion", type=int, default=1, choices=[0, 1],
                    help="mrts_set_bot_fusion: 0 k_bot at every step, 1 k_step decides the next tick's bot actions")
    ap.add_argument("--api", default="tensor", choices=["tensor", "numpy", "sharedmem"],
                    help="numpy: the reference's host contract (numpy obs / masks / rewards out, host int64 actions in), "
                         "i.e. the PCIe-inclusive rate; sharedmem: the same through MicroRTSGridModeSharedMemVecEnv's "
                         "page-locked buffers; tensor: device tensors (the headline)")
    ap.add_argument("--no-eager-masks", action="store_true",
                    help="get_action_mask() launches k_masks instead of k_step writing the next tick's masks")
    ap.add_argument("--sampler", default="src", choices=["src", "dense"],
                    help="src: mrts_sample_actions_src (reads the mask rows of source cells only); dense: every row")
    ap.add_argument("--workload", default="selfplay", choices=sorted(WORKLOADS),
                    help="selfplay = the BASELINE metric; the others are the secondary BASELINE.json configs")
    ap.add_argument("--preroll", type=int, default=-1,
                    help="untimed ticks played before --warmup with staggered game resets, so the timed window sees "
                         "games at every phase of an episode (mid-game states, gameovers, auto-resets); "
                         "-1 = max_steps, 0 = off (every game starts fresh at the first warmup step)")
    ap.add_argument("--dist-backend", default="gloo", choices=["nccl", "gloo"],
                    help="process group of the timing barrier / max-over-ranks / per-rank gather.  gloo (default): on "
                         "the host -- the env shards exchange no data, so nothing on the data path needs RCCL and an RCCL "
                         "init or topology problem cannot cost the scaling curve; nccl = RCCL over xGMI (each rank "
                         "synchronises its own device first either way)")
    ap.add_argument("--rank-timeout", type=float, default=None,
                    help="seconds: a self-launched parent terminates every rank and exits 124 when they have not all "
                         "exited by then (or STRAGGLE_S after rank 0 exited); each rank also exits 124 by itself "
                         "after this long, so a hang under an external launcher ends too.  Default: derived from the "
                         "requested work (rank_deadline: 900 s + 50 ms per pre-roll / warm-up / timed tick per seed, "
                         "about 100x the real tick time); the value in force is in the line's window.rank_timeout_s. "
                         "A longer run than that needs a larger value, or 0 = no deadline")
    ap.add_argument("--bucket-streams", type=int, default=0, choices=[0, 1],
                    help="mixed workload: 1 = each size bucket on its own HIP stream (concurrent), 0 = back to back")
    ap.add_argument("--group-policy", default="default",
                    help="mixed workload: the buckets' steps in one mrts_step_group call with this policy "
                         "(MRTS_GROUP_* bits, include/microrts_amd.h; default = merge-fit | bots-first), "
                         "or 'none' = one step launch per bucket")
    ap.add_argument("--sampler-group", type=int, default=1, choices=[0, 1],
                    help="mixed workload, src sampler: 1 = every bucket's actions in one "
                         "mrts_sample_actions_src_group launch, 0 = one launch per bucket (same actions)")
    ap.add_argument("--dump", default=None,
                    help="save each rank's final obs / masks / raw rewards / dones to DUMP.rank<r>.npz (shard tests)")
    a = ap.parse_args(argv)
    if a.rank_timeout is None:
        a.rank_timeout = rank_deadline(a)
    return a


def rank_deadline(a):
    """--rank-timeout's default: 900 s of start-up (torch import, rendezvous, env build,
    the CPU-side cpu_baseline is rank 0 at N=1 only) plus 50 ms per tick the run asks
    for -- pre-roll (max_steps by default), warm-up and timed steps, for every seed.
    A tick takes about 0.2-0.5 ms, so only a hang reaches it."""
    pre = a.max_steps if a.preroll < 0 else a.preroll
    return 900.0 + 0.05 * max(1, a.seeds) * (pre + a.warmup + a.steps)


# BASELINE.json configs as bench workloads: (map, selfplay envs, bot envs, bot, partial_obs).
# The headline metric is "selfplay" (8192 envs / GPU of 16x16 basesWorkers).
WORKLOADS = {
    "selfplay": (MAP, "all", 0, None, False),
    "coac": (MAP, 0, "all", "coacAI", False),          # configs[1]: envs vs device-side coacAI
    "passive": (MAP, 0, "all", "passiveAI", False),    # envs vs passiveAI
    "workerrush": (MAP, 0, "all", "workerRushAI", False),
    "partial_obs": (MAP, "all", 0, None, True),       # configs[3]: partial_obs=True, 31 planes
    "8x8": ("maps/8x8/basesWorkers8x8.xml", "all", 0, None, False),
    "24x24": ("maps/24x24/basesWorkers24x24.xml", "all", 0, None, False),
    "mixed": (None, None, None, None, False),           # configs[4]: 8x8 / 16x16 / 24x24 buckets, bots + selfplay
}

# configs[4]: mixed sizes bucketed in one batch; per bucket (map, selfplay envs, bot envs per bot kind)
MIXED = [("maps/8x8/basesWorkers8x8.xml", 0.25), ("maps/16x16/basesWorkers16x16.xml", 0.5),
         ("maps/24x24/basesWorkers24x24.xml", 0.25)]


def stagger_plan(G, ticks, game0=0, G_total=None):
    """Global game g of G_total is reset at pre-roll tick floor(g * ticks / G_total):
    after `ticks` ticks the games' episode ages spread evenly over (0, ticks]
    (time-limit resets then fall at every tick of the timed window, not all at
    once).  A shard holds global games [game0, game0 + G); returns its local
    indices per tick, so shards reset exactly the games one unsharded run would."""
    G_total = G if G_total is None else G_total
    plan = [[] for _ in range(ticks)]
    if ticks <= 0:
        return plan
    for g in range(G):
        plan[(game0 + g) * ticks // G_total].append(g)
    return plan


def preroll(envs, one_step, ticks, rank=0, world=1):
    """`ticks` untimed steps of the bench loop; each env resets its share of games
    at staggered ticks (stagger_plan; every rank holds an equal slice of the global
    games).  Returns the number of ticks played."""
    plans = [stagger_plan(e._n_games(), ticks, rank * e._n_games(), world * e._n_games()) for e in envs]
    for s in range(ticks):
        one_step(s)
        for e, plan in zip(envs, plans):
            e.reset_games(plan[s])
    return ticks


def window_stats(before, after, steps):
    """What the timed window covered, from mrts_game_stats before / after it:
    episode phase (game time) at its start and end, auto-resets, and the serial
    one-lane work (ordered execution ticks, ordered-path issue rows)."""
    import numpy as np

    b, a = np.concatenate(before), np.concatenate(after)
    G = a.shape[0]
    return {"games": int(G),
            "game_tick_start": {"min": int(b[:, 0].min()), "mean": round(float(b[:, 0].mean()), 1), "max": int(b[:, 0].max())},
            "game_tick_end": {"min": int(a[:, 0].min()), "mean": round(float(a[:, 0].mean()), 1), "max": int(a[:, 0].max())},
            "auto_resets": int((a[:, 5] - b[:, 5]).sum()),
            "serial_exec_games_per_step": round(float((a[:, 3] - b[:, 3]).sum()) / steps, 1),
            "ordered_issue_rows_per_step": round(float((a[:, 4] - b[:, 4]).sum()) / steps, 1)}


def roofline_pass(args, one_step, timing, s1):
    """The event-timed pass priced by `roofline`: --roofline-steps more steps of the
    same loop right after the timed window (which itself records no events), with
    HIP events around every launch of every step."""
    import torch

    if args.no_kernel_events or args.roofline_steps <= 0:
        return
    timing[0] = True
    for s in range(s1, s1 + args.roofline_steps):
        one_step(s)
    torch.cuda.synchronize()
    timing[0] = False


def run_mixed(args, rank, world, dev):
    """BASELINE configs[4]: one MicroRTSMixedMapVecEnv with an 8x8, a 16x16 and a 24x24
    bucket, each half selfplay envs, a quarter vs device workerRushAI, a quarter vs
    device coacAI; envs_per_gpu split 1:2:1 over the buckets."""
    import numpy as np
    import torch

    from gym_microrts import _native, microrts_ai
    from gym_microrts.envs.vec_env import MicroRTSMixedMapVecEnv

    n = args.envs_per_gpu
    buckets = []
    for m, frac in MIXED:
        nb = int(n * frac) // 4 * 4
        bots = [microrts_ai.workerRushAI] * (nb // 4) + [microrts_ai.coacAI] * (nb // 4)
        buckets.append(dict(map_paths=[m], num_selfplay_envs=nb // 2, num_bot_envs=len(bots), ai2s=bots))
    gp = args.group_policy
    gp = None if gp == "none" else gp if gp == "default" else int(gp)
    env = MicroRTSMixedMapVecEnv(buckets, concurrent=bool(args.bucket_streams), group_policy=gp, max_steps=args.max_steps, device=dev,
                                 return_tensors=True,
                                 reward_weight=np.array([10.0, 1.0, 1.0, 0.2, 1.0, 4.0]), eager_masks=not args.no_eager_masks)
    lib = _native.lib()
    acts = [torch.empty((e.num_envs, e.height * e.width, 7), dtype=torch.int64, device=dev) for e in env.envs]
    seed = args.seed
    ev = {}
    timing = [False]

    # the stand-in policy over every bucket in one launch (mrts_sample_actions_src_group:
    # each bucket's actions are those of its own mrts_sample_actions_src call)
    grouped_sampler = bool(args.sampler_group) and args.sampler == "src" and len(env.envs) <= _native.SAMPLE_GROUP_MAX

    def one_step(s):
        masks = env.get_action_mask()
        rec = timing[0]
        for e in env.envs:
            e.kernel_events = ev.setdefault(e.height, {}) if rec else None
        if grouped_sampler:
            if rec:
                s0e, s1e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s0e.record()
            segs = (_native.SampleSeg * len(env.envs))(*[
                _native.SampleSeg(m.data_ptr(), e.source_unit_mask.data_ptr(), e.num_envs, e.height * e.width, rank * e.num_envs,
                                  a.data_ptr()) for e, m, a in zip(env.envs, masks, acts)])
            _native.check(lib.mrts_sample_actions_src_group(torch.cuda.current_stream().cuda_stream, segs, len(env.envs), seed, s),
                          None, "sample_group")
            if rec:
                s1e.record()
                ev.setdefault("sample", []).append((s0e, s1e))
        else:
            for e, m, a in zip(env.envs, masks, acts):
                _native.check(sample(lib, args.sampler, m, e.source_unit_mask, e.num_envs, e.height * e.width, rank * e.num_envs,
                                     seed, s, a), None, "sample")
        if not rec:
            return env.step(acts)
        # the buckets' step kernels run concurrently: time them together too
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = env.step(acts)
        e1.record()
        ev.setdefault("all", []).append((e0, e1))
        return out

    env.reset()
    s0 = preroll(env.envs, one_step, args.max_steps if args.preroll < 0 else args.preroll, rank, world)
    for s in range(s0, s0 + args.warmup):
        one_step(s)
    torch.cuda.synchronize()
    before = [e.game_stats() for e in env.envs]
    barrier(world, dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(s0 + args.warmup, s0 + args.warmup + args.steps):
        one_step(s)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    barrier(world, dev)
    after = [e.game_stats() for e in env.envs]
    roofline_pass(args, one_step, timing, s0 + args.warmup + args.steps)
    for e in env.envs:
        e.kernel_events = None
    # per bucket: mean step-kernel launch time and its algorithmic bytes
    buckets = []
    for e in env.envs:
        hw, G = e.height * e.width, e._n_games()
        kb = kernel_bytes(G, e.num_envs, hw, sum(e.num_planes))
        k = {name: float(np.mean([a.elapsed_time(b) for a, b in v])) for name, v in ev.get(e.height, {}).items()}
        buckets.append({"map": f"{e.height}x{e.width}", "envs": e.num_envs, "games": G, "step_ms": k.get("step"),
                        "step_bytes": kb["step"]})
    stats = window_stats(before, after, args.steps)
    stats["buckets"] = buckets
    stats["roofline_samples"] = len(ev.get("all", []))
    stats["buckets_concurrent"] = env.concurrent
    stats["group_policy"] = env.group_policy if env.grouped else None
    stats["bucket_launch"], stats["launches_per_step"] = env.launch_plan()
    stats["sampler_launches_per_step"] = 1 if grouped_sampler else len(env.envs)
    if ev.get("all"):
        stats["step_all_buckets_ms"] = float(np.mean([a.elapsed_time(b) for a, b in ev["all"]]))
    if ev.get("sample"):   # the grouped sampler: source read + actions written + the source rows' mask rows
        src = sum(int(e.source_unit_mask.sum().item()) for e in env.envs)
        sb = sum(e.num_envs * e.height * e.width * (4 + 7 * 8) for e in env.envs) + src * 78 * 4
        sms = float(np.mean([a.elapsed_time(b) for a, b in ev["sample"]]))
        stats["sampler_group"] = {"avg_ms": round(sms, 4), "bytes": sb, "gbs": round(sb / (sms * 1e-3) / 1e9, 1)}
    return elapsed, {}, env.error_flags(), 256, sum(e._n_games() for e in env.envs), env.num_envs, 29, 0, stats


WORKLOAD_DESC = {
    "selfplay": "16x16 basesWorkers selfplay, random masked actions (device Philox sampler), get_action_mask+sample+step per env-step",
    "coac": "16x16 basesWorkers, every env vs device coacAI (k_bot), random masked agent actions",
    "passive": "16x16 basesWorkers, every env vs passiveAI, random masked agent actions",
    "workerrush": "16x16 basesWorkers, every env vs device workerRushAI (k_bot), random masked agent actions",
    "partial_obs": "16x16 basesWorkers selfplay, partial_obs=True (31 planes), random masked actions",
    "8x8": "8x8 basesWorkers selfplay, random masked actions",
    "24x24": "24x24 basesWorkers selfplay, random masked actions",
    "mixed": "8x8 / 16x16 / 24x24 basesWorkers buckets (1:2:1) in one batch, each half selfplay, a quarter vs "
             "device workerRushAI, a quarter vs device coacAI; random masked agent actions",
}


def sample(lib, kind, mask, source, n, hw, env0, seed, step, act):
    """The bench's stand-in policy: a uniform pick among the valid entries of
    every component of every cell (hello_world.py:27-64), on the device; env0 =
    the global index of the shard's first env (Philox counter)."""
    import torch

    st = torch.cuda.current_stream().cuda_stream
    if kind == "src":
        return lib.mrts_sample_actions_src(st, mask.data_ptr(), source.data_ptr(), n, hw, env0, seed, step, act.data_ptr())
    return lib.mrts_sample_actions(st, mask.data_ptr(), n, hw, env0, seed, step, act.data_ptr())


def shard(rank, n, nsp, nbot):
    """rank r owns global envs [r*n, (r+1)*n) of one batch of world*n envs: its
    selfplay envs / bot envs are that slice of the global selfplay / bot envs.
    Returns (env0, game_offset): the sampler's global env index of the shard's
    first env and the global index of its first game (bot RNG streams), so
    shard r plays exactly the games of that slice of one unsharded run.  n even:
    selfplay pairs never straddle ranks."""
    assert n % 2 == 0, "envs per GPU must be even (selfplay pairs)"
    assert nsp == 0 or nbot == 0, "a shard is all selfplay or all bot envs"
    return rank * n, rank * (nsp // 2 + nbot)


def kernel_bytes(G, N, HW, P=29, eager=True, sampler="src", src_rows=0):
    """Algorithmic bytes per launch.
    masks: game state read (16 B/cell/game) + mask write (78*4 B/cell/env) + source write (4 B/cell/env).
    step : game state read+write (32 B/cell/game) + source read (4 B/cell/env) + obs write (4P B/cell/env)
           + raw reward (48 B/env) + done (6 B/env) + fused reward / done0 (9 B/env); action rows (56 B
           per acting unit) not counted.  Eager masks: + the next tick's mask and source writes.
    sample: dense -- every mask row read + actions written; src -- source read, the mask rows of
           `src_rows` source cells read, actions written."""
    masks = N * HW * (78 * 4 + 4)
    step = G * HW * 32 + N * HW * (4 + 4 * P) + N * (48 + 6 + 8 + 1) + (masks if eager else 0)
    if sampler == "dense":
        samp = N * HW * (78 * 4 + 7 * 8)
    else:
        samp = N * HW * (4 + 7 * 8) + src_rows * 78 * 4
    return {"get_masks": G * HW * 16 + masks, "step": step, "sample": samp}


# rocprofv3 kernel names -> bench kernel names
PMC_NAMES = {"get_masks": "k_masks", "step": "k_step", "sample": "k_sample"}


LIB = os.path.join(REPO, "microrts-py_amd", "gym_microrts", "libmicrorts_amd.so")


def lib_sha256():
    import hashlib

    h = hashlib.sha256()
    with open(LIB, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


def pmc_traffic(kernel, workload):
    """HBM bytes per launch of `kernel` from the committed PMC summary
    (profiles/pmc_latest.json, written by scripts/pmc_summary.py from separate
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this bench command, filed
    under `workload` = <workload>@<envs per gpu>).  Only counters of THIS build
    count: the summary's library sha256 must equal the running library's, else
    (None, reason)."""
    path = os.path.join(REPO, "profiles", "pmc_latest.json")
    if not os.path.exists(path):
        return None, "no profiles/pmc_latest.json"
    d = json.load(open(path))
    if d.get("_meta", {}).get("lib_sha256") != lib_sha256():
        return None, "profiles/pmc_latest.json is of another build (lib sha256 differs): traffic not reported"
    w = d.get("workloads", {}).get(workload)
    if not w:
        return None, f"no PMC passes for {workload} in profiles/pmc_latest.json"
    for k, v in w["kernels"].items():
        if k.startswith(PMC_NAMES.get(kernel, "?")) and v.get("hbm_bytes"):
            return v["hbm_bytes"], f"profiles/pmc_latest.json [{workload}] {k}, lib sha256 {d['_meta']['lib_sha256'][:12]}"
    return None, f"no {kernel} counters for {workload}"


def run_gpu(args, rank, world, local_rank):
    import numpy as np
    import torch

    from gym_microrts import _native
    from gym_microrts.envs.vec_env import MicroRTSGridModeVecEnv

    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)
    n = args.envs_per_gpu
    from gym_microrts import microrts_ai

    wmap, nsp, nbot, bot, po = WORKLOADS[args.workload]
    nsp = n if nsp == "all" else nsp
    nbot = n if nbot == "all" else nbot
    env0, game_offset = shard(rank, n, nsp, nbot)
    if args.api == "sharedmem":
        from gym_microrts.envs.vec_env import MicroRTSGridModeSharedMemVecEnv as Env
        extra = {}
    else:
        Env = MicroRTSGridModeVecEnv
        extra = dict(return_tensors=args.api == "tensor", eager_masks=not args.no_eager_masks,
                     bot_fusion=args.bot_fusion, game_offset=game_offset)
    env = Env(num_selfplay_envs=nsp, num_bot_envs=nbot, max_steps=args.max_steps, map_paths=[wmap],
              ai2s=[getattr(microrts_ai, bot)] * nbot if nbot else [], partial_obs=po,
              reward_weight=np.array([10.0, 1.0, 1.0, 0.2, 1.0, 4.0]), device=dev, **extra)
    hw = env.height * env.width
    act = torch.empty((n, hw, 7), dtype=torch.int64, device=dev)
    act_host = torch.empty((n, hw, 7), dtype=torch.int64, pin_memory=True) if args.api != "tensor" else None
    lib = _native.lib()
    seed = args.seed   # one stream over global env indices: rank r samples envs [env0, env0 + n)
    ev = {}

    def one_step(s):
        # HIP events around every launch, in the roofline pass only (each event is a
        # queue packet between dependent kernels: ~7 % of the step, kept out of the
        # timed window)
        env.kernel_events = ev if timing[0] else None
        m = env.get_action_mask()   # numpy api: the (N, HW, 78) host copy ppo_gridnet.py:466 makes
        if env.kernel_events is not None:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        rc = sample(lib, args.sampler, env._mask, env._src, n, hw, env0, seed, s, act)
        if env.kernel_events is not None:
            e1.record()
            env.kernel_events.setdefault("sample", []).append((e0, e1))
        _native.check(rc, None, "sample")
        if args.api != "tensor":   # ppo_gridnet.py:475: host int64 actions (N, HW*7)
            # the stand-in policy's action.cpu(): into a page-locked buffer (the driver's
            # choice; a fresh pageable array would add first-touch faults + a staged copy
            # that are the driver's cost, not the env's), synchronous like .cpu()
            act_host.copy_(act, non_blocking=True)
            torch.cuda.current_stream().synchronize()
            return env.step(act_host.numpy().reshape(n, -1))
        return env.step(act)

    timing = [False]
    env.reset()
    s0 = preroll([env], one_step, args.max_steps if args.preroll < 0 else args.preroll, rank, world)
    for s in range(s0, s0 + args.warmup):
        one_step(s)
    torch.cuda.synchronize()
    before = [env.game_stats()]
    barrier(world, dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(s0 + args.warmup, s0 + args.warmup + args.steps):
        obs, rew, done, infos = one_step(s)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier(world, dev)
    elapsed = t1 - t0
    stats = window_stats(before, [env.game_stats()], args.steps)
    stats["preroll_ticks"] = s0
    if args.dump:
        np.savez(f"{args.dump}.rank{rank}.npz", obs=obs.cpu().numpy(), mask=env._mask.cpu().numpy(),
                 src=env._src.cpu().numpy(), raw=env._raw.cpu().numpy(), done=env._done.cpu().numpy(),
                 stats=env.game_stats(), env0=env0)
    roofline_pass(args, one_step, timing, s0 + args.warmup + args.steps)
    env.kernel_events = None
    stats["roofline_samples"] = len(ev.get("step", []))
    flags = env.error_flags()
    kern = {k: float(np.mean([a.elapsed_time(b) for a, b in v])) for k, v in ev.items()}  # ms per launch
    G = nsp // 2 + nbot
    src_rows = int(env._src.sum().item())   # source cells of the last step (sampler bytes)
    if not args.no_kernel_events and rank == 0:
        stats["box_write_ceiling"] = write_ceiling(dev, kernel_bytes(G, n, hw, sum(env.num_planes))["step"])
    return elapsed, kern, flags, env.height * env.width, G, env.num_envs, sum(env.num_planes), src_rows, stats


def write_ceiling(dev, nbytes, reps=20):
    """This box's write rate for the step kernel's byte count, measured in the same run:
    back-to-back torch fill_ of one buffer of that size (HIP events around each fill on
    the current stream; each fill pays the previous one's dirty lines, as k_step pays the
    sampler's).  Context for roofline.frac, which is priced against the 8 TB/s peak: box
    states differ by ~10-15 %."""
    import torch

    buf = torch.empty(int(nbytes) // 4, dtype=torch.int32, device=dev)
    buf.fill_(1)
    t = []
    for i in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        buf.fill_(i)
        b.record()
        t.append((a, b))
    torch.cuda.synchronize()
    ms = sorted(a.elapsed_time(b) for a, b in t)[reps // 2]
    del buf
    return {"bytes": int(nbytes), "fill_ms": round(ms, 4), "GBps": round(nbytes / (ms * 1e-3) / 1e9, 1)}


def _coll_device(dev):
    """collectives run on the GPU under RCCL, on the host under gloo"""
    import torch.distributed as dist

    return dev if dist.get_backend() == "nccl" else "cpu"


def barrier(world, dev):
    if world > 1:
        import torch
        import torch.distributed as dist

        t = torch.ones(1, device=_coll_device(dev))
        dist.all_reduce(t)
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)


def max_over_ranks(x, world, dev):
    if world == 1:
        return x
    import torch
    import torch.distributed as dist

    t = torch.tensor([x], dtype=torch.float64, device=_coll_device(dev))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


# workloads with a CPU leg (M1 selfplay, M2 vs passiveAI, M3 vs coacAI)
CPU_WORKLOADS = ("selfplay", "passive", "coac")


def cpu_baseline(seconds, envs=512, one_core_seconds=6.0, workload="selfplay"):
    """The oracle (C restatement, OpenMP over games) on a bounded sample of the
    same workload (16x16 basesWorkers; selfplay, or every env vs the workload's
    bot; random masked actions); all host cores, plus a 1-core sample in a child
    process (OMP_NUM_THREADS=1)."""
    import subprocess

    res = cpu_sample(seconds, envs, workload)
    if one_core_seconds > 0:
        env = dict(os.environ, OMP_NUM_THREADS="1")
        out = subprocess.run([sys.executable, os.path.abspath(__file__), "--cpu-sample", str(one_core_seconds), workload],
                             env=env, capture_output=True, text=True, timeout=120)
        one = json.loads(out.stdout.strip().splitlines()[-1])
        res["value_1core"] = one["value"]
        res["sample_1core"] = one["sample"]
    return res


def cpu_sample(seconds, envs=512, workload="selfplay"):
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    from oracle_py import OracleVecEnv

    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    os.environ.setdefault("OMP_NUM_THREADS", str(threads))
    path = os.path.join(REPO, "microrts-py_amd", "gym_microrts", "microrts", MAP)
    _, nsp, nbot, bot, _ = WORKLOADS[workload]
    nsp = envs if nsp == "all" else nsp
    nbot = envs if nbot == "all" else nbot
    o = OracleVecEnv(nsp, nbot, [path], max_steps=2000, ai2s=[bot] * nbot)
    o.reset()
    o.bench_steps(5, 1, 0)
    steps = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds or steps < 5:
        o.bench_steps(5, 1, 5 + steps)
        steps += 5
    dt = time.perf_counter() - t0
    o.close()
    return {"value": envs * steps / dt, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": f"oracle/libmrts_oracle.so ovec_bench_steps, {envs} {'selfplay envs' if nsp else f'envs vs {bot}'} x "
                      f"{steps} steps ({dt:.1f} s), 16x16 basesWorkers, masks + sampler + step{' + bot' if nbot else ''} + obs "
                      f"encode in C, OpenMP over envs, OMP_NUM_THREADS={threads}"}


def _free_port():
    import socket

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


# a self-launched parent waits at most this long for the other ranks once rank 0 has exited
STRAGGLE_S = 60.0


def _stop(procs, rcs, grace_s=30):
    """terminate every rank still running, then kill what ignores it"""
    import subprocess

    for r, p in enumerate(procs):
        if rcs[r] is None:
            p.terminate()
    for r, p in enumerate(procs):
        if rcs[r] is None:
            try:
                rcs[r] = p.wait(timeout=grace_s)
            except subprocess.TimeoutExpired:
                p.kill()
                rcs[r] = p.wait()


def launch_ranks(n, argv, popen=None, poll_s=0.2, deadline_s=900.0, clock=time.monotonic):
    """`bench.py --gpus N` without a launcher: start ranks 0..N-1 of this same
    command as fresh child processes (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*
    in their environment, as torch.distributed.run sets them), relay their output,
    and return the worst exit status.  Runs before the parent imports torch, so the
    parent never initialises HIP (children start from a clean process; no exec).
    Every rank is terminated, the per-rank statuses printed and a non-zero status
    returned when
      * a rank fails (the others would wait in the barrier): that rank's status;
      * `deadline_s` passes with a rank still running (0 = no deadline): 124;
      * rank 0 (which prints the line) exited and another rank is still running
        STRAGGLE_S later: 124."""
    import subprocess

    popen = popen or subprocess.Popen
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port, MICRORTS_BENCH_SELF_LAUNCHED="1")
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    t0 = clock()
    rcs = [None] * n
    cause, why = 0, ""
    rank0_done = None
    while any(rc is None for rc in rcs):
        for r, p in enumerate(procs):
            if rcs[r] is None:
                rcs[r] = p.poll()
                if rcs[r] not in (None, 0) and not cause:
                    cause, why = rcs[r], f"rank {r} failed"
        now = clock()
        if rcs[0] is not None and rank0_done is None:
            rank0_done = now
        if not cause and any(rc is None for rc in rcs):
            if deadline_s and now - t0 > deadline_s:
                cause, why = 124, f"deadline of {deadline_s:g} s passed"
            elif rank0_done is not None and now - rank0_done > STRAGGLE_S:
                cause, why = 124, f"rank 0 exited {STRAGGLE_S:g} s ago"
        if cause:
            hung = [r for r, rc in enumerate(rcs) if rc is None]
            _stop(procs, rcs)
            print(f"bench.py: {why}; ranks still running then: {hung}; rank exit statuses {rcs}", file=sys.stderr,
                  flush=True)
            return cause if cause > 0 else 128 - cause   # killed by signal k: 128 + k, as a shell reports it
        time.sleep(poll_s)
    return 0


def _rank_watchdog(seconds, rank):
    """A rank's own deadline (--rank-timeout): under an external launcher nothing else
    ends a rank stuck in a rendezvous, a collective or a kernel.  Exits the process
    with 124 (no exec; the GPU context is torn down as at any exit)."""
    import threading

    def fire():
        print(f"bench.py: rank {rank} still running after --rank-timeout {seconds:g} s; exiting 124", file=sys.stderr,
              flush=True)
        os._exit(124)

    t = threading.Timer(seconds, fire)
    t.daemon = True
    t.start()
    return t


def gather_per_rank(elapsed, n_envs, steps, world, dev):
    """Every rank's elapsed time and env-steps/s (one all_gather), so a straggler can be
    told from a uniform slowdown in the one line rank 0 prints."""
    if world == 1:
        vals = [elapsed]
    else:
        import torch
        import torch.distributed as dist

        t = torch.tensor([elapsed], dtype=torch.float64, device=_coll_device(dev))
        out = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(out, t)
        vals = [float(x.item()) for x in out]
    return [{"rank": r, "elapsed_s": round(v, 6), "env_steps_per_s": round(n_envs * steps / v, 1)} for r, v in enumerate(vals)]


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if len(argv) == 3 and argv[0] == "--cpu-sample":   # child of cpu_baseline (no GPU use)
        print(json.dumps(cpu_sample(float(argv[1]), envs=64, workload=argv[2])), flush=True)
        return 0
    args = parse(argv)
    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            return launch_ranks(args.gpus, argv, deadline_s=args.rank_timeout)
        world = 1
    else:
        world = int(os.environ["WORLD_SIZE"])
        if world != args.gpus:
            print(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks", file=sys.stderr)
            return 2
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and args.rank_timeout > 0:
        _rank_watchdog(args.rank_timeout, rank)
    import torch

    # one GPU per rank; ranks beyond the visible GPUs share them (gloo shard tests on a 1-GPU box)
    ndev = max(1, torch.cuda.device_count())
    local_rank %= ndev
    pg = None
    if world > 1:
        import torch.distributed as dist

        import datetime

        torch.cuda.set_device(local_rank)
        # rendezvous / collective timeout well inside the rank's own deadline
        tmo = datetime.timedelta(seconds=max(60.0, min(600.0, args.rank_timeout or 600.0)))
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank), timeout=tmo)
        else:
            dist.init_process_group("gloo", timeout=tmo)
        pg = {"backend": dist.get_backend(), "world_size": dist.get_world_size(), "visible_devices": ndev,
              "launcher": "bench.py (self-launched ranks)" if os.environ.get("MICRORTS_BENCH_SELF_LAUNCHED")
              else "external (torch.distributed.run or equivalent)"}
    if args.workload == "mixed":
        torch.cuda.set_device(local_rank)
        elapsed, kern, flags, hw, G, N, P, src_rows, stats = run_mixed(args, rank, world, torch.device("cuda", local_rank))
    else:
        runs = []
        for i in range(max(1, args.seeds)):
            a = argparse.Namespace(**vars(args))
            a.seed = args.seed + i
            runs.append((a.seed, run_gpu(a, rank, world, local_rank)))
        order = sorted(range(len(runs)), key=lambda i: runs[i][1][0])
        elapsed, kern, flags, hw, G, N, P, src_rows, stats = runs[order[len(order) // 2]][1]
        if len(runs) > 1:
            stats["seeds"] = {"median_of": len(runs), "seed_of_median": runs[order[len(order) // 2]][0],
                              "values": {str(sd): round(N * args.steps / r[0], 1) for sd, r in runs},
                              "note": "per-rank values; the reported line is the median-elapsed run"}
            flags = 0
            for _, r in runs:
                flags |= r[2]
    dev = torch.device("cuda", local_rank)
    elapsed_max = max_over_ranks(elapsed, world, dev)
    per_rank = gather_per_rank(elapsed, N, args.steps, world, dev)
    total_env_steps = world * N * args.steps
    value = total_env_steps / elapsed_max
    out = None
    if rank == 0:
        eager = not args.no_eager_masks
        kb = kernel_bytes(G, N, hw, P, eager=eager, sampler=args.sampler, src_rows=src_rows)
        roof = None
        kernels = {}
        for k, ms in kern.items():
            entry = {"avg_ms": ms}
            if k in kb:
                entry["gbs"] = kb[k] / (ms * 1e-3) / 1e9
                entry["bytes"] = kb[k]
            kernels[k] = entry
        dom = max((k for k in kern if k in kb), key=lambda k: kern[k], default=None)
        if dom:
            achieved = kb[dom] / (kern[dom] * 1e-3) / 1e9
            # the committed PMC summary covers the default bench commands of a workload
            # (tensor api, eager masks, source-guided sampler) at one env count
            default_cmd = args.api == "tensor" and eager and args.sampler == "src"
            traffic, tsrc = pmc_traffic(dom, f"{args.workload}@{N}") if default_cmd else (None, "non-default bench options")
            roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBS, 4),
                    "traffic": None if traffic is None else round(traffic / (kern[dom] * 1e-3) / 1e9, 1),
                    "traffic_bytes_per_launch": traffic, "traffic_source": tsrc,
                    "algorithmic_bytes_per_launch": kb[dom], "kernel": dom, "avg_launch_ms": round(kern[dom], 4),
                    "samples": stats.get("roofline_samples"),
                    "timing": f"HIP events around every launch of a separate {args.roofline_steps}-step pass after the "
                              "timed window (the timed window records none)"}
        bk = stats.get("buckets")
        if bk and (stats.get("step_all_buckets_ms") or all(b["step_ms"] for b in bk)):
            # configs[4]: one step kernel per size bucket -- the algorithmic bytes of all
            # buckets over the time their launches take together (concurrent streams:
            # the span from the first launch's start to the last one's end; back to back:
            # the sum of their mean launch times; one mrts_step_group call: its launches)
            tb = sum(b["step_bytes"] for b in bk)
            tms = stats.get("step_all_buckets_ms") or sum(b["step_ms"] for b in bk)
            achieved = tb / (tms * 1e-3) / 1e9
            # PMC: the step kernel's mean bytes per launch x launches per step (each
            # step makes every launch of the group's plan once)
            nl = stats.get("launches_per_step") or len(bk)
            default_cmd = args.api == "tensor" and eager and args.sampler == "src" and args.group_policy == "default"
            traffic, tsrc = pmc_traffic("step", f"{args.workload}@{N}") if default_cmd else (None, "non-default bench options")
            traffic = None if traffic is None else traffic * nl
            roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBS, 4),
                    "traffic": None if traffic is None else round(traffic / (tms * 1e-3) / 1e9, 1),
                    "traffic_bytes_per_step": traffic, "traffic_source": tsrc, "algorithmic_bytes_per_launch": tb,
                    "kernel": "step (all size buckets)", "launches": nl, "avg_launch_ms": round(tms, 4),
                    "samples": stats.get("roofline_samples"),
                    "timing": f"HIP events around every step call of a separate {args.roofline_steps}-step pass after "
                              "the timed window (the timed window records none)"}
        wc = stats.get("box_write_ceiling")
        if roof and wc and roof.get("kernel") == "step":
            roof["frac_of_box_write_ceiling"] = round(roof["achieved"] / wc["GBps"], 4)
        env_step_bytes = hw * (4 * P + 312 + 56 + 32) + 64   # SURVEY.md §8d whole-step formula
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "env-steps/s",
            "n_gpus": world,
            "process_group": pg,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed_max / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic",
            "config": {"workload": WORKLOAD_DESC[args.workload],
                       "envs_per_gpu": N, "games_per_gpu": G, "map": WORKLOADS[args.workload][0], "max_steps": args.max_steps,
                       "obs": f"float32 device tensor, {P} planes", "parallelism": f"env-shard x{world}",
                       "masks": "next-tick masks written by k_step (eager)" if eager else "k_masks per get_action_mask()",
                       "sampler": {"src": "mrts_sample_actions_src (mask rows of source cells)",
                                   "dense": "mrts_sample_actions (every mask row)"}[args.sampler]},
            "roofline": roof,
            "kernels": kernels,
            "env_step_bytes": env_step_bytes,
            "env_step_roofline_frac": round(value / world * env_step_bytes / (HBM_PEAK_GBS * 1e9), 4),
            "engine_error_flags": flags,
            "window": stats,
        }
        stats["per_rank"] = per_rank
        if world > 1:
            stats["rank_timeout_s"] = args.rank_timeout
            el = [p["elapsed_s"] for p in per_rank]
            stats["per_rank_spread"] = round(max(el) / min(el), 4)   # slowest / fastest rank
        if args.workload != "selfplay":
            out["metric"] = f"env-steps/sec, workload {args.workload} (secondary config, not the BASELINE metric)"
        if args.api != "tensor":
            out["config"]["api"] = args.api
            out["metric"] = ("env-steps/sec, reference numpy contract (obs / masks / rewards copied to the host, host "
                             "actions in: PCIe-inclusive; not the headline)")
        if world == 1 and not args.no_cpu_baseline and args.workload in CPU_WORKLOADS:
            out["cpu_baseline"] = cpu_baseline(args.cpu_baseline_seconds, workload=args.workload)
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
