"""Time the reference's own per-step Python stage beside the oracle's C encoder
(SURVEY §8d "Optionally (in this container only)").

CONTAINER ONLY: imports /root/reference (tests/golden/make_golden.py's stubs for the
JVM / gym / rdflib modules); nothing of it travels to the GPU box,
and no product path or bench line uses it.

Input: 8192 envs of 16x16 raw planes (the headline shape, BASELINE.json configs[2])
taken from the oracle's raw_obs() in mid-game -- 4096 selfplay games of
basesWorkers16x16 stepped 300 ticks by the bench's masked sampler (ovec_bench_steps).

Timed, on the same inputs and this container's cores:
* ref_stage: the reference's step_wait obs assembly,
  /root/reference/gym_microrts/envs/vec_env.py:1035 + :1058 -- one `_encode_obs`
  (:284-321) per env over `np.array(ro)` of the JNI response, then `np.array(obs)`.
  Pure numpy per env, single-threaded (the reference runs it in the training
  process), so "all-core" is measured by running the same loop in N worker processes,
  each on its own slice of the envs.
* oracle_c: oracle/libmrts_oracle.so ovec_encode_obs (the C restatement), 1 thread
  and all threads (OpenMP).
Both outputs are checked equal before any number is reported.

    python scripts/time_ref_encode.py [--envs 8192] [--reps 3] [--out profiles/r06_ref_encode.json]
"""
import argparse
import ctypes
import json
import multiprocessing as mp
import os
import platform
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "oracle"), os.path.join(REPO, "tests", "golden"), os.path.join(REPO, "microrts-py_amd")):
    sys.path.insert(0, p)
MAP = os.path.join(REPO, "microrts-py_amd", "gym_microrts", "microrts", "maps", "16x16", "basesWorkers16x16.xml")

_RAW = None


def _ref_encoder(h, w):
    from make_golden import encoder, load_reference_env

    return encoder(load_reference_env(), h, w, False)


def _ref_stage(raw):
    """vec_env.py:1035 (+ the np.array of :1058): the obs list of step_wait."""
    e = _ref_encoder(raw.shape[2], raw.shape[3])
    obs = [e._encode_obs(np.array(ro), i) for i, ro in enumerate(raw)]
    return np.array(obs)


def _worker(bounds):
    lo, hi = bounds
    raw = _RAW[lo:hi]
    e = _ref_encoder(raw.shape[2], raw.shape[3])
    t0 = time.perf_counter()
    obs = np.array([e._encode_obs(np.array(ro), i) for i, ro in enumerate(raw)])
    return time.perf_counter() - t0, int(obs.sum())


def _cpu_model():
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def main():
    global _RAW
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=8192)
    ap.add_argument("--ticks", type=int, default=300)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "r06_ref_encode.json"))
    a = ap.parse_args()
    if not os.path.isdir("/root/reference"):
        sys.exit("container only: /root/reference is absent here")

    from oracle_py import OracleVecEnv

    o = OracleVecEnv(a.envs, 0, [MAP], max_steps=2000)
    o.reset()
    o.bench_steps(a.ticks, 1, 0)   # mid-game: the bench's masked sampler, 300 ticks
    raw = o.raw_obs()
    _RAW = raw
    print(f"raw planes {raw.shape}, units on the map: {int((raw[:, 3] > 0).sum())}", flush=True)

    cores = os.cpu_count()
    gomp = ctypes.CDLL("libgomp.so.1")
    res = {"input": f"{a.envs} envs x 6 x 16 x 16 raw planes, oracle raw_obs() after {a.ticks} ticks of basesWorkers16x16 "
                    "selfplay (ovec_bench_steps sampler)", "cpu_model": _cpu_model(), "cores": cores,
           "scope": "container only (the GPU box has no /root/reference); reference Python stage vs the oracle's C encoder"}

    # oracle C encoder: 1 thread, all threads
    for nt in (1, cores):
        gomp.omp_set_num_threads(nt)
        o.encode(raw[:64])
        best = 1e9
        for _ in range(a.reps):
            t0 = time.perf_counter()
            oc = o.encode(raw)
            best = min(best, time.perf_counter() - t0)
        res[f"oracle_c_{nt}t"] = {"s_per_step": best, "envs_per_s": a.envs / best, "threads": nt}
        print(f"oracle C encoder, {nt} thread(s): {best * 1e3:.1f} ms / step = {a.envs / best / 1e6:.3f} M envs/s", flush=True)

    # the reference's stage, one process
    ref = _ref_stage(raw[:64])
    best = 1e9
    for _ in range(a.reps):
        t0 = time.perf_counter()
        ref = _ref_stage(raw)
        best = min(best, time.perf_counter() - t0)
    assert ref.dtype == np.int32 and np.array_equal(ref, oc), "reference _encode_obs != oracle encoder"
    res["ref_stage_1core"] = {"s_per_step": best, "envs_per_s": a.envs / best, "processes": 1}
    print(f"reference _encode_obs stage, 1 core: {best * 1e3:.1f} ms / step = {a.envs / best / 1e3:.1f} k envs/s", flush=True)

    # the reference's stage, every core (one process per core, each on its slice)
    sl = np.linspace(0, a.envs, cores + 1).astype(int)
    ctx = mp.get_context("fork")
    with ctx.Pool(cores) as pool:
        pool.map(_worker, [(0, 8)] * cores)   # import the reference in every worker first
        best = 1e9
        for _ in range(a.reps):
            t0 = time.perf_counter()
            out = pool.map(_worker, list(zip(sl[:-1], sl[1:])))
            best = min(best, time.perf_counter() - t0)
    assert sum(s for _, s in out) == int(oc.sum())
    res[f"ref_stage_{cores}core"] = {"s_per_step": best, "envs_per_s": a.envs / best, "processes": cores,
                                     "note": "wall time of the pool map incl. its IPC of the obs sums (not the obs)"}
    print(f"reference _encode_obs stage, {cores} processes: {best * 1e3:.1f} ms / step = {a.envs / best / 1e3:.1f} k envs/s",
          flush=True)
    res["outputs_equal"] = True
    o.close()
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
        f.write("\n")
    print("wrote", a.out)


if __name__ == "__main__":
    main()
