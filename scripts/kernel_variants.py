"""A/B kernel timing of libmicrorts_amd.so variants (scripts/build_variants.sh).

  python scripts/kernel_variants.py [names...]     (on the GPU box)

Each variant runs in its own subprocess (the engine library binds once per
process): 8192-env 16x16 selfplay, per-kernel HIP-event timing of
get_action_mask / sample / step over 100 steps.  Experiment tooling only.
"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXP = os.path.join(REPO, "scripts", "_exp")


def child(lib_path, workload, envs=8192):
    sys.path.insert(0, os.path.join(REPO, "microrts-py_amd"))
    sys.path.insert(0, REPO)
    import numpy as np
    import torch

    from gym_microrts import _native

    _native.LIB_PATH = lib_path
    import bench

    class A:
        pass

    a = A()
    a.envs_per_gpu, a.max_steps, a.seed, a.warmup, a.steps, a.no_kernel_events = int(envs), 2000, 1, 30, 100, False
    a.workload = workload
    a.no_eager_masks, a.sampler, a.event_every = False, "src", 1
    elapsed, kern, flags, hw, G, N, P, _ = bench.run_gpu(a, 0, 1, 0)
    print(json.dumps({"lib": os.path.basename(lib_path), "workload": workload, "envs": int(envs), "ms_per_step": 1e3 * elapsed / a.steps,
                      "kernels_ms": kern, "flags": flags}))


def fill_rate(nbytes=948428800, reps=30):
    """Write ceiling of this box: torch's fill kernel over the bytes one k_step launch writes."""
    import torch

    buf = torch.empty(nbytes // 4, dtype=torch.int32, device="cuda")
    for _ in range(3):
        buf.fill_(0)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        buf.fill_(1)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(json.dumps({"fill_bytes": nbytes, "fill_ms": ms, "fill_TBps": nbytes / ms / 1e9}))


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--fill":
        fill_rate()
        return
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(*sys.argv[2:])
        return
    names = sys.argv[1:] or sorted(f[4:-3] for f in os.listdir(EXP) if f.startswith("lib_"))
    for n in names:
        parts = n.split(":")   # name[:workload[:envs]]
        n, wl, envs = parts[0], (parts[1] if len(parts) > 1 else "") or "selfplay", parts[2] if len(parts) > 2 else "8192"
        out = subprocess.run([sys.executable, __file__, "--child", os.path.join(EXP, f"lib_{n}.so"), wl, envs],
                             capture_output=True, text=True, timeout=300)
        line = [l for l in out.stdout.splitlines() if l.startswith("{")]
        print(line[-1] if line else f"{n}: FAILED {out.stderr[-800:]}", flush=True)


if __name__ == "__main__":
    main()
