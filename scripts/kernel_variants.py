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


def child(lib_path, workload):
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
    a.envs_per_gpu, a.max_steps, a.seed, a.warmup, a.steps, a.no_kernel_events = 8192, 2000, 1, 30, 100, False
    a.workload = workload
    a.no_eager_masks, a.sampler = False, "src"
    elapsed, kern, flags, hw, G, N, P, _ = bench.run_gpu(a, 0, 1, 0)
    print(json.dumps({"lib": os.path.basename(lib_path), "workload": workload, "ms_per_step": 1e3 * elapsed / a.steps,
                      "kernels_ms": kern, "flags": flags}))


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(sys.argv[2], sys.argv[3])
        return
    names = sys.argv[1:] or sorted(f[4:-3] for f in os.listdir(EXP) if f.startswith("lib_"))
    for n in names:
        wl = "selfplay"
        if ":" in n:
            n, wl = n.split(":")
        out = subprocess.run([sys.executable, __file__, "--child", os.path.join(EXP, f"lib_{n}.so"), wl],
                             capture_output=True, text=True, timeout=300)
        line = [l for l in out.stdout.splitlines() if l.startswith("{")]
        print(line[-1] if line else f"{n}: FAILED {out.stderr[-800:]}", flush=True)


if __name__ == "__main__":
    main()
