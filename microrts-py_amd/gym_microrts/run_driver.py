"""Run a reference driver script unmodified on the MI355X engine.

    python -m gym_microrts.run_driver [--contract numpy|tensors|hybrid] experiments/ppo_gridnet.py --num-selfplay-envs 24 ...

`--contract hybrid` (the same as MICRORTS_AMD_RETURN=hybrid in the environment)
gives every MicroRTSGridModeVecEnv the script constructs the zero-copy contract an
unmodified ppo_gridnet.py can consume: obs / masks stay device tensors, rewards /
dones / infos are numpy (gym_microrts/envs/vec_env.py module docstring).

The reference's drivers (experiments/ppo_gridnet.py:17-23, ppo_gridnet_eval.py,
hello_world.py) import `gym.spaces`, `stable_baselines3.common.vec_env` and
`torch.utils.tensorboard` besides `gym_microrts`.  None of the three is installed in
this image (nor on the GPU host).  This runner
1. puts this package first on sys.path, so `gym_microrts` is the MI355X engine;
2. appends `compat/` (gym, stable_baselines3 stand-ins) to the END of sys.path, so a
   real installation always wins;
3. if `import torch.utils.tensorboard` fails, registers compat/tensorboard_shim as
   that module (SummaryWriter writing JSON lines);
4. executes the script as `__main__` with the remaining argv (runpy), in the
   current working directory, so relative map / static-file paths resolve as they
   do for the reference.
"""
import os
import runpy
import sys

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))   # microrts-py_amd/
_COMPAT = os.path.join(_PKG_ROOT, "compat")


def install():
    """Make the reference drivers' third-party imports resolvable (idempotent).
    Returns the list of stand-ins in use (for logs and tests)."""
    used = []
    if _PKG_ROOT not in sys.path:
        sys.path.insert(0, _PKG_ROOT)
    if _COMPAT not in sys.path:
        sys.path.append(_COMPAT)
    for mod in ("gym", "stable_baselines3"):
        try:
            m = __import__(mod)
        except ImportError:
            continue
        if getattr(m, "__microrts_compat__", False):
            used.append(mod)
    try:
        import torch.utils.tensorboard  # noqa: F401
    except ImportError:
        import torch.utils

        sys.modules.pop("torch.utils.tensorboard", None)
        import tensorboard_shim

        sys.modules["torch.utils.tensorboard"] = tensorboard_shim
        torch.utils.tensorboard = tensorboard_shim
        used.append("torch.utils.tensorboard")
    return used


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv or argv[0] in ("-h", "--help"):
        print(__doc__)
        return 0
    if argv[0].startswith("--contract"):
        if "=" in argv[0]:
            contract, argv = argv[0].split("=", 1)[1], argv[1:]
        elif len(argv) >= 2:
            contract, argv = argv[1], argv[2:]
        else:
            print("--contract needs a value: numpy | tensors | hybrid", file=sys.stderr)
            print(__doc__)
            return 2
        if contract not in ("numpy", "tensors", "hybrid"):
            print(f"unknown contract {contract!r}: numpy | tensors | hybrid", file=sys.stderr)
            return 2
        os.environ["MICRORTS_AMD_RETURN"] = contract
    if not argv:
        print(__doc__)
        return 2
    script = argv[0]
    used = install()
    if used:
        print(f"[gym_microrts.run_driver] stand-ins: {', '.join(used)}", file=sys.stderr)
    sys.argv = [script] + argv[1:]
    runpy.run_path(script, run_name="__main__")
    return 0


if __name__ == "__main__":
    sys.exit(main())
