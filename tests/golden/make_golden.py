"""Generate tests/golden/encode_obs_golden.npz from the REFERENCE's own encoder.

Runs only in the build container (where /root/reference exists): imports
/root/reference/gym_microrts/envs/vec_env.py with the JVM / gym / rdflib modules
stubbed, and calls MicroRTSGridModeVecEnv._encode_obs
(vec_env.py:284-321) on seeded random raw planes, including out-of-range and
negative values to exercise the clipping.  The fixture holds inputs and
outputs only; no reference source is copied.

    python tests/golden/make_golden.py
"""
import os
import sys
import types

import numpy as np

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "encode_obs_golden.npz")


def load_reference_env():
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    gym = types.ModuleType("gym")
    gym.spaces = types.ModuleType("gym.spaces")
    jp = types.ModuleType("jpype")
    jpi = types.ModuleType("jpype.imports")
    jpi.registerDomain = lambda *a, **k: None
    jpt = types.ModuleType("jpype.types")
    jpt.JArray = object
    jpt.JInt = int
    jp.imports, jp.types = jpi, jpt
    for name, mod in {"gym": gym, "gym.spaces": gym.spaces, "jpype": jp, "jpype.imports": jpi, "jpype.types": jpt,
                      "rdflib": types.ModuleType("rdflib")}.items():
        sys.modules.setdefault(name, mod)
    from gym_microrts.envs.vec_env import MicroRTSGridModeVecEnv as E

    return E


def encoder(E, h, w, partial):
    e = E.__new__(E)
    e.prior_mode = E.PriorMode("none")
    e.height, e.width = h, w
    e.num_planes = [5, 5, 3, 8, 6, 2] + ([2] if partial else [])
    e.num_planes_len = len(e.num_planes)
    e.num_planes_prefix_sum = [0]
    for n in e.num_planes:
        e.num_planes_prefix_sum.append(e.num_planes_prefix_sum[-1] + n)
    return e


def main():
    E = load_reference_env()
    rng = np.random.default_rng(20250117)
    out = {}
    cases = [("16x16", 16, 16, False, 8), ("4x4", 4, 4, False, 4), ("10x10", 10, 10, False, 4), ("24x24", 24, 24, False, 2),
             ("16x16_po", 16, 16, True, 4)]
    for name, h, w, partial, n in cases:
        P_raw = 7 if partial else 6
        # realistic-range planes plus out-of-range / negative values
        raw = rng.integers(-3, 12, size=(n, P_raw, h, w)).astype(np.int32)
        raw[0, 0, 0, 0] = 10_000
        raw[0, 1, 0, 1] = -10_000
        enc = encoder(E, h, w, partial)
        obs = np.stack([enc._encode_obs(raw[i].copy(), i) for i in range(n)])
        out[f"{name}_raw"] = raw
        out[f"{name}_obs"] = obs.astype(np.int32)
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
