"""The oracle's host-side sanitizer build: the C restatement built
with AddressSanitizer + UndefinedBehaviorSanitizer (oracle/Makefile `asan`,
-fno-sanitize-recover) drives rollouts of every code path the GPU parity tests
lean on -- selfplay, every device bot, partial observability, auto-resets, map
cycling, adversarial unmasked actions -- on 8x8, 16x16 and 24x24 maps, in a child
python with the ASan runtime preloaded.  CPU only."""
import os
import subprocess
import sys

import pytest

from conftest import MAPS, REPO

CHILD = r"""
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(sys.argv[1], "oracle"))
from oracle_py import OracleVecEnv, sample_actions
maps = sys.argv[2]
bots = ["workerRushAI", "lightRushAI", "randomBiasedAI", "coacAI", "POWorkerRush", "POLightRush", "POHeavyRush",
        "PORangedRush", "randomAI", "passiveAI"]
for m, extra, po in (("maps/8x8/basesWorkers8x8.xml", [], False), ("maps/16x16/basesWorkers16x16.xml",
                     ["maps/16x16/melee16x16Mixed8.xml"], True), ("maps/24x24/basesWorkers24x24.xml", [], False)):
    paths = [os.path.join(maps, p) for p in [m] + extra]
    o = OracleVecEnv(4, len(bots), paths, max_steps=150, partial_obs=po, ai2s=bots)
    o.reset()
    rng = np.random.default_rng(0)
    for s in range(220):
        mask = o.get_action_mask()
        a = sample_actions(mask, 9, s)
        if s % 3 == 0:   # unmasked rows: illegal types, out-of-range parameters, conflicts
            a = a.reshape(o.num_envs, -1, 7)
            a[:, :, :] = rng.integers(-1, 50, size=a.shape)
            o.source_unit_mask = rng.integers(0, 2, size=o.source_unit_mask.shape).astype(np.int32)
        o.step_raw(a)
        o.raw_obs()
        if s % 40 == 39 and len(paths) > 1:
            o.reset_game(1, 1)
    o.close()
maps_loaded = open("/proc/self/maps").read()
assert "libmrts_oracle_asan.so" in maps_loaded and "libasan" in maps_loaded
print("ok")
"""


def _libasan():
    out = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True)
    p = out.stdout.strip()
    return p if os.path.isabs(p) and os.path.exists(p) else None


@pytest.mark.timeout(600)
def test_oracle_under_asan_ubsan():
    asan = _libasan()
    if asan is None:
        pytest.skip("gcc's libasan is not installed")
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "asan"], check=True)
    env = dict(os.environ, LD_PRELOAD=asan, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1",
               MRTS_ORACLE_LIB=os.path.join(REPO, "oracle", "libmrts_oracle_asan.so"))
    r = subprocess.run([sys.executable, "-c", CHILD, REPO, MAPS], env=env, capture_output=True, text=True, timeout=560)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stderr[-4000:]
    assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
