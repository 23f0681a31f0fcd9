"""Seeded random maps (tests/random_maps.py): walls, resources and every unit type of both
players scattered over 8x8, 12x20, 16x16 and 24x24 maps, up to 150 units per game -- past one
wavefront of units, so the bots take their serial unit-list / abstract-action paths
(rush_serial, coac_serial, the serial translateActions) -- with every device bot, full and
partial observability, masked and partly unmasked agent actions: GPU == oracle every step
(obs, masks, raw rewards, dones).  Engine and bot rules stay parity unpinned against Java
(DESIGN.md §4 / §4b); these maps widen the GPU == oracle coverage past the authored maps."""
import pytest

from random_maps import write_random_map
from test_gpu_bots import lockstep

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]   # per-test limits below override
BOTS = ["coacAI", "workerRushAI", "lightRushAI", "randomBiasedAI", "POWorkerRush", "PORangedRush", "POHeavyRush",
        "POLightRush", "randomAI", "passiveAI"]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("partial_obs", [False, True])
@pytest.mark.parametrize("w,h,n_units,seed", [(16, 16, 90, 1), (12, 20, 80, 2), (24, 24, 150, 3), (8, 8, 40, 4),
                                              (16, 16, 60, 5)])
def test_random_map_lockstep(tmp_path, w, h, n_units, seed, partial_obs):
    path = write_random_map(str(tmp_path / f"r{w}x{h}_{seed}.xml"), w, h, seed, n_units=n_units)
    f32 = dict(return_tensors=True, obs_dtype="float32") if seed % 2 else {}   # odd seeds: the bench's dtype, as bits
    lockstep(BOTS * 2, path, 4, 300, partial_obs=partial_obs, seed=seed, max_steps=200, mode="mixed", **f32)
