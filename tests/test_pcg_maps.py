"""Maps written by the reference's own generator, /root/reference/PCG/pcg.py:17-153
(VERDICT r5 item 3), as fixtures under tests/golden/maps/pcg/ (made by
tests/golden/make_pcg_maps.py, which records each map's seed and the generator's sha256).

They carry the format variation the generator produces and the builder's authored maps
do not: ElementTree's self-closing tags on one line, unit IDs from 16, 0-9 concentric
wall rings, random interior obstacles, non-square maps whose "right" rings sit on
interior columns (pcg.py:57 tests x against the height), and -- via the generator's own
initiate_bases called twice -- two bases per side.

CPU: both loaders (the oracle's parse_map and the C ABI's mrts_create) accept every map,
and the oracle's reset observation puts every unit and wall where the XML says.  GPU
(-m gpu): HIP == oracle lock-steps on every map, selfplay + device coacAI + workerRushAI,
with and without fog.
"""
import hashlib
import json
import os

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PCG = os.path.join(REPO, "tests", "golden", "maps", "pcg")
MANIFEST = json.load(open(os.path.join(PCG, "MANIFEST.json")))
NAMES = [m["name"] for m in MANIFEST["maps"]]
UNIT_TYPES = ["Resource", "Base", "Barracks", "Worker", "Light", "Heavy", "Ranged"]


def _path(name):
    return os.path.join(PCG, name)


def test_manifest_covers_the_generators_variation():
    maps = MANIFEST["maps"]
    assert len(maps) >= 16
    assert MANIFEST["generator"].endswith("PCG/pcg.py") and len(MANIFEST["generator_sha256"]) == 64
    for w in (12, 16):   # every wallRings value the generator allows at 12x12 and 16x16 (pcg.py:23)
        assert sorted(m["wallRings"] for m in maps if m["width"] == m["height"] == w and m["bases_per_side"] == 1) == \
            list(range(w // 2 - 2))
    assert any(m["width"] != m["height"] for m in maps)
    assert any(m["bases_per_side"] == 2 for m in maps)
    for m in maps:
        data = open(_path(m["name"]), "rb").read()
        assert hashlib.sha256(data).hexdigest() == m["sha256"], m["name"]


@pytest.mark.parametrize("name", NAMES)
def test_both_loaders_accept_pcg_map(name):
    from gym_microrts import _native
    from oracle_py import OracleVecEnv, parse_map

    m = parse_map(_path(name))
    meta = next(x for x in MANIFEST["maps"] if x["name"] == name)
    w, h, r = meta["width"], meta["height"], meta["wallRings"]
    assert (m["width"], m["height"]) == (w, h) and m["res"] == [5, 5]
    units = m["units"]
    nb = meta["bases_per_side"]
    assert len(units) == 4 + 2 * nb + 2
    assert sorted(units[:, 0].tolist()) == sorted([0] * 4 + [1] * (2 * nb) + [3] * 2)
    wall = m["terrain"].reshape(h, w)
    # the rings pcg.py:50-60 writes: rows [0, r) and [h - r, h); columns [0, r) and [h - r, h) (sic: height)
    for y in range(h):
        for x in range(w):
            if y < r or y >= h - r or x < r or h - r <= x < h:
                assert wall[y, x] == 1, (name, x, y)
    assert all(wall[u[3], u[2]] == 0 for u in units)   # no unit on a wall

    # the C ABI's loader (mrts_create parses; no device work)
    hd = _native.create(2, 2, 100, False, [_path(name)], [0, 0, 0], [0, 4], 1)
    i = _native.info(hd)
    assert (i.height, i.width, i.num_envs) == (h, w, 4)
    _native.lib().mrts_destroy(hd)

    # the oracle's reset: every unit's type plane and every wall's terrain plane
    o = OracleVecEnv(2, 0, [_path(name)], max_steps=100)
    obs = o.reset()
    assert obs.shape == (2, h, w, 29)
    for t, owner, x, y, res, hp in units:
        assert obs[0, y, x, 13 + t + 1] == 1, (name, t, x, y)
        assert obs[0, y, x, 10 + (0 if owner < 0 else 1 + owner)] == 1
        assert obs[1, y, x, 10 + (0 if owner < 0 else 2 - owner)] == 1   # player 2's view: owners swapped
    np.testing.assert_array_equal(obs[:, :, :, 28], np.broadcast_to(wall, (2, h, w)))
    o.close()


@pytest.mark.gpu
@pytest.mark.timeout(300)
@pytest.mark.parametrize("partial_obs", [False, True])
@pytest.mark.parametrize("name", NAMES)
def test_gpu_lockstep_pcg_map(name, partial_obs):
    """HIP == oracle every tick for 400 ticks: 4 selfplay envs + device coacAI and
    workerRushAI (two of each), max_steps 150 so every game auto-resets inside the window."""
    from test_gpu_bots import lockstep

    out = lockstep(["coacAI", "workerRushAI"] * 2, _path(name), 4, 400, partial_obs=partial_obs, seed=31, max_steps=150)
    assert out.sum() >= 8   # every game ended (gameover or time limit) at least once


# ---- campaign: 300 more generator maps (tests/golden/make_pcg_maps.py --campaign 300) ----
CAMPAIGN = json.load(open(os.path.join(REPO, "tests", "golden", "maps", "pcg_campaign.json")))
NCAMP = int(os.environ.get("MRTS_PCG_CAMPAIGN", "8"))   # GPU cases by default (the full set: 300)


def _campaign_map(tmp_path, k):
    m = CAMPAIGN["maps"][k]
    p = tmp_path / f"pcg_campaign_{k}.xml"
    p.write_text(m["xml"])
    return str(p), m


def test_campaign_maps_load_in_both_loaders(tmp_path):
    from gym_microrts import _native
    from oracle_py import parse_map

    assert len(CAMPAIGN["maps"]) == 300 and CAMPAIGN["generator_sha256"] == MANIFEST["generator_sha256"]
    shapes = set()
    for k in range(len(CAMPAIGN["maps"])):
        p, m = _campaign_map(tmp_path, k)
        pm = parse_map(p)
        assert (pm["width"], pm["height"]) == (m["width"], m["height"])
        assert len(pm["units"]) == 4 + 2 * m["bases_per_side"] + 2
        hd = _native.create(2, 2, 100, False, [p], [0, 0, 0], [0, 4], 1)
        _native.lib().mrts_destroy(hd)
        shapes.add((m["width"], m["height"], m["wallRings"], m["bases_per_side"]))
    assert len(shapes) > 100


@pytest.mark.gpu
@pytest.mark.timeout(600)
@pytest.mark.parametrize("k", range(NCAMP))
def test_gpu_lockstep_pcg_campaign(tmp_path, k):
    """Campaign map k: 4 selfplay envs + coacAI / workerRushAI / lightRushAI / randomBiasedAI,
    300 ticks, max_steps 120, fog on odd k, the tensor path with float32 obs (the bench's
    dtype, compared as bits) on k % 4 >= 2: HIP == oracle every tick."""
    from test_gpu_bots import lockstep

    p, m = _campaign_map(tmp_path, k)
    f32 = dict(return_tensors=True, obs_dtype="float32") if k % 4 >= 2 else {}
    lockstep(["coacAI", "workerRushAI", "lightRushAI", "randomBiasedAI"], p, 4, 300, partial_obs=bool(k % 2), seed=k,
             max_steps=120, **f32)
