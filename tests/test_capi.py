"""The drop-in boundary on CPU: libmicrorts_amd.so loads, exports every entry
point include/microrts_amd.h declares, and its host-only calls (config
validation, map XML loading, unit-type JSON) behave -- no kernel launches."""
import ctypes
import json
import os
import re

import numpy as np
import pytest

from conftest import MAPS, REPO

HEADER = os.path.join(REPO, "include", "microrts_amd.h")


def declared_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"\b(mrts_[a-z_]+)\s*\(", txt)))


def test_header_declares_the_api():
    syms = declared_symbols()
    for s in ["mrts_create", "mrts_reset", "mrts_step", "mrts_get_masks", "mrts_destroy", "mrts_last_error"]:
        assert s in syms


def test_library_exports_every_declared_symbol():
    from gym_microrts import _native

    L = _native.lib()
    missing = [s for s in declared_symbols() if not hasattr(L, s)]
    assert not missing, missing
    assert set(_native.SIGNATURES) == set(declared_symbols())


def _create(**kw):
    from gym_microrts import _native

    args = dict(num_selfplay_envs=4, num_bot_envs=2, max_steps=2000, partial_obs=False,
                map_paths=[os.path.join(MAPS, "maps/16x16/basesWorkers16x16.xml")], game_map=[0, 0, 0, 0], bot_ai=[0, 0],
                obs_dtype=1)
    args.update(kw)
    return _native.create(**args)


def test_create_and_info():
    from gym_microrts import _native

    h = _create()
    i = _native.info(h)
    assert (i.height, i.width, i.num_envs, i.num_games, i.obs_planes, i.mask_channels) == (16, 16, 6, 4, 29, 78)
    assert i.workspace_bytes >= 4 * 256 * 16
    utt = json.loads(_native.lib().mrts_utt_json(h).decode())
    names = [u["name"] for u in utt["unitTypes"]]
    assert names == ["Resource", "Base", "Barracks", "Worker", "Light", "Heavy", "Ranged"]
    assert len(utt["unitTypes"]) + 1 == 8   # num_planes unit-type group (vec_env.py:235)
    _native.lib().mrts_destroy(h)


@pytest.mark.parametrize("kw,err", [
    (dict(num_selfplay_envs=3), "MicroRTSError"),
    (dict(max_steps=0), "MicroRTSError"),
    (dict(map_paths=["/nonexistent.xml"]), "MicroRTSError"),
    (dict(bot_ai=[99, 0]), "MicroRTSError"),
])
def test_create_rejects_bad_config(kw, err):
    from gym_microrts import _native

    with pytest.raises(getattr(_native, err)):
        _create(**kw)


def test_mixed_map_sizes_rejected():
    with pytest.raises(Exception, match="share height"):
        _create(map_paths=[os.path.join(MAPS, "maps/16x16/basesWorkers16x16.xml"), os.path.join(MAPS, "maps/8x8/basesWorkers8x8.xml")])


def test_unbound_calls_fail_loudly():
    from gym_microrts import _native

    h = _create()
    rc = _native.lib().mrts_reset(h, None, ctypes.c_void_p(16))
    assert rc != 0 and b"not bound" in _native.lib().mrts_last_error(h)


def test_map_loader_matches_python_parser():
    """C++ PhysicalGameState loader vs the oracle harness' python parser on every
    authored map: same size and unit count (workspace size reflects maps)."""
    from gym_microrts import _native
    from oracle_py import parse_map

    for root, _, files in os.walk(os.path.join(MAPS, "maps")):
        for f in files:
            p = os.path.join(root, f)
            m = parse_map(p)
            h = _native.create(2, 0, 100, False, [p], [0], [], 1)
            i = _native.info(h)
            assert (i.height, i.width) == (m["height"], m["width"])
            _native.lib().mrts_destroy(h)
            assert len(m["units"]) > 0 and np.all(m["units"][:, 5] >= 1)


def test_env_requires_gpu_when_absent():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from gym_microrts.envs.vec_env import MicroRTSGridModeVecEnv

    with pytest.raises(RuntimeError, match="GPU"):
        MicroRTSGridModeVecEnv(num_selfplay_envs=2, num_bot_envs=0, map_paths=["maps/16x16/basesWorkers16x16.xml"])


def test_fused_early_bot_layout_is_race_free_for_every_size():
    """the bot-fused k_step's early bot (wave 0) runs beside
    emit_outputs' phase A (waves 1..).  For every map size the engine fuses (W <= 32,
    H <= 64, H*W > 64, LDS within 160 KB) the bot's LDS writes must miss phase A's
    reads (unit / act / wall / scalars) and phase A's writes (output words, counter)
    must miss everything the bot touches -- in particular on sizes whose cell count
    is not a multiple of 4, where the bot's own wall slot lands inside the step's
    terrain (the bot now reads the step's terrain in place).  Checked by the
    library from the two LDS carves the kernels use."""
    from gym_microrts import _native

    f = _native.lib().mrts_fused_layout_ok
    fusable = [(w, h) for w in range(1, 33) for h in range(1, 65) if f(w, h) >= 0]
    # every size up to 32 x 64 whose fused LDS fits and whose bot LDS mrts_create accepts (<= 64 KB:
    # HW <= ~1130); maps of <= 64 cells take a 128-lane step
    assert 1700 < len(fusable) < 1900 and f(32, 32) == 1 and f(32, 64) == -1
    bad = [(w, h) for w, h in fusable if f(w, h) != 1]
    assert not bad, bad[:20]
    odd = [(w, h) for w, h in fusable if (w * h) % 4]
    assert (15, 15) in odd and (9, 13) in odd and (3, 5) in odd
    assert f(8, 8) == 1 and f(4, 4) == 1 and f(33, 16) == -1 and f(0, 5) == -1


def test_step_group_plan_merges_what_fits():
    """mrts_step_group_plan (host logic, no workspace needed): configs[4]'s buckets -- 8x8
    and 16x16 share a launch under merge-fit (members that keep >= 6 workgroups per CU),
    24x24 (40 KB fused workgroups: four per CU) and 32x32 keep their own; merge-all puts
    all in one; separate gives one each; engines of other planes or bot fusion never share;
    a handle listed twice is rejected."""
    from gym_microrts import _native

    lib = _native.lib()

    def mk(m, bots=2, partial=False):
        return _create(map_paths=[os.path.join(MAPS, m)], game_map=[0] * (2 + bots), bot_ai=[4] * bots, num_bot_envs=bots,
                       partial_obs=partial)

    def plan(hs, policy):
        arr = (ctypes.c_void_p * len(hs))(*hs)
        lo, nl = (ctypes.c_int32 * len(hs))(), ctypes.c_int32()
        rc = lib.mrts_step_group_plan(arr, len(hs), policy, lo, ctypes.byref(nl))
        return rc, list(lo), nl.value

    h8, h16, h24 = mk("maps/8x8/basesWorkers8x8.xml"), mk("maps/16x16/basesWorkers16x16.xml"), mk("maps/24x24/basesWorkers24x24.xml")
    hs = [h8, h16, h24]
    assert plan(hs, _native.GROUP_MERGE_FIT | _native.GROUP_BOTS_FIRST) == (0, [0, 0, 1], 2)
    h32 = mk("maps/32x32/basesWorkers32x32.xml")
    assert plan([h8, h16, h32], _native.GROUP_MERGE_FIT) == (0, [0, 0, 1], 2)
    assert plan([h8, h16, h32], _native.GROUP_MERGE_ALL) == (0, [0, 0, 0], 1)
    lib.mrts_destroy(h32)
    assert plan(hs, _native.GROUP_MERGE_ALL) == (0, [0, 0, 0], 1)
    assert plan(hs, _native.GROUP_SEPARATE) == (0, [0, 1, 2], 3)
    hp = mk("maps/10x10/basesTwoWorkers10x10.xml", partial=True)   # 31 planes: its own launch
    hsp = mk("maps/4x4/baseTwoWorkers4x4.xml", bots=0)             # no bots: not fused, its own launch
    assert plan([h16, hp, hsp], _native.GROUP_MERGE_ALL) == (0, [0, 1, 2], 3)
    rc, _, _ = plan([h16, h16], _native.GROUP_MERGE_ALL)
    assert rc != 0 and b"twice" in lib.mrts_last_error(h16)
    for bad in (3, 8):
        rc, _, _ = plan(hs, bad)
        assert rc != 0 and b"policy" in lib.mrts_last_error(h8)
    for h in hs + [hp, hsp]:
        lib.mrts_destroy(h)
