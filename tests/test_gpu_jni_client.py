"""gym_microrts.jni_client.JNIGridnetVecClient (the ts.JNIGridnetVecClient-shaped
client over the C ABI) driven the way the reference's vec_env.py drives the Java
client (reset :279, getMasks :1097, ragged gameStep rows :968-984 / :1002), raw
Response.observation compared with the oracle's getVectorObservation."""
import os

import numpy as np
import pytest

from conftest import MAPS

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]   # per-test limits below override


def pack_rows(actions, source_unit_mask, hw):
    """vec_env.py:968-984: prepend the cell index, keep rows of source units."""
    out = []
    idx = np.arange(hw)[:, None]
    for i in range(actions.shape[0]):
        a = np.concatenate([idx, actions[i].reshape(hw, 7)], axis=1)
        out.append(a[source_unit_mask[i] == 1])
    return out


@pytest.mark.parametrize("partial_obs", [False, True])
def test_jni_client_matches_oracle(partial_obs):
    from gym_microrts import microrts_ai
    from gym_microrts.jni_client import JNIGridnetVecClient
    from oracle_py import OracleVecEnv, sample_actions

    m = "maps/16x16/basesWorkers16x16.xml"
    ais = [microrts_ai.coacAI, microrts_ai.workerRushAI, microrts_ai.randomBiasedAI, microrts_ai.passiveAI]
    c = JNIGridnetVecClient(4, len(ais), 300, None, os.path.join(MAPS), [m], ais, None, partial_obs)
    o = OracleVecEnv(4, len(ais), [os.path.join(MAPS, m)], max_steps=300, partial_obs=partial_obs,
                     ai2s=["coacAI", "workerRushAI", "randomBiasedAI", "passiveAI"])
    r = c.reset([0] * 8)
    o.reset()
    np.testing.assert_array_equal(r.observation, o.raw_obs())
    hw = 256
    for s in range(400):
        mk = c.getMasks(0)
        mo = o.get_action_mask_full()
        np.testing.assert_array_equal(mk.reshape(8, hw, 79), mo)
        src = mk.reshape(8, hw, 79)[:, :, 0]
        a = sample_actions(np.ascontiguousarray(mo[:, :, 1:]), 21, s)
        r = c.gameStep(pack_rows(a, src, hw), [0] * 8)
        o.source_unit_mask = np.ascontiguousarray(src)
        ro, do = o.step_raw(a)
        np.testing.assert_array_equal(r.observation, o.raw_obs(), err_msg=f"step {s}")
        np.testing.assert_array_equal(r.reward, ro)
        np.testing.assert_array_equal(r.done, do)
    c.close()


CYCLE = ["maps/16x16/basesWorkers16x16A.xml", "maps/16x16/melee16x16Mixed8.xml", "maps/16x16/basesWorkers16x16C.xml",
         "maps/16x16/EightBasesWorkers16x16.xml"]


@pytest.mark.parametrize("kind", ["selfplay", "bots"])
def test_jni_client_cycle_maps_branch(kind):
    """The reference's map-cycling branch of step_wait (vec_env.py:1038-1056), run
    verbatim against the client's per-game objects: `clients[i].mapPath = ...;
    clients[i].reset(0)` for bot envs, `selfPlayClients[k].mapPath = ...; .reset();
    .getResponse(0/1)` for selfplay pairs.  The maps named by mapPath were not in the
    constructor's map list (mrts_add_map loads them).  Raw observations of every
    step and of every reset response equal the oracle's, which resets the same
    games onto the same maps."""
    from itertools import cycle

    from gym_microrts import microrts_ai
    from gym_microrts.jni_client import JNIGridnetVecClient
    from oracle_py import OracleVecEnv, sample_actions

    m = "maps/16x16/basesWorkers16x16.xml"
    if kind == "selfplay":
        nsp, ais, names = 8, [], []
    else:
        nsp = 0
        ais = [microrts_ai.coacAI, microrts_ai.workerRushAI, microrts_ai.randomBiasedAI, microrts_ai.lightRushAI,
               microrts_ai.passiveAI, microrts_ai.coacAI]
        names = ["coacAI", "workerRushAI", "randomBiasedAI", "lightRushAI", "passiveAI", "coacAI"]
    n, hw = nsp + len(ais), 256
    max_steps = 40
    c = JNIGridnetVecClient(nsp, len(ais), max_steps, None, MAPS, [m], ais, None, False)
    table = [m] + CYCLE
    o = OracleVecEnv(nsp, len(ais), [os.path.join(MAPS, p) for p in table], max_steps=max_steps, ai2s=names)
    r = c.reset([0] * n)
    o.reset()
    np.testing.assert_array_equal(r.observation, o.raw_obs())
    # vec_env.py:156-157 (cycle_maps joined to microrts_path) and the python-side state of the branch
    cycle_maps = [os.path.join(MAPS, p) for p in CYCLE]
    next_map = cycle(cycle_maps)
    next_oracle = cycle(range(1, len(table)))
    num_bot_envs = len(ais)
    resets = 0
    for s in range(260):
        mk = c.getMasks(0).reshape(n, hw, 79)
        mo = o.get_action_mask_full()
        np.testing.assert_array_equal(mk, mo)
        a = sample_actions(np.ascontiguousarray(mo[:, :, 1:]), 5, s)
        responses = c.gameStep(pack_rows(a, mk[:, :, 0], hw), [0] * n)
        o.source_unit_mask = np.ascontiguousarray(mk[:, :, 0])
        ro, do = o.step_raw(a)
        np.testing.assert_array_equal(responses.reward, ro)
        np.testing.assert_array_equal(responses.done, do)
        obs = [np.array(x) for x in responses.observation]
        done = np.array(responses.done)
        # ---- vec_env.py:1038-1056, as the reference writes it
        for done_idx, d in enumerate(done[:, 0]):
            if done_idx < num_bot_envs:
                if d:
                    c.clients[done_idx].mapPath = next(next_map)
                    response = c.clients[done_idx].reset(0)
                    obs[done_idx] = np.array(response.observation)
                    o.reset_game(done_idx, next(next_oracle))
                    resets += 1
            else:
                if d and done_idx % 2 == 0:
                    done_idx -= num_bot_envs
                    c.selfPlayClients[done_idx // 2].mapPath = next(next_map)
                    c.selfPlayClients[done_idx // 2].reset()
                    p0_response = c.selfPlayClients[done_idx // 2].getResponse(0)
                    p1_response = c.selfPlayClients[done_idx // 2].getResponse(1)
                    obs[done_idx] = np.array(p0_response.observation)
                    obs[done_idx + 1] = np.array(p1_response.observation)
                    o.reset_game(done_idx // 2, next(next_oracle))
                    resets += 1
        np.testing.assert_array_equal(np.array(obs), o.raw_obs(), err_msg=f"step {s}")
    assert resets >= 4
    # the maps the clients now play are the cycled ones
    assert {x.mapPath for x in c.clients + c.selfPlayClients} <= set(cycle_maps) | {os.path.join(MAPS, m)}
    c.close()


def test_jni_client_render_client():
    """render_client = selfPlayClients[0] (else clients[0]) (vec_env.py:272-276):
    sendUTT() is the UnitTypeTable JSON, and render(True) returns the BGR bytes that
    vec_env.py:1082-1084 turn back into the RGB frame -- the one k_render draws and
    oracle_py.render_frame restates."""
    import json

    from gym_microrts import microrts_ai
    from gym_microrts.jni_client import JNIGridnetVecClient
    from oracle_py import OracleVecEnv, parse_map, render_frame

    m = "maps/16x16/basesWorkers16x16.xml"
    for nsp, ais in ((2, []), (0, [microrts_ai.workerRushAI])):
        c = JNIGridnetVecClient(nsp, len(ais), 100, None, MAPS, [m], ais, None, False)
        c.reset([0] * (nsp + len(ais)))
        rc = c.selfPlayClients[0] if len(c.selfPlayClients) > 0 else c.clients[0]
        utt = json.loads(str(rc.sendUTT()))
        assert [u["name"] for u in utt["unitTypes"]][:2] == ["Resource", "Base"]
        assert rc.render(False) is None
        bytes_array = np.array(rc.render(True))
        assert bytes_array.shape == (640 * 640 * 3,)
        frame = bytes_array.reshape(640, 640, 3)[:, :, ::-1]   # Image.frombytes("RGB", ...) then [:, :, ::-1]
        o = OracleVecEnv(nsp, len(ais), [os.path.join(MAPS, m)], max_steps=100, ai2s=["workerRushAI"] * len(ais))
        o.reset()
        wall = parse_map(os.path.join(MAPS, m))["terrain"]
        np.testing.assert_array_equal(frame, render_frame(o.dump_cells(0), wall, 16, 16))
        o.close()
        c.close()
