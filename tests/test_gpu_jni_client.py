"""gym_microrts.jni_client.JNIGridnetVecClient (the ts.JNIGridnetVecClient-shaped
client over the C ABI) driven the way the reference's vec_env.py drives the Java
client (reset :279, getMasks :1097, ragged gameStep rows :968-984 / :1002), raw
Response.observation compared with the oracle's getVectorObservation."""
import os

import numpy as np
import pytest

from conftest import MAPS

pytestmark = pytest.mark.gpu


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
