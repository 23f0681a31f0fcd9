"""The agent_sota.pt fixture (tests/golden/make_agent_sota.py) loads into the
driver's GridNet under the reference's layer names and acts legally (CPU)."""
import json
import os

import numpy as np
import torch

from conftest import MAPS

HERE = os.path.dirname(os.path.abspath(__file__))


def test_fixture_matches_its_record():
    meta = json.load(open(os.path.join(HERE, "golden", "agent_sota_policy.json")))
    with np.load(os.path.join(HERE, "golden", "agent_sota_policy.npz")) as z:
        assert {k: list(z[k].shape) for k in z.files} == meta["tensors"]
        assert all(z[k].dtype == np.float32 for k in z.files)
    assert meta["loader"] == "torch.load(weights_only=True)"


def test_policy_acts_within_masks_on_the_oracle():
    from oracle_py import OracleVecEnv
    from policy import load_policy, policy_actions

    net = load_policy("cpu")
    o = OracleVecEnv(4, 2, [os.path.join(MAPS, "maps/16x16/basesWorkers16x16A.xml")], max_steps=200,
                     ai2s=["coacAI", "workerRushAI"])
    obs = o.reset()
    gen = torch.Generator().manual_seed(3)
    nvec = np.array([6, 4, 4, 4, 4, 7, 49])
    off = np.r_[0, np.cumsum(nvec)[:-1]]
    for s in range(60):
        m = o.get_action_mask()
        a = policy_actions(net, torch.from_numpy(obs), torch.from_numpy(m), gen).numpy()
        assert a.shape == (6, 256, 7) and a.dtype == np.int64
        e, c = np.nonzero(o.source_unit_mask)
        for k in range(7):
            valid = m[e, c, off[k] + a[e, c, k]]
            has_any = m[e, c, off[k]:off[k] + nvec[k]].any(-1)
            assert (valid[has_any] == 1).all(), f"component {k} picked an invalid entry at tick {s}"
        obs, _, _, _ = o.step(a)
    o.close()
