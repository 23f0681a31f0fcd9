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


def _full_reference_state_dict():
    """A synthetic full ppo_gridnet Agent state_dict (experiments/ppo_gridnet.py:191-212
    names: encoder.{1,4}, actor.{0,2} and critic.{1,3}) -- 12 tensors, as agent_sota.pt holds."""
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "examples"))
    from ppo_gridnet_driver import GridNet

    src = GridNet(29, 16, 16).state_dict()
    inv = {v: k for k, v in GridNet.REFERENCE_NAMES.items()}
    out = {}
    for name, t in src.items():
        layer, _, field = name.rpartition(".")
        out[f"{inv[layer]}.{field}"] = t.clone() + 0.25
    assert len(out) == 12 and "critic.3.bias" in out
    return GridNet, out


def test_full_agent_state_dict_loads_with_critic(tmp_path):
    """a full reference state_dict (critic included) is the documented
    --agent-model-path input; load_reference_policy takes all 12 tensors, through
    load_weights' torch.load(weights_only=True) path."""
    GridNet, sd = _full_reference_state_dict()
    from ppo_gridnet_driver import load_weights

    p = tmp_path / "agent_full.pt"
    torch.save(sd, p)
    net = GridNet(29, 16, 16)
    done = net.load_reference_policy(load_weights(str(p)))
    assert sorted(done) == sorted(sd)
    assert torch.equal(net.state_dict()["v.3.bias"], sd["critic.3.bias"])
    assert torch.equal(net.state_dict()["pi.2.weight"], sd["actor.2.weight"])


def test_policy_state_dict_missing_actor_raises():
    import pytest

    GridNet, sd = _full_reference_state_dict()
    del sd["actor.2.bias"]
    with pytest.raises(ValueError, match="actor.2.bias"):
        GridNet(29, 16, 16).load_reference_policy(sd)
    _, sd = _full_reference_state_dict()
    sd["encoder.1.weight"] = sd["encoder.1.weight"][:, :5]
    with pytest.raises(ValueError, match="encoder.1.weight"):
        GridNet(29, 16, 16).load_reference_policy(sd)
