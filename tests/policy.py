"""The reference's trained GridNet policy (agent_sota.pt, via the committed fixture
tests/golden/agent_sota_policy.npz, see tests/golden/make_agent_sota.py) as an action
source for lock-step parity runs.  Actions are computed once, on whatever device the
obs live on, and the same int64 array goes to the engine and to the oracle: floating
point never enters the comparison, it only steers the games into the states a trained
player reaches (economies, barracks, army production, focused attacks)."""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
NVEC = [6, 4, 4, 4, 4, 7, 49]


def load_policy(device, planes=29, h=16, w=16):
    sys.path.insert(0, os.path.join(REPO, "examples"))
    from ppo_gridnet_driver import GridNet

    net = GridNet(planes, h, w)
    with np.load(os.path.join(HERE, "golden", "agent_sota_policy.npz")) as z:
        loaded = net.load_reference_state({k: z[k] for k in z.files})
    assert len(loaded) == 8, loaded
    return net.to(device).eval()


@torch.no_grad()
def policy_actions(net, obs, mask, gen):
    """Sample every component of every cell from the policy's masked categorical
    (ppo_gridnet.py's CategoricalMasked: invalid logits -> -1e8) by the Gumbel-max
    trick with a seeded generator.  obs (N, H, W, P) any dtype, mask (N, HW, 78);
    returns int64 (N, HW, 7) on the obs' device."""
    logits, _ = net(obs.float())
    m = mask.reshape(logits.shape).bool()
    logits = torch.where(m, logits, torch.full_like(logits, -1e8))
    u = torch.rand(logits.shape, generator=gen, device=logits.device).clamp_(1e-20, 1.0)
    z = logits - torch.log(-torch.log(u))
    acts = torch.stack([c.argmax(-1) for c in torch.split(z, NVEC, dim=-1)], -1)
    return acts.reshape(mask.shape[0], mask.shape[1], 7)
