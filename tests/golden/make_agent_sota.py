"""Extract the reference's trained GridNet policy as a test fixture.

Source: /root/reference/experiments/gym-microrts-static-files/agent_sota.pt, the
state_dict ppo_gridnet_eval.py loads (experiments/ppo_gridnet_eval.py:49-52, 149)
into ppo_gridnet.py's Agent (experiments/ppo_gridnet.py:185-213).  It is loaded with
torch.load(weights_only=True) -- tensors only, nothing in the file is executed --
and its encoder.* / actor.* tensors (the policy; the critic plays no part in acting)
are written unchanged, float32, under their reference names to
tests/golden/agent_sota_policy.npz (numpy.load needs no pickle for it), with the
source file's sha256 in agent_sota_policy.json.

  python tests/golden/make_agent_sota.py
"""
import hashlib
import json
import os

import numpy as np
import torch

SRC = "/root/reference/experiments/gym-microrts-static-files/agent_sota.pt"
HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    sd = torch.load(SRC, map_location="cpu", weights_only=True)
    keep = {k: v.numpy().astype(np.float32) for k, v in sd.items() if k.startswith(("encoder.", "actor."))}
    np.savez_compressed(os.path.join(HERE, "agent_sota_policy.npz"), **keep)
    meta = {"source": "experiments/gym-microrts-static-files/agent_sota.pt",
            "source_sha256": hashlib.sha256(open(SRC, "rb").read()).hexdigest(),
            "loader": "torch.load(weights_only=True)",
            "tensors": {k: list(v.shape) for k, v in keep.items()},
            "dropped": sorted(k for k in sd if k not in keep)}
    with open(os.path.join(HERE, "agent_sota_policy.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(json.dumps(meta))


if __name__ == "__main__":
    main()
