"""BASELINE.json configs[0] on the MI355X engine: the reference's hello_world.py
loop (/root/reference/hello_world.py:11-67) -- 16x16 basesWorkers, random masked
actions drawn on the host with the softmax-over-{0, -9e8} sampler, render() every
step -- with the configuration BASELINE.json states (2 selfplay envs + 2 bot envs
vs coacAI; the reference script's own `prior=True, graph_depth, graph_vector_length`
kwargs are rejected by its vec env).

Provenance: `softmax`, `sample` and the body of the loop are a near-verbatim
adaptation of the reference's /root/reference/hello_world.py:27-67 -- the
workload definition of configs[0] (SURVEY.md §8d names that sampler), kept as
the reference wrote it on purpose; this file is an example, not engine code.

  python examples/hello_world.py [--steps N]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "microrts-py_amd"))

from gym_microrts import microrts_ai  # noqa: E402
from gym_microrts.envs.vec_env import MicroRTSGridModeVecEnv  # noqa: E402


def softmax(x, axis=None):
    x = x - x.max(axis=axis, keepdims=True)
    y = np.exp(x)
    return y / y.sum(axis=axis, keepdims=True)


def sample(logits, rng):
    p = softmax(logits, axis=1)
    c = p.cumsum(axis=1)
    u = rng.random((len(c), 1))
    return (u < c).argmax(axis=1).reshape(-1, 1)


def main(steps=10000, seed=0, render=True, trace=None):
    """Runs the loop; returns the number of finished episodes.  `trace` (a list)
    receives (mask, action, obs, reward, done) of every step (tests replay it
    through the oracle)."""
    envs = MicroRTSGridModeVecEnv(
        num_selfplay_envs=2,
        num_bot_envs=2,
        max_steps=2000,
        render_theme=2,
        ai2s=[microrts_ai.coacAI for _ in range(2)],
        map_paths=["maps/16x16/basesWorkers16x16.xml"],
        reward_weight=np.array([10.0, 1.0, 1.0, 0.2, 1.0, 4.0]),
        autobuild=False,
    )
    envs.action_space.seed(seed)
    rng = np.random.default_rng(seed)
    envs.reset()
    nvec = envs.action_space.nvec
    episodes = 0
    for _ in range(steps):
        if render:
            envs.render()
        action_mask = envs.get_action_mask()
        action_mask = action_mask.reshape(-1, action_mask.shape[-1])
        action_mask[action_mask == 0] = -9e8
        action = np.concatenate(
            (
                sample(action_mask[:, 0:6], rng),
                sample(action_mask[:, 6:10], rng),
                sample(action_mask[:, 10:14], rng),
                sample(action_mask[:, 14:18], rng),
                sample(action_mask[:, 18:22], rng),
                sample(action_mask[:, 22:29], rng),
                sample(action_mask[:, 29: sum(envs.action_space.nvec[1:])], rng),   # attack target (as the reference slices)
            ),
            axis=1,
        )
        if trace is not None:
            mask = np.where(action_mask == -9e8, 0, action_mask).reshape(envs.num_envs, -1, action_mask.shape[-1])
        next_obs, reward, done, info = envs.step(action)
        if trace is not None:
            trace.append((mask, action.reshape(envs.num_envs, -1), next_obs.copy(), reward.copy(), done.copy()))
        episodes += int(done.sum())
    envs.close()
    return episodes


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10000)
    a = ap.parse_args()
    print("episodes finished:", main(a.steps))
