"""The reference drivers' third-party imports (gym.spaces, stable_baselines3 vec-env
wrappers, torch.utils.tensorboard; experiments/ppo_gridnet.py:17-20) resolved by
gym_microrts.run_driver's stand-ins.

CPU: the stand-ins' semantics on a host-only VecEnv, and -- in the container that
holds the reference -- the unmodified ppo_gridnet.py importing through them.
GPU: ppo_gridnet.py's wrapper stack (VecEnvWrapper subclass -> VecMonitor) over
MicroRTSGridModeVecEnv, with episodes ending at max_steps.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "microrts-py_amd")
REF_PPO = "/root/reference/experiments/ppo_gridnet.py"


@pytest.fixture(scope="module")
def compat():
    from gym_microrts import run_driver

    used = run_driver.install()
    from stable_baselines3.common import vec_env as sb3

    return used, sb3


class _CountdownEnv:
    """Host-only VecEnv: env i ends its episode every `period[i]` steps, reward 1 per step."""

    def __init__(self, period):
        from gym_microrts._spaces import Box, MultiDiscrete

        self.period = np.asarray(period)
        self.num_envs = len(period)
        self.observation_space = Box(0, 1, (2, 2, 1), np.int32)
        self.action_space = MultiDiscrete([2] * 4)
        self.t = np.zeros(self.num_envs, int)
        self.marker = "reached"

    def reset(self):
        self.t[:] = 0
        return np.zeros((self.num_envs, 2, 2, 1), np.int32)

    def step_async(self, a):
        self.a = a

    def step_wait(self):
        self.t += 1
        done = self.t % self.period == 0
        return (np.zeros((self.num_envs, 2, 2, 1), np.int32), np.ones(self.num_envs), done,
                [{"raw_rewards": np.ones(6)} for _ in range(self.num_envs)])

    def get_action_mask(self):
        return np.ones((self.num_envs, 4, 2), np.int32)

    def close(self):
        self.closed = True


def test_stand_ins_resolve(compat):
    used, sb3 = compat
    import gym.spaces
    from gym_microrts._spaces import MultiDiscrete
    from torch.utils.tensorboard import SummaryWriter  # noqa: F401

    assert {"VecEnvWrapper", "VecMonitor", "VecVideoRecorder"} <= set(dir(sb3))
    # isinstance(envs.action_space, MultiDiscrete) (ppo_gridnet.py:390) holds for our spaces
    assert gym.spaces.MultiDiscrete is MultiDiscrete or "gym" not in used


def test_vec_monitor_episode_info_and_forwarding(compat):
    _, sb3 = compat

    class Recorder(sb3.VecEnvWrapper):   # the shape of ppo_gridnet.py:126-162's MicroRTSStatsRecorder
        def reset(self):
            self.n = 0
            return self.venv.reset()

        def step_wait(self):
            obs, r, d, infos = self.venv.step_wait()
            self.n += 1
            return obs, r, d, list(infos[:])

    base = _CountdownEnv([3, 5])
    env = sb3.VecMonitor(Recorder(base))
    env.reset()
    assert env.num_envs == 2 and env.marker == "reached"          # attribute lookup down the chain
    assert env.get_action_mask().shape == (2, 4, 2)
    eps = []
    for _ in range(15):
        _, _, d, infos = env.step(np.zeros((2, 4)))
        eps += [(i, infos[i]["episode"]) for i in np.flatnonzero(d)]
    assert [(i, e["l"], e["r"]) for i, e in eps] == [(0, 3, 3.0), (1, 5, 5.0), (0, 3, 3.0), (0, 3, 3.0), (1, 5, 5.0),
                                                     (0, 3, 3.0), (0, 3, 3.0), (1, 5, 5.0)]
    env.close()
    assert base.closed


def test_summary_writer_stand_in(compat, tmp_path):
    import json

    from torch.utils.tensorboard import SummaryWriter

    w = SummaryWriter(str(tmp_path / "run"))
    w.add_text("hyperparameters", "|a|b|")
    w.add_scalar("charts/sps", 123, 7)
    w.close()
    if getattr(sys.modules["torch.utils.tensorboard"], "__microrts_compat__", False):
        rows = [json.loads(x) for x in open(tmp_path / "run" / "events.jsonl")]
        assert rows[1] == {**rows[1], "tag": "charts/sps", "value": 123.0, "step": 7}


def test_video_recorder_writes_frames(compat, tmp_path):
    _, sb3 = compat

    class Frames(_CountdownEnv):
        def render(self, mode="human"):
            return np.full((4, 4, 3), self.t[0], np.uint8)

    env = sb3.VecVideoRecorder(Frames([100]), str(tmp_path), record_video_trigger=lambda s: s == 0, video_length=3)
    env.reset()
    for _ in range(5):
        env.step(np.zeros((1, 4)))
    env.close()
    (clip,) = os.listdir(tmp_path)
    assert np.load(tmp_path / clip)["frames"][:, 0, 0, 0].tolist() == [0, 1, 2]


@pytest.mark.skipif(not os.path.exists(REF_PPO), reason="reference checkout only in the build container")
@pytest.mark.parametrize("script,flag", [("ppo_gridnet.py", "--num-selfplay-envs"), ("ppo_gridnet_eval.py", "--model-type"),
                                         ("ppo_gridnet_large.py", "--num-selfplay-envs")])
def test_reference_drivers_import_unmodified(tmp_path, script, flag):
    """The unmodified experiments/ drivers get through every import
    (gym, stable_baselines3, torch.utils.tensorboard, gym_microrts = this package) and their
    argument parsers under the runner (the env itself needs the GPU)."""
    env = dict(os.environ, PYTHONPATH=PKG)
    path = os.path.join(os.path.dirname(REF_PPO), script)
    p = subprocess.run([sys.executable, "-m", "gym_microrts.run_driver", path, "--help"], cwd=tmp_path, env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    assert flag in p.stdout


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_ppo_gridnet_wrapper_stack_on_device(compat, tmp_path):
    """ppo_gridnet.py:364-389: env -> VecEnvWrapper subclass -> VecMonitor; masks through
    both wrappers (:466), host int64 actions (:475), info["episode"] when an env hits
    max_steps (:486-488)."""
    import torch

    _, sb3 = compat
    from gym_microrts import microrts_ai
    from gym_microrts.envs.vec_env import MicroRTSGridModeVecEnv
    from torch.utils.tensorboard import SummaryWriter

    class Stats(sb3.VecEnvWrapper):
        def reset(self):
            self.raw = np.zeros((self.num_envs, 6))
            return self.venv.reset()

        def step_wait(self):
            obs, r, d, infos = self.venv.step_wait()
            infos = list(infos[:])
            for i in range(len(d)):
                self.raw[i] += infos[i]["raw_rewards"]
                if d[i]:
                    infos[i] = dict(infos[i], microrts_stats=dict(zip([str(rf) for rf in self.rfs], self.raw[i])))
                    self.raw[i] = 0
            return obs, r, d, infos

    max_steps = 24
    base = MicroRTSGridModeVecEnv(num_selfplay_envs=4, num_bot_envs=2, max_steps=max_steps,
                                  ai2s=[microrts_ai.workerRushAI, microrts_ai.coacAI],
                                  map_paths=["maps/16x16/basesWorkers16x16A.xml"],
                                  reward_weight=np.array([10.0, 1.0, 1.0, 0.2, 1.0, 4.0]))
    envs = sb3.VecMonitor(Stats(base))
    writer = SummaryWriter(str(tmp_path / "runs"))
    obs = envs.reset()
    n, hw = envs.num_envs, base.height * base.width
    rng = np.random.default_rng(0)
    returns = np.zeros(n)
    episodes = []
    for step in range(max_steps + 2):
        mask = torch.tensor(envs.get_action_mask())           # (N, HW, 78) through both wrappers
        assert mask.shape == (n, hw, 78)
        logits = torch.from_numpy(rng.standard_normal((n, hw, 78)))
        acts = []
        off = 0
        for k in envs.action_plane_space.nvec.tolist():
            lg = torch.where(mask[..., off:off + k].bool(), logits[..., off:off + k], torch.tensor(-1e8, dtype=torch.float64))
            acts.append(lg.argmax(-1))
            off += k
        a = torch.stack(acts, -1).numpy().reshape(n, -1)
        obs, rew, done, infos = envs.step(a)
        returns += rew
        for i in np.flatnonzero(done):
            ep = infos[i]["episode"]
            episodes.append((i, ep["l"]))
            assert abs(ep["r"] - returns[i]) < 1e-3 and "microrts_stats" in infos[i]
            writer.add_scalar("charts/episodic_return", ep["r"], step)
            returns[i] = 0
    writer.close()
    assert obs.shape == (n, 16, 16, 29)
    assert {i for i, _ in episodes} == set(range(n))                   # every env hit max_steps once
    assert all(l <= max_steps for _, l in episodes)
    assert base.error_flags() == 0
    envs.close()


def test_return_contract_from_environment(monkeypatch):
    """MICRORTS_AMD_RETURN selects the return contract of an env constructed without
    `return_tensors` (an unmodified ppo_gridnet.py); the keyword wins when given."""
    from gym_microrts.envs.vec_env import contract_of

    monkeypatch.delenv("MICRORTS_AMD_RETURN", raising=False)
    assert contract_of(None) == "numpy"
    monkeypatch.setenv("MICRORTS_AMD_RETURN", "hybrid")
    assert contract_of(None) == "hybrid"
    assert contract_of(False) == "numpy" and contract_of(True) == "tensors" and contract_of("hybrid") == "hybrid"
    monkeypatch.setenv("MICRORTS_AMD_RETURN", "bogus")
    with pytest.raises(ValueError):
        contract_of(None)


def test_run_driver_contract_flag(tmp_path, monkeypatch):
    """`run_driver --contract hybrid script.py` exports MICRORTS_AMD_RETURN before the
    script runs, so the script itself is not edited."""
    from gym_microrts import run_driver

    out = tmp_path / "seen.txt"
    script = tmp_path / "probe.py"
    script.write_text(f"import os\nopen({str(out)!r}, 'w').write(os.environ.get('MICRORTS_AMD_RETURN', ''))\n")
    monkeypatch.delenv("MICRORTS_AMD_RETURN", raising=False)
    assert run_driver.main(["--contract", "hybrid", str(script)]) == 0
    assert out.read_text() == "hybrid"
    assert run_driver.main(["--contract=tensors", str(script)]) == 0
    assert out.read_text() == "tensors"
    assert run_driver.main(["--contract", "nope", str(script)]) == 2
    assert run_driver.main(["--contract"]) == 2   # no value: usage, not IndexError
