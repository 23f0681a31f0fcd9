"""EXPERIMENT: bench.py with MicroRTSGridModeSharedMemVecEnv.step_wait as it was before the
overlapped copies (three blocking copies, infos after them) -- same-box A/B baseline."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "microrts-py_amd"))
from gym_microrts.envs import vec_env  # noqa: E402


def step_wait(self):
    obs, _, done0, infos = vec_env.MicroRTSGridModeVecEnv.step_wait(self)
    self._obs_host.copy_(obs)
    reward = infos._raw.cpu().numpy()
    return self.obs, reward @ self.reward_weight, done0.cpu().numpy(), [{"raw_rewards": r} for r in reward]


vec_env.MicroRTSGridModeSharedMemVecEnv.step_wait = step_wait
import bench  # noqa: E402

sys.argv = ["bench.py"] + sys.argv[1:]
bench.main()
