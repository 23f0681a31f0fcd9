"""VecEnvWrapper / VecMonitor / VecVideoRecorder with the semantics the reference
drivers rely on (ppo_gridnet.py:126-162 subclasses VecEnvWrapper, :385-389 wraps in
VecMonitor and optionally VecVideoRecorder, :487-490 reads info["episode"]).

Behaviour follows stable-baselines3's public VecEnv API:
* `step(a)` = `step_async(a)` then `step_wait()`;
* unknown attributes resolve down the wrapper chain (so `envs.get_action_mask()`,
  `envs.rfs`, `envs.action_plane_space` reach MicroRTSGridModeVecEnv through both
  wrappers, as ppo_gridnet.py:466 / :222 / :145 need);
* VecMonitor adds `info["episode"] = {"r", "l", "t"}` to the info of every env whose
  episode ended this step and resets that env's running return / length.
Rewards and dones may be numpy arrays (the reference contract) or device tensors
(`return_tensors=True`); the monitor keeps its accumulators in the same form.
"""
import time

import numpy as np

__all__ = ["VecEnv", "VecEnvWrapper", "VecMonitor", "VecVideoRecorder"]


class VecEnv:
    """Base class: num_envs, observation_space, action_space."""

    def __init__(self, num_envs, observation_space, action_space):
        self.num_envs = num_envs
        self.observation_space = observation_space
        self.action_space = action_space

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def reset(self):
        raise NotImplementedError

    def step_async(self, actions):
        raise NotImplementedError

    def step_wait(self):
        raise NotImplementedError

    def close(self):
        pass

    def seed(self, seed=None):
        return [None] * self.num_envs

    @property
    def unwrapped(self):
        return self


class VecEnvWrapper(VecEnv):
    def __init__(self, venv, observation_space=None, action_space=None):
        self.venv = venv
        VecEnv.__init__(self, venv.num_envs, observation_space or venv.observation_space,
                        action_space or venv.action_space)

    def reset(self):
        return self.venv.reset()

    def step_async(self, actions):
        self.venv.step_async(actions)

    def step_wait(self):
        return self.venv.step_wait()

    def close(self):
        return self.venv.close()

    def render(self, mode="human"):
        return self.venv.render(mode=mode)

    def seed(self, seed=None):
        s = getattr(self.venv, "seed", None)
        return s(seed) if callable(s) else [None] * self.num_envs

    @property
    def unwrapped(self):
        return getattr(self.venv, "unwrapped", self.venv)

    def __getattr__(self, name):
        # only reached when normal lookup fails; never recurse on our own fields
        if name in ("venv", "__setstate__", "__getstate__"):
            raise AttributeError(name)
        return getattr(self.venv, name)


def _to_host(x):
    if hasattr(x, "detach"):
        return x.detach().cpu().numpy()
    return np.asarray(x)


class VecMonitor(VecEnvWrapper):
    """Episode return / length / wall time per env (stable-baselines3 VecMonitor)."""

    def __init__(self, venv, filename=None, info_keywords=()):
        super().__init__(venv)
        self.t_start = time.time()
        self.info_keywords = tuple(info_keywords)
        self.episode_returns = None
        self.episode_lengths = None
        self.episode_count = 0
        self._file = open(filename, "w") if filename else None
        if self._file:
            self._file.write("r,l,t\n")

    def reset(self):
        obs = self.venv.reset()
        self.episode_returns = np.zeros(self.num_envs, dtype=np.float32)
        self.episode_lengths = np.zeros(self.num_envs, dtype=np.int32)
        return obs

    def step_wait(self):
        obs, rewards, dones, infos = self.venv.step_wait()
        if self.episode_returns is None:
            self.episode_returns = np.zeros(self.num_envs, dtype=np.float32)
            self.episode_lengths = np.zeros(self.num_envs, dtype=np.int32)
        r = _to_host(rewards)
        d = _to_host(dones).astype(bool)
        self.episode_returns += r
        self.episode_lengths += 1
        ended = np.flatnonzero(d)
        if len(ended) == 0:
            return obs, rewards, dones, infos
        new_infos = list(infos[:])
        now = round(time.time() - self.t_start, 6)
        for i in ended:
            info = dict(new_infos[i])
            ep = {"r": float(self.episode_returns[i]), "l": int(self.episode_lengths[i]), "t": now}
            for k in self.info_keywords:
                ep[k] = info.get(k)
            info["episode"] = ep
            new_infos[i] = info
            self.episode_count += 1
            if self._file:
                self._file.write(f"{ep['r']},{ep['l']},{ep['t']}\n")
            self.episode_returns[i] = 0
            self.episode_lengths[i] = 0
        return obs, rewards, dones, new_infos

    def close(self):
        if self._file:
            self._file.close()
            self._file = None
        return super().close()


class VecVideoRecorder(VecEnvWrapper):
    """Records `render("rgb_array")` frames while `record_video_trigger(step)` fires,
    for `video_length` steps.  stable-baselines3 encodes mp4 through moviepy, which
    is not in this image; the frames of each clip are written as a compressed
    `.npz` (`frames`: (T, H, W, 3) uint8) in `video_folder` instead."""

    def __init__(self, venv, video_folder, record_video_trigger, video_length=200, name_prefix="rl-video"):
        super().__init__(venv)
        import os

        self.video_folder = os.path.abspath(video_folder)
        os.makedirs(self.video_folder, exist_ok=True)
        self.record_video_trigger = record_video_trigger
        self.video_length = int(video_length)
        self.name_prefix = name_prefix
        self.step_id = 0
        self.recording = False
        self.frames = []
        self.clip_start = 0

    def reset(self):
        obs = self.venv.reset()
        self._maybe_start()
        return obs

    def _maybe_start(self):
        if not self.recording and self.record_video_trigger(self.step_id):
            self.recording = True
            self.frames = []
            self.clip_start = self.step_id
        if self.recording:
            self.frames.append(np.asarray(self.venv.render(mode="rgb_array")))

    def _flush(self):
        import os

        if self.frames:
            path = os.path.join(self.video_folder, f"{self.name_prefix}-step-{self.clip_start}-to-step-{self.step_id}.npz")
            np.savez_compressed(path, frames=np.stack(self.frames))
        self.frames = []
        self.recording = False

    def step_wait(self):
        out = self.venv.step_wait()
        self.step_id += 1
        if self.recording and len(self.frames) >= self.video_length:
            self._flush()
        self._maybe_start()
        return out

    def close(self):
        if self.recording:
            self._flush()
        return super().close()
