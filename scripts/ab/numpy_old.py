"""EXPERIMENT: bench.py with MicroRTSGridModeVecEnv.step_wait as it was before the infos
were built during the D2H copies -- same-box A/B baseline for the numpy contract."""
import os
import sys

import numpy as np  # noqa: F401

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "microrts-py_amd"))
from gym_microrts import _native  # noqa: E402,F401
from gym_microrts.envs import vec_env  # noqa: E402
from gym_microrts.envs.vec_env import LazyInfos  # noqa: E402,F401


def step_wait(self):
    """vec_env.py:1001-1057"""
    if not self._mask_fresh:
        # the reference reads the source mask of the last get_action_mask
        # (vec_env.py:974); compute it if the caller skipped that call
        self.get_action_mask()
    a = self._actions_in
    self._mask_fresh = self.eager_masks
    if self.return_tensors:
        # reward @ reward_weight and done[:, 0] are fused into the step kernel
        self._launch("step", _native.lib().mrts_step_weighted, self._h, self._stream(), a.data_ptr(), self._src.data_ptr(),
                     self._obs.data_ptr(), self._raw.data_ptr(), self._done.data_ptr(), self._rew.data_ptr(),
                     self._done0.data_ptr())
        return self._tensor_outputs()
    self._launch("step", _native.lib().mrts_step, self._h, self._stream(), a.data_ptr(), self._src.data_ptr(),
                 self._obs.data_ptr(), self._raw.data_ptr(), self._done.data_ptr())
    self._mask_prefetch = None
    # numpy contract + eager masks, when the caller reads the masks every step (the
    # rollout loop does: ppo_gridnet.py:466): the next get_action_mask()'s host copy
    # rides behind the obs copy, in this call's one sync
    prefetch = self._host_outputs and self.eager_masks and self._mask_wanted
    self._mask_wanted = False
    reward = self._host("raw", self._raw)
    done = self._host("done", self._done)
    cycling = len(self.cycle_maps) > self._cycle_min
    obs = self._obs   # hybrid contract: obs stay in HBM
    if not cycling and self._host_outputs:   # one stream sync for every output
        obs = self._host("obs", self._obs)
        if prefetch:
            self._mask_prefetch = self._host("mask", self._mask)
    self._sync()
    self._act_src = None
    done = done.astype(bool)
    if not self.reward_shaping:
        reward[:, 1:] = 0
    if cycling:
        self._cycle(done[:, 0])
        if self._host_outputs:
            obs = self._host("obs", self._obs)
            if prefetch:
                self._mask_prefetch = self._host("mask", self._mask)
            self._sync()
    infos = [{"raw_rewards": item} for item in reward]
    return obs, reward @ self.reward_weight, done[:, 0], infos

def _step_io(self):
    """The tensor contract's step buffers (mrts_step_io) after step_async, for a
    step launched by mrts_step_group (MicroRTSMixedMapVecEnv); _tensor_outputs()
    afterwards returns what step_wait would."""
    if not self._mask_fresh:
        self.get_action_mask()
    self._mask_fresh = self.eager_masks
    return _native.StepIO(self._actions_in.data_ptr(), self._src.data_ptr(), self._obs.data_ptr(), self._raw.data_ptr(),
                          self._done.data_ptr(), self._rew.data_ptr(), self._done0.data_ptr())

def _tensor_outputs(self):
    raw = self._raw
    if not self.reward_shaping:
        raw = raw.clone()
        raw[:, 1:] = 0
    if len(self.cycle_maps) > self._cycle_min:
        self._cycle(self._done0.cpu().numpy())
    return self._obs, self._rew, self._done0, LazyInfos(raw)



vec_env.MicroRTSGridModeVecEnv.step_wait = step_wait
import bench  # noqa: E402

sys.argv = ["bench.py"] + sys.argv[1:]
bench.main()
