"""JNIGridnetVecClient-shaped client over libmicrorts_amd.so.

The reference's MicroRTSGridModeVecEnv talks to Java through one object,
`ts.JNIGridnetVecClient` (constructed at
/root/reference/gym_microrts/envs/vec_env.py:259-271, called at :279, :1002,
:1088, :1097).  This class has the same constructor arguments and the same
four calls, so a maintainer can keep the reference's own vec_env.py (its
python `_encode_obs`, action packing and reward weighting) and swap only the
client (INTEGRATION.md shows the three-line diff).  The engine behind it is the
same HIP path as gym_microrts.envs.vec_env: the arrays it returns are copied
back from device buffers, exactly as JPype copied them out of the JVM.

  Client(num_selfplay, num_bot, max_steps, rfs, micrortsPath, mapPaths, ai2s, utt, partialObs)
  .reset(players)            -> Response(observation int32 [N][P_raw][H][W], reward f64 [N][6], done bool [N][6])
  .gameStep(actions, players)-> Response   (actions: per env a [k_i][8] array of (cell, 7 components) rows)
  .getMasks(player)          -> int32 [N][H][W][79]
  .close()
"""
import ctypes
import os

import numpy as np
import torch

from gym_microrts import _native


class Response:
    """ts.Response: the fields vec_env.py reads (observation, reward, done)."""

    def __init__(self, observation, reward, done):
        self.observation = observation
        self.reward = reward
        self.done = done


class JNIGridnetVecClient:
    def __init__(self, num_selfplay_envs, num_bot_envs, max_steps, rfs, microrts_path, map_paths, ai2s, utt=None,
                 partial_obs=False, device=None):
        if device is None:
            if not torch.cuda.is_available():
                raise _native.MicroRTSError("JNIGridnetVecClient needs a GPU (HIP) device: the engine has no CPU fallback")
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        self.num_envs = num_selfplay_envs + num_bot_envs
        self.rfs = rfs
        full = [p if os.path.isabs(p) else os.path.join(microrts_path, p) for p in map_paths]
        table = []
        for p in full:
            if p not in table:
                table.append(p)
        nsp_games = num_selfplay_envs // 2
        game_env = [2 * k for k in range(nsp_games)] + [num_selfplay_envs + j for j in range(num_bot_envs)]
        game_map = [table.index(full[e] if len(full) > 1 else full[0]) for e in game_env]
        bot_ai = []
        for a in ai2s:
            d = a(utt) if callable(a) else a
            if getattr(d, "ai_id", None) is None:
                raise _native.MicroRTSNotImplemented(f"bot {d} has no device implementation")
            bot_ai.append(d.ai_id)
        self._h = _native.create(num_selfplay_envs, num_bot_envs, max_steps, partial_obs, table, game_map, bot_ai,
                                 _native.MRTS_OBS_INT32)
        info = _native.info(self._h)
        self.height, self.width, self.P_raw = info.height, info.width, 7 if partial_obs else 6
        hw = self.height * self.width
        n = self.num_envs
        with torch.cuda.device(self.device):
            self._ws = torch.empty(int(info.workspace_bytes), dtype=torch.uint8, device=self.device)
            self._obs = torch.empty((n, hw, info.obs_planes), dtype=torch.int32, device=self.device)
            self._raw_obs = torch.empty((n, self.P_raw, self.height, self.width), dtype=torch.int32, device=self.device)
            self._mask = torch.empty((n, hw, 78), dtype=torch.int32, device=self.device)
            self._src = torch.empty((n, hw), dtype=torch.int32, device=self.device)
            self._rew = torch.zeros((n, 6), dtype=torch.float64, device=self.device)
            self._done = torch.zeros((n, 6), dtype=torch.uint8, device=self.device)
        L = _native.lib()
        _native.check(L.mrts_bind_workspace(self._h, self._ws.data_ptr(), self._stream()), self._h, "bind_workspace")

    def _stream(self):
        return torch.cuda.current_stream(self.device).cuda_stream

    def _response(self):
        _native.check(_native.lib().mrts_get_raw_obs(self._h, self._stream(), self._raw_obs.data_ptr()), self._h, "raw_obs")
        return Response(self._raw_obs.cpu().numpy(), self._rew.cpu().numpy(), self._done.cpu().numpy().astype(bool))

    def reset(self, players):
        _native.check(_native.lib().mrts_reset(self._h, self._stream(), self._obs.data_ptr()), self._h, "reset")
        self._rew.zero_()
        self._done.zero_()
        return self._response()

    def getMasks(self, player):  # noqa: N802 (Java name)
        _native.check(_native.lib().mrts_get_masks(self._h, self._stream(), self._mask.data_ptr(), self._src.data_ptr()),
                      self._h, "get_masks")
        m = torch.cat([self._src.unsqueeze(-1), self._mask], dim=-1)
        return m.reshape(self.num_envs, self.height, self.width, 79).cpu().numpy()

    def gameStep(self, actions, players):  # noqa: N802 (Java name)
        """actions: the reference's ragged int[N][k_i][8] rows (vec_env.py:968-984)."""
        hw = self.height * self.width
        dense = np.zeros((self.num_envs, hw, 7), np.int64)
        src = np.zeros((self.num_envs, hw), np.int32)
        for i, rows in enumerate(actions):
            r = np.asarray(rows, dtype=np.int64).reshape(-1, 8)
            if r.size:
                dense[i, r[:, 0]] = r[:, 1:]
                src[i, r[:, 0]] = 1
        a = torch.from_numpy(dense).to(self.device)
        s = torch.from_numpy(src).to(self.device)
        _native.check(_native.lib().mrts_step(self._h, self._stream(), a.data_ptr(), s.data_ptr(), self._obs.data_ptr(),
                                              self._rew.data_ptr(), self._done.data_ptr()), self._h, "step")
        return self._response()

    def close(self):
        if getattr(self, "_h", None):
            torch.cuda.synchronize(self.device)
            _native.lib().mrts_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
