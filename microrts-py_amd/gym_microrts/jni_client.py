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
  .clients[j]                -> bot env j's game client (JNIGridnetClient): .mapPath, .reset(p), .getResponse(p)
  .selfPlayClients[k]        -> selfplay game k (JNIGridnetClientSelfPlay, envs 2k / 2k+1): .mapPath, .reset(),
                                .getResponse(p)
  .render(True) / .sendUTT() on either kind (the reference's render_client, vec_env.py:272-276, 1077-1083)
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


RENDER_SIZE = 640   # PhysicalGameStatePanel frame of the reference (vec_env.py:1083)
MAP_SLOTS = 64      # map-table slots for maps set later through .mapPath


class GameClient:
    """One game of the vec client: ts.JNIGridnetClient (a bot env, `envs` = [env])
    or ts.JNIGridnetClientSelfPlay (`envs` = [2k, 2k + 1]).  The calls the
    reference's map cycling and render make (vec_env.py:272-276, 1044-1054,
    1077-1083):

      c.mapPath = path       the map of the game's next reset (Java re-reads the
                             file; here mrts_add_map loads it into a free slot)
      c.reset(p=0)           the game back to mapPath (mrts_reset_games); a bot
                             client returns player p's Response, a selfplay one
                             nothing (then getResponse(0) / getResponse(1))
      c.getResponse(p)       Response of the game's player p: raw observation of
                             this state, reward and done of the last step (zero after a reset)
      c.render(True)         the frame as BGR bytes [640*640*3] (the reference turns
                             them into an image and flips them back to RGB); render(False)
                             opens no window on a headless GPU host and returns None
      c.sendUTT()            UnitTypeTable JSON
    """

    def __init__(self, vec, game, envs, map_path):
        self._vec = vec
        self.game = game
        self.envs = envs
        self._map_path = map_path

    @property
    def mapPath(self):  # noqa: N802 (Java name)
        return self._map_path

    @mapPath.setter
    def mapPath(self, path):  # noqa: N802
        self._vec._map_id(path)   # load now: a bad path fails at the assignment
        self._map_path = path

    def reset(self, player=None):
        self._vec._reset_game(self.game, self._vec._map_id(self._map_path))
        if len(self.envs) == 1:
            return self.getResponse(0 if player is None else player)
        return None

    def getResponse(self, player):  # noqa: N802
        env = self.envs[player] if len(self.envs) > 1 else self.envs[0]
        return self._vec._env_response(env)

    def render(self, rgb):
        return self._vec._render(self.envs[0], rgb)

    def sendUTT(self):  # noqa: N802
        return self._vec.utt_json


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
                                 _native.MRTS_OBS_INT32, map_capacity=len(table) + MAP_SLOTS)
        self.microrts_path = microrts_path
        self._map_table = list(table)
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
        self._raw_cache = None   # host copy of _raw_obs for the current engine state (_raw_host)
        L = _native.lib()
        _native.check(L.mrts_bind_workspace(self._h, self._ws.data_ptr(), self._stream()), self._h, "bind_workspace")
        self.utt_json = L.mrts_utt_json(self._h).decode()
        # per-game clients (Java: JNIGridnetClientSelfPlay per pair, JNIGridnetClient per bot env)
        self.selfPlayClients = [GameClient(self, k, [2 * k, 2 * k + 1], table[game_map[k]]) for k in range(nsp_games)]
        self.clients = [GameClient(self, nsp_games + j, [num_selfplay_envs + j], table[game_map[nsp_games + j]])
                        for j in range(num_bot_envs)]
        self._frame = None

    def _stream(self):
        return torch.cuda.current_stream(self.device).cuda_stream

    def _raw_host(self):
        """Every env's raw observation as a host array, computed (k_raw + one D2H) once
        per engine state: reset, gameStep and per-game resets invalidate it, so the
        reference's cycling loop (one getResponse per finished env, vec_env.py:1044-1054)
        costs one kernel per tick, not one per finished env."""
        if self._raw_cache is None:
            _native.check(_native.lib().mrts_get_raw_obs(self._h, self._stream(), self._raw_obs.data_ptr()), self._h, "raw_obs")
            self._raw_cache = self._raw_obs.cpu().numpy()
        return self._raw_cache

    def _response(self):
        return Response(self._raw_host().copy(), self._rew.cpu().numpy(), self._done.cpu().numpy().astype(bool))

    def reset(self, players):
        self._raw_cache = None
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
        self._raw_cache = None
        _native.check(_native.lib().mrts_step(self._h, self._stream(), a.data_ptr(), s.data_ptr(), self._obs.data_ptr(),
                                              self._rew.data_ptr(), self._done.data_ptr()), self._h, "step")
        return self._response()

    # ---- per-game calls (GameClient)
    def _map_id(self, path):
        full = path if os.path.isabs(path) else os.path.join(self.microrts_path, path)
        return _native.add_map(self._h, self._stream(), full)

    def _reset_game(self, game, map_id):
        self._raw_cache = None
        g = (ctypes.c_int32 * 1)(game)
        m = (ctypes.c_int32 * 1)(map_id)
        _native.check(_native.lib().mrts_reset_games(self._h, self._stream(), g, m, 1, self._obs.data_ptr()), self._h,
                      "reset_games")
        envs = [e for c in self.selfPlayClients + self.clients if c.game == game for e in c.envs]
        self._rew[envs] = 0
        self._done[envs] = 0

    def _env_response(self, env):
        return Response(self._raw_host()[env].copy(), self._rew[env].cpu().numpy(),
                        self._done[env].cpu().numpy().astype(bool))

    def _render(self, env, rgb):
        if not rgb:
            return None   # render(False): the Swing window; no display on the GPU host
        if self._frame is None:
            self._frame = torch.empty((RENDER_SIZE, RENDER_SIZE, 3), dtype=torch.uint8, device=self.device)
        _native.check(_native.lib().mrts_render(self._h, self._stream(), env, self._frame.data_ptr(), RENDER_SIZE), self._h,
                      "render")
        return self._frame.flip(-1).contiguous().cpu().numpy().reshape(-1)   # BGR byte order, as the Java returns

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
