"""ctypes binding of the CPU restatement (oracle/libmrts_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, never by the product package (microrts-py_amd/).

OracleVecEnv mirrors the JNIGridnetVecClient + MicroRTSGridModeVecEnv pair of
/root/reference/gym_microrts/envs/vec_env.py (reset 278-282, step_async/step_wait
968-1057, get_action_mask 1091-1101) closely enough that the ported reference
tests read the same against it.
"""
import ctypes
import os
import subprocess
import xml.etree.ElementTree as ET

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# MRTS_ORACLE_LIB: another build of the same sources (the ASan/UBSan one, tests/test_oracle_asan.py)
LIB_PATH = os.environ.get("MRTS_ORACLE_LIB") or os.path.join(HERE, "libmrts_oracle.so")
UNIT_TYPES = ["Resource", "Base", "Barracks", "Worker", "Light", "Heavy", "Ranged"]
AI_IDS = {"passiveAI": 0, "workerRushAI": 1, "lightRushAI": 2, "randomBiasedAI": 3, "coacAI": 4,
          "POWorkerRush": 5, "POLightRush": 6, "POHeavyRush": 7, "PORangedRush": 8, "randomAI": 9}

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        L.ovec_create.restype = P
        L.ovec_create.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, P, ctypes.c_int, P, P, P]
        L.ovec_destroy.argtypes = [P]
        L.ovec_reset.argtypes = [P]
        L.ovec_reset_game.argtypes = [P, ctypes.c_int, ctypes.c_int]
        L.ovec_get_masks.argtypes = [P, P]
        L.ovec_step.argtypes = [P, P, P, P, P]
        L.ovec_raw_obs.argtypes = [P, P]
        L.ovec_encode_obs.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, P]
        L.ovec_game_time.argtypes = [P, ctypes.c_int]
        L.ovec_game_time.restype = ctypes.c_int
        L.ovec_game_resources.argtypes = [P, ctypes.c_int, P]
        L.ovec_dump_cells.argtypes = [P, ctypes.c_int, P]
        L.ovec_sample_actions.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint32, P]
        L.ovec_bench_steps.argtypes = [P, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint32, P, P, P, P, P, P]
        L.ovec_event_counts.argtypes = [P, P]
        _lib = L
    return _lib


class _OMap(ctypes.Structure):
    _fields_ = [
        ("width", ctypes.c_int32),
        ("height", ctypes.c_int32),
        ("terrain", ctypes.c_void_p),
        ("player_res", ctypes.c_int32 * 2),
        ("num_units", ctypes.c_int32),
        ("units", ctypes.c_void_p),
    ]


def parse_map(path):
    """PhysicalGameState.load restated in Python (XML order kept)."""
    root = ET.parse(path).getroot()
    w, h = int(root.get("width")), int(root.get("height"))
    terrain = np.array([int(ch) for ch in root.find("terrain").text.strip()], dtype=np.uint8)
    assert terrain.size == w * h
    res = [0, 0]
    for p in root.find("players"):
        res[int(p.get("ID"))] = int(p.get("resources"))
    units = []
    for u in root.find("units"):
        units.append([UNIT_TYPES.index(u.get("type")), int(u.get("player")), int(u.get("x")), int(u.get("y")),
                      int(u.get("resources")), int(u.get("hitpoints"))])
    return {"width": w, "height": h, "terrain": terrain, "res": res, "units": np.array(units, dtype=np.int32).reshape(-1, 6)}


def ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


class OracleVecEnv:
    """The oracle behind a MicroRTSGridModeVecEnv-shaped surface."""

    def __init__(self, num_selfplay_envs, num_bot_envs, map_paths, max_steps=2000, partial_obs=False,
                 ai2s=None, reward_weight=None, game_maps=None, ai1s=None):
        self.num_selfplay_envs, self.num_bot_envs = num_selfplay_envs, num_bot_envs
        self.num_envs = num_selfplay_envs + num_bot_envs
        self.num_games = num_selfplay_envs // 2 + num_bot_envs
        self.partial_obs = partial_obs
        self.maps = [parse_map(p) for p in map_paths]
        self.height, self.width = self.maps[0]["height"], self.maps[0]["width"]
        self._keep = []
        arr = (_OMap * len(self.maps))()
        for i, m in enumerate(self.maps):
            arr[i].width, arr[i].height = m["width"], m["height"]
            arr[i].terrain = ptr(m["terrain"])
            arr[i].player_res[0], arr[i].player_res[1] = m["res"]
            arr[i].num_units = len(m["units"])
            arr[i].units = ptr(m["units"])
        gm = np.zeros(self.num_games, np.int32) if game_maps is None else np.asarray(game_maps, np.int32)
        ai = np.array([AI_IDS[a] if isinstance(a, str) else a for a in (ai2s or [0] * num_bot_envs)], np.int32)
        if ai.size == 0:
            ai = np.zeros(1, np.int32)
        # bot-vs-bot games (MicroRTSBotVecEnv): ai1s[j] plays player 0 of bot env j
        ai0 = np.array([AI_IDS[a] if isinstance(a, str) else a for a in ai1s], np.int32) if ai1s else None
        self._ai0 = ai0
        self._h = lib().ovec_create(num_selfplay_envs, num_bot_envs, max_steps, int(partial_obs),
                                    ctypes.cast(arr, ctypes.c_void_p), len(self.maps), ptr(gm), ptr(ai),
                                    ptr(ai0) if ai0 is not None else None)
        self.reward_weight = np.asarray(reward_weight if reward_weight is not None else [10.0, 1.0, 1.0, 0.2, 1.0, 4.0])
        hw = self.height * self.width
        self.P_raw = 7 if partial_obs else 6
        self.source_unit_mask = np.zeros((self.num_envs, hw), np.int32)

    def close(self):
        if self._h:
            lib().ovec_destroy(self._h)
            self._h = None

    __del__ = close

    def raw_obs(self):
        raw = np.zeros((self.num_envs, self.P_raw, self.height, self.width), np.int32)
        lib().ovec_raw_obs(self._h, ptr(raw))
        return raw

    def encode(self, raw):
        P = 31 if self.partial_obs else 29
        out = np.zeros((raw.shape[0], self.height, self.width, P), np.int32)
        lib().ovec_encode_obs(ptr(np.ascontiguousarray(raw)), raw.shape[0], self.height, self.width, int(self.partial_obs), ptr(out))
        return out

    def reset(self):
        lib().ovec_reset(self._h)
        return self.encode(self.raw_obs())

    def reset_game(self, game, map_id):
        lib().ovec_reset_game(self._h, game, map_id)

    def get_action_mask_full(self):
        m = np.zeros((self.num_envs, self.height * self.width, 79), np.int32)
        lib().ovec_get_masks(self._h, ptr(m))
        return m

    def get_action_mask(self):
        m = self.get_action_mask_full()
        self.source_unit_mask = np.ascontiguousarray(m[:, :, 0])
        return np.ascontiguousarray(m[:, :, 1:])

    def step_raw(self, actions):
        a = np.ascontiguousarray(np.asarray(actions).reshape(self.num_envs, self.height * self.width, 7).astype(np.int64))
        reward = np.zeros((self.num_envs, 6), np.float64)
        done = np.zeros((self.num_envs, 6), np.uint8)
        lib().ovec_step(self._h, ptr(a), ptr(self.source_unit_mask), ptr(reward), ptr(done))
        return reward, done.astype(bool)

    def step(self, actions):
        reward, done = self.step_raw(actions)
        obs = self.encode(self.raw_obs())
        infos = [{"raw_rewards": r} for r in reward]
        return obs, reward @ self.reward_weight, done[:, 0], infos

    def game_time(self, g):
        return lib().ovec_game_time(self._h, g)

    def game_resources(self, g):
        r = np.zeros(2, np.int32)
        lib().ovec_game_resources(self._h, g, ptr(r))
        return r

    def bench_steps(self, steps, seed, step0):
        """`steps` whole env-steps in C (masks, sampler, step, encode; OpenMP):
        the bench's CPU baseline.  Returns the last (obs, raw rewards, dones)."""
        n, hw = self.num_envs, self.height * self.width
        if getattr(self, "_bench_bufs", None) is None:
            P = 31 if self.partial_obs else 29
            self._bench_bufs = (np.zeros((n, hw, 79), np.int32), np.zeros((n, hw, 7), np.int64), np.zeros((n, hw), np.int32),
                                np.zeros((n, 6), np.float64), np.zeros((n, 6), np.uint8),
                                np.zeros((n, self.height, self.width, P), np.int32))
        m, a, src, rew, done, obs = self._bench_bufs
        lib().ovec_bench_steps(self._h, steps, ctypes.c_uint64(seed), ctypes.c_uint32(step0), ptr(m), ptr(a), ptr(src),
                               ptr(rew), ptr(done), ptr(obs))
        return obs, rew, done.astype(bool)

    def event_counts(self):
        """Trajectory statistics summed over every game (ovec_event_counts): CANCEL_BOTH and
        inconsistent-issue conflicts, units produced per player and type, hits, kills."""
        c = np.zeros(20, np.int64)
        lib().ovec_event_counts(self._h, ptr(c))
        prod = c[2:16].reshape(2, 7)
        return {"cancel_both": int(c[0]), "inconsistent": int(c[1]),
                "produced": [{t: int(prod[p, i]) for i, t in enumerate(UNIT_TYPES)} for p in range(2)],
                "hits": [int(c[16]), int(c[17])], "kills": [int(c[18]), int(c[19])]}

    def dump_cells(self, g):
        out = np.zeros((self.height * self.width, 8), np.int32)
        lib().ovec_dump_cells(self._h, g, ptr(out))
        return out


def sample_actions(masks78, seed, step, env0=0):
    """Philox-keyed masked sampler (same stream as the GPU bench sampler); env0 =
    global index of row 0's env (a shard of a larger batch)."""
    m = np.ascontiguousarray(masks78, dtype=np.int32)
    n, hw = m.shape[0], m.shape[1]
    out = np.zeros((n, hw, 7), np.int64)
    lib().ovec_sample_actions(ptr(m), n, hw, env0, ctypes.c_uint64(seed), ctypes.c_uint32(step), ptr(out))
    return out


# render("rgb_array") drawing rules, restated in numpy from the
# rule list -- the device k_render must match it pixel for pixel.
_RENDER_RGB = {0: 0x00A000, 1: 0xFFFFFF, 2: 0xA0A0A0, 3: 0x808080, 4: 0xFF8000, 5: 0xFFFF00, 6: 0x00FFFF}
_MAX_HP = {0: 1, 1: 10, 2: 4, 3: 1, 4: 4, 5: 4, 6: 1}


def render_frame(cells, wall, W, H, size=640):
    """cells: OracleVecEnv.dump_cells(g) (type, player, hp, ...) per cell; wall: u8 [H*W]."""
    col = np.zeros((size, size), np.int64)
    cs = size // max(W, H)
    ox, oy = (size - cs * W) // 2, (size - cs * H) // 2
    py, px = np.mgrid[0:size, 0:size]
    gx, gy = px - ox, py - oy
    ing = (gx >= 0) & (gy >= 0) & (gx < cs * W) & (gy < cs * H)
    cx, cy = np.where(ing, gx // cs, 0), np.where(ing, gy // cs, 0)
    lx, ly = gx - cx * cs, gy - cy * cs
    c = cy * W + cx
    wall = np.asarray(wall).reshape(-1)
    col = np.where(ing, np.where(wall[c] != 0, 0x205020, 0), 0)
    col = np.where(ing & ((lx == 0) | (ly == 0)), 0x303030, col)
    t, owner, hp = cells[c, 0], cells[c, 1], cells[c, 2]
    m, b = cs // 8, max(1, cs // 16)
    building = (t == 0) | (t == 1) | (t == 2)
    sq_in = (lx >= m) & (ly >= m) & (lx < cs - m) & (ly < cs - m)
    sq_rim = (lx < m + b) | (ly < m + b) | (lx >= cs - m - b) | (ly >= cs - m - b)
    r2 = cs * 3 // 4
    d2 = (2 * lx + 1 - cs) ** 2 + (2 * ly + 1 - cs) ** 2
    ci_in, ci_rim = d2 <= r2 * r2, d2 > (r2 - 2 * b) ** 2
    inside = np.where(building, sq_in, ci_in)
    rim = np.where(building, sq_rim, ci_rim)
    unit = ing & (t >= 0)
    fill = np.vectorize(lambda k: _RENDER_RGB.get(int(k), 0))(np.clip(t, 0, 6))
    rimc = np.where(owner == 0, 0x0000FF, 0xFF0000)
    ucol = np.where(rim & (owner >= 0), rimc, fill)
    col = np.where(unit & inside, ucol, col)
    mhp = np.vectorize(lambda k: _MAX_HP.get(int(k), 1))(np.clip(t, 0, 6))
    bar = unit & (t != 0) & (hp < mhp) & (ly >= cs - m - 2 * b) & (ly < cs - m) & (lx >= m) & (lx < m + (cs - 2 * m) * hp // mhp)
    col = np.where(bar, 0xFF0000, col)
    rgb = np.stack([(col >> 16) & 255, (col >> 8) & 255, col & 255], -1).astype(np.uint8)
    return rgb
