"""ctypes binding of libmicrorts_amd.so (include/microrts_amd.h).

The library is built in-tree (`make -C microrts-py_amd/csrc`, or
`python __graft_entry__.py`) and resolves `libamdhip64.so.7` to the copy torch
already loaded, so kernels run on torch's HIP runtime and streams.  There is no
CPU fallback: if the library is missing this module raises MicroRTSError.
"""
import ctypes
import os

import torch  # noqa: F401  (load torch's HIP runtime before the engine library)

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libmicrorts_amd.so")

MRTS_OK = 0
MRTS_OBS_INT32 = 0
MRTS_OBS_FLOAT32 = 1
MRTS_GAME_STATS = 6
ERROR_NAMES = {-1: "EINVAL", -2: "EIO", -3: "EHIP", -4: "ENOTIMPL", -5: "ESTATE"}


class MicroRTSError(RuntimeError):
    """Engine error.  Also answers printStackTrace(): the reference's callers
    invoke that Java method on exceptions raised through JPype
    (/root/reference/experiments/ppo_gridnet.py:477-479, tests/test_mask.py:24)."""

    def printStackTrace(self):  # noqa: N802 (Java name kept on purpose)
        import traceback

        traceback.print_exception(type(self), self, self.__traceback__)


class MicroRTSNotImplemented(MicroRTSError, NotImplementedError):
    pass


class Config(ctypes.Structure):
    _fields_ = [
        ("num_selfplay_envs", ctypes.c_int32),
        ("num_bot_envs", ctypes.c_int32),
        ("max_steps", ctypes.c_int32),
        ("partial_obs", ctypes.c_int32),
        ("num_maps", ctypes.c_int32),
        ("map_paths", ctypes.POINTER(ctypes.c_char_p)),
        ("game_map", ctypes.POINTER(ctypes.c_int32)),
        ("bot_ai", ctypes.POINTER(ctypes.c_int32)),
        ("obs_dtype", ctypes.c_int32),
        ("bot_ai0", ctypes.POINTER(ctypes.c_int32)),
        ("game_offset", ctypes.c_int32),
        ("map_capacity", ctypes.c_int32),
    ]


class Info(ctypes.Structure):
    _fields_ = [
        ("height", ctypes.c_int32),
        ("width", ctypes.c_int32),
        ("num_envs", ctypes.c_int32),
        ("num_games", ctypes.c_int32),
        ("obs_planes", ctypes.c_int32),
        ("mask_channels", ctypes.c_int32),
        ("action_components", ctypes.c_int32),
        ("workspace_bytes", ctypes.c_size_t),
    ]


P = ctypes.c_void_p


class StepIO(ctypes.Structure):
    """mrts_step_io: one engine's buffers of an mrts_step_group call."""
    _fields_ = [("actions", P), ("source", P), ("obs", P), ("raw_reward", P), ("done", P), ("reward", P), ("done0", P)]


STEP_GROUP_MAX = 4


class SampleSeg(ctypes.Structure):
    """mrts_sample_seg: one batch of an mrts_sample_actions_src_group call."""
    _fields_ = [("mask", P), ("source", P), ("num_envs", ctypes.c_int32), ("hw", ctypes.c_int32), ("env0", ctypes.c_int32),
                ("actions", P)]


SAMPLE_GROUP_MAX = 4
GROUP_SEPARATE, GROUP_MERGE_FIT, GROUP_MERGE_ALL, GROUP_BOTS_FIRST = 0, 1, 2, 4

# every entry point of include/microrts_amd.h: (restype, argtypes)
SIGNATURES = {
    "mrts_create": (ctypes.c_int, [ctypes.POINTER(Config), ctypes.POINTER(P)]),
    "mrts_info": (ctypes.c_int, [P, ctypes.POINTER(Info)]),
    "mrts_bind_workspace": (ctypes.c_int, [P, P, P]),
    "mrts_reset": (ctypes.c_int, [P, P, P]),
    "mrts_get_masks": (ctypes.c_int, [P, P, P, P]),
    "mrts_step": (ctypes.c_int, [P, P, P, P, P, P, P]),
    "mrts_get_raw_obs": (ctypes.c_int, [P, P, P]),
    "mrts_set_reward_weight": (ctypes.c_int, [P, P, ctypes.c_int32]),
    "mrts_step_weighted": (ctypes.c_int, [P, P, P, P, P, P, P, P, P]),
    "mrts_step_group": (ctypes.c_int, [P, ctypes.c_int32, P, P, ctypes.c_int32]),
    "mrts_step_group_plan": (ctypes.c_int, [P, ctypes.c_int32, ctypes.c_int32, P, P]),
    "mrts_reset_games": (ctypes.c_int, [P, P, P, P, ctypes.c_int32, P]),
    "mrts_add_map": (ctypes.c_int, [P, P, ctypes.c_char_p, P]),
    "mrts_park_games": (ctypes.c_int, [P, P, P, ctypes.c_int32, P]),
    "mrts_sample_actions": (ctypes.c_int, [P, P, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint64, ctypes.c_uint32, P]),
    "mrts_sample_actions_src": (ctypes.c_int, [P, P, P, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint64,
                                               ctypes.c_uint32, P]),
    "mrts_sample_actions_src_group": (ctypes.c_int, [P, P, ctypes.c_int32, ctypes.c_uint64, ctypes.c_uint32]),
    "mrts_game_stats": (ctypes.c_int, [P, P, P]),
    "mrts_bind_mask_outputs": (ctypes.c_int, [P, P, P]),
    "mrts_set_bot_fusion": (ctypes.c_int, [P, ctypes.c_int32]),
    "mrts_render": (ctypes.c_int, [P, P, ctypes.c_int32, P, ctypes.c_int32]),
    "mrts_error_flags": (ctypes.c_int, [P, P, P]),
    "mrts_state_bytes": (ctypes.c_size_t, [P]),
    "mrts_save_state": (ctypes.c_int, [P, P, P]),
    "mrts_load_state": (ctypes.c_int, [P, P, P, P]),
    "mrts_fused_layout_ok": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32]),
    "mrts_utt_json": (ctypes.c_char_p, [P]),
    "mrts_last_error": (ctypes.c_char_p, [P]),
    "mrts_destroy": (None, [P]),
    "mrts_version": (ctypes.c_char_p, []),
}

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise MicroRTSError(
                f"{LIB_PATH} is not built: run `make -C microrts-py_amd/csrc` (or __graft_entry__.build()); "
                "there is no CPU fallback for the engine"
            )
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(rc, handle=None, what="call"):
    if rc != MRTS_OK:
        msg = lib().mrts_last_error(handle).decode() if handle else ""
        cls = MicroRTSNotImplemented if rc == -4 else MicroRTSError
        raise cls(f"libmicrorts_amd {what} failed ({ERROR_NAMES.get(rc, rc)}): {msg}")


def create(num_selfplay_envs, num_bot_envs, max_steps, partial_obs, map_paths, game_map, bot_ai, obs_dtype, bot_ai0=None,
           game_offset=0, map_capacity=0):
    cfg = Config()
    cfg.num_selfplay_envs = num_selfplay_envs
    cfg.num_bot_envs = num_bot_envs
    cfg.max_steps = max_steps
    cfg.partial_obs = int(bool(partial_obs))
    cfg.num_maps = len(map_paths)
    paths = (ctypes.c_char_p * len(map_paths))(*[p.encode() for p in map_paths])
    cfg.map_paths = ctypes.cast(paths, ctypes.POINTER(ctypes.c_char_p))
    gm = (ctypes.c_int32 * max(1, len(game_map)))(*game_map)
    ai = (ctypes.c_int32 * max(1, len(bot_ai)))(*bot_ai)
    cfg.game_map = ctypes.cast(gm, ctypes.POINTER(ctypes.c_int32))
    cfg.bot_ai = ctypes.cast(ai, ctypes.POINTER(ctypes.c_int32))
    cfg.obs_dtype = obs_dtype
    cfg.game_offset = int(game_offset)
    cfg.map_capacity = int(map_capacity)
    if bot_ai0 is not None:
        a0 = (ctypes.c_int32 * max(1, len(bot_ai0)))(*bot_ai0)
        cfg.bot_ai0 = ctypes.cast(a0, ctypes.POINTER(ctypes.c_int32))
    h = P()
    rc = lib().mrts_create(ctypes.byref(cfg), ctypes.byref(h))
    if rc != MRTS_OK:
        msg = lib().mrts_last_error(h).decode() if h else ""
        if h:
            lib().mrts_destroy(h)
        cls = MicroRTSNotImplemented if rc == -4 else MicroRTSError
        raise cls(f"libmicrorts_amd create failed ({ERROR_NAMES.get(rc, rc)}): {msg}")
    return h


def add_map(h, stream, path):
    """mrts_add_map: the map-table index of `path`, loading it if new."""
    idx = ctypes.c_int32(-1)
    check(lib().mrts_add_map(h, stream, path.encode(), ctypes.byref(idx)), h, "add_map")
    return int(idx.value)


def info(h):
    i = Info()
    check(lib().mrts_info(h, ctypes.byref(i)), h, "info")
    return i
