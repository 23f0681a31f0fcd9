"""MicroRTSGridModeVecEnv on the MI355X engine.

Keeps the constructor signature and the reset / get_action_mask / step surface of
/root/reference/gym_microrts/envs/vec_env.py:38-1101 so that
experiments/ppo_gridnet.py runs unmodified.  Everything the reference does in
Java (JNIGridnetVecClient over JPype) and in the per-env numpy loops
(_encode_obs, action packing, reward weighting) happens in libmicrorts_amd.so
kernels on the GPU; this class only moves buffers and keeps the Python contract.

Return types (`return_tensors`, or the environment variable MICRORTS_AMD_RETURN
when the keyword is not given -- so an unmodified driver script can select one)
  * "numpy" (False, the default): exactly the reference's -- numpy int32 obs
    (N,H,W,29), numpy int32 masks (N,H*W,78), numpy float64 rewards, numpy bool
    dones, a list of {"raw_rewards": row} dicts.
  * "tensors" (True): device-resident torch tensors (obs float32 by default,
    masks int32, rewards float64, dones bool) and a lazily materialised infos
    sequence.  Tensors alias engine-owned buffers that are overwritten by the
    next call (the ownership rule of the reference's shared-memory env,
    vec_env.py:1331-1362).
  * "hybrid": the contract an unmodified experiments/ppo_gridnet.py needs to keep
    obs and masks in HBM: obs (float32 device tensor: its
    `torch.Tensor(x)` aliases a float32 tensor, ppo_gridnet.py:421, 476) and masks
    (int32 device tensor: `torch.tensor(x).to(device)`, :466) stay on the GPU,
    while rewards (numpy float64, `raw @ reward_weight` in numpy as the
    reference), dones (numpy bool) and infos (a list of {"raw_rewards": numpy
    row}) are host objects, because MicroRTSStatsRecorder indexes dones[i] /
    infos[i] per env and VecMonitor accumulates with numpy (:138-160).  Host
    actions (:475) are accepted as in the numpy contract.
"""
import json
import os
import warnings
import xml.etree.ElementTree as ET
from enum import Enum

import numpy as np
import torch

import gym_microrts
from gym_microrts import _native
from gym_microrts._native import MicroRTSError, MicroRTSNotImplemented
from gym_microrts._spaces import Box, Discrete, MultiDiscrete

# Tracing: MICRORTS_AMD_MARKERS=1 puts a named roctx range ("mrts_step",
# "mrts_masks", "mrts_reset", ...) around every engine launch, for rocprofv3 --marker-trace /
# --sys-trace timelines next to the kernel trace; off by default (no call at all)
MARKERS = os.environ.get("MICRORTS_AMD_MARKERS", "0").strip() not in ("", "0")

RENDER_SIZE = 640   # vec_env.py:1083: Image.frombytes("RGB", (640, 640), ...)

RF_NAMES = [
    "WinLossRewardFunction",
    "ResourceGatherRewardFunction",
    "ProduceWorkerRewardFunction",
    "ProduceBuildingRewardFunction",
    "AttackRewardFunction",
    "ProduceCombatUnitRewardFunction",
]


class RewardFunction:
    """Stand-in for the ai.reward.* Java objects of vec_env.py:185-195; callers
    only use str(rf) (ppo_gridnet.py:145-147, league.py:278)."""

    def __init__(self, name):
        self.name = name

    def __str__(self):
        return self.name

    __repr__ = __str__


class LazyInfos:
    """list[dict] view over the (N,6) raw-reward tensor, materialised on access
    (the per-env dict creation of vec_env.py:1036 is the host cost avoided)."""

    def __init__(self, raw):
        self._raw = raw
        self._np = None

    def _rows(self):
        if self._np is None:
            self._np = self._raw.detach().cpu().numpy()
        return self._np

    def __len__(self):
        return self._raw.shape[0]

    def __getitem__(self, i):
        rows = self._rows()
        if isinstance(i, slice):
            return [{"raw_rewards": r} for r in rows[i]]
        return {"raw_rewards": rows[i]}

    def __iter__(self):
        for r in self._rows():
            yield {"raw_rewards": r}


class HostArrayPool:
    """Page-locked host arrays handed out as fresh numpy arrays.

    The reference's numpy contract returns a new array from every call
    (`np.array(...)` of the JPype result, vec_env.py:280, 1003, 1097), and a
    caller may keep it as long as it likes.  Copying the device outputs into
    fresh pageable arrays costs a staged D2H plus first-touch page faults on
    every call (hundreds of MB per step at 8192 envs).  This pool keeps a few
    page-locked buffers per output and hands out a numpy view of one; a buffer
    is reused only when no array derived from it is still alive (every numpy
    view, and torch.from_numpy of one, keeps the owning array referenced), so a
    returned array is never overwritten behind the caller's back.  When every
    buffer is held, the pool grows up to `limit`, then falls back to plain
    fresh arrays."""

    def __init__(self, pinned=True, limit=3):
        import sys

        self._refs = sys.getrefcount
        self.pinned = pinned
        self.limit = limit
        self._bufs = {}   # key -> [(tensor, owner ndarray, idle refcount)]

    def d2h(self, key, src):
        """Enqueue src (device tensor) -> a free host buffer on the current stream;
        the returned numpy array is valid after the stream is synchronised."""
        bufs = self._bufs.setdefault(key, [])
        for t, n, idle in bufs:
            if self._refs(n) == idle and t.shape == src.shape and t.dtype == src.dtype:
                t.copy_(src, non_blocking=True)
                return n[...]
        if len(bufs) < self.limit:
            t = torch.empty(tuple(src.shape), dtype=src.dtype, pin_memory=self.pinned)
            n = t.numpy()
            entry = [t, n, 0]
            bufs.append(entry)
            entry[2] = self._refs(n)   # the pool's slot + this frame's name + the call (as in the loop above)
            t.copy_(src, non_blocking=True)
            return n[...]
        out = torch.empty(tuple(src.shape), dtype=src.dtype)
        out.copy_(src)
        return out.numpy()


CONTRACTS = {False: "numpy", "numpy": "numpy", True: "tensors", "tensors": "tensors", "hybrid": "hybrid"}


def contract_of(return_tensors):
    """The return contract for a `return_tensors` keyword value; None = the
    environment variable MICRORTS_AMD_RETURN (numpy | tensors | hybrid), default numpy."""
    if return_tensors is None:
        return_tensors = os.environ.get("MICRORTS_AMD_RETURN", "numpy").strip().lower() or "numpy"
    try:
        return CONTRACTS[return_tensors]
    except (KeyError, TypeError):
        raise ValueError(f"return_tensors must be one of False / True / 'numpy' / 'tensors' / 'hybrid', got {return_tensors!r}")


class MicroRTSGridModeVecEnv:
    metadata = {"render.modes": ["human", "rgb_array"], "video.frames_per_second": 150}
    _cycle_min = 0   # map cycling when len(cycle_maps) > _cycle_min (vec_env.py:1038)

    class PriorMode(Enum):
        """vec_env.py:48-84.  Only NONE is supported (the KG prior is out of
        scope)."""

        NONE = "none"
        APPEND_ENCODED = "append_encoded"
        APPEND_RAW = "append_raw"
        REWARD_ADVICE = "reward_advice"
        REWARD_SHAPING = "reward_shaping"

        def __bool__(self):
            return self != self.NONE

    def __init__(
        self,
        num_selfplay_envs,
        num_bot_envs,
        partial_obs=False,
        max_steps=2000,
        render_theme=2,
        frame_skip=0,
        ai2s=[],
        map_paths=["maps/10x10/basesTwoWorkers10x10.xml"],
        reward_shaping=True,
        reward_weight=np.array([0.0, 1.0, 0.0, 0.0, 0.0, 5.0]),
        cycle_maps=[],
        autobuild=False,
        jvm_args=[],
        prior_mode="none",
        reward_prior_weight=0.01,
        prior_advice_freq=1,
        seed=1,
        runs_dir=".",
        graph_ttl_file="graph.ttl",
        graph_triples_file="triples.tsv",
        *,
        device=None,
        return_tensors=None,
        obs_dtype=None,
        eager_masks=True,
        bot_fusion=True,
        game_offset=0,
        _ai1s=None,
        _extra_maps=(),
    ):
        # vec_env.py:110-127
        self.num_selfplay_envs = num_selfplay_envs
        self.num_bot_envs = num_bot_envs
        self.num_envs = num_selfplay_envs + num_bot_envs
        assert self.num_bot_envs == len(ai2s), "for each environment, a microrts ai should be provided"
        self.partial_obs = partial_obs
        self.max_steps = max_steps
        self.render_theme = render_theme  # stored, unused (as in the reference)
        self.frame_skip = frame_skip      # stored, unused (vec_env.py:116-117)
        self.ai2s = ai2s
        self.map_paths = map_paths
        if len(map_paths) == 1:
            self.map_paths = [map_paths[0] for _ in range(self.num_envs)]
        else:
            assert len(map_paths) == self.num_envs, "if multiple maps are provided, they should be provided for each environment"
        self.reward_shaping = reward_shaping
        self.reward_weight = reward_weight
        self.prior_mode = self.PriorMode(prior_mode)
        if self.prior_mode:
            raise MicroRTSNotImplemented("prior_mode other than 'none' (KG prior) is out of scope")
        self.microrts_path = os.path.join(gym_microrts.__path__[0], "microrts")
        self.cycle_maps = list(map(lambda i: os.path.join(self.microrts_path, i), cycle_maps))
        self.next_map = MapCycle(self.cycle_maps)

        # read map (vec_env.py:148-150)
        first = os.path.join(self.microrts_path, self.map_paths[0])
        root = ET.parse(first).getroot()
        self.height, self.width = int(root.get("height")), int(root.get("width"))

        # map table: one entry per distinct path; envs of a selfplay pair share game 2k's map
        full = [os.path.join(self.microrts_path, p) for p in self.map_paths]
        self._map_table = []
        for p in full + self.cycle_maps + [os.path.join(self.microrts_path, m) for m in _extra_maps]:
            if p not in self._map_table:
                self._map_table.append(p)
        self._map_index = {p: i for i, p in enumerate(self._map_table)}
        nsp_games = num_selfplay_envs // 2
        game_env = [2 * k for k in range(nsp_games)] + [num_selfplay_envs + j for j in range(num_bot_envs)]
        game_map = [self._map_index[full[e]] for e in game_env]

        # opponents (vec_env.py:268): factories -> device bot ids
        def device_ids(factories):
            ids = []
            for f in factories:
                d = f(None) if callable(f) else f
                ai_id = getattr(d, "ai_id", None)
                if ai_id is None:
                    raise MicroRTSNotImplemented(f"bot {d} has no device implementation")
                ids.append(ai_id)
            return ids

        bot_ai = device_ids(ai2s)
        bot_ai0 = device_ids(_ai1s) if _ai1s is not None else None   # MicroRTSBotVecEnv: player-0 bots

        # device + return contract
        if device is None:
            if not torch.cuda.is_available():
                raise MicroRTSError("MicroRTSGridModeVecEnv needs a GPU (HIP) device: the engine has no CPU fallback")
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise MicroRTSError(f"device must be a HIP/cuda device, got {self.device}")
        self.contract = contract_of(return_tensors)
        self.return_tensors = self.contract == "tensors"
        self._host_outputs = self.contract == "numpy"   # obs / masks copied to numpy
        if obs_dtype is None:
            obs_dtype = torch.int32 if self._host_outputs else torch.float32
        if obs_dtype not in (torch.float32, torch.int32):
            raise ValueError("obs_dtype must be torch.float32 or torch.int32")
        self.obs_dtype = obs_dtype

        # new JNIGridnetVecClient(...) (vec_env.py:256-276)
        self._h = _native.create(num_selfplay_envs, num_bot_envs, max_steps, partial_obs, self._map_table, game_map,
                                 bot_ai, _native.MRTS_OBS_FLOAT32 if obs_dtype == torch.float32 else _native.MRTS_OBS_INT32,
                                 bot_ai0=bot_ai0, game_offset=game_offset)
        self._game_map = list(game_map)
        info = _native.info(self._h)
        assert (info.height, info.width) == (self.height, self.width)
        self.utt = json.loads(_native.lib().mrts_utt_json(self._h).decode())
        self.rfs = [RewardFunction(n) for n in RF_NAMES]
        self.real_utt = self.utt
        self.vec_client = self  # reference attribute; the client is the engine itself

        with torch.cuda.device(self.device):
            self._ws = torch.empty(int(info.workspace_bytes), dtype=torch.uint8, device=self.device)
            hw = self.height * self.width
            self.num_planes = [5, 5, 3, len(self.utt["unitTypes"]) + 1, 6, 2]
            if partial_obs:
                self.num_planes = [5, 5, 3, len(self.utt["unitTypes"]) + 1, 6, 2, 2]
            P = sum(self.num_planes)
            self._obs = torch.empty((self.num_envs, self.height, self.width, P), dtype=obs_dtype, device=self.device)
            self._mask = torch.zeros((self.num_envs, hw, 78), dtype=torch.int32, device=self.device)
            self._src = torch.zeros((self.num_envs, hw), dtype=torch.int32, device=self.device)
            self._raw = torch.zeros((self.num_envs, 6), dtype=torch.float64, device=self.device)
            self._done = torch.zeros((self.num_envs, 6), dtype=torch.uint8, device=self.device)
            self._actions = torch.zeros((self.num_envs, hw, 7), dtype=torch.int64, device=self.device)
            self._rew = torch.zeros((self.num_envs,), dtype=torch.float64, device=self.device)
            self._done0 = torch.zeros((self.num_envs,), dtype=torch.bool, device=self.device)
        _native.check(_native.lib().mrts_bind_workspace(self._h, self._ws.data_ptr(), self._stream()), self._h, "bind_workspace")
        self.reward_weight = reward_weight   # the setter sends it to the engine
        # eager masks: reset / step / map-cycling resets also write getMasks(0) of
        # the state they leave (mrts_bind_mask_outputs), in the same kernel pass, so
        # get_action_mask() after them launches nothing (the rollout loop calls it
        # once per step, ppo_gridnet.py:448-466)
        self.eager_masks = bool(eager_masks)
        if self.eager_masks:
            _native.check(_native.lib().mrts_bind_mask_outputs(self._h, self._mask.data_ptr(), self._src.data_ptr()), self._h,
                          "bind_mask_outputs")
        # bot fusion: the step kernel decides the next tick's device-bot actions in
        # the same pass (mrts_set_bot_fusion; outputs identical either way)
        self.bot_fusion = bool(bot_fusion)
        _native.check(_native.lib().mrts_set_bot_fusion(self._h, int(self.bot_fusion)), self._h, "set_bot_fusion")

        # computed properties (vec_env.py:230-254)
        self.action_space_dims = [6, 4, 4, 4, 4, len(self.utt["unitTypes"]), 7 * 7]
        self.observation_space = Box(low=0.0, high=1.0, shape=(self.height, self.width, P), dtype=np.int32)
        self.num_planes_len = len(self.num_planes)
        self.num_planes_prefix_sum = [0]
        for num_plane in self.num_planes:
            self.num_planes_prefix_sum.append(self.num_planes_prefix_sum[-1] + num_plane)
        self.action_space = MultiDiscrete(np.array([self.action_space_dims] * self.height * self.width).flatten())
        self.action_plane_space = MultiDiscrete(self.action_space_dims)
        self.source_unit_idxs = np.tile(np.arange(self.height * self.width), (self.num_envs, 1))
        self.source_unit_idxs = self.source_unit_idxs.reshape((self.source_unit_idxs.shape + (1,)))
        self._mask_fresh = False   # _mask / _src hold getMasks(0) of the current state
        self._pool = None          # numpy contract: page-locked output arrays (HostArrayPool)
        self._act_stage = None     # host actions: page-locked int64 staging buffer
        self._act_copied = None    # event after the staging buffer's last H2D copy (reused only once it fired)
        self._act_src = None       # a caller's page-locked action array being copied (kept alive until step_wait's sync)
        self._mask_prefetch = None # numpy contract: host masks of the current state, copied in step_wait's sync
        self._mask_wanted = False  # get_action_mask() was called since the last step (the rollout loop's pattern)
        # optional {kernel name: [(start, end) torch.cuda.Event]} filled around
        # each engine launch on the launch stream (bench.py roofline timing)
        self.kernel_events = None

    # ------------------------------------------------------------------ utils
    @property
    def reward_weight(self):
        return self._reward_weight

    @reward_weight.setter
    def reward_weight(self, w):
        """vec_env.py:1057 reads self.reward_weight on every step_wait; the tensor
        path's fused `raw @ w` reads the engine's copy, so a reassignment is sent
        to the engine at once."""
        self._reward_weight = w
        if getattr(self, "_h", None):
            rw = np.ascontiguousarray(np.asarray(w, dtype=np.float64).reshape(6))
            _native.check(_native.lib().mrts_set_reward_weight(self._h, rw.ctypes.data, int(bool(self.reward_shaping))), self._h,
                          "set_reward_weight")

    def _launch(self, name, fn, *args):
        ev = self.kernel_events
        if MARKERS:   # a named host range around the C-ABI call (rocprofv3 --marker-trace)
            torch.cuda.nvtx.range_push(f"mrts_{name}")
        if ev is None:
            rc = fn(*args)
        else:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            rc = fn(*args)
            e.record()
            ev.setdefault(name, []).append((s, e))
        if MARKERS:
            torch.cuda.nvtx.range_pop()
        _native.check(rc, self._h, name)
    def _stream(self):
        return torch.cuda.current_stream(self.device).cuda_stream

    def _host(self, key, t):
        """numpy contract: a fresh host array of device tensor t (HostArrayPool),
        enqueued on the current stream; valid after _sync()."""
        if self._pool is None:
            self._pool = HostArrayPool(pinned=self.device.type == "cuda")
        return self._pool.d2h(key, t)

    def _sync(self):
        torch.cuda.current_stream(self.device).synchronize()

    def _obs_out(self):
        if not self._host_outputs:
            return self._obs
        obs = self._host("obs", self._obs)
        self._sync()
        return obs

    # ------------------------------------------------------------------- API
    def reset(self):
        """vec_env.py:278-282"""
        self._mask_prefetch = None
        _native.check(_native.lib().mrts_reset(self._h, self._stream(), self._obs.data_ptr()), self._h, "reset")
        self._mask_fresh = self.eager_masks
        return self._obs_out()

    def get_action_mask(self):
        """vec_env.py:1091-1101: (N, H*W, 78); channel 0 kept as source_unit_mask.
        With eager masks the last reset / step already wrote them."""
        if not self._mask_fresh:
            self._launch("get_masks", _native.lib().mrts_get_masks, self._h, self._stream(), self._mask.data_ptr(),
                         self._src.data_ptr())
            self._mask_fresh = True
        if not self._host_outputs:
            return self._mask
        self._mask_wanted = True
        if self._mask_prefetch is not None:   # copied behind the obs in the last step_wait's one sync
            mask, self._mask_prefetch = self._mask_prefetch, None
            return mask
        mask = self._host("mask", self._mask)
        self._sync()
        return mask

    @property
    def source_unit_mask(self):
        return self._src.cpu().numpy() if self._host_outputs else self._src

    def step_async(self, actions):
        """vec_env.py:968-984: actions (N, H*W*7) (or any shape with N*H*W*7 elements)."""
        hw = self.height * self.width
        if isinstance(actions, torch.Tensor):
            a = actions.reshape(self.num_envs, hw, 7)
            if a.device == self.device and a.dtype == torch.int64 and a.is_contiguous():
                self._actions_in = a
                return
            self._actions.copy_(a)
        else:
            a = np.asarray(actions)
            if self.contract != "tensors" and a.dtype == np.int64 and a.size == self._actions.numel() and a.flags.c_contiguous:
                t = torch.from_numpy(a.reshape(-1))
                if t.is_pinned():
                    # the caller's array is page-locked already (e.g. a view of a pinned
                    # tensor the policy copied its actions into): one DMA straight from it,
                    # no host pass.  step_wait syncs the stream before returning (numpy /
                    # hybrid contracts), so the array is free again once step() returns.
                    self._actions.view(-1).copy_(t, non_blocking=True)
                    self._act_src = t
                    self._actions_in = self._actions
                    return
            a = a.reshape(self.num_envs, hw, 7)
            if self._act_stage is None:
                self._act_stage = torch.empty(tuple(self._actions.shape), dtype=torch.int64, pin_memory=True)
                self._act_copied = torch.cuda.Event()
            else:
                # the previous step's DMA may still be queued (the tensor contract
                # never syncs the stream): the staging buffer is rewritten only after it
                self._act_copied.synchronize()
            # one host pass into page-locked memory, then a DMA at full PCIe rate (a
            # pageable source would be staged by the runtime in small chunks)
            np.copyto(self._act_stage.numpy(), a, casting="unsafe")
            self._actions.copy_(self._act_stage, non_blocking=True)
            self._act_copied.record(torch.cuda.current_stream(self.device))
        self._actions_in = self._actions

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
        # vec_env.py:1036: one dict per env around a row VIEW of the raw rewards -- built
        # while the copies above are in flight (views read nothing; they see the rows
        # the copy lands and the shaping mask below, as the reference's do)
        infos = [{"raw_rewards": item} for item in reward]
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

    def game_of_env(self, e):
        """env index -> game index (selfplay pairs 2k / 2k+1 share game k, then bot envs)."""
        nsp = self.num_selfplay_envs
        return e // 2 if e < nsp else nsp // 2 + (e - nsp)

    def reset_games(self, games, maps=None):
        """Reset the given games (their envs' obs, and masks when eager) onto `maps`
        (map-table indices; default: each game's current map) -- the per-client
        reset of the reference's map cycling (vec_env.py:1044-1054)."""
        import ctypes

        games = [int(g) for g in games]
        if not games:
            return
        self._mask_prefetch = None
        maps = [self._game_map[g] for g in games] if maps is None else [int(m) for m in maps]
        for g, m in zip(games, maps):
            self._game_map[g] = m
        ga = (ctypes.c_int32 * len(games))(*games)
        ma = (ctypes.c_int32 * len(maps))(*maps)
        _native.check(_native.lib().mrts_reset_games(self._h, self._stream(), ga, ma, len(games), self._obs.data_ptr()), self._h,
                      "reset_games")

    def park_games(self, games):
        """Park the given games (mrts_park_games): they stop ticking and their envs'
        obs, masks, rewards and dones read zero until reset_games() restarts them on
        a map.  MicroRTSSizeCyclingVecEnv parks an env's game in every size engine
        but the one it plays in."""
        import ctypes

        games = [int(g) for g in games]
        if not games:
            return
        self._mask_prefetch = None
        ga = (ctypes.c_int32 * len(games))(*games)
        _native.check(_native.lib().mrts_park_games(self._h, self._stream(), ga, len(games), self._obs.data_ptr()), self._h,
                      "park_games")
        envs = [e for g in games for e in self.envs_of_game(g)]
        for t in (self._raw, self._done, self._rew, self._done0):
            t[envs] = 0

    def envs_of_game(self, g):
        nsp2 = self.num_selfplay_envs // 2
        return [2 * g, 2 * g + 1] if g < nsp2 else [self.num_selfplay_envs + g - nsp2]

    def get_state(self):
        """Env-state checkpoint (mrts_save_state; no reference counterpart):
        a device uint8 tensor holding every game's state, the bots' pending decisions and
        the host-side mirrors.  set_state(s) on this env brings it back."""
        n = int(_native.lib().mrts_state_bytes(self._h))
        if n <= 0:
            raise _native.MicroRTSError("get_state: engine not bound")
        buf = torch.empty(n + 256, dtype=torch.uint8, device=self.device)
        off = (-buf.data_ptr()) % 256   # 256-byte aligned view
        state = buf[off:off + n]
        _native.check(_native.lib().mrts_save_state(self._h, self._stream(), state.data_ptr()), self._h, "save_state")
        return EnvState(state, list(self._game_map), self.next_map.drawn)

    def _check_state(self, state):
        """The snapshot tensor of a get_state() EnvState that fits this env, or ValueError
        (the engine's own fingerprint check runs in mrts_load_state)."""
        t = state.tensor if isinstance(state, EnvState) else None
        if t is None or t.device != self.device or t.dtype != torch.uint8 or t.data_ptr() % 256:
            raise ValueError("set_state expects an EnvState returned by get_state() of this env")
        if t.numel() != int(_native.lib().mrts_state_bytes(self._h)) or not t.is_contiguous():
            raise ValueError("set_state: the snapshot's size differs from this env's (another configuration)")
        return t

    def set_state(self, state):
        """Restore a get_state() snapshot of this env (mrts_load_state) and return the
        restored state's obs, as reset() does; the next get_action_mask() / step()
        continue from it bit for bit as the saved run did (map cycling included)."""
        t = self._check_state(state)
        self._mask_prefetch = None
        _native.check(_native.lib().mrts_load_state(self._h, self._stream(), t.data_ptr(), self._obs.data_ptr()), self._h,
                      "load_state")
        self._game_map = list(state.game_map)
        if state.next_map is not None:
            self.next_map = MapCycle(self.cycle_maps, state.next_map)
        self._mask_fresh = self.eager_masks
        return self._obs_out()

    def game_stats(self):
        """(num_games, 6) int32: game time, episode env steps, steps since creation, serial
        ticks, ordered-path rows, auto-resets (mrts_game_stats)."""
        out = np.zeros((self._n_games(), _native.MRTS_GAME_STATS), np.int32)
        _native.check(_native.lib().mrts_game_stats(self._h, self._stream(), out.ctypes.data), self._h, "game_stats")
        return out

    def _n_games(self):
        return self.num_selfplay_envs // 2 + self.num_bot_envs

    def _cycle(self, done0):
        """vec_env.py:1038-1056 map cycling, indexed the engine's way (selfplay
        pairs first, then bot envs)."""
        games, maps = [], []
        nsp = self.num_selfplay_envs
        for e in np.nonzero(done0)[0]:
            if e < nsp and e % 2:
                continue
            games.append(self.game_of_env(e))
            maps.append(self._map_index[next(self.next_map)])
        self.reset_games(games, maps)

    def step(self, ac):
        self.step_async(ac)
        return self.step_wait()

    def getattr_depth_check(self, name, already_found):
        """vec_env.py:1063-1073 (stable-baselines3 VecEnvWrapper protocol)."""
        if hasattr(self, name) and already_found:
            return "{0}.{1}".format(type(self).__module__, type(self).__name__)
        return None

    def render(self, mode="human"):
        """vec_env.py:1075-1084 on render_client = game 0 (selfPlayClients[0], else
        clients[0]: env 0 either way).  "rgb_array": a 640x640x3 uint8 RGB frame drawn
        on the device (k_render).  "human": the Java Swing window has no
        counterpart on a headless GPU host; warns once and draws nothing."""
        if mode == "human":
            if not getattr(self, "_human_warned", False):
                warnings.warn("render(mode='human') has no display on the GPU engine; use render('rgb_array') frames")
                self._human_warned = True
            return None
        if mode != "rgb_array":
            raise ValueError(f"unsupported render mode {mode!r}")
        if getattr(self, "_frame", None) is None:
            self._frame = torch.empty((RENDER_SIZE, RENDER_SIZE, 3), dtype=torch.uint8, device=self.device)
        _native.check(_native.lib().mrts_render(self._h, self._stream(), 0, self._frame.data_ptr(), RENDER_SIZE), self._h, "render")
        return self._frame.cpu().numpy()

    def error_flags(self):
        import ctypes

        f = ctypes.c_int32(0)
        _native.check(_native.lib().mrts_error_flags(self._h, self._stream(), ctypes.byref(f)), self._h, "error_flags")
        return int(f.value)

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


class MapCycle:
    """itertools.cycle(maps) (vec_env.py's `self.next_map`) that counts the maps drawn,
    so an env-state checkpoint stores the cycling position as an integer and restores
    it without copying an iterator (copying itertools objects is gone in Python 3.14)."""

    def __init__(self, maps, drawn=0):
        self.maps, self.drawn = list(maps), int(drawn)

    def __iter__(self):
        return self

    def __next__(self):
        if not self.maps:
            raise StopIteration
        m = self.maps[self.drawn % len(self.maps)]
        self.drawn += 1
        return m


def _set_states_atomic(envs, states):
    """set_state on several engines as one operation: every snapshot is checked first, and if
    an engine still refuses its snapshot (mrts_load_state's configuration fingerprint), the
    engines restored before it -- and the refusing engine itself, which mrts_load_state may
    have left half-restored if it failed after its header checks -- are rolled back to
    where they were."""
    for e, st in zip(envs, states):
        e._check_state(st)
    before = [e.get_state() for e in envs]
    out = []
    try:
        for e, st in zip(envs, states):
            out.append(e.set_state(st))
    except Exception:
        for e, st in zip(envs[:len(out) + 1], before):
            e.set_state(st)
        raise
    return out


class EnvState:
    """An env-state checkpoint (MicroRTSGridModeVecEnv.get_state): the engine's
    snapshot (a 256-byte aligned device uint8 tensor, mrts_save_state) and the
    Python-side map-cycling position (maps drawn from `next_map` so far)."""

    def __init__(self, tensor, game_map, next_map):
        self.tensor, self.game_map, self.next_map = tensor, game_map, next_map


class MicroRTSBotVecEnv(MicroRTSGridModeVecEnv):
    """Bot vs bot (vec_env.py:1104-1236; league.py:236-245 plays its matches with
    it): env j is a game of ai1s[j] (player 0) against ai2s[j] (player 1), both
    device bots computed by k_bot on the same pre-issue state each tick
    (JNIBotClient.gameStep).  Observations are the reference's dummy
    np.ones((N, 2)); rewards / dones are player 0's."""

    metadata = {"render.modes": ["human", "rgb_array"], "video.frames_per_second": 150}

    def __init__(
        self,
        ai1s=[],
        ai2s=[],
        partial_obs=False,
        max_steps=2000,
        render_theme=2,
        map_paths="maps/10x10/basesTwoWorkers10x10.xml",
        reward_weight=np.array([0.0, 1.0, 0.0, 0.0, 0.0, 5.0]),
        autobuild=True,
        jvm_args=[],
        *,
        device=None,
    ):
        assert len(ai1s) == len(ai2s), "for each environment, a microrts ai should be provided"
        if isinstance(map_paths, str):
            map_paths = [map_paths]
        super().__init__(num_selfplay_envs=0, num_bot_envs=len(ai1s), partial_obs=partial_obs, max_steps=max_steps,
                         render_theme=render_theme, ai2s=ai2s, map_paths=map_paths, reward_weight=reward_weight,
                         device=device, eager_masks=False, return_tensors=False, _ai1s=ai1s)
        self.ai1s = ai1s
        self.observation_space = Discrete(2)
        self.action_space = Discrete(2)

    def reset(self):
        """vec_env.py:1223-1226"""
        super().reset()
        return np.ones((self.num_envs, 2))

    def step_async(self, actions):
        """vec_env.py:1228-1229: the actions are not used"""
        self._actions_in = self._actions

    def step_wait(self):
        """vec_env.py:1231-1235"""
        self._launch("step", _native.lib().mrts_step, self._h, self._stream(), self._actions.data_ptr(), self._src.data_ptr(),
                     self._obs.data_ptr(), self._raw.data_ptr(), self._done.data_ptr())
        reward = self._raw.cpu().numpy()
        done = self._done.cpu().numpy().astype(bool)
        infos = [{"raw_rewards": item} for item in reward]
        return np.ones((self.num_envs, 2)), reward @ self.reward_weight, done[:, 0], infos


class MicroRTSGridModeSharedMemVecEnv(MicroRTSGridModeVecEnv):
    """vec_env.py:1238-1362: the zero-copy variant.  The reference allocates three
    direct buffers shared with the JVM (`self.obs` (N, H, W, P) int32,
    `self.action_mask` (N, H*W, 78) int32, `self.actions` (N, H*W, 7) int32) and
    returns them from reset / step / get_action_mask, overwritten in place by every
    call; all envs play one map.

    Here the three are page-locked host arrays: the engine's device outputs are
    copied into them (one DMA each, no allocation) and `self.actions` is copied to
    the device by `step_wait`, with the same aliasing contract.  Rewards are
    `raw @ reward_weight` in numpy, dones `done[:, 0]`, infos `[{"raw_rewards": r}]`.
    The reference forwards its arguments to the base class by position, which
    shifts `reward_weight` into `reward_shaping`; they are
    forwarded by name here.  It cycles maps only with more than one cycle map
    (vec_env.py:1344), not with one as the base class (vec_env.py:1038)."""

    _cycle_min = 1

    def __init__(
        self,
        num_selfplay_envs,
        num_bot_envs,
        partial_obs=False,
        max_steps=2000,
        render_theme=2,
        frame_skip=0,
        ai2s=[],
        map_paths=["maps/10x10/basesTwoWorkers10x10.xml"],
        reward_weight=np.array([0.0, 1.0, 0.0, 0.0, 0.0, 5.0]),
        cycle_maps=[],
        *,
        device=None,
    ):
        if len(map_paths) > 1 and len(set(map_paths)) > 1:
            raise ValueError("Mem shared environment requires all games to be played on the same map.")
        super().__init__(num_selfplay_envs, num_bot_envs, partial_obs=partial_obs, max_steps=max_steps,
                         render_theme=render_theme, frame_skip=frame_skip, ai2s=ai2s, map_paths=map_paths,
                         reward_weight=reward_weight, cycle_maps=cycle_maps, device=device, return_tensors=True,
                         obs_dtype=torch.int32)
        hw = self.height * self.width
        self.num_feature_planes = self._obs.shape[-1]
        self.masks_dim = sum(self.action_space_dims)
        self.action_dim = len(self.action_space_dims)
        pin = self.device.type == "cuda"
        self._obs_host = torch.empty(tuple(self._obs.shape), dtype=torch.int32, pin_memory=pin)
        self._mask_host = torch.empty((self.num_envs, hw, self.masks_dim), dtype=torch.int32, pin_memory=pin)
        self._act_host = torch.zeros((self.num_envs, hw, self.action_dim), dtype=torch.int32, pin_memory=pin)
        self._act_dev32 = torch.empty((self.num_envs, hw, self.action_dim), dtype=torch.int32, device=self.device)
        self.obs = self._obs_host.numpy()
        self.action_mask = self._mask_host.numpy()
        self.actions = self._act_host.numpy()

    def reset(self):
        self._obs_host.copy_(super().reset())
        return self.obs

    def get_action_mask(self):
        self._mask_host.copy_(super().get_action_mask())
        return self.action_mask

    def step_async(self, actions):
        actions = np.asarray(actions).reshape((self.num_envs, self.width * self.height, self.action_dim))
        np.copyto(self.actions, actions)
        # int32 over PCIe from the page-locked buffer, widened to int64 on the device
        self._act_dev32.copy_(self._act_host, non_blocking=True)
        super().step_async(self._act_dev32)

    def step_wait(self):
        obs, _, done0, infos = super().step_wait()
        self._obs_host.copy_(obs)
        reward = infos._raw.cpu().numpy()
        return self.obs, reward @ self.reward_weight, done0.cpu().numpy(), [{"raw_rewards": r} for r in reward]


class MicroRTSMixedMapVecEnv:
    """Maps of several sizes in one batch (BASELINE.json config 5), bucketed by
    height x width: one MicroRTSGridModeVecEnv engine per bucket, all launched on
    the caller's HIP stream back to back.  The reference's vec env requires one
    map size per env (vec_env.py:148-150), so each bucket keeps the reference's
    exact shapes and contract; the mixed env returns one entry per bucket.

      buckets = [dict(map_paths=[...], num_selfplay_envs=..., num_bot_envs=..., ai2s=[...]), ...]
      env = MicroRTSMixedMapVecEnv(buckets, max_steps=2000, return_tensors=True)
      obs  = env.reset()                       # list over buckets
      mask = env.get_action_mask()             # list over buckets
      obs, rew, done, infos = env.step(actions)  # actions: list over buckets
    """

    def __init__(self, buckets, concurrent=False, group_policy="default", **common):
        self.envs = []
        for b in buckets:
            kw = dict(common)
            kw.update(b)
            kw.setdefault("num_bot_envs", len(kw.get("ai2s", [])))
            kw.setdefault("num_selfplay_envs", 0)
            self.envs.append(MicroRTSGridModeVecEnv(**kw))
        sizes = [(e.height, e.width) for e in self.envs]
        if len(set(sizes)) != len(sizes):
            raise ValueError(f"one bucket per map size, got {sizes}")
        self.num_envs = sum(e.num_envs for e in self.envs)
        self.shapes = sizes
        # concurrent=True: each bucket launches on its own HIP stream, forked from and
        # joined back into the caller's stream.  Off by default: every bucket's step
        # kernel fills the GPU by itself, and side by side they measured slower
        # (configs[4] 22.6 vs 23.8 M env-steps/s, profiles/r02i/)
        self.concurrent = bool(concurrent) and len(self.envs) > 1
        self._streams = [torch.cuda.Stream(device=e.device) for e in self.envs] if self.concurrent else None
        # group_policy (tensor contract, no map cycling, <= 4 buckets): every bucket's
        # step in one mrts_step_group call -- buckets whose kernels fit one launch
        # share it (include/microrts_amd.h MRTS_GROUP_*); None = one step_wait per bucket
        if group_policy == "default":
            group_policy = _native.GROUP_MERGE_FIT | _native.GROUP_BOTS_FIRST
        self.group_policy = group_policy
        # (one launch runs on one device: buckets placed on different GPUs step one by one)
        self.grouped = (group_policy is not None and not self.concurrent and 1 < len(self.envs) <= _native.STEP_GROUP_MAX
                        and all(e.contract == "tensors" and len(e.cycle_maps) <= e._cycle_min for e in self.envs)
                        and all(e.device == self.envs[0].device for e in self.envs))

    def launch_plan(self):
        """(launch index of each bucket, launches per step) of the grouped step
        (mrts_step_group_plan); one launch per bucket when not grouped."""
        if not self.grouped:
            return list(range(len(self.envs))), len(self.envs)
        import ctypes

        n = len(self.envs)
        hs = (ctypes.c_void_p * n)(*[e._h for e in self.envs])
        lo, nl = (ctypes.c_int32 * n)(), ctypes.c_int32()
        _native.check(_native.lib().mrts_step_group_plan(hs, n, self.group_policy, lo, ctypes.byref(nl)), self.envs[0]._h,
                      "step_group_plan")
        return list(lo), int(nl.value)

    def reset(self):
        return [e.reset() for e in self.envs]

    def get_action_mask(self):
        return [e.get_action_mask() for e in self.envs]

    def step_async(self, actions):
        assert len(actions) == len(self.envs)
        for e, a in zip(self.envs, actions):
            e.step_async(a)

    def step_wait(self):
        if self.grouped:
            import ctypes

            io = (_native.StepIO * len(self.envs))(*[e._step_io() for e in self.envs])
            hs = (ctypes.c_void_p * len(self.envs))(*[e._h for e in self.envs])
            e0 = self.envs[0]
            e0._launch("step", _native.lib().mrts_step_group, hs, len(self.envs), e0._stream(), io, self.group_policy)
            outs = [e._tensor_outputs() for e in self.envs]
            return tuple(list(x) for x in zip(*outs))
        if not self.concurrent:
            outs = [e.step_wait() for e in self.envs]
            return tuple(list(x) for x in zip(*outs))
        cur = torch.cuda.current_stream(self.envs[0].device)
        fork = torch.cuda.Event()
        fork.record(cur)   # the actions (and anything else) the caller enqueued
        outs = []
        for e, st in zip(self.envs, self._streams):
            st.wait_event(fork)
            with torch.cuda.stream(st):
                outs.append(e.step_wait())
        for st in self._streams:
            cur.wait_stream(st)   # outputs are ready on the caller's stream
        return tuple(list(x) for x in zip(*outs))

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def error_flags(self):
        f = 0
        for e in self.envs:
            f |= e.error_flags()
        return f

    def get_state(self):
        """Env-state checkpoint of every bucket (MicroRTSGridModeVecEnv.get_state, in bucket order)."""
        return [e.get_state() for e in self.envs]

    def set_state(self, states):
        """Restore a get_state() list of this env; returns the restored obs per bucket."""
        if len(states) != len(self.envs):
            raise ValueError(f"set_state expects {len(self.envs)} bucket states, got {len(states)}")
        return _set_states_atomic(self.envs, states)

    def close(self):
        for e in self.envs:
            e.close()


class MicroRTSSizeCyclingVecEnv:
    """Map cycling across map sizes: vec_env.py:1038-1056 (a finished game restarts
    on next(cycle_maps)) with cycle_maps of several sizes.

    One engine (MicroRTSGridModeVecEnv) per map size in map_paths + cycle_maps,
    each holding EVERY env of the batch at the same index (selfplay pairs first,
    then bot envs -- the engine order).  An env plays in exactly one
    engine and is parked (mrts_park_games: no tick, zero obs / masks / rewards /
    dones) in the others.  When its game ends, the env restarts on the next cycle
    map; if that map has another size, its game is parked in the old engine and
    reset onto the map in the new one (an env of a selfplay pair moves with its
    partner).  The terminal reward and done of the tick are reported first.

      env = MicroRTSSizeCyclingVecEnv(4, 2, ai2s=[...], map_paths=[...], cycle_maps=[8x8, 16x16, ...])
      obs  = env.reset()                     # list over env.sizes: (N, H_i, W_i, P) device tensors
      mask = env.get_action_mask()           # list over env.sizes: (N, H_i*W_i, 78)
      obs, rew, done, infos = env.step(acts) # acts: list over env.sizes; rew / done: (N,) over all envs
      env.bucket                             # (N,) index into env.sizes of each env's current map

    Random bots (randomBiasedAI, randomAI) key their Philox stream on (unit, the
    game's tick counter in the engine it plays in, game).  A parked game's counter
    does not advance, so after a move to another size the stream continues from
    that engine's counter for the game, not from the ticks played elsewhere.  No
    reference fixture holds these streams (the Java bots draw from an unseeded
    java.util.Random): parity unpinned, and tests/test_gpu_size_cycling.py uses
    deterministic bots.

    Rows of envs that play in another engine are zero in every list entry, so a
    policy can run each size's batch as it is.  Device tensors only (the
    return_tensors=True contract)."""

    def __init__(self, num_selfplay_envs, num_bot_envs, ai2s=[], map_paths=["maps/16x16/basesWorkers16x16.xml"], cycle_maps=[],
                 max_steps=2000, partial_obs=False, reward_weight=np.array([0.0, 1.0, 0.0, 0.0, 0.0, 5.0]), device=None,
                 obs_dtype=None):
        self.num_selfplay_envs, self.num_bot_envs = num_selfplay_envs, num_bot_envs
        self.num_envs = num_selfplay_envs + num_bot_envs
        root = os.path.join(gym_microrts.__path__[0], "microrts")
        per_env = list(map_paths) * self.num_envs if len(map_paths) == 1 else list(map_paths)
        assert len(per_env) == self.num_envs, "if multiple maps are provided, they should be provided for each environment"

        def size(m):
            r = ET.parse(os.path.join(root, m)).getroot()
            return int(r.get("height")), int(r.get("width"))

        self.sizes = sorted({size(m) for m in per_env + list(cycle_maps)})
        self._size_of = {m: size(m) for m in per_env + list(cycle_maps)}
        self.cycle_maps = list(cycle_maps)
        self.next_map = MapCycle(self.cycle_maps)
        self.bucket = np.array([self.sizes.index(self._size_of[m]) for m in per_env], np.int64)
        self.envs = []
        for i, sz in enumerate(self.sizes):
            own = [m for m in per_env + self.cycle_maps if self._size_of[m] == sz]
            maps_i = [m if self._size_of[m] == sz else own[0] for m in per_env]   # placeholders are parked at reset
            self.envs.append(MicroRTSGridModeVecEnv(num_selfplay_envs, num_bot_envs, partial_obs=partial_obs, max_steps=max_steps,
                                                    ai2s=ai2s, map_paths=maps_i, reward_weight=reward_weight, device=device,
                                                    return_tensors=True, obs_dtype=obs_dtype, _extra_maps=own))
        self.device = self.envs[0].device
        self.reward_weight = reward_weight

    def _games_in(self, i, inside):
        e0 = self.envs[0]
        return [g for g in range(e0._n_games()) if (self.bucket[e0.envs_of_game(g)[0]] == i) == inside]

    def reset(self):
        out = []
        for i, e in enumerate(self.envs):
            e.reset()
            e.park_games(self._games_in(i, False))
            out.append(e._obs)
        return out

    def get_action_mask(self):
        return [e.get_action_mask() for e in self.envs]

    def step_async(self, actions):
        assert len(actions) == len(self.envs)
        for e, a in zip(self.envs, actions):
            e.step_async(a)

    def step_wait(self):
        outs = [e.step_wait() for e in self.envs]
        # each env's row is non-zero in the engine it played the tick in only
        rew = outs[0][1].clone()
        done = outs[0][2].clone()
        raw = outs[0][3]._raw.clone()
        for _, r, d, inf in outs[1:]:
            rew += r
            done |= d
            raw += inf._raw
        self._cycle(done.cpu().numpy())
        return [e._obs for e in self.envs], rew, done, LazyInfos(raw)

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def _cycle(self, done0):
        if not self.cycle_maps:
            return
        e0 = self.envs[0]
        moves = {}   # (from, to) -> (games, maps)
        for e in np.nonzero(done0)[0]:
            if e < self.num_selfplay_envs and e % 2:
                continue
            g = e0.game_of_env(e)
            m = next(self.next_map)
            src, dst = int(self.bucket[e]), self.sizes.index(self._size_of[m])
            gl, ml = moves.setdefault((src, dst), ([], []))
            gl.append(g)
            ml.append(self.envs[dst]._map_index[os.path.join(self.envs[dst].microrts_path, m)])
            for x in e0.envs_of_game(g):
                self.bucket[x] = dst
        for (src, dst), (gl, ml) in moves.items():
            if src != dst:
                self.envs[src].park_games(gl)
            self.envs[dst].reset_games(gl, ml)

    def error_flags(self):
        f = 0
        for e in self.envs:
            f |= e.error_flags()
        return f

    def get_state(self):
        """Env-state checkpoint: every size engine's snapshot (its played and parked games),
        the size each env plays in and the cycle position."""
        return SizeCyclingState([e.get_state() for e in self.envs], self.bucket.copy(), self.next_map.drawn)

    def set_state(self, state):
        """Restore a get_state() snapshot of this env; returns the restored obs per size."""
        if not isinstance(state, SizeCyclingState) or len(state.engines) != len(self.envs) or \
                len(state.bucket) != self.num_envs:
            raise ValueError("set_state expects a SizeCyclingState returned by get_state() of this env")
        out = _set_states_atomic(self.envs, state.engines)
        self.bucket = state.bucket.copy()
        self.next_map = MapCycle(self.cycle_maps, state.drawn)
        return out

    def close(self):
        for e in self.envs:
            e.close()


class SizeCyclingState:
    """MicroRTSSizeCyclingVecEnv.get_state: one EnvState per size engine, the env -> size
    index map and the maps drawn from cycle_maps so far."""

    def __init__(self, engines, bucket, drawn):
        self.engines, self.bucket, self.drawn = engines, bucket, drawn
