"""EXPERIMENT (not product): configs[4] with the grouped step's launches on two HIP
streams -- the merged 8x8 + 16x16 launch on one, the 24x24 launch on another, forked from
and joined back into the caller's stream -- vs the product's back-to-back launches.
Runs bench.py's mixed workload with MicroRTSMixedMapVecEnv.step_wait patched.

  python scripts/ab/mixed_concurrent.py [bench args...]
"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "microrts-py_amd"))
import torch  # noqa: E402

from gym_microrts import _native  # noqa: E402
from gym_microrts.envs import vec_env  # noqa: E402

_streams = {}


def step_wait(self):
    lib = _native.lib()
    launch_of, nl = self.launch_plan()
    ios = [e._step_io() for e in self.envs]
    cur = torch.cuda.current_stream(self.envs[0].device)
    fork = torch.cuda.Event()
    fork.record(cur)
    if not _streams:
        _streams.update({l: torch.cuda.Stream(device=self.envs[0].device) for l in range(nl)})
    for l in range(nl):
        idx = [i for i in range(len(self.envs)) if launch_of[i] == l]
        st = _streams[l]
        st.wait_stream(cur)
        with torch.cuda.stream(st):
            hs = (ctypes.c_void_p * len(idx))(*[self.envs[i]._h for i in idx])
            io = (_native.StepIO * len(idx))(*[ios[i] for i in idx])
            _native.check(lib.mrts_step_group(hs, len(idx), st.cuda_stream, io, self.group_policy), self.envs[idx[0]]._h, "group")
    for st in _streams.values():
        cur.wait_stream(st)
    outs = [e._tensor_outputs() for e in self.envs]
    return tuple(list(x) for x in zip(*outs))


if os.environ.get("MIXED_CONCURRENT") == "1":
    vec_env.MicroRTSMixedMapVecEnv.step_wait = step_wait
import bench  # noqa: E402

sys.argv = ["bench.py"] + sys.argv[1:]
bench.main()
