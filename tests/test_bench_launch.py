"""bench.py --gpus N starts its own N ranks when no launcher did.

The parent must not initialise HIP before the children start (a process that
touched the GPU must not fork/exec the ranks' runtime state, and the children
each pick their own device): these tests run bench.main with `torch` replaced
by a module that raises on any attribute access, and with subprocess.Popen
replaced by a recorder, so they need no GPU.  The GPU end-to-end check (the
self-launched ranks' dumps are the slices of a 1-rank run) is
tests/test_gpu_shard.py::test_bench_sharding_end_to_end.
"""
import os
import subprocess
import sys
import time
import types

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


class _NoTorch(types.ModuleType):
    def __getattr__(self, name):
        raise AssertionError(f"the launching parent touched torch.{name}")


class _FakeProc:
    def __init__(self, rc):
        self.rc, self.terminated = rc, False

    def poll(self):
        return self.rc

    def terminate(self):
        self.terminated = True
        self.rc = -15

    def wait(self, timeout=None):
        return self.rc

    def kill(self):
        self.rc = -9


@pytest.fixture
def no_torch(monkeypatch):
    monkeypatch.setitem(sys.modules, "torch", _NoTorch("torch"))
    monkeypatch.setitem(sys.modules, "torch.cuda", _NoTorch("torch.cuda"))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MICRORTS_BENCH_SELF_LAUNCHED"):
        monkeypatch.delenv(k, raising=False)


def _recorder(monkeypatch, rcs):
    calls = []

    def popen(cmd, env=None, **kw):
        calls.append((cmd, env))
        return _FakeProc(rcs[len(calls) - 1])

    monkeypatch.setattr(subprocess, "Popen", popen)
    return calls


def test_self_launch_starts_n_ranks_without_touching_torch(no_torch, monkeypatch):
    calls = _recorder(monkeypatch, [0] * 8)
    argv = ["--gpus", "8", "--steps", "20", "--warmup", "5"]
    assert bench.main(argv) == 0
    assert len(calls) == 8
    ports = set()
    for r, (cmd, env) in enumerate(calls):
        assert cmd[0] == sys.executable and cmd[1].endswith("bench.py") and cmd[2:] == argv
        assert env["RANK"] == env["LOCAL_RANK"] == str(r) and env["WORLD_SIZE"] == "8"
        assert env["MASTER_ADDR"] == "127.0.0.1" and env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
        ports.add(env["MASTER_PORT"])
    assert len(ports) == 1   # one rendezvous


def test_self_launch_failed_rank_stops_the_others(no_torch, monkeypatch):
    procs = []

    def popen(cmd, env=None, **kw):
        p = _FakeProc(3 if env["RANK"] == "1" else None)
        procs.append(p)
        return p

    monkeypatch.setattr(subprocess, "Popen", popen)
    assert bench.main(["--gpus", "4"]) == 3
    assert [p.terminated for p in procs] == [True, False, True, True]


def test_world_size_must_match_gpus(no_torch, monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("RANK", "0")
    assert bench.main(["--gpus", "4"]) == 2   # an error, before torch is imported


def test_one_gpu_does_not_spawn(monkeypatch):
    """--gpus 1 with no launcher runs in process (no child): the parse step only."""
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    args = bench.parse(["--gpus", "1", "--roofline-steps", "64"])
    assert args.gpus == 1 and args.roofline_steps == 64 and not args.no_kernel_events


def test_self_launch_hung_rank_hits_the_deadline(no_torch, monkeypatch, capsys):
    """A rank that neither exits nor fails (an RCCL init hang, a stuck kernel): the
    parent terminates every rank and exits non-zero once --rank-timeout passes."""
    procs = []

    def popen(cmd, env=None, **kw):
        p = _FakeProc(None)   # never exits until terminated
        procs.append(p)
        return p

    monkeypatch.setattr(subprocess, "Popen", popen)
    t0 = time.monotonic()
    rc = bench.main(["--gpus", "4", "--rank-timeout", "0.5"])
    assert rc == 124 and time.monotonic() - t0 < 5
    assert all(p.terminated for p in procs)
    err = capsys.readouterr().err
    assert "deadline" in err and "[0, 1, 2, 3]" in err


def test_self_launch_straggler_after_rank0(no_torch, monkeypatch, capsys):
    """Rank 0 (which prints the line) exited but rank 2 never does: the parent stops it
    STRAGGLE_S later and exits 124 rather than waiting for the driver's time limit."""
    monkeypatch.setattr(bench, "STRAGGLE_S", 0.3)
    procs = []

    def popen(cmd, env=None, **kw):
        p = _FakeProc(None if env["RANK"] == "2" else 0)
        procs.append(p)
        return p

    monkeypatch.setattr(subprocess, "Popen", popen)
    t0 = time.monotonic()
    assert bench.main(["--gpus", "4"]) == 124
    assert time.monotonic() - t0 < 5
    assert [p.terminated for p in procs] == [False, False, True, False]
    assert "rank 0 exited" in capsys.readouterr().err


def test_dist_backend_defaults_to_gloo():
    """The timing barrier / max-over-ranks / per-rank gather run on gloo unless asked:
    no data-path collective exists, so RCCL is not needed for the curve."""
    a = bench.parse(["--gpus", "8"])
    assert a.dist_backend == "gloo"
    assert bench.parse(["--dist-backend", "nccl"]).dist_backend == "nccl"


def test_rank_timeout_default_scales_with_the_requested_work():
    """the default deadline grows with steps / warm-up / pre-roll / seeds, so a
    legitimately long scale run is not killed at a fixed 15 minutes; an explicit value wins."""
    a = bench.parse(["--gpus", "8"])   # 2000 pre-roll + 50 warm-up + 300 steps
    assert a.rank_timeout == 900.0 + 0.05 * 2350
    long = bench.parse(["--gpus", "8", "--steps", "100000", "--seeds", "3"])
    assert long.rank_timeout == 900.0 + 0.05 * 3 * (2000 + 50 + 100000)
    assert long.rank_timeout > 60 * 60 * 4   # > 100x the ~0.25 ms a tick takes
    assert bench.parse(["--rank-timeout", "0"]).rank_timeout == 0
    assert bench.parse(["--rank-timeout", "42"]).rank_timeout == 42


def test_per_rank_single():
    import torch as _t  # noqa: F401  (real torch: gather_per_rank at world 1 makes no collective)

    pr = bench.gather_per_rank(0.5, 8192, 100, 1, None)
    assert pr == [{"rank": 0, "elapsed_s": 0.5, "env_steps_per_s": 8192 * 100 / 0.5}]
