import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "microrts-py_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

MAPS = os.path.join(REPO, "microrts-py_amd", "gym_microrts", "microrts")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); runs through libmicrorts_amd.so")


@pytest.fixture(scope="session")
def maps_root():
    return MAPS


ONE_F32 = 0x3f800000   # 1.0f as stored bits


def obs_bits_equal(gpu, host):
    """Bit-level obs parity.  `host` is the oracle's int32 one-hot; an int32 `gpu`
    tensor must equal it, a float32 one must hold exactly 0x3f800000 (1.0f) where
    the one-hot is 1 and 0x00000000 (+0.0f) where it is 0 -- the bits the bench's
    float kernels store (mrts_engine.hip stream_obs: ONE, and the unaligned
    fallback's cast)."""
    import numpy as np
    import torch

    h = torch.from_numpy(np.ascontiguousarray(host, dtype=np.int32)).to(gpu.device)
    if gpu.dtype == torch.int32:
        return torch.equal(gpu, h)
    assert gpu.dtype == torch.float32, gpu.dtype
    assert bool(((h == 0) | (h == 1)).all()), "oracle obs is not one-hot"
    return torch.equal(gpu.view(torch.int32), h * ONE_F32)


OBS_DTYPES = ("float32", "int32")   # the bench's dtype first


def gpu_available():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if gpu_available():
        return
    skip = pytest.mark.skip(reason="no HIP device in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)
