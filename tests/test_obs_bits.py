"""conftest.obs_bits_equal, the float32-obs parity check of the -m gpu lock-steps: exact
bit patterns (1.0f = 0x3f800000, +0.0f = 0), so a -0.0f, a 1.0000001f or a non-one-hot
oracle plane fails it (CPU tensors here; the GPU tests pass device tensors)."""
import numpy as np
import pytest
import torch

from conftest import obs_bits_equal


def _pair():
    rng = np.random.default_rng(0)
    host = (rng.random((3, 4, 4, 29)) < 0.2).astype(np.int32)
    return host, torch.from_numpy(host.astype(np.float32))


def test_float_ones_and_zeros_pass():
    host, dev = _pair()
    assert obs_bits_equal(dev, host)
    assert obs_bits_equal(torch.from_numpy(host), host)   # the int32 arm


def test_negative_zero_and_near_one_fail():
    host, dev = _pair()
    z = np.argwhere(host == 0)[0]
    bad = dev.clone()
    bad[tuple(z)] = -0.0
    assert bad[tuple(z)] == 0.0 and not obs_bits_equal(bad, host)   # equal as floats, not as bits
    o = np.argwhere(host == 1)[0]
    bad = dev.clone()
    bad[tuple(o)] = float(np.nextafter(np.float32(1), np.float32(2)))
    assert not obs_bits_equal(bad, host)


def test_non_onehot_oracle_is_an_error():
    host, dev = _pair()
    host[0, 0, 0, 0] = 2
    with pytest.raises(AssertionError, match="one-hot"):
        obs_bits_equal(dev, host)
