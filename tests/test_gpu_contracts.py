"""The zero-copy return contract an UNMODIFIED experiments/ppo_gridnet.py can
select: with MICRORTS_AMD_RETURN=hybrid in
the environment (or `python -m gym_microrts.run_driver --contract hybrid`), the
env constructed with the reference's own arguments returns obs and masks as
device tensors while rewards, dones and infos stay numpy -- what
MicroRTSStatsRecorder (ppo_gridnet.py:138-160) and VecMonitor index per env.

Checked at BASELINE.json configs[3]'s size (4096 envs, partial_obs, 31 planes,
ppo_gridnet.py:370-373's bot mix) against the reference's numpy contract, through
both wrappers, with ppo_gridnet.py's own call forms (:421, 466, 475-490)."""
import importlib.util
import os

import numpy as np
import pytest

from conftest import REPO

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]   # per-test limits below override

NVEC = [6, 4, 4, 4, 4, 7, 49]


def _driver():
    spec = importlib.util.spec_from_file_location("ppo_gridnet_driver", os.path.join(REPO, "examples", "ppo_gridnet_driver.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _sample(mask, gen):
    """uniform over the valid entries of each action component (random when none is)"""
    import torch

    m = mask.reshape(-1, sum(NVEC)).float()
    out = []
    for seg in torch.split(m, NVEC, 1):
        w = seg + (seg.sum(1, keepdim=True) == 0).float()
        out.append(torch.multinomial(w, 1, generator=gen))
    return torch.cat(out, 1).reshape(mask.shape[0], -1)


def test_hybrid_contract_by_env_var_equals_numpy_contract_4096(monkeypatch):
    import torch

    d = _driver()
    dev = torch.device("cuda", 0)
    nsp, nbot = 4072, 24
    monkeypatch.setenv("MICRORTS_AMD_RETURN", "hybrid")
    eh, bh = d.make_envs(nsp, nbot, True, dev, max_steps=40)
    monkeypatch.setenv("MICRORTS_AMD_RETURN", "numpy")
    en, bn = d.make_envs(nsp, nbot, True, dev, max_steps=40)
    assert (bh.contract, bn.contract) == ("hybrid", "numpy") and bh.num_envs == 4096
    oh, on = eh.reset(), en.reset()
    assert torch.is_tensor(oh) and oh.is_cuda and oh.dtype == torch.float32 and oh.shape == (4096, 16, 16, 31)
    assert isinstance(on, np.ndarray) and on.dtype == np.int32
    assert torch.Tensor(oh).data_ptr() == oh.data_ptr()   # ppo_gridnet.py:421 / 476 alias, no copy
    np.testing.assert_array_equal(oh.cpu().numpy(), on)
    gen = torch.Generator(device=dev)
    gen.manual_seed(3)
    episodes = stats = 0
    for s in range(60):
        mh, mn = eh.get_action_mask(), en.get_action_mask()
        assert torch.is_tensor(mh) and mh.is_cuda and mh.dtype == torch.int32
        np.testing.assert_array_equal(mh.cpu().numpy(), mn, err_msg=f"mask step {s}")
        im = torch.tensor(mh).to(dev)   # ppo_gridnet.py:466's form
        assert torch.equal(im, mh)
        a = _sample(mh, gen).cpu().numpy()   # host int64 (N, H*W*7), ppo_gridnet.py:475
        oh, rh, dh, ih = eh.step(a)
        on, rn, dn, inn = en.step(a)
        assert torch.is_tensor(oh) and oh.is_cuda
        assert isinstance(rh, np.ndarray) and rh.dtype == np.float64 and isinstance(dh, np.ndarray) and dh.dtype == bool
        assert isinstance(ih, list) and len(ih) == 4096
        np.testing.assert_array_equal(oh.cpu().numpy(), on, err_msg=f"obs step {s}")
        np.testing.assert_array_equal(rh, rn, err_msg=f"reward step {s}")
        np.testing.assert_array_equal(dh, dn, err_msg=f"done step {s}")
        for i in range(4096):
            np.testing.assert_array_equal(ih[i]["raw_rewards"], inn[i]["raw_rewards"])
            assert ("episode" in ih[i]) == ("episode" in inn[i])
            if "episode" in ih[i]:
                episodes += 1
                assert (ih[i]["episode"]["r"], ih[i]["episode"]["l"]) == (inn[i]["episode"]["r"], inn[i]["episode"]["l"])
                assert ih[i]["microrts_stats"] == inn[i]["microrts_stats"]
                stats += 1
    assert episodes >= 4096 and stats == episodes   # every env finished its 40-step episode at least once
    assert bh.error_flags() == 0 and bn.error_flags() == 0
    bh.close()
    bn.close()


@pytest.mark.parametrize("api", ["hybrid", "numpy"])
def test_ppo_driver_configs3_4096(api):
    """configs[3] end to end at its stated size: GridNet PPO over 4096 envs
    (partial obs, ppo_gridnet.py's bot mix) through StatsRecorder + VecMonitor."""
    s = _driver().run(num_selfplay_envs=4072, num_bot_envs=24, partial_obs=True, num_steps=4, updates=1, api=api,
                      log=lambda _: None)
    assert s["global_step"] == 4 * 4096 and s["finite"] and s["engine_error_flags"] == 0
    assert s["num_envs"] == 4096 and s["api"] == api


@pytest.mark.parametrize("cycle", [False, True])
def test_numpy_contract_pinned_actions_and_mask_prefetch(cycle):
    """The numpy contract's fast paths change no byte: host
    actions handed over in a page-locked array (one DMA, no staging pass) vs a
    pageable one, masks copied behind the obs in step_wait's sync vs on demand;
    a returned mask array is never overwritten by later calls."""
    import torch

    from gym_microrts.envs.vec_env import MicroRTSGridModeVecEnv

    m = "maps/16x16/basesWorkers16x16A.xml"
    kw = dict(max_steps=25, map_paths=[m], reward_weight=np.array([10.0, 1.0, 1.0, 0.2, 1.0, 4.0]), return_tensors=False,
              cycle_maps=[m] if cycle else [])
    ea = MicroRTSGridModeVecEnv(64, 0, **kw)
    eb = MicroRTSGridModeVecEnv(64, 0, **kw)
    et = MicroRTSGridModeVecEnv(64, 0, **dict(kw, return_tensors=True, obs_dtype=torch.int32))
    np.testing.assert_array_equal(ea.reset(), eb.reset())
    et.reset()
    pinned = torch.empty((64, 256 * 7), dtype=torch.int64, pin_memory=True)
    gen = torch.Generator(device=et.device)
    gen.manual_seed(5)
    kept = []
    for s in range(60):
        ma, mb = ea.get_action_mask(), eb.get_action_mask()
        mt = et.get_action_mask()
        np.testing.assert_array_equal(ma, mb)
        np.testing.assert_array_equal(ma, mt.cpu().numpy())
        kept.append((ma, ma.copy()))
        a = _sample(mt, gen)
        pinned.copy_(a.cpu())
        oa, ra, da, ia = ea.step(pinned.numpy().copy())   # pageable: staging pass
        ob, rb, db, ib = eb.step(pinned.numpy())          # page-locked: direct DMA
        ot, rt, dt, it = et.step(a)
        for x, y in ((oa, ob), (ra, rb), (da, db)):
            np.testing.assert_array_equal(x, y, err_msg=f"step {s}")
        np.testing.assert_array_equal(oa, ot.cpu().numpy())
        np.testing.assert_array_equal(da, dt.cpu().numpy())
    for arr, saved in kept:
        np.testing.assert_array_equal(arr, saved)
    for e in (ea, eb, et):
        assert e.error_flags() == 0
        e.close()
