"""End-to-end drivers on the HIP engine (the reference's tests/test_e2e.py runs
experiments/ppo_gridnet.py with 2 selfplay envs, 16 steps, 32 timesteps).

examples/ppo_gridnet_driver.py drives the env through the same calls
ppo_gridnet.py makes; these tests run it on the GPU with the
reference's test sizes and with BASELINE configs[3]'s shape (partial_obs, bot
mix of ppo_gridnet.py:370-373) at a small env count."""
import importlib.util
import os

import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]   # per-test limits below override

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _driver():
    spec = importlib.util.spec_from_file_location("ppo_gridnet_driver", os.path.join(REPO, "examples", "ppo_gridnet_driver.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_ppo_gridnet_selfplay_numpy_api():
    """test_e2e.py:4-14: --num-bot-envs 0 --num-selfplay-envs 2 --num-steps 16 --total-timesteps 32."""
    s = _driver().run(num_selfplay_envs=2, num_bot_envs=0, num_steps=16, updates=1, api="numpy", log=lambda _: None)
    assert s["global_step"] == 32 and s["finite"] and s["engine_error_flags"] == 0


@pytest.mark.parametrize("api", ["numpy", "tensor"])
def test_ppo_gridnet_partial_obs_with_bots(api):
    """configs[3] shape: partial_obs (31 planes) + the bot envs ppo_gridnet.py builds."""
    s = _driver().run(num_selfplay_envs=8, num_bot_envs=8, partial_obs=True, num_steps=8, updates=2, api=api, log=lambda _: None)
    assert s["global_step"] == 2 * 8 * 16 and s["finite"] and s["engine_error_flags"] == 0


def test_ppo_gridnet_eval_selfplay():
    """test_e2e.py:17-26: ppo_gridnet_eval.py --num-steps 16 --total-timesteps 32 (2 selfplay
    envs, the reference's agent_sota.pt on both sides, render() every step)."""
    out = _driver().evaluate(num_steps=16, total_timesteps=32, log=lambda _: None)
    assert out["global_step"] == 32 and out["engine_error_flags"] == 0


def test_ppo_gridnet_eval_bot():
    """test_e2e.py:29-35: ppo_gridnet_eval.py --ai coacAI --num-steps 16 --total-timesteps 32;
    and a longer run in which agent_sota.pt finishes games against the device coacAI."""
    d = _driver()
    out = d.evaluate(ai="coacAI", num_steps=16, total_timesteps=32, log=lambda _: None)
    assert out["global_step"] == 32 and out["engine_error_flags"] == 0
    lines = []
    out = d.evaluate(ai="coacAI", num_steps=500, total_timesteps=3000, log=lines.append, render=False)
    assert out["engine_error_flags"] == 0 and out["results"], "no episode ended in 3000 steps"
    assert all(x.startswith("against coacAI ") for x in lines)
    assert all(r in (-1.0, 0.0, 1.0) for _, r in out["results"])
