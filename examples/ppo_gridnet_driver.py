"""A GridNet PPO driver over the MI355X engine (BASELINE.json configs[3]).

The reference trains with experiments/ppo_gridnet.py, whose third-party imports
(gym, stable_baselines3, tensorboard) and whose file itself are absent from the
GPU host.  This driver exercises the engine through exactly the calls that
script makes on the env (SURVEY.md §8b callers; ppo_gridnet.py:364-383 the
constructor, :421 reset, :460-466 get_action_mask, :475-476 step with host int64
actions, numpy rewards / dones, infos[i]["raw_rewards"]) and runs the same
algorithm family -- a GridNet encoder / deconvolution actor / critic, a masked
categorical per action component, GAE and the clipped PPO objective -- so the
rollout + update loop of configs[3] (16x16, partial_obs=True, 31 planes, 4096
envs) runs end to end on the GPU.

  --api numpy  : the reference's return contract (numpy obs / masks / rewards),
                 i.e. the host round trips ppo_gridnet.py performs every step
  --api hybrid : the contract an UNMODIFIED ppo_gridnet.py gets with
                 MICRORTS_AMD_RETURN=hybrid (or `run_driver --contract hybrid`):
                 obs / masks stay device tensors, rewards / dones / infos numpy
  --api tensor : return_tensors=True, every buffer stays in HBM

With --api numpy / hybrid the rollout makes ppo_gridnet.py's own calls in its own
forms (`torch.Tensor(envs.reset()).to(device)`, `torch.tensor(envs.get_action_mask())
.to(device)`, `envs.step(action.cpu().numpy().reshape(n, -1))`, `torch.Tensor(rs)`,
the `info["episode"]` scan; ppo_gridnet.py:421, 466, 475-490) through its wrapper
stack: MicroRTSStatsRecorder (restated below, ppo_gridnet.py:126-160) inside
VecMonitor (ppo_gridnet.py:384-385).  The contract is chosen by the environment
variable alone: the env is constructed without `return_tensors`.

  python examples/ppo_gridnet_driver.py --num-selfplay-envs 4072 --num-bot-envs 24 --partial-obs --num-steps 8 --updates 2 --api hybrid

`--eval` runs experiments/ppo_gridnet_eval.py's loop instead (`evaluate`): the reference's
trained agent_sota.pt (committed as tests/golden/agent_sota_policy.npz) against a device bot
(`--ai coacAI`) or against itself in selfplay:

  python examples/ppo_gridnet_driver.py --eval --ai coacAI --num-steps 16 --total-timesteps 32
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.nn as nn

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "microrts-py_amd"))

from gym_microrts import microrts_ai  # noqa: E402
from gym_microrts.envs.vec_env import MicroRTSGridModeVecEnv  # noqa: E402
from gym_microrts.run_driver import install as _install_compat  # noqa: E402

_install_compat()   # stable_baselines3 stand-ins when the real package is absent (as on the GPU host)
from stable_baselines3.common.vec_env import VecEnvWrapper, VecMonitor  # noqa: E402

NVEC = [6, 4, 4, 4, 4, 7, 49]   # action_plane_space.nvec (vec_env.py:234)


def orthogonal(m, gain=np.sqrt(2)):
    nn.init.orthogonal_(m.weight, gain)
    nn.init.zeros_(m.bias)
    return m


class GridNet(nn.Module):
    """Encoder (two conv + max-pool stages, H x W -> H/4 x W/4), a transposed-conv
    actor back to one 78-logit vector per cell, and a value head on the code."""

    def __init__(self, planes, h, w):
        super().__init__()
        self.hw = h * w
        self.enc = nn.Sequential(orthogonal(nn.Conv2d(planes, 32, 3, padding=1)), nn.MaxPool2d(3, 2, 1), nn.ReLU(),
                                 orthogonal(nn.Conv2d(32, 64, 3, padding=1)), nn.MaxPool2d(3, 2, 1), nn.ReLU())
        self.pi = nn.Sequential(orthogonal(nn.ConvTranspose2d(64, 32, 3, 2, 1, 1)), nn.ReLU(),
                                orthogonal(nn.ConvTranspose2d(32, sum(NVEC), 3, 2, 1, 1)))
        self.v = nn.Sequential(nn.Flatten(), orthogonal(nn.Linear(64 * (h // 4) * (w // 4), 128)), nn.ReLU(),
                               orthogonal(nn.Linear(128, 1), 1.0))

    # ppo_gridnet.py's Agent (experiments/ppo_gridnet.py:191-212) names the same layers
    # encoder.{1,4} (after its Transpose), actor.{0,2}, critic.{1,3}
    REFERENCE_NAMES = {"encoder.1": "enc.0", "encoder.4": "enc.3", "actor.0": "pi.0", "actor.2": "pi.2",
                       "critic.1": "v.1", "critic.3": "v.3"}

    def load_reference_state(self, tensors):
        """Load a reference Agent state_dict (name -> tensor / array, e.g. the
        tests/golden/agent_sota_policy.npz fixture of agent_sota.pt); layers it does
        not hold keep their values.  Returns the names loaded."""
        own = self.state_dict()
        done = []
        for k, v in tensors.items():
            layer, _, field = k.rpartition(".")
            if layer in self.REFERENCE_NAMES:
                name = f"{self.REFERENCE_NAMES[layer]}.{field}"
                t = torch.as_tensor(np.asarray(v))
                if own[name].shape != t.shape:
                    raise ValueError(f"{k}: shape {tuple(t.shape)}, this GridNet's {name} is {tuple(own[name].shape)}")
                own[name] = t
                done.append(k)
        self.load_state_dict(own)
        return done

    # what a policy needs to act: the encoder and the actor (the critic is optional --
    # the trimmed fixture omits it, a full agent_sota.pt state_dict carries it)
    POLICY_NAMES = [f"{layer}.{f}" for layer in ("encoder.1", "encoder.4", "actor.0", "actor.2") for f in ("weight", "bias")]

    def load_reference_policy(self, tensors):
        """load_reference_state, then require every encoder / actor tensor: a state_dict
        missing one raises ValueError (not an assert, so it holds under python -O).
        Critic tensors are accepted as extras.  Returns the names loaded."""
        done = self.load_reference_state(tensors)
        missing = [k for k in self.POLICY_NAMES if k not in done]
        if missing:
            raise ValueError(f"policy state_dict lacks {missing}")
        return done

    def forward(self, obs):
        z = self.enc(obs.permute(0, 3, 1, 2))
        logits = self.pi(z).permute(0, 2, 3, 1).reshape(obs.shape[0] * self.hw, sum(NVEC))
        return logits, self.v(z).squeeze(-1)


class StatsRecorder(VecEnvWrapper):
    """MicroRTSStatsRecorder (ppo_gridnet.py:126-160), restated: per env it keeps the
    raw reward rows of the running episode and the same rows scaled by gamma**t with
    their sum appended; when the env's episode ends, a copy of its info gets
    "microrts_stats" = the summed rows under the reward functions' names (and
    "discounted_<name>", "discounted"), and the env's record starts afresh.  Reads
    dones[i] and infos[i]["raw_rewards"] per env, as the reference does."""

    def __init__(self, env, gamma=0.99):
        super().__init__(env)
        self.gamma = gamma

    def reset(self):
        obs = self.venv.reset()
        self._rows = [[] for _ in range(self.num_envs)]
        self._disc = [[] for _ in range(self.num_envs)]
        self._t = np.zeros(self.num_envs, dtype=np.float32)
        return obs

    def step_wait(self):
        obs, rews, dones, infos = self.venv.step_wait()
        out = list(infos[:])
        names = [str(rf) for rf in self.rfs]
        dnames = ["discounted_" + k for k in names] + ["discounted"]
        for i in range(len(dones)):
            r = infos[i]["raw_rewards"]
            self._rows[i].append(r)
            self._disc[i].append((self.gamma ** self._t[i]) * np.concatenate((r, r.sum()), axis=None))
            self._t[i] += 1
            if dones[i]:
                info = infos[i].copy()
                stats = dict(zip(names, np.array(self._rows[i]).sum(0)))
                stats.update(zip(dnames, np.array(self._disc[i]).sum(0)))
                info["microrts_stats"] = stats
                self._rows[i], self._disc[i], self._t[i] = [], [], 0
                out[i] = info
        return obs, rews, dones, out


def make_envs(num_selfplay_envs, num_bot_envs, partial_obs, dev, max_steps=2000, **kw):
    """ppo_gridnet.py:364-385's env: its constructor arguments (one training map,
    cycling over it, reward_weight [10, 1, 1, 0.2, 1, 4], its bot mix), no
    `return_tensors` (the contract comes from MICRORTS_AMD_RETURN), wrapped in
    StatsRecorder and VecMonitor."""
    env = MicroRTSGridModeVecEnv(num_selfplay_envs=num_selfplay_envs, num_bot_envs=num_bot_envs, partial_obs=partial_obs,
                                 max_steps=max_steps, render_theme=2, ai2s=bot_list(num_bot_envs) if num_bot_envs else [],
                                 map_paths=["maps/16x16/basesWorkers16x16A.xml"],
                                 reward_weight=np.array([10.0, 1.0, 1.0, 0.2, 1.0, 4.0]),
                                 cycle_maps=["maps/16x16/basesWorkers16x16A.xml"], device=dev, **kw)
    return VecMonitor(StatsRecorder(env, 0.99)), env


def masked_log_softmax(logits, mask):
    """Per action component: the logit where the mask allows it, -1e8 elsewhere
    (ppo_gridnet's CategoricalMasked rule), as log-probabilities."""
    out = []
    for lg, mk in zip(torch.split(logits, NVEC, 1), torch.split(mask, NVEC, 1)):
        out.append(torch.log_softmax(torch.where(mk.bool(), lg, torch.full_like(lg, -1e8)), -1))
    return out


def policy(net, obs, mask, hw, action=None):
    logits, value = net(obs)
    heads = masked_log_softmax(logits, mask.reshape(-1, sum(NVEC)))
    if action is None:
        action = torch.stack([torch.multinomial(h.exp(), 1).squeeze(-1) for h in heads], -1)
    a = action.reshape(-1, len(NVEC))
    logp = sum(h.gather(1, a[:, k:k + 1]).squeeze(-1) for k, h in enumerate(heads))
    ent = sum(-(h.exp() * h).sum(-1) for h in heads)
    return a.reshape(-1, hw, len(NVEC)), logp.reshape(-1, hw).sum(1), ent.reshape(-1, hw).sum(1), value


def bot_list(n):
    """ppo_gridnet.py:370-373's opponents (n >= 6 bot envs)."""
    return ([microrts_ai.coacAI] * (n - 6) + [microrts_ai.randomBiasedAI] * min(n, 2) + [microrts_ai.lightRushAI] * min(n, 2)
            + [microrts_ai.workerRushAI] * min(n, 2))


def run(num_selfplay_envs=2, num_bot_envs=0, partial_obs=False, num_steps=16, updates=2, api="numpy", minibatches=4,
        epochs=2, seed=1, device="cuda", log=print, max_steps=2000):
    torch.manual_seed(seed)
    np.random.seed(seed)
    dev = torch.device(device)
    ref_calls = api in ("numpy", "hybrid")   # ppo_gridnet.py's own call forms + wrapper stack
    if ref_calls:
        prev = os.environ.get("MICRORTS_AMD_RETURN")
        os.environ["MICRORTS_AMD_RETURN"] = api
        try:
            envs, base = make_envs(num_selfplay_envs, num_bot_envs, partial_obs, dev, max_steps=max_steps)
        finally:
            if prev is None:
                os.environ.pop("MICRORTS_AMD_RETURN", None)
            else:
                os.environ["MICRORTS_AMD_RETURN"] = prev
        assert base.contract == api
    else:
        base = envs = MicroRTSGridModeVecEnv(num_selfplay_envs=num_selfplay_envs, num_bot_envs=num_bot_envs,
                                             partial_obs=partial_obs, max_steps=max_steps, render_theme=2,
                                             ai2s=bot_list(num_bot_envs) if num_bot_envs else [],
                                             map_paths=["maps/16x16/basesWorkers16x16A.xml"],
                                             reward_weight=np.array([10.0, 1.0, 1.0, 0.2, 1.0, 4.0]),
                                             cycle_maps=["maps/16x16/basesWorkers16x16A.xml"], device=dev, return_tensors=True)
    n, hw = envs.num_envs, envs.height * envs.width
    h, w, planes = envs.observation_space.shape
    net = GridNet(planes, h, w).to(dev)
    opt = torch.optim.Adam(net.parameters(), lr=2.5e-4, eps=1e-5)
    buf_obs = torch.zeros((num_steps, n, h, w, planes), device=dev)
    buf_mask = torch.zeros((num_steps, n, hw, sum(NVEC)), device=dev)
    buf_act = torch.zeros((num_steps, n, hw, len(NVEC)), dtype=torch.long, device=dev)
    buf_logp, buf_rew, buf_done, buf_val = (torch.zeros((num_steps, n), device=dev) for _ in range(4))

    def as_dev(x):
        return (x if torch.is_tensor(x) else torch.from_numpy(np.asarray(x))).to(dev).float()

    next_obs = torch.Tensor(envs.reset()).to(dev) if ref_calls else as_dev(envs.reset())   # ppo_gridnet.py:421
    next_done = torch.zeros(n, device=dev)
    ep_ret, finished = torch.zeros(n, device=dev), []
    steps, t0, stats, stats_seen = 0, time.time(), {}, 0
    rollout_s = 0.0
    for update in range(updates):
        tr = time.time()
        for t in range(num_steps):
            buf_obs[t], buf_done[t] = next_obs, next_done
            with torch.no_grad():
                if ref_calls:   # ppo_gridnet.py:466
                    buf_mask[t] = torch.tensor(envs.get_action_mask()).to(dev)
                else:
                    buf_mask[t] = as_dev(envs.get_action_mask())
                a, logp, _, v = policy(net, next_obs, buf_mask[t], hw)
            buf_act[t], buf_logp[t], buf_val[t] = a, logp, v
            if ref_calls:   # ppo_gridnet.py:475-490: host int64 actions (N, H*W*7), numpy rewards / dones, info scan
                obs, rs, ds, infos = envs.step(a.cpu().numpy().reshape(n, -1))
                next_obs = torch.Tensor(obs).to(dev)
                buf_rew[t], next_done = torch.Tensor(rs).to(dev), torch.Tensor(ds).to(dev)
                for info in infos:
                    if "episode" in info.keys():
                        finished.append(info["episode"]["r"])
                        stats_seen += "microrts_stats" in info
            else:
                obs, rew, done, infos = envs.step(a)
                raw = infos._raw
                next_obs, buf_rew[t], next_done = as_dev(obs), as_dev(rew), as_dev(done)
                ep_ret += (raw @ torch.as_tensor(envs.reward_weight, device=dev)).float()
                if bool(next_done.any()):
                    finished += ep_ret[next_done.bool()].tolist()
                    ep_ret[next_done.bool()] = 0
            steps += n
        torch.cuda.synchronize(dev)
        rollout_s += time.time() - tr
        with torch.no_grad():   # GAE (gamma 0.99, lambda 0.95)
            _, last_v = net(next_obs)
            adv = torch.zeros_like(buf_rew)
            gae = torch.zeros(n, device=dev)
            for t in reversed(range(num_steps)):
                nv, nd = (last_v, next_done) if t == num_steps - 1 else (buf_val[t + 1], buf_done[t + 1])
                delta = buf_rew[t] + 0.99 * nv * (1 - nd) - buf_val[t]
                gae = delta + 0.99 * 0.95 * (1 - nd) * gae
                adv[t] = gae
            ret = adv + buf_val
        B = num_steps * n
        flat = [x.reshape((B,) + x.shape[2:]) for x in (buf_obs, buf_mask, buf_act, buf_logp, adv, ret, buf_val)]
        mb = max(1, B // minibatches)
        for _ in range(epochs):
            perm = torch.randperm(B, device=dev)
            for s in range(0, B, mb):
                idx = perm[s:s + mb]
                o, m, a, lp0, ad, rt, v0 = (x[idx] for x in flat)
                ad = (ad - ad.mean()) / (ad.std() + 1e-8)
                _, lp, ent, v = policy(net, o, m, hw, action=a)
                ratio = (lp - lp0).exp()
                pg = torch.max(-ad * ratio, -ad * ratio.clamp(0.9, 1.1)).mean()
                vc = v0 + (v - v0).clamp(-0.1, 0.1)
                vl = 0.5 * torch.max((v - rt) ** 2, (vc - rt) ** 2).mean()
                loss = pg - 0.01 * ent.mean() + 0.5 * vl
                opt.zero_grad()
                loss.backward()
                nn.utils.clip_grad_norm_(net.parameters(), 0.5)
                opt.step()
        torch.cuda.synchronize(dev)
        stats = {"update": update + 1, "global_step": steps, "sps": round(steps / (time.time() - t0), 1),
                 "rollout_env_steps_per_s": round(steps / rollout_s, 1), "loss": float(loss.detach()), "policy_loss": float(pg.detach()),
                 "value_loss": float(vl.detach()), "entropy": float(ent.detach().mean()), "episodes": len(finished),
                 "microrts_stats_infos": stats_seen, "api": api, "num_envs": n, "partial_obs": bool(partial_obs)}
        log(stats)
    stats["engine_error_flags"] = base.error_flags()
    stats["finite"] = bool(np.isfinite([stats["loss"], stats["value_loss"], stats["entropy"]]).all())
    envs.close()
    return stats


def load_weights(path):
    """A reference Agent state_dict as name -> tensor: the committed .npz fixture of
    agent_sota.pt (tests/golden/make_agent_sota.py), or a .pt file read with
    torch.load(weights_only=True) (never an unpickling load)."""
    if path.endswith(".npz"):
        with np.load(path) as z:
            return {k: torch.from_numpy(z[k]) for k in z.files}
    return torch.load(path, map_location="cpu", weights_only=True)


SOTA = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "agent_sota_policy.npz")


def evaluate(ai="", num_steps=256, total_timesteps=1000000, agent_model_path=SOTA, agent2_model_path=SOTA, seed=1,
             device="cuda", log=print, render=True):
    """experiments/ppo_gridnet_eval.py's loop over this engine: a trained GridNet (default
    the reference's agent_sota.pt) against a device bot (`ai`, 1 bot env; :60-61) or
    against a second trained GridNet in selfplay (2 selfplay envs, player 0 = agent and
    player 1 = agent2 on the even / odd envs; :62-63, 170-186), basesWorkers16x16A,
    max_steps 5000, reward_weight [10, 1, 1, 0.2, 1, 4] (:113-123), StatsRecorder +
    VecMonitor (:124-125), render() every step (:161), the masks and steps in the
    script's own call forms (:168, :189-190), and one WinLoss line per finished
    episode (:195-201).  Returns the win / loss records and the step count."""
    torch.manual_seed(seed)
    np.random.seed(seed)
    dev = torch.device(device)
    ais = [getattr(microrts_ai, ai)] if ai else []
    nbot, nsp = (1, 0) if ai else (0, 2)
    env = MicroRTSGridModeVecEnv(num_bot_envs=nbot, num_selfplay_envs=nsp, partial_obs=False, max_steps=5000, render_theme=2,
                                 ai2s=ais, map_paths=["maps/16x16/basesWorkers16x16A.xml"],
                                 reward_weight=np.array([10.0, 1.0, 1.0, 0.2, 1.0, 4.0]), device=dev)
    envs = VecMonitor(StatsRecorder(env, 0.99))
    n, hw = envs.num_envs, envs.height * envs.width
    h, w, planes = envs.observation_space.shape
    agent, agent2 = GridNet(planes, h, w).to(dev), GridNet(planes, h, w).to(dev)
    agent.load_reference_policy(load_weights(agent_model_path))
    agent.eval()
    if not ai:
        agent2.load_reference_policy(load_weights(agent2_model_path))
        agent2.eval()
    num_updates = total_timesteps // (n * num_steps)
    next_obs = torch.Tensor(envs.reset()).to(dev)
    results, global_step = [], 0
    for _ in range(num_updates):
        for _ in range(num_steps):
            if render:
                envs.render()
            global_step += n
            with torch.no_grad():
                masks = torch.tensor(np.array(envs.get_action_mask())).to(dev)
                if ai:
                    action, _, _, _ = policy(agent, next_obs, masks, hw)
                else:
                    p1, _, _, _ = policy(agent, next_obs[::2], masks[::2], hw)
                    p2, _, _, _ = policy(agent2, next_obs[1::2], masks[1::2], hw)
                    action = torch.zeros((n,) + tuple(p2.shape[1:]), dtype=torch.long, device=dev)
                    action[::2], action[1::2] = p1, p2
            obs, rs, ds, infos = envs.step(action.cpu().numpy().reshape(n, -1))
            next_obs = torch.Tensor(obs).to(dev)
            for idx, info in enumerate(infos):
                if "episode" in info.keys():
                    wl = float(info["microrts_stats"]["WinLossRewardFunction"])
                    if ai:
                        log(f"against {ai} {wl}")
                        results.append(("agent", wl))
                    elif idx % 2 == 0:
                        log(f"player{idx % 2} {wl}")
                        results.append(("player0", wl))
    out = {"global_step": global_step, "results": results, "engine_error_flags": env.error_flags()}
    envs.close()
    return out


if __name__ == "__main__":
    if "--eval" in sys.argv:   # ppo_gridnet_eval.py's flags
        ap = argparse.ArgumentParser()
        ap.add_argument("--eval", action="store_true")
        ap.add_argument("--ai", type=str, default="")
        ap.add_argument("--num-steps", type=int, default=256)
        ap.add_argument("--total-timesteps", type=int, default=1000000)
        ap.add_argument("--agent-model-path", type=str, default=SOTA)
        ap.add_argument("--agent2-model-path", type=str, default=SOTA)
        ap.add_argument("--seed", type=int, default=1)
        a = ap.parse_args()
        out = evaluate(a.ai, a.num_steps, a.total_timesteps, a.agent_model_path, a.agent2_model_path, a.seed)
        print(json.dumps(out))
        sys.exit(0)
    ap = argparse.ArgumentParser()
    ap.add_argument("--num-selfplay-envs", type=int, default=2)
    ap.add_argument("--num-bot-envs", type=int, default=0)
    ap.add_argument("--partial-obs", action="store_true")
    ap.add_argument("--num-steps", type=int, default=16)
    ap.add_argument("--updates", type=int, default=2)
    ap.add_argument("--minibatches", type=int, default=4)
    ap.add_argument("--api", choices=["numpy", "hybrid", "tensor"], default="numpy")
    ap.add_argument("--max-steps", type=int, default=2000)
    a = ap.parse_args()
    out = run(a.num_selfplay_envs, a.num_bot_envs, a.partial_obs, a.num_steps, a.updates, a.api, a.minibatches,
              log=lambda s: print(json.dumps(s), flush=True), max_steps=a.max_steps)
    print(json.dumps(out))
