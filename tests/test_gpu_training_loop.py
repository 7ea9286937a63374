"""The reference's training loop, shaped as main.py:19-101 runs it, on
rcbf_amd's surfaces end to end on the device.

Per env step: select_action (policy sample -> RCBF_SAC.get_safe_action,
sac_cbf.py:59-91, 218-238: get_state -> predict_disturbance -> CBFQPLayer)
-> env.step (the single-env gym class, rcbf_env_step_sync) -> ReplayMemory.push
-> DynamicsModel.append_transition every 2nd step (a GP refit every
gp_model_size / 10 appended transitions, dynamics.py:303-304) -> when the
buffers hold a batch, update_parameters (sac_cbf.py:95-158: target safe
actions under no_grad, the policy's safe actions with the gradient through
the differentiable CBF-QP) and, for cars, generate_model_rollouts every 5th
step (main.py:52-57) into a second ReplayMemory.

The SAC networks are out of scope, so the agent here is the
reference's shape with small MLPs (model.py's GaussianPolicy / QNetwork at
hidden 32) -- only the safety layer, the envs, the dynamics model and the
buffers are the product.  The GP variance is forced to a Lanczos (LOVE) root
of size 16 (gp_rank) so the fast_pred_var path runs at the loop's small
gp_model_size; the B = 1 query takes the one-launch GEMV, the update's
B = 256 query the MFMA path.

Asserted: the reference's observable contract -- info['cost'] as the
reference envs report it, the refit cadence, every safe action inside
safe_action_space, no 'QP Failed to solve', finite losses and gradients.
The per-env-step time is recorded (gpurun_out/training_loop_r06.json when
that directory exists) for DESIGN §5.5 against BASELINE.md's reference
pre-solve path (1.21 ms cars / 0.45 ms unicycle per RCBF_SAC.get_safe_action
at B = 1)."""
import json
import os
import time
import types

import numpy as np
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.distributions import Normal

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class _Policy(nn.Module):
    """model.py GaussianPolicy (tanh-squashed, rescaled to the action space)."""

    def __init__(self, n_in, n_act, hidden, space):
        super().__init__()
        self.l1, self.l2 = nn.Linear(n_in, hidden), nn.Linear(hidden, hidden)
        self.mean, self.log_std = nn.Linear(hidden, n_act), nn.Linear(hidden, n_act)
        self.register_buffer("scale", torch.as_tensor((space.high - space.low) / 2.0, dtype=torch.float32))
        self.register_buffer("bias", torch.as_tensor((space.high + space.low) / 2.0, dtype=torch.float32))

    def sample(self, s):
        x = F.relu(self.l2(F.relu(self.l1(s))))
        mean, log_std = self.mean(x), self.log_std(x).clamp(-20, 2)
        normal = Normal(mean, log_std.exp())
        x_t = normal.rsample()
        y_t = torch.tanh(x_t)
        action = y_t * self.scale + self.bias
        log_prob = (normal.log_prob(x_t) - torch.log(self.scale * (1 - y_t.pow(2)) + 1e-6)).sum(1, keepdim=True)
        return action, log_prob, torch.tanh(mean) * self.scale + self.bias


class _Q(nn.Module):
    """model.py QNetwork (twin Q)."""

    def __init__(self, n_in, n_act, hidden):
        super().__init__()
        self.q1 = nn.Sequential(nn.Linear(n_in + n_act, hidden), nn.ReLU(), nn.Linear(hidden, hidden), nn.ReLU(),
                                nn.Linear(hidden, 1))
        self.q2 = nn.Sequential(nn.Linear(n_in + n_act, hidden), nn.ReLU(), nn.Linear(hidden, hidden), nn.ReLU(),
                                nn.Linear(hidden, 1))

    def forward(self, s, a):
        xu = torch.cat([s, a], 1)
        return self.q1(xu), self.q2(xu)


class _Agent:
    """RCBF_SAC's select_action / update_parameters / get_safe_action
    (sac_cbf.py:12-158, 218-238) over rcbf_amd.diff_cbf_qp.CBFQPLayer."""

    def __init__(self, env, args):
        from rcbf_amd.diff_cbf_qp import CBFQPLayer
        n_o, n_a = env.observation_space.shape[0], env.action_space.shape[0]
        self.dev = torch.device("cuda")
        self.action_space = env.action_space
        self.gamma, self.tau, self.alpha = 0.99, 0.005, 0.2
        self.policy = _Policy(n_o, n_a, 32, env.action_space).to(self.dev)
        self.critic, self.critic_target = _Q(n_o, n_a, 32).to(self.dev), _Q(n_o, n_a, 32).to(self.dev)
        self.critic_target.load_state_dict(self.critic.state_dict())
        self.policy_optim = torch.optim.Adam(self.policy.parameters(), lr=3e-4)
        self.critic_optim = torch.optim.Adam(self.critic.parameters(), lr=3e-4)
        self.cbf_layer = CBFQPLayer(env, args, args.gamma_b, args.k_d, args.l_p)
        self.safe_action_s = []
        self.grads_finite = []

    def get_safe_action(self, obs_batch, action_batch, dynamics_model):
        from rcbf_amd.sac_cbf import get_safe_action
        return get_safe_action(self.cbf_layer, obs_batch, action_batch, dynamics_model)

    def select_action(self, state, dynamics_model, evaluate=False, warmup=False):
        state = torch.as_tensor(np.asarray(state), dtype=torch.float32, device=self.dev)
        expand = state.dim() == 1
        if expand:
            state = state.unsqueeze(0)
        if warmup:
            action = torch.stack([torch.as_tensor(self.action_space.sample()) for _ in range(state.shape[0])])
            action = action.to(self.dev, torch.float32)
        else:
            with torch.no_grad():
                a, _, m = self.policy.sample(state)
            action = m if evaluate else a
        torch.cuda.synchronize()  # the policy's launches are not the safety layer's time
        t0 = time.perf_counter()
        # the per-env-step path: with the fitted GP one launch that leaves the action in pinned host memory
        from rcbf_amd.sac_cbf import get_safe_action_host
        out = get_safe_action_host(self.cbf_layer, state, action, dynamics_model)
        self.safe_action_s.append(time.perf_counter() - t0)
        return out[0] if expand else out

    def update_parameters(self, memory, batch_size, updates, dynamics_model, memory_model=None, real_ratio=None):
        if memory_model and real_ratio:
            s, a, r, ns, m, _, _ = memory.sample(batch_size=int(real_ratio * batch_size))
            s2, a2, r2, ns2, m2, _, _ = memory_model.sample(batch_size=int((1 - real_ratio) * batch_size))
            s, a, r, ns, m = np.vstack((s, s2)), np.vstack((a, a2)), np.hstack((r, r2)), np.vstack((ns, ns2)), \
                np.hstack((m, m2))
        else:
            s, a, r, ns, m, _, _ = memory.sample(batch_size=batch_size)
        f = lambda v: torch.as_tensor(np.asarray(v), dtype=torch.float32, device=self.dev)  # noqa: E731
        s, ns, a, r, m = f(s), f(ns), f(a), f(r).unsqueeze(1), f(m).unsqueeze(1)
        with torch.no_grad():
            na, nlp, _ = self.policy.sample(ns)
            na = self.get_safe_action(ns, na, dynamics_model)  # diff_qp (sac_cbf.py:133)
            q1t, q2t = self.critic_target(ns, na)
            target = r + m * self.gamma * (torch.min(q1t, q2t) - self.alpha * nlp)
        q1, q2 = self.critic(s, a)
        qf_loss = F.mse_loss(q1, target) + F.mse_loss(q2, target)
        self.critic_optim.zero_grad()
        qf_loss.backward()
        self.critic_optim.step()
        pi, log_pi, _ = self.policy.sample(s)
        pi = self.get_safe_action(s, pi, dynamics_model)  # the gradient flows back through the CBF-QP (:149)
        q1p, q2p = self.critic(s, pi)
        policy_loss = (self.alpha * log_pi - torch.min(q1p, q2p)).mean()
        self.policy_optim.zero_grad()
        policy_loss.backward()
        grads = [p.grad for p in self.policy.parameters() if p.grad is not None]
        self.grads_finite.append(bool(grads) and all(bool(torch.isfinite(g).all()) for g in grads)
                                 and bool(torch.isfinite(qf_loss)) and bool(torch.isfinite(policy_loss)))
        self.policy_optim.step()
        with torch.no_grad():
            for tp, p in zip(self.critic_target.parameters(), self.critic.parameters()):
                tp.mul_(1 - self.tau).add_(self.tau * p)
        return float(qf_loss), float(policy_loss)


def _train(env_name, episodes, model_based):
    """main.py train() for `episodes` episodes; returns the loop's record."""
    from rcbf_amd.build_env import build_env
    from rcbf_amd.dynamics import DynamicsModel
    from rcbf_amd.generate_rollouts import generate_model_rollouts
    from rcbf_amd.replay_memory import ReplayMemory
    torch.manual_seed(0)
    np.random.seed(0)
    args = types.SimpleNamespace(env_name=env_name, cuda=True, gamma_b=20.0, k_d=3.0, l_p=0.03, gp_model_size=300,
                                 gp_rank=16, batch_size=256, start_steps=100, updates_per_step=1, replay_size=100000,
                                 model_based=model_based, k_horizon=1, rollout_batch_size=5, real_ratio=0.3, seed=0)
    env = build_env(args)
    env.seed(0)
    dm = DynamicsModel(env, args)
    fits = []
    fit = dm.fit_gp_model
    dm.fit_gp_model = lambda *a, **k: (fits.append(dm.history_counter), fit(*a, **k))
    agent = _Agent(env, args)
    memory, memory_model = ReplayMemory(args.replay_size, args.seed), ReplayMemory(args.replay_size, args.seed)
    rec = {"steps": 0, "updates": 0, "episodes": [], "step_s": [], "update_s": [], "rollout_calls": 0}
    lo, hi = env.safe_action_space.low, env.safe_action_space.high
    total = 0
    for _ in range(episodes):
        obs, done, ep_steps, ep_r, ep_c = env.reset(), False, 0, 0.0, 0.0
        while not done:
            state = dm.get_state(obs)
            if model_based and ep_steps % 5 == 0 and len(memory) > dm.max_history_count / 3:
                memory_model = generate_model_rollouts(env, memory_model, memory, agent, dm, k_horizon=args.k_horizon,
                                                       batch_size=min(len(memory), 5 * args.rollout_batch_size),
                                                       warmup=args.start_steps > total)
                rec["rollout_calls"] += 1
            if len(memory) + len(memory_model) * model_based > args.batch_size:
                t_up = time.perf_counter()
                for _ in range(args.updates_per_step):
                    if model_based:
                        rr = max(min(args.real_ratio, len(memory) / args.batch_size),
                                 1 - len(memory_model) / args.batch_size)
                        agent.update_parameters(memory, args.batch_size, rec["updates"], dm, memory_model, rr)
                    else:
                        agent.update_parameters(memory, args.batch_size, rec["updates"], dm)
                    rec["updates"] += 1
                torch.cuda.synchronize()  # the update's queued tail stays out of the env step's time
                rec["update_s"].append(time.perf_counter() - t_up)
            t0 = time.perf_counter()
            action = agent.select_action(obs, dm, warmup=args.start_steps > total)
            next_obs, reward, done, info = env.step(action)
            rec["step_s"].append(time.perf_counter() - t0)
            if env_name == "SimulatedCars":
                assert "cost" in info and info["goal_met"] is False  # simulated_cars_env.py:84-87
            else:
                assert info.get("cost", 0) in (0, 0.1)  # unicycle_env.py:100-104: the key only on contact
            assert np.all(action >= lo - 1e-6) and np.all(action <= hi + 1e-6)
            ep_steps += 1
            total += 1
            ep_r += float(reward)
            ep_c += float(info.get("cost", 0))
            mask = 1 if ep_steps == env.max_episode_steps else float(not done)
            memory.push(obs, action, reward, next_obs, mask, t=ep_steps * env.dt, next_t=(ep_steps + 1) * env.dt)
            next_state = dm.get_state(next_obs)
            if ep_steps % 2 == 0:
                dm.append_transition(state, action, next_state, t_batch=np.array([ep_steps * env.dt]))
            obs = next_obs
        rec["episodes"].append({"steps": ep_steps, "reward": ep_r, "cost": ep_c})
        rec["steps"] += ep_steps
        if dm.disturb_estimators is not None:  # the GP hand-off's counters are clean after the episode
            dm.disturb_estimators.check_failures()
    rec.update(fits=fits, agent=agent, dm=dm, memory_len=len(memory), memory_model_len=len(memory_model))
    return rec


def _record(name, rec):
    out_dir = os.path.join(ROOT, "gpurun_out")
    warm = np.asarray(rec["step_s"][200:]) * 1e6  # past the warm-up actions and first launches
    sa = np.asarray(rec["agent"].safe_action_s[200:]) * 1e6
    up = np.asarray(rec["update_s"]) * 1e6
    row = {"env_steps": rec["steps"], "updates": rec["updates"], "gp_fits": len(rec["fits"]),
           "rollout_calls": rec["rollout_calls"],
           "env_step_us_median": round(float(np.median(warm)), 1),
           "env_step_us_p90": round(float(np.percentile(warm, 90)), 1),
           "safe_action_us_median": round(float(np.median(sa)), 1),
           "update_us_median": round(float(np.median(up)), 1) if up.size else None,
           "what": "env_step: select_action (policy MLP sample, synchronize, RCBF_SAC.get_safe_action with the GP "
                   "posterior at B = 1, to numpy) + env.step (rcbf_env_step_sync), after the update's queued work "
                   "has drained; safe_action: get_safe_action + .cpu() alone; update: update_parameters at "
                   "B = 256 (two safe-action calls, one with the gradient through the CBF-QP) to its drained end",
           "episodes": rec["episodes"]}
    if os.path.isdir(out_dir):
        path = os.path.join(out_dir, "training_loop_r06.json")
        data = json.load(open(path)) if os.path.exists(path) else {}
        data[name] = row
        json.dump(data, open(path, "w"), indent=1)
    print(name, json.dumps(row))


def _check(rec, every):
    assert rec["fits"] and all(c % every == 0 for c in rec["fits"])  # dynamics.py:303-304
    assert rec["fits"] == [every * (k + 1) for k in range(len(rec["fits"]))]
    gpm = rec["dm"].disturb_estimators
    assert gpm is not None and gpm.rank == 16 and gpm.love_init is not None  # the Lanczos (LOVE) factor
    assert rec["updates"] > 0 and all(rec["agent"].grads_finite)


def test_training_loop_cars_model_based():
    """Two SimulatedCars episodes (300 steps each) with model-based rollouts."""
    rec = _train("SimulatedCars", 2, model_based=True)
    assert [e["steps"] for e in rec["episodes"]] == [300, 300]
    _check(rec, 30)
    assert rec["rollout_calls"] > 0 and rec["memory_model_len"] > 0
    assert rec["memory_len"] == 600
    _record("SimulatedCars", rec)


def test_training_loop_unicycle():
    """One Unicycle episode (the reference's 5 hazards, up to 1000 steps)."""
    rec = _train("Unicycle", 1, model_based=False)
    assert 1 <= rec["episodes"][0]["steps"] <= 1000
    _check(rec, 30)
    _record("Unicycle", rec)
