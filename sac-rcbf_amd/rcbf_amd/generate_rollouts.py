"""Model-based rollouts (rcbf_sac/generate_rollouts.py:6-81)
on the device.

Each k-step of the reference (get_state -> predict_next_state -> Gaussian
sample -> get_obs -> reward / done -> batch_push) is ONE launch of
rcbf_model_step over the whole batch (fp64, the reference's operation
order), fed by the device ReplayMemory and pushing into it; the disturbance
mean/std come from the GP kernel (rcbf_gp_predict) once the dynamics model
has been fitted, else the MAX_STD prior in-kernel.  The policy is the
agent's own select_action on the host, as in the reference.  The N(0,1)
draws are Philox4x32-10 keyed by (seed, row, call counter) instead of
numpy's global RNG.
"""
import ctypes

import numpy as np
import torch

from . import _lib
from .params import make_params

_counter = [0]


def model_step(env, obs, act, t=None, mean=None, std=None, z=None, seed=0, counter=None):
    """One rcbf_model_step launch.  obs (B,n_o), act (B,n_u), t (B,) f64;
    mean/std (B,n_s) f32 disturbance (None: prior); z (B,n_s) f64 N(0,1)
    draws (None: in-kernel Philox).  Returns next_obs, reward, mask, next_t
    (device f64 tensors)."""
    dev = torch.device("cuda", torch.cuda.current_device())

    def d64(v):
        return None if v is None else torch.as_tensor(v).to(device=dev, dtype=torch.float64).contiguous()

    def d32(v):
        return None if v is None else torch.as_tensor(v).to(device=dev, dtype=torch.float32).contiguous()

    obs, act, t, z = d64(obs), d64(act), d64(t), d64(z)
    mean, std = d32(mean), d32(std)
    B = obs.shape[0]
    if act.dim() == 1:
        act = act.reshape(B, -1).contiguous()
    prm = make_params(env, 1.0)
    nobs = torch.empty_like(obs)
    rew = torch.empty(B, dtype=torch.float64, device=dev)
    mask = torch.empty_like(rew)
    nt = torch.empty_like(rew)
    if counter is None:
        counter = _counter[0]
        _counter[0] += 1
    rc = _lib.load().rcbf_model_step(ctypes.byref(prm), B, _lib.ptr(obs), _lib.ptr(act), _lib.ptr(t), _lib.ptr(mean),
                                     _lib.ptr(std), _lib.ptr(z), seed, counter, _lib.ptr(nobs), _lib.ptr(rew),
                                     _lib.ptr(mask), _lib.ptr(nt), _lib.stream_of(dev))
    _lib.check(rc, "rcbf_model_step")
    return nobs, rew, mask, nt


def generate_model_rollouts(env, memory_model, memory, agent, dynamics_model, k_horizon=1, batch_size=20,
                            warmup=False, seed=0):
    """Same signature and semantics as the reference (memory / memory_model
    are rcbf_amd.replay_memory.ReplayMemory)."""

    def policy(observation):
        if warmup and env.action_space:
            return agent.select_action(observation, dynamics_model, warmup=True)
        return agent.select_action(observation, dynamics_model, evaluate=False)

    obs_b, act_b, rew_b, nobs_b, mask_b, t_b, nt_b = memory.sample_tensors(batch_size)
    obs_ = obs_b
    t_ = t_b
    for _ in range(k_horizon):
        action = policy(obs_.cpu().numpy())
        action = torch.as_tensor(np.asarray(action, np.float64), device=obs_.device).reshape(obs_.shape[0], -1)
        mean = std = None
        if getattr(dynamics_model, "disturb_estimators", None):
            state = dynamics_model.get_state(obs_.cpu().numpy())
            mean, std = dynamics_model.disturb_estimators.predict(torch.as_tensor(state, dtype=torch.float32))
        # predict_next_state is called with the sampled t_batch at every k (generate_rollouts.py:31)
        nobs, rew, mask, nt = model_step(env, obs_, action, t_b[:obs_.shape[0]], mean, std, seed=seed)
        memory_model.batch_push(obs_, action, rew, nobs, mask, t_[:obs_.shape[0]], nt)
        t_ = nt
        keep = mask > 0.5  # delete done trajectories (:77-79)
        obs_ = nobs[keep] if not bool(keep.all()) else nobs
    return memory_model
