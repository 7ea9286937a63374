"""Dynamics-model glue on the hot path (rcbf_sac/dynamics.py).

Only the pieces the safe step uses are here: DYNAMICS_MODE / MAX_STD
(dynamics.py:22-24), get_state / get_obs (:190-261), the zero-mean MAX_STD
prior of predict_disturbance (:381-384) and the model prior of
predict_next_state (:60-105, :125-188).  GP learning (:263-340, gp_model.py)
is out of scope (SURVEY.md section 8f ranks it "next"): a model with GP
estimators attached raises instead of silently using the prior.

Inside the fused step (rcbf_safe_step) get_state and the prior run in-kernel;
this module serves the un-fused API: torch device tensors stay on device (no
numpy round trip, unlike dynamics.py:208-211), numpy inputs keep the
reference's numpy behaviour.
"""
import numpy as np
import torch

DYNAMICS_MODE = {"Unicycle": {"n_s": 3, "n_u": 2},
                 "SimulatedCars": {"n_s": 10, "n_u": 1}}
MAX_STD = {"Unicycle": [2e-1, 2e-1, 2e-1], "SimulatedCars": [0, 0.2, 0, 0.2, 0, 0.2, 0, 0.2, 0, 0.2]}


class DynamicsModel:
    """Prior-only DynamicsModel with the reference's constructor and methods."""

    def __init__(self, env, args):
        self.env = env
        if env.dynamics_mode not in DYNAMICS_MODE:
            raise Exception("Unknown Dynamics mode.")
        self.n_s = DYNAMICS_MODE[env.dynamics_mode]["n_s"]
        self.n_u = DYNAMICS_MODE[env.dynamics_mode]["n_u"]
        self.disturb_estimators = None
        self.max_history_count = getattr(args, "gp_model_size", 2000)
        if hasattr(args, "l_p"):
            self.l_p = args.l_p
        self.device = torch.device("cuda" if getattr(args, "cuda", False) else "cpu")

    # -- obs <-> state (dynamics.py:190-261) -------------------------------
    def get_state(self, obs):
        expand = len(obs.shape) == 1
        if torch.is_tensor(obs):
            o = obs.unsqueeze(0) if expand else obs
            # the reference rescales in fp64 numpy then casts back to obs.dtype
            o64 = o.to(torch.float64)
            if self.env.dynamics_mode == "Unicycle":
                s = torch.stack([o64[:, 0], o64[:, 1], torch.atan2(o64[:, 3], o64[:, 2])], dim=1)
            else:
                s = o64.clone()
                s[:, ::2] *= 100.0
                s[:, 1::2] *= 30.0
            s = s.to(obs.dtype)
            return s.squeeze(0) if expand else s
        o = np.atleast_2d(np.asarray(obs, np.float64))
        if self.env.dynamics_mode == "Unicycle":
            s = np.stack([o[:, 0], o[:, 1], np.arctan2(o[:, 3], o[:, 2])], axis=1)
        else:
            s = o.copy()
            s[:, ::2] *= 100.0
            s[:, 1::2] *= 30.0
        return s[0] if expand else s

    def get_obs(self, state_batch):
        s = np.atleast_2d(np.asarray(state_batch, np.float64))
        if self.env.dynamics_mode == "Unicycle":
            return np.stack([s[:, 0], s[:, 1], np.cos(s[:, 2]), np.sin(s[:, 2])], axis=1)
        o = s.copy()
        o[:, ::2] /= 100.0
        o[:, 1::2] /= 30.0
        return o

    # -- disturbance prior (dynamics.py:342-390) ----------------------------
    def predict_disturbance(self, test_x):
        if self.disturb_estimators:
            raise NotImplementedError("GP disturbance posterior is out of scope (SURVEY 8f row 1)")
        std = MAX_STD[self.env.dynamics_mode]
        if torch.is_tensor(test_x):
            mean = torch.zeros_like(test_x)
            sig = torch.tensor(std, dtype=torch.float64).to(test_x.dtype).to(test_x.device)
            sig = sig.expand_as(test_x).contiguous()
            return mean, sig
        x = np.asarray(test_x, np.float64)
        mean = np.zeros(x.shape)
        sig = np.ones(x.shape) * np.asarray(std)
        return mean, sig

    # -- model prior step (dynamics.py:60-105, 125-188) ---------------------
    def predict_next_state(self, state_batch, u_batch, t_batch=None, use_gps=True):
        if use_gps and self.disturb_estimators:
            raise NotImplementedError("GP disturbance posterior is out of scope (SURVEY 8f row 1)")
        x = np.asarray(state_batch, np.float64)
        expand = x.ndim == 1
        x = np.atleast_2d(x)
        u = np.atleast_2d(np.asarray(u_batch, np.float64))
        dt = self.env.dt
        if self.env.dynamics_mode == "Unicycle":
            f = np.zeros_like(x)
            gu = np.stack([np.cos(x[:, 2]) * u[:, 0], np.sin(x[:, 2]) * u[:, 0], u[:, 1]], axis=1)
        else:
            pos, vel = x[:, ::2], x[:, 1::2]
            vdes = np.full_like(vel, 30.0)
            vdes[:, 0] -= 10 * np.sin(0.2 * np.asarray(t_batch))
            acc = 4.0 * (vdes - vel)
            d01, d12, d24 = pos[:, 0] - pos[:, 1], pos[:, 1] - pos[:, 2], pos[:, 2] - pos[:, 4]
            acc[:, 1] -= 20.0 * d01 * (d01 < 6.0)
            acc[:, 2] -= 20.0 * d12 * (d12 < 6.0)
            acc[:, 3] = 0.0
            acc[:, 4] -= 20.0 * d24 * (d24 < 13.0)
            f = np.zeros_like(x)
            f[:, ::2] = vel
            f[:, 1::2] = acc
            gu = np.zeros_like(x)
            gu[:, 7] = 50.0 * u[:, 0]
        nxt = x + dt * (f + gu)
        std = np.zeros(x.shape)
        if expand:
            nxt, std = nxt[0], std[0]
        if t_batch is not None:
            return nxt, dt * std, t_batch + dt
        return nxt, dt * std, t_batch
