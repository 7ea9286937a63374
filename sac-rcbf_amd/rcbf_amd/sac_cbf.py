"""`RCBF_SAC.get_safe_action` (rcbf_sac/sac_cbf.py:218-238) on device.

The SAC update calls it on replay batches (B = batch_size, 256 by default;
sac_cbf.py:133 for the target actions under no_grad, :149 for the policy
actions with gradients flowing back into the policy).  The reference goes
obs -> numpy -> get_state -> predict_disturbance (numpy) -> torch ->
CBFQPLayer, two host round trips per call (dynamics.py:205-232, 357-390).
Here the prior-disturbance case is ONE kernel (rcbf_obs_safe_action:
get_state + rows + normalise + exact QP + clamp) and its backward one more;
with a fitted GP disturbance model, three launches: rcbf_state_from_obs (the
GP's query state), rcbf_gp_predict (the posterior) and the same safe-action
kernel reading the per-env mean / sigma rows.

get_safe_action_host is select_action's per-env-step call (main.py:93 ->
sac_cbf.py:59-91, whose result goes to numpy for env.step): with the fitted
GP, ONE launch (rcbf_gp_obs_safe_action: get_state, the GP posterior and the
safe action in one kernel) writes the action into pinned host memory and a
completion word, so no device-to-host copy or stream synchronisation follows.
"""
import ctypes
import threading

import numpy as np
import torch

from . import _lib
from .diff_cbf_qp import _QP_FAILED, CBFQPLayer, _dev, _f32, safe_action_op
from .dynamics import DYNAMICS_MODE


def get_safe_action(cbf_layer, obs_batch, action_batch, dynamics_model):
    """Drop-in body for RCBF_SAC.get_safe_action(obs_batch, action_batch,
    dynamics_model): returns the safe actions (same device as the action),
    differentiable w.r.t. action_batch."""
    if not isinstance(cbf_layer, CBFQPLayer):
        raise TypeError("cbf_layer must be an rcbf_amd CBFQPLayer")
    gpm = getattr(dynamics_model, "disturb_estimators", None)
    if gpm and not hasattr(gpm, "predict"):  # not rcbf_amd's GP model: the reference's three calls
        state = dynamics_model.get_state(obs_batch)
        mean, sigma = dynamics_model.predict_disturbance(state)
        return cbf_layer.get_safe_action(state, action_batch, mean, sigma)
    expand = len(obs_batch.shape) == 1
    if expand:
        obs_batch = obs_batch.unsqueeze(0)
        action_batch = action_batch.unsqueeze(0)
    out_device = action_batch.device
    dev = _dev()
    obs = _f32(obs_batch, dev)
    if action_batch.requires_grad:
        u = action_batch.to(device=dev, dtype=torch.float32)
        u = u if u.is_contiguous() else u.contiguous()
    else:
        u = _f32(action_batch, dev)
    n_o = cbf_layer.env.observation_space.shape[0]
    if obs.dim() != 2 or obs.shape[1] != n_o or u.shape != (obs.shape[0], cbf_layer.action_dim):
        raise ValueError(f"expected obs (B,{n_o}) and action (B,{cbf_layer.action_dim}), got "
                         f"{tuple(obs.shape)} / {tuple(u.shape)}")
    mean = sigma = None
    if gpm:
        # with the GP fitted (dynamics.py:342-390): the state from the observation (rcbf_state_from_obs, the
        # state the safe-action kernel forms itself), the GP posterior on it (rcbf_gp_predict), then the same
        # one-launch safe action reading the per-env mean / sigma rows -- three launches, no host round trip
        state = dynamics_model.get_state(obs)
        mean, sigma = gpm.predict(state)
    out = safe_action_op(cbf_layer, obs, u, mean, sigma, True)
    if out.device != out_device:
        out = out.to(out_device)
    return out.squeeze(0) if expand else out


class _HostSlot:
    """A pinned host block per device and thread for rcbf_gp_obs_safe_action: the action
    (<= 2 floats) at byte 0, the QP status at byte 32, the completion word at
    byte 64 (its own line)."""

    def __init__(self):
        lib = _lib.load()
        p = ctypes.c_void_p()
        _lib.check(lib.rcbf_host_alloc(128, ctypes.byref(p)), "rcbf_host_alloc")
        self.ptr = p.value
        self.u = (ctypes.c_float * 2).from_address(self.ptr)
        self.status = ctypes.c_int32.from_address(self.ptr + 32)
        self.word = ctypes.c_uint32.from_address(self.ptr + 64)
        self.word.value = 0
        self.seq = 0


_SLOTS = {}


class _NoGuard:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


_NO_GUARD = _NoGuard()


def _ready(t, dev):
    """A contiguous fp32 tensor on `dev` the kernel can read as it is."""
    return t.dtype == torch.float32 and t.device == dev and t.is_contiguous()


def _slot(dev):
    """The calling thread's host slot on `dev` (two threads must not share a
    completion word)."""
    key = (dev.index, threading.get_ident())
    s = _SLOTS.get(key)
    if s is None:
        s = _SLOTS[key] = _HostSlot()
    return s


def get_safe_action_host(cbf_layer, obs, action, dynamics_model):
    """select_action's safe action for ONE observation as a numpy array (n_u,)
    (or (1, n_u) for a (1, n_o) batch) -- what main.py:93 passes to env.step.
    With rcbf_amd's fitted GP and the exact solver: one launch
    (rcbf_gp_obs_safe_action) that ends with the action in pinned host memory;
    the result equals get_safe_action(...) bit for bit.  Otherwise
    get_safe_action(...).cpu().numpy().  Raises Exception('QP Failed to solve')
    like the reference."""
    gpm = getattr(dynamics_model, "disturb_estimators", None)
    obs_t = obs if torch.is_tensor(obs) else torch.as_tensor(np.asarray(obs))
    act_t = action if torch.is_tensor(action) else torch.as_tensor(np.asarray(action))
    single = obs_t.dim() == 1 or (obs_t.dim() == 2 and obs_t.shape[0] == 1)
    n_o = cbf_layer.env.observation_space.shape[0]
    fused = (gpm is not None and hasattr(gpm, "_m") and single and obs_t.shape[-1] == n_o
             and act_t.numel() == cbf_layer.action_dim and cbf_layer._prm.solver == _lib.SOLVER_ACTIVE_SET
             and gpm.n_s == DYNAMICS_MODE[cbf_layer.env.dynamics_mode]["n_s"])
    if not fused:
        out = get_safe_action(cbf_layer, obs_t, act_t, dynamics_model)
        return out.detach().cpu().numpy()
    dev = gpm.device
    o = obs_t if _ready(obs_t, dev) else _f32(obs_t.reshape(1, n_o), dev)
    u = act_t if _ready(act_t, dev) else _f32(act_t.reshape(1, cbf_layer.action_dim), dev)
    slot = _slot(dev)
    slot.seq = (slot.seq + 1) & 0xFFFFFFFF or 1
    stream = torch._C._cuda_getCurrentRawStream(dev.index)
    ent = gpm.__dict__.get("_sa_ws")
    if ent is None or ent[0] != stream:  # the B = 1 workspace of this stream (zero-filled when made)
        ws = gpm._workspace(1)[0]
        ent = gpm._sa_ws = (stream, ws.data_ptr(), ws)
    fast = _lib.fast()
    guard = torch.cuda.device(dev) if torch.cuda.current_device() != dev.index else _NO_GUARD
    with guard:
        if fast is not None:  # CPython binding: ~1 us instead of ~4 us of ctypes argument handling
            rc = fast.gp_obs_safe_action(ctypes.addressof(cbf_layer._prm), ctypes.addressof(gpm._m), o.data_ptr(),
                                         u.data_ptr(), ent[1], stream, slot.ptr, slot.seq)
        else:
            rc = _lib.load().rcbf_gp_obs_safe_action(ctypes.byref(cbf_layer._prm), ctypes.byref(gpm._m), 1,
                                                     _lib.ptr(o), _lib.ptr(u), None, None, None, slot.ptr,
                                                     slot.ptr + 64, slot.seq, slot.ptr + 32, None, ent[1],
                                                     stream or None)
    _lib.check(rc, "rcbf_gp_obs_safe_action")
    if slot.status.value != _lib.QP_OK:
        raise Exception(_QP_FAILED)
    res = np.array(slot.u[:cbf_layer.action_dim], dtype=np.float32)
    return res if obs_t.dim() == 1 else res[None, :]
