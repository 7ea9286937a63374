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
"""
import torch

from .diff_cbf_qp import CBFQPLayer, _dev, _f32, safe_action_op


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
