"""Build the `rcbf_params` record from a reference-style env + layer args.

Reads exactly the env attributes the reference layers read
(rcbf_sac/diff_cbf_qp.py:12-42, 205-208, 286-290, 392-393;
rcbf_sac/cbf_qp.py:20-27, 93, 167-171, 336-337).
"""
import numpy as np

from . import _lib
from .dynamics import DYNAMICS_MODE


def mode_id(dynamics_mode):
    if dynamics_mode == "SimulatedCars":
        return _lib.MODE_SIMULATED_CARS
    if dynamics_mode == "Unicycle":
        return _lib.MODE_UNICYCLE
    raise Exception("Dynamics mode not supported.")


def make_params(env, gamma_b, k_d=1.5, l_p=0.03, formulation=_lib.FORM_DIFF,
                solver=_lib.SOLVER_ACTIVE_SET, max_iter=0, eps=0.0):
    if env.dynamics_mode not in DYNAMICS_MODE:
        raise Exception("Dynamics mode not supported.")
    p = _lib.RcbfParams()
    p.mode = mode_id(env.dynamics_mode)
    p.formulation = formulation
    p.solver = solver
    p.max_iter = max_iter
    p.eps = eps
    p.gamma_b = float(gamma_b)
    p.k_d = float(k_d)
    p.l_p = float(l_p)
    p.kp = float(getattr(env, "kp", 4.0))
    p.k_brake = float(getattr(env, "k_brake", 20.0))
    lo = np.asarray(env.safe_action_space.low, np.float64).ravel()
    hi = np.asarray(env.safe_action_space.high, np.float64).ravel()
    for c in range(min(2, lo.size)):
        p.u_min[c] = lo[c]
        p.u_max[c] = hi[c]
    if p.mode == _lib.MODE_UNICYCLE:
        hz = np.asarray(env.hazards_locations, np.float64).reshape(-1, 2)
        if not 1 <= hz.shape[0] <= _lib.MAX_HAZARDS:
            raise ValueError(f"1..{_lib.MAX_HAZARDS} hazards supported, got {hz.shape[0]}")
        p.num_hazards = hz.shape[0]
        for j in range(hz.shape[0]):
            p.hazards_xy[2 * j] = hz[j, 0]
            p.hazards_xy[2 * j + 1] = hz[j, 1]
        p.hazards_radius = float(env.hazards_radius)
    else:
        p.num_hazards = 0
        p.hazards_radius = 0.0
    return p
