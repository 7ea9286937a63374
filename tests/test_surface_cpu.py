"""The drop-in surfaces keep the reference's parameter names, so keyword
callers work unchanged (CPU: signatures only, no compute).

The table is the reference's own signatures (file:line in yemam3/SAC-RCBF);
an extra trailing keyword of ours (the QP `solver`, the replay `device`, the
rollout `seed`) is allowed, a renamed or reordered one is not.
"""
import inspect

import pytest

REFERENCE = {
    # rcbf_sac/diff_cbf_qp.py
    ("diff_cbf_qp", "CBFQPLayer", "__init__"): ("env", "args", "gamma_b", "k_d", "l_p"),  # :12
    ("diff_cbf_qp", "CBFQPLayer", "get_safe_action"): ("state_batch", "action_batch", "mean_pred_batch",
                                                       "sigma_batch"),  # :44
    ("diff_cbf_qp", "CBFQPLayer", "solve_qp"): ("Ps", "qs", "Gs", "hs"),  # :81
    ("diff_cbf_qp", "CBFQPLayer", "cbf_layer"): ("Qs", "ps", "Gs", "hs", "As", "bs", "solver_args"),  # :111
    ("diff_cbf_qp", "CBFQPLayer", "get_cbf_qp_constraints"): ("state_batch", "action_batch", "mean_pred_batch",
                                                              "sigma_pred_batch"),  # :146
    ("diff_cbf_qp", "CBFQPLayer", "get_control_bounds"): (),  # :381
    # rcbf_sac/cbf_qp.py
    ("cbf_qp", "CascadeCBFLayer", "__init__"): ("env", "gamma_b", "k_d", "l_p"),  # :7
    ("cbf_qp", "CascadeCBFLayer", "get_u_safe"): ("u_nom", "s", "mean_pred", "sigma"),  # :29
    ("cbf_qp", "CascadeCBFLayer", "get_cbf_qp_constraints"): ("u_nom", "state", "mean_pred", "sigma_pred"),  # :55
    ("cbf_qp", "CascadeCBFLayer", "solve_qp"): ("P", "q", "G", "h"),  # :242
    ("cbf_qp", "CascadeCBFLayer", "get_cbfs"): ("hazards_locations", "hazards_radius"),  # :288
    ("cbf_qp", "CascadeCBFLayer", "get_control_bounds"): (),  # :325
    ("cbf_qp", "CascadeCBFLayer", "get_min_h_val"): ("state",),  # :341
    # rcbf_sac/dynamics.py
    ("dynamics", "DynamicsModel", "__init__"): ("env", "args"),  # :29
    ("dynamics", "DynamicsModel", "predict_next_state"): ("state_batch", "u_batch", "t_batch", "use_gps"),  # :60
    ("dynamics", "DynamicsModel", "predict_next_obs"): ("state", "u"),  # :107
    ("dynamics", "DynamicsModel", "get_dynamics"): (),  # :125
    ("dynamics", "DynamicsModel", "get_state"): ("obs",),  # :190
    ("dynamics", "DynamicsModel", "get_obs"): ("state_batch",),  # :234
    ("dynamics", "DynamicsModel", "append_transition"): ("state_batch", "u_batch", "next_state_batch",
                                                         "t_batch"),  # :263
    ("dynamics", "DynamicsModel", "fit_gp_model"): ("training_iter",),  # :306
    ("dynamics", "DynamicsModel", "predict_disturbance"): ("test_x",),  # :342
    ("dynamics", "DynamicsModel", "load_disturbance_models"): ("output",),  # :392
    ("dynamics", "DynamicsModel", "save_disturbance_models"): ("output",),  # :409
    ("dynamics", "DynamicsModel", "seed"): ("s",),  # :421
    # rcbf_sac/replay_memory.py
    ("replay_memory", "ReplayMemory", "__init__"): ("capacity", "seed"),  # :6
    ("replay_memory", "ReplayMemory", "push"): ("state", "action", "reward", "next_state", "mask", "t",
                                                "next_t"),  # :12
    ("replay_memory", "ReplayMemory", "batch_push"): ("state_batch", "action_batch", "reward_batch",
                                                      "next_state_batch", "mask_batch", "t_batch",
                                                      "next_t_batch"),  # :20
    ("replay_memory", "ReplayMemory", "sample"): ("batch_size",),  # :28
    # rcbf_sac/generate_rollouts.py
    ("generate_rollouts", None, "generate_model_rollouts"): ("env", "memory_model", "memory", "agent",
                                                             "dynamics_model", "k_horizon", "batch_size",
                                                             "warmup"),  # :6
}


@pytest.mark.parametrize("key", sorted(REFERENCE, key=str), ids=lambda k: ".".join(x for x in k if x))
def test_parameter_names_match_the_reference(key):
    import importlib
    mod_name, cls_name, fn_name = key
    mod = importlib.import_module("rcbf_amd." + mod_name)
    fn = getattr(getattr(mod, cls_name), fn_name) if cls_name else getattr(mod, fn_name)
    params = [p for p in inspect.signature(fn).parameters if p != "self"]
    ref = REFERENCE[key]
    assert tuple(params[:len(ref)]) == ref, (key, params)
    # anything of ours past the reference's parameters has a default (keyword-optional)
    sig = inspect.signature(fn).parameters
    for extra in params[len(ref):]:
        assert sig[extra].default is not inspect.Parameter.empty, (key, extra)


def test_cbf_layer_solver_args_follow_qpfunction():
    """solver_args carry qpth QPFunction's keywords (diff_cbf_qp.py:132-139):
    an unknown key raises TypeError before any device work; the exact solver
    reads none of them, the interior point takes maxIter / eps into a copy of
    its parameters (the layer's own record is untouched)."""
    from types import SimpleNamespace

    import numpy as np

    from rcbf_amd import _lib
    from rcbf_amd.diff_cbf_qp import CBFQPLayer
    box = SimpleNamespace(low=np.full(1, -10.0, np.float32), high=np.full(1, 10.0, np.float32), shape=(1,))
    env = SimpleNamespace(dynamics_mode="SimulatedCars", safe_action_space=box, action_space=box, kp=4.0,
                          k_brake=20.0)
    exact = CBFQPLayer(env, SimpleNamespace(cuda=False), gamma_b=20.0)
    with pytest.raises(TypeError, match="unexpected keyword argument 'maxiter'"):
        exact.cbf_layer(None, None, None, None, solver_args={"maxiter": 5})
    ref_args = {"check_Q_spd": False, "maxIter": 100000, "notImprovedLim": 10, "eps": 1e-4}  # diff_cbf_qp.py:107
    assert exact._solver_params(ref_args) is exact._prm
    pd = CBFQPLayer(env, SimpleNamespace(cuda=False), gamma_b=20.0, solver=_lib.SOLVER_PDIPM)
    p = pd._solver_params(ref_args)
    assert p is not pd._prm and (p.max_iter, p.eps) == (100000, 1e-4) and (pd._prm.max_iter, pd._prm.eps) == (0, 0.0)
    assert p.gamma_b == pd._prm.gamma_b and p.solver == _lib.SOLVER_PDIPM
    # the reference passes verbose=0 itself (diff_cbf_qp.py:139): a second one is a duplicate keyword
    with pytest.raises(TypeError, match="multiple values for keyword argument 'verbose'"):
        pd._solver_params({"verbose": 0})
    with pytest.raises(TypeError, match="multiple values for keyword argument 'verbose'"):
        exact.cbf_layer(None, None, None, None, solver_args={"eps": 1e-4, "verbose": 0})
