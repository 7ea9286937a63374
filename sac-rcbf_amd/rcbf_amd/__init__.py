"""rcbf_amd -- MI355X-native batched safe-env step of SAC-RCBF.

Hot path: SimulatedCars / Unicycle control-affine dynamics + the RCBF
safety-layer QP, as hand-written HIP kernels for gfx950 behind a C-ABI
(include/rcbf_hip.h, librcbf_hip.so) and the reference's own Python surfaces:

  rcbf_amd.diff_cbf_qp.CBFQPLayer       <- rcbf_sac/diff_cbf_qp.py
  rcbf_amd.cbf_qp.CascadeCBFLayer       <- rcbf_sac/cbf_qp.py
  rcbf_amd.dynamics.DynamicsModel (prior), DYNAMICS_MODE, MAX_STD <- rcbf_sac/dynamics.py
  rcbf_amd.envs.SimulatedCarsEnv / UnicycleEnv   <- envs/*_env.py
  rcbf_amd.envs.Batched*Env (+ safe_step / rollout: the fused kernels)
  rcbf_amd.build_env.build_env          <- build_env.py
"""
from . import _lib  # noqa: F401

__version__ = "0.1.0"
