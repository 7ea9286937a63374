"""ctypes binding of librcbf_hip.so (C-ABI declared in include/rcbf_hip.h).

The product path is HIP only: if the shared library is missing or fails to
load, every entry point raises -- there is no CPU or PyTorch fallback.
torch is imported first so the process has exactly one HIP runtime
(torch's libamdhip64.so.7; ours binds to the same soname).
"""
import ctypes
import os
import warnings

import torch  # noqa: F401  (loads the HIP runtime the library binds to)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RCBF_HIP_LIB", os.path.join(_HERE, "librcbf_hip.so"))

MODE_SIMULATED_CARS = 0
MODE_UNICYCLE = 1
FORM_DIFF = 0
FORM_CASCADE = 1
SOLVER_ACTIVE_SET = 0
SOLVER_PDIPM = 1
SOLVER_GI = 2
QP_OK, QP_MAX_ITER, QP_INFEASIBLE, QP_NONFINITE = 0, 1, 2, 3
MAX_HAZARDS = 8
ABI_VERSION = 12

_ERRORS = {1001: "RCBF_E_BAD_MODE", 1002: "RCBF_E_BAD_SHAPE", 1003: "RCBF_E_NULL", 1004: "RCBF_E_HSA",
           1005: "RCBF_E_TIMEOUT", 1006: "RCBF_E_GP_HANDOFF"}


class RcbfParams(ctypes.Structure):
    """Mirror of `rcbf_params` (include/rcbf_hip.h)."""
    _fields_ = [
        ("mode", ctypes.c_int32),
        ("formulation", ctypes.c_int32),
        ("num_hazards", ctypes.c_int32),
        ("solver", ctypes.c_int32),
        ("max_iter", ctypes.c_int32),
        ("_pad", ctypes.c_int32),
        ("gamma_b", ctypes.c_double),
        ("k_d", ctypes.c_double),
        ("l_p", ctypes.c_double),
        ("kp", ctypes.c_double),
        ("k_brake", ctypes.c_double),
        ("u_min", ctypes.c_double * 2),
        ("u_max", ctypes.c_double * 2),
        ("hazards_radius", ctypes.c_double),
        ("hazards_xy", ctypes.c_double * (2 * MAX_HAZARDS)),
        ("eps", ctypes.c_double),
    ]


_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_I32 = ctypes.c_int32
_U64 = ctypes.c_uint64
_PRM = ctypes.POINTER(RcbfParams)


# rcbf_safe_action_jac: the f64 bit pattern (as int64) of a saturated row's "no gradient" marker
JAC_NO_GRAD = 0x7FFCD0C0FFEE0000
GP_RT_UPPER = 1  # rcbf_gp_model.flags: [R | alpha] upper triangular (exact posterior)


class RcbfGpModel(ctypes.Structure):
    """include/rcbf_hip.h rcbf_gp_model (device pointers as integers)."""
    _fields_ = [("n_s", ctypes.c_int32), ("N", ctypes.c_int32), ("N_pad", ctypes.c_int32), ("r", ctypes.c_int32),
                ("C_pad", ctypes.c_int32), ("flags", ctypes.c_int32),
                ("xt", ctypes.c_void_p), ("tn2", ctypes.c_void_p), ("Rt", ctypes.c_void_p),
                ("x_std", ctypes.c_void_p), ("inv_sl", ctypes.c_void_p), ("outscale", ctypes.c_void_p),
                ("noise", ctypes.c_void_p), ("y_scale", ctypes.c_void_p)]


_GPM = ctypes.POINTER(RcbfGpModel)

SIGNATURES = {
    "rcbf_build": [_PRM, _I64, _P, _P, _P, _P, _P, _P, _P, _P, _P],
    "rcbf_build_f64": [_PRM, _I64, _P, _P, _P, _P, _P, _P, _P, _P, _P],
    "rcbf_qp_solve": [_PRM, _I64, _I32, _I32, _P, _P, _P, _P, _I32, _P, _P, _P, _P, _P],
    "rcbf_qp_solve_f64": [_PRM, _I64, _I32, _I32, _P, _P, _P, _P, _I32, _P, _P, _P, _P, _P],
    "rcbf_qp_backward": [_PRM, _I64, _I32, _I32, _P, _P, _P, _P, _I32, _P, _P, _P, _P, _P, _P],
    "rcbf_qp_solve_saved": [_PRM, _I64, _I32, _I32, _P, _P, _P, _P, _I32, _P, _P, _P, _P, _P],
    "rcbf_qp_backward_saved": [_PRM, _I64, _I32, _I32, _P, _P, _P, _P, _I32, _P, _P, _P, _P, _P, _P, _P],
    "rcbf_safe_action": [_PRM, _I64, _P, _P, _P, _P, _P, _P, _P, _P],
    "rcbf_safe_action_backward": [_PRM, _I64, _P, _P, _P, _P, _P, _P, _P],
    "rcbf_obs_safe_action": [_PRM, _I64, _P, _P, _P, _P, _P, _P, _P, _P],
    "rcbf_gp_workspace_floats": [_GPM, _I64],
    "rcbf_gp_workspace_init": [_GPM, _P, _P],
    "rcbf_gp_workspace_check": [_GPM, _P, _P],
    "rcbf_predict_next_state": [_PRM, _I64, _P, _P, _P, _P, _P, _I32, _P, _P, _P, _P],
    "rcbf_model_step": [_PRM, _I64, _P, _P, _P, _P, _P, _P, _U64, _U64, _P, _P, _P, _P, _P],
    "rcbf_state_from_obs": [_PRM, _I64, _P, _P, _P],
    "rcbf_ring_scatter_f64": [_P, _I64, _I64, _I64, _P, _I64, _P],
    "rcbf_gather_rows_f64": [_P, _P, _I64, _P, _I64, _P],
    "rcbf_gp_predict": [_GPM, _I64, _P, _P, _P, _P, _P],
    "rcbf_gp_obs_safe_action": [_PRM, _GPM, _I64, _P, _P, _P, _P, _P, _P, _P, ctypes.c_uint32, _P, _P, _P, _P],
    "rcbf_gp_predict_cols": [_GPM, _I64, _P, _P, _P, _P, _I32, _P, _P, _P, _P],
    "rcbf_obs_safe_action_backward": [_PRM, _I64, _P, _P, _P, _P, _P, _P, _P],
    "rcbf_safe_action_jac": [_PRM, _I64, _P, _P, _P, _P, _P, _P, _P, _P, _P],
    "rcbf_obs_safe_action_jac": [_PRM, _I64, _P, _P, _P, _P, _P, _P, _P, _P, _P],
    "rcbf_safe_action_apply_jac": [_I64, _I32, _P, _P, _P, _P],
    "rcbf_cascade_u_safe": [_PRM, _I64, _P, _P, _P, _P, _P, _P, _P, _P, _P],
    "rcbf_cascade_u_safe_sync": [_PRM, _I64, _P, _P, _P, _P, _P, _P, _P, _P, ctypes.c_uint32, _P],
    "rcbf_env_reset": [_PRM, _I64, _P, _P, _U64, _I64, _P, _P, _P, _P, _P, _P],
    "rcbf_env_step": [_PRM, _I64, _P, _P, _P, _P, _P, _I32, _P, _P, _P, _P, _P, _P, _I32, _U64, _I64, _P],
    "rcbf_safe_step": [_PRM, _I64, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I32, _U64, _I64, _P],
    "rcbf_safe_step_cols": [_PRM, _I64, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I32, _U64, _I64,
                            _P],
    "rcbf_safe_rollout": [_PRM, _I64, _I32, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _U64, _I64, _P],
    "rcbf_safe_step_seq": [_PRM, _I64, _I32, _P, _P, _P, _P, _P, _I32, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                           _I32, _U64, _I64, _P],
    "rcbf_safe_step_seq_cols": [_PRM, _I64, _I32, _P, _P, _P, _P, _P, _I32, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                                _I32, _U64, _I64, _P],
    "rcbf_safe_step_span": [_PRM, _I64, _P, _P, _P, _P, _P, _P, _P, _I32, _P, _P, _P, _P, _P, _P, _P, _P, _I32, _U64,
                            _I64, _P, _P],
    "rcbf_env_step_sync": [_PRM, _I64, _P, _P, _P, _P, _P, _I32, _P, _I32, _U64, _I64, _P],
    "rcbf_host_alloc": [_I64, ctypes.POINTER(ctypes.c_void_p)],
    # the AQL dispatch path (csrc/rcbf_aql.hip; rcbf_amd.aql)
    "rcbf_aql_open": [_I32, ctypes.c_char_p, _I32, ctypes.POINTER(ctypes.c_void_p)],
    "rcbf_aql_close": [_P],
    "rcbf_aql_kernel_count": [_P],
    "rcbf_aql_safe_step_plan": [_P, _PRM, _I64, _I32, _P, _P, _P, _P, _P, _I32, _P, _P, _I32, _P, _P, _P, _P, _P, _P,
                                _P, _P, _I32, _U64, _I64, _P, _I32, ctypes.POINTER(ctypes.c_void_p)],
    "rcbf_aql_run": [_P, _U64],
    "rcbf_aql_plan_times": [_P, _P],
    "rcbf_aql_plan_free": [_P],
    "rcbf_host_free": [_P],
    "rcbf_version": [],
    "rcbf_abi_version": [],
    "rcbf_params_size": [],
}

_lib = None
_load_error = None


def load():
    """Load the library once; raise (never fall back) if it is unavailable."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    if _load_error is not None:
        raise _load_error
    if not os.path.exists(LIB_PATH):
        _load_error = RuntimeError(
            f"librcbf_hip.so not found at {LIB_PATH}: build it with `python __graft_entry__.py build` "
            "(hipcc --offload-arch=gfx950). There is no CPU fallback.")
        raise _load_error
    lib = ctypes.CDLL(LIB_PATH)
    for name, argtypes in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = ctypes.c_int32
    lib.rcbf_version.restype = ctypes.c_char_p
    lib.rcbf_gp_workspace_floats.restype = ctypes.c_int64
    if lib.rcbf_abi_version() != ABI_VERSION or lib.rcbf_params_size() != ctypes.sizeof(RcbfParams):
        raise RuntimeError("librcbf_hip.so ABI mismatch (rebuild with `python __graft_entry__.py build`)")
    _bind_fast(lib)
    _bind_torch_op(lib)
    _lib = lib
    return lib


FAST_ENTRY_POINTS = ("rcbf_safe_step", "rcbf_safe_step_seq", "rcbf_env_step_sync", "rcbf_gp_obs_safe_action")
_fast = None


def _bind_fast(lib):
    """Point the CPython binding (csrc/rcbf_pyfast.cpp, optional) at the entry
    points of THIS library copy -- the one ctypes loaded, RCBF_HIP_LIB
    included -- so both bindings always launch the same code."""
    global _fast
    try:
        from . import _rcbf_fast
        _rcbf_fast.bind(*(entry_address(lib, n) for n in FAST_ENTRY_POINTS))
    except (ImportError, AttributeError, TypeError) as e:
        # not built, or a stale build without this bind(): the ctypes path serves
        if not isinstance(e, ImportError):
            warnings.warn(f"_rcbf_fast unusable ({e}); rebuild with `python __graft_entry__.py build`")
        _fast = None
        return
    _fast = _rcbf_fast


TORCH_OP_ENTRY_POINTS = ("rcbf_safe_action", "rcbf_safe_action_backward", "rcbf_obs_safe_action",
                         "rcbf_obs_safe_action_backward", "rcbf_safe_action_jac", "rcbf_obs_safe_action_jac",
                         "rcbf_safe_action_apply_jac")
_torch_op = None


def _bind_torch_op(lib):
    """The C++ autograd op of the safe action (csrc/rcbf_torch_op.cpp,
    optional), bound like the CPython binding to THIS library copy."""
    global _torch_op
    try:
        from . import _rcbf_torch
        _rcbf_torch.bind(*(entry_address(lib, n) for n in TORCH_OP_ENTRY_POINTS))
    except (ImportError, AttributeError, TypeError) as e:
        if not isinstance(e, ImportError):
            warnings.warn(f"_rcbf_torch unusable ({e}); rebuild with `python __graft_entry__.py build`")
        _torch_op = None
        return
    _torch_op = _rcbf_torch


def torch_op():
    """The C++ autograd op bound to the loaded library, or None if not built."""
    load()
    return _torch_op


def entry_address(lib, name):
    return ctypes.cast(getattr(lib, name), ctypes.c_void_p).value


def fast():
    """The CPython binding bound to the loaded library, or None if not built."""
    load()
    return _fast


def check(rc, what):
    if rc != 0:
        msg = _ERRORS.get(rc, f"hipError_t {rc}")
        raise RuntimeError(f"{what} failed: {msg}")


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


def stream_of(device):
    """torch's current HIP stream on `device` (raw handle, without building a
    torch.cuda.Stream object: ~0.3 us instead of ~2.4 us per call)."""
    idx = device.index if isinstance(device, torch.device) else device
    if idx is None:
        idx = torch.cuda.current_device()
    return ctypes.c_void_p(torch._C._cuda_getCurrentRawStream(idx))


def require_device(t, name):
    if not t.is_cuda:
        raise ValueError(f"{name} must be a HIP device tensor")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
