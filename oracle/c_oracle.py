"""ctypes wrapper of oracle/_build/librcbf_oracle.so -- TEST INFRASTRUCTURE ONLY
(tests/ and bench.py's cpu_baseline leg).  Same algorithm as oracle.py in C,
OpenMP over envs; built by __graft_entry__.build_oracle()."""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(_HERE, "_build", "librcbf_oracle.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(SO):
            import subprocess
            import sys
            subprocess.run([sys.executable, os.path.join(os.path.dirname(_HERE), "__graft_entry__.py"), "build_oracle"],
                           check=True)
        _lib = ctypes.CDLL(SO)
        P = ctypes.c_void_p
        _lib.oracle_safe_action.argtypes = [ctypes.c_int, ctypes.c_int, P, ctypes.c_double, ctypes.c_int64,
                                            P, P, P, P, P, ctypes.c_int]
        _lib.oracle_safe_step.argtypes = [ctypes.c_int, ctypes.c_int, P, ctypes.c_double, ctypes.c_int64,
                                          P, P, P, P, P, P, P, P, ctypes.c_int]
        _lib.oracle_cars_cascade_loop.argtypes = [ctypes.c_double, ctypes.c_int, ctypes.c_double, P, P, P]
        _lib.oracle_safe_step_ex.argtypes = [ctypes.c_int, ctypes.c_int, P, ctypes.c_double, ctypes.c_int64,
                                             P, P, P, P, P, P, P, P, P, P, P, P, ctypes.c_int, P, P, ctypes.c_int]
        _lib.oracle_safe_action_grad.argtypes = [ctypes.c_int, ctypes.c_int, P, ctypes.c_double, ctypes.c_int64,
                                                 P, P, P, P, P, P, P, ctypes.c_int]
        _lib.oracle_max_threads.restype = ctypes.c_int
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _hz(hazards):
    if hazards is None:
        return np.zeros(2), 0
    h = np.ascontiguousarray(np.asarray(hazards, np.float64).reshape(-1, 2))
    return h, h.shape[0]


def safe_action(mode, x, u, mu, sigma, gamma_b, hazards=None, threads=0):
    m = 0 if mode == "SimulatedCars" else 1
    x = np.ascontiguousarray(x, np.float32); u = np.ascontiguousarray(u, np.float32)
    mu = np.ascontiguousarray(mu, np.float32); sigma = np.ascontiguousarray(sigma, np.float32)
    hz, K = _hz(hazards)
    out = np.empty_like(u)
    fails = lib().oracle_safe_action(m, K, _p(hz), float(gamma_b), x.shape[0], _p(x), _p(u), _p(mu), _p(sigma),
                                     _p(out), int(threads))
    return out, fails


def safe_action_grad(mode, x, u, mu, sigma, gamma_b, w, hazards=None, threads=0):
    """CBFQPLayer.get_safe_action and d(sum w * final)/d u (oracle.safe_action_diff_grad
    restated in C): returns (final (B, n_u) f32, grad (B, n_u) f64, fails)."""
    m = 0 if mode == "SimulatedCars" else 1
    x = np.ascontiguousarray(x, np.float32); u = np.ascontiguousarray(u, np.float32)
    mu = np.ascontiguousarray(mu, np.float32); sigma = np.ascontiguousarray(sigma, np.float32)
    w = np.ascontiguousarray(w, np.float32)
    hz, K = _hz(hazards)
    out = np.empty_like(u)
    grad = np.empty(u.shape, np.float64)
    fails = lib().oracle_safe_action_grad(m, K, _p(hz), float(gamma_b), x.shape[0], _p(x), _p(u), _p(mu), _p(sigma),
                                          _p(w), _p(out), _p(grad), int(threads))
    return out, grad, fails


def safe_step(mode, x, aux, step, u, gamma_b, hazards=None, threads=0):
    """In-place fused step on x (B,n_s) f64, aux (B,) f64, step (B,) i32."""
    m = 0 if mode == "SimulatedCars" else 1
    u = np.ascontiguousarray(u, np.float32)
    hz, K = _hz(hazards)
    B = x.shape[0]
    uo = np.empty_like(u)
    rew = np.empty(B, np.float32); cost = np.empty(B, np.float32); done = np.empty(B, np.uint8)
    fails = lib().oracle_safe_step(m, K, _p(hz), float(gamma_b), B, _p(x), _p(aux), _p(step), _p(u), _p(uo),
                                   _p(rew), _p(cost), _p(done), int(threads))
    return uo, rew, cost, done, fails


def safe_step_ex(mode, x, aux, step, u, gamma_b, hazards=None, mean=None, sigma=None, auto_reset=False,
                 reset_noise=None, env_action=None, threads=0):
    """In-place fused step with the kernel's full output set: mean/sigma
    (B, n_s) f32 or None (prior), auto-reset with the cars reset draw injected
    (reset_noise (B,) f64 = the N(0, 0.5) sample an env takes if it resets).
    env_action (B, n_u) f32 or None: step the env with this action instead of
    the oracle's own safe action (still returned as "u").
    Returns dict(u, reward, cost, done, goal, obs, fails)."""
    m = 0 if mode == "SimulatedCars" else 1
    n_o = 10 if m == 0 else 7
    u = np.ascontiguousarray(u, np.float32)
    hz, K = _hz(hazards)
    B = x.shape[0]
    assert x.flags.c_contiguous and x.dtype == np.float64 and aux.dtype == np.float64 and step.dtype == np.int32
    mu = None if mean is None else np.ascontiguousarray(mean, np.float32)
    sg = None if sigma is None else np.ascontiguousarray(sigma, np.float32)
    nz = None if reset_noise is None else np.ascontiguousarray(reset_noise, np.float64)
    ea = None if env_action is None else np.ascontiguousarray(env_action, np.float32).reshape(u.shape)
    out = dict(u=np.empty_like(u), reward=np.empty(B, np.float32), cost=np.empty(B, np.float32),
               done=np.empty(B, np.uint8), goal=np.empty(B, np.uint8), obs=np.empty((B, n_o), np.float32))

    def pp(a):
        return None if a is None else _p(a)
    out["fails"] = lib().oracle_safe_step_ex(m, K, _p(hz), float(gamma_b), B, _p(x), _p(aux), _p(step), _p(u),
                                             pp(mu), pp(sg), _p(out["u"]), _p(out["reward"]), _p(out["cost"]),
                                             _p(out["done"]), _p(out["goal"]), _p(out["obs"]), int(auto_reset),
                                             pp(nz), pp(ea), int(threads))
    return out


def max_threads():
    return lib().oracle_max_threads()


def cars_cascade_loop(noise, steps=300, gamma_b=20.0):
    """BASELINE config 1 (envs/simulated_cars_env.py:161-228): the hand
    controller + CascadeCBFLayer.get_u_safe + env.step closed loop of one
    SimulatedCars env from reset with velocity noise `noise`, in C (one
    thread).  Returns (u_nom (steps,), u_safe (steps,), states (steps+1, 10))."""
    un, us = np.zeros(steps), np.zeros(steps)
    xs = np.zeros((steps + 1, 10))
    rc = lib().oracle_cars_cascade_loop(float(noise), int(steps), float(gamma_b), _p(un), _p(us), _p(xs))
    if rc:
        raise RuntimeError(f"oracle_cars_cascade_loop: no QP solution at step {rc - 1}")
    return un, us, xs
