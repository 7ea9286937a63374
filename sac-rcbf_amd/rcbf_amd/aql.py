"""The fused safe step on the library's own AQL queue (csrc/rcbf_aql.hip).

`AqlQueue(device)` owns one user-mode HSA queue on a HIP device and the
code object the HIP path launches the fused step from (librcbf_steps.co,
identical machine code).  `AqlQueue.safe_step_plan(env, u_rl_seq, layer, ...)`
is the AQL analogue of capturing K `BatchedEnv.safe_step` calls into a
hipGraph: the K kernel-argument blocks go to device memory once, the K
dispatch packets are pre-built, and `plan.run()` submits them with one
doorbell and returns when the K steps have completed -- a synchronous
env.step() (main.py:93-95, sac_cbf.py:218-238) of K steps.

The queue is not a HIP stream: `run()` first waits for all HIP work queued
on the env's device unless `sync_hip=False` is
passed by a caller that has synchronised itself (bench.py's timed region
follows torch.cuda.synchronize()).
"""
import ctypes
import weakref

import torch

from . import _lib

PROFILE = 1  # RCBF_AQL_PROFILE
PROFILE_ENDS = 64  # RCBF_AQL_PROFILE_ENDS: timestamps of the first and last dispatch only


def _bind():
    return _lib.load()


def _check(rc, what):
    _lib.check(rc, what)


class AqlQueue:
    """One AQL queue on HIP device `device` (int or torch.device)."""

    def __init__(self, device=None, profile=False, code_object=None):
        lib = _bind()
        dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        if dev.type != "cuda":
            raise ValueError("AqlQueue needs a HIP device")
        self.device = torch.device("cuda", dev.index if dev.index is not None else torch.cuda.current_device())
        self.profile = bool(profile)
        h = ctypes.c_void_p()
        _check(lib.rcbf_aql_open(self.device.index, code_object.encode() if code_object else None,
                                 PROFILE if profile else 0, ctypes.byref(h)), "rcbf_aql_open")
        self._h = h
        self._plans = weakref.WeakSet()  # live plans: freed before the queue (they point into it)
        self._fin = weakref.finalize(self, lib.rcbf_aql_close, h)

    @property
    def handle(self):
        if not self._fin.alive:
            raise RuntimeError("the AQL queue is closed")
        return self._h

    def kernel_count(self):
        return int(_lib.load().rcbf_aql_kernel_count(self.handle))

    def close(self):
        for p in list(self._plans):
            p.free()
        self._fin()

    def safe_step_plan(self, env, u_rl_seq, layer, steps=None, mean=None, sigma=None, outputs=None,
                       auto_reset=True, prior_layout="rows", span=None, profile=False, fence_flags=0):
        """K = steps (default len(u_rl_seq)) fused safe steps of `env` with
        `layer`, step j reading u_rl_seq[j % len(u_rl_seq)]: the same
        arguments and results as env.safe_step_seq (span: the measurement
        instantiation of env.safe_step_span, step j stamping span[j])."""
        if env.device != self.device:
            raise ValueError(f"env on {env.device}, queue on {self.device}")
        o = outputs if outputs is not None else env.make_outputs()
        us = [env._u_arg(u) for u in u_rl_seq]
        if not us:
            raise ValueError("u_rl_seq is empty")
        K = len(us) if steps is None else int(steps)
        if prior_layout not in ("rows", "cols"):
            raise ValueError(f"prior_layout must be 'rows' or 'cols', got {prior_layout!r}")
        cols = prior_layout == "cols"
        if cols:
            if mean is not None and env.dynamics_mode == "SimulatedCars":
                raise ValueError("the cars CBF rows read no mean (diff_cbf_qp.py:298-299): pass mean=None")
            mean, sigma = env._prior_cols_arg(mean, "mean"), env._prior_cols_arg(sigma, "sigma")
        else:
            mean, sigma = env._prior_arg(mean, "mean"), env._prior_arg(sigma, "sigma")
        if span is not None:
            nw = (env.num_envs + 63) // 64
            if not (torch.is_tensor(span) and span.dtype == torch.int64 and span.device == env.device
                    and span.is_contiguous() and span.numel() >= 4 * nw * K):
                raise ValueError(f"span must be a contiguous int64 tensor of >= {4 * nw * K} entries "
                                 f"(K blocks of ceil(B / 64) x 4) on {env.device}")
        a = env._step_args(layer, o, auto_reset)
        arr = (ctypes.c_void_p * len(us))(*[u.data_ptr() for u in us])
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _check(_lib.load().rcbf_aql_safe_step_plan(
                self.handle, ctypes.byref(layer._prm), env.num_envs, K, *[v or None for v in a[2:6]], arr, len(us),
                None if mean is None else mean.data_ptr(), None if sigma is None else sigma.data_ptr(), int(cols),
                *[v or None for v in a[9:17]], *a[17:20], None if span is None else span.data_ptr(),
                (PROFILE if profile else 0) | int(fence_flags), ctypes.byref(h)), "rcbf_aql_safe_step_plan")
        # the plan holds raw pointers: keep every tensor it reads or writes alive with it
        keep = (env, layer, o, us, mean, sigma, span)
        plan = AqlPlan(self, h, K, keep, bool(profile), env)
        self._plans.add(plan)
        return plan


class AqlPlan:
    """K pre-built dispatches of the fused step (see AqlQueue.safe_step_plan)."""

    def __init__(self, queue, handle, K, keep, profiled, env):
        self.queue, self.K, self.profiled = queue, K, profiled
        self._h, self._keep, self._env = handle, keep, env
        self._fin = weakref.finalize(self, _lib.load().rcbf_aql_plan_free, handle)

    def run(self, sync_hip=True, timeout_us=0):
        """Submit the K steps and return when they have completed."""
        if sync_hip:
            torch.cuda.synchronize(self.queue.device)
        if not self._fin.alive or not self.queue._fin.alive:
            raise RuntimeError("the AQL plan (or its queue) was freed")
        # ctypes, not the CPython binding: a 20-step run measured the same through both (85.1 / 85.5 us, r06w)
        _check(_lib.load().rcbf_aql_run(self._h, timeout_us), "rcbf_aql_run")
        return self._env.obs, self._keep[2]["reward"], self._keep[2]["done"], self._keep[2]

    def times_ns(self):
        """(K, 2) int64 numpy array: each dispatch's start and end (ns, HSA
        system clock) from the last run; profiled plans only."""
        import numpy as np
        if not self._fin.alive or not self.queue._fin.alive:
            raise RuntimeError("the AQL plan (or its queue) was freed")
        out = np.zeros((self.K, 2), dtype=np.uint64)
        _check(_lib.load().rcbf_aql_plan_times(self._h, out.ctypes.data), "rcbf_aql_plan_times")
        return out.astype(np.int64)

    def free(self):
        self._fin()
