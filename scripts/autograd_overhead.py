"""Break down the host time of the SAC-update safe action under autograd
(rcbf_amd.sac_cbf.get_safe_action forward + backward, bench.py --extra
'autograd_us'): each stage timed over 200 calls, microseconds per call."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "sac-rcbf_amd")):
    sys.path.insert(0, p)

import ctypes  # noqa: E402

import torch  # noqa: E402


def us(fn, n=200):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return round((time.perf_counter() - t0) * 1e6 / n, 1)


def main():
    from rcbf_amd import _lib
    from rcbf_amd.diff_cbf_qp import CBFQPLayer
    from rcbf_amd.dynamics import DynamicsModel
    from rcbf_amd.envs import BatchedSimulatedCarsEnv
    from rcbf_amd.sac_cbf import get_safe_action

    class A:
        cuda = True

    B = 256
    env = BatchedSimulatedCarsEnv(B)
    layer = CBFQPLayer(env, A(), gamma_b=20.0)
    dyn = DynamicsModel(env, A())
    obs = env.obs.clone()
    u = torch.rand(B, 1, device="cuda") * 2 - 1
    w = torch.randn(B, 1, device="cuda")
    lib = _lib.load()
    out = torch.empty_like(u)
    flag = torch.zeros(1, dtype=torch.int32, device="cuda")
    s = _lib.stream_of(torch.device("cuda", 0))
    r = {}
    r["raw_launch"] = us(lambda: lib.rcbf_obs_safe_action(ctypes.byref(layer._prm), B, _lib.ptr(obs), _lib.ptr(u),
                                                          None, None, _lib.ptr(out), None, _lib.ptr(flag), s))
    r["raw_launch_and_flag_read"] = us(lambda: (lib.rcbf_obs_safe_action(
        ctypes.byref(layer._prm), B, _lib.ptr(obs), _lib.ptr(u), None, None, _lib.ptr(out), None, _lib.ptr(flag),
        s), flag.item()))
    r["stream_of"] = us(lambda: _lib.stream_of(torch.device("cuda", 0)))
    r["fwd_no_grad"] = us(lambda: get_safe_action(layer, obs, u, dyn))
    uu = u.clone().requires_grad_(True)
    r["fwd_requires_grad"] = us(lambda: get_safe_action(layer, obs, uu, dyn))

    def fwd_loss():
        return (get_safe_action(layer, obs, uu, dyn) * w).sum()
    r["fwd_plus_loss"] = us(fwd_loss)

    def full():
        uu.grad = None
        fwd_loss().backward()
    r["fwd_loss_backward"] = us(full)

    def torch_only():
        uu.grad = None
        (uu * 2.0 * w).sum().backward()
    r["torch_only_mul_sum_backward"] = us(torch_only)

    def torch_only_clamp():
        uu.grad = None
        (torch.clamp(uu + 0.1, -10, 10) * w).sum().backward()
    r["torch_only_clamp_mul_sum_backward"] = us(torch_only_clamp)
    gu = torch.empty_like(u)
    r["raw_backward_launch"] = us(lambda: lib.rcbf_obs_safe_action_backward(
        ctypes.byref(layer._prm), B, _lib.ptr(obs), _lib.ptr(u), None, None, _lib.ptr(w), _lib.ptr(gu), s))
    layer.check_failures = False
    r["full_without_nan_check"] = us(full)
    layer.check_failures = True
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
