"""Model-rollout step (rcbf_model_step) and DynamicsModel.predict_next_state
(rcbf_predict_next_state) at B = 65 536, hipGraph-timed
(20 calls per graph, best of 3 replays, HIP events): cars and unicycle, with
the MAX_STD prior and with per-row GP mean / std (f32).  `GBs` = the
algorithmic bytes (rows read and written once) / time.
Usage: python scripts/model_step_bench.py   (RCBF_HIP_LIB=<variant.so> for an A/B)"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sac-rcbf_amd")]
import torch  # noqa: E402

from rcbf_amd import _lib  # noqa: E402
from rcbf_amd.envs import BatchedSimulatedCarsEnv, BatchedUnicycleEnv  # noqa: E402
from rcbf_amd.params import make_params  # noqa: E402


def time_graph(fn, reps=20):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        assert fn() == 0
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = None
    for _ in range(3):
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / reps
        best = us if best is None else min(best, us)
    return best


def main():
    lib = _lib.load()
    dev = torch.device("cuda")
    B = 65536
    out = {}
    for name, env in (("cars", BatchedSimulatedCarsEnv(4, device=dev)), ("uni", BatchedUnicycleEnv(4, device=dev))):
        prm = make_params(env, 1.0)
        n_s, n_o, n_u = (10, 10, 1) if name == "cars" else (3, 7, 2)
        g = torch.Generator(device=dev)
        g.manual_seed(0)
        obs = torch.rand(B, n_o, dtype=torch.float64, device=dev, generator=g) + 0.1
        act = torch.rand(B, n_u, dtype=torch.float64, device=dev, generator=g)
        t = torch.rand(B, dtype=torch.float64, device=dev, generator=g)
        mean = torch.rand(B, n_s, dtype=torch.float32, device=dev, generator=g) * 0.1
        std = torch.rand(B, n_s, dtype=torch.float32, device=dev, generator=g) * 0.2
        nobs = torch.empty_like(obs)
        r, m, nt = (torch.empty(B, dtype=torch.float64, device=dev) for _ in range(3))
        nx, so = torch.empty(B, n_s, dtype=torch.float64, device=dev), torch.empty(B, n_s, dtype=torch.float64,
                                                                                   device=dev)
        for gp_rows in (False, True):
            mp, sp = (_lib.ptr(mean), _lib.ptr(std)) if gp_rows else (None, None)
            us = time_graph(lambda: lib.rcbf_model_step(ctypes.byref(prm), B, _lib.ptr(obs), _lib.ptr(act),
                                                        _lib.ptr(t), mp, sp, None, 1, 0, _lib.ptr(nobs), _lib.ptr(r),
                                                        _lib.ptr(m), _lib.ptr(nt), _lib.stream_of(dev)))
            nbytes = B * (8 * (2 * n_o + n_u + 1 + 3) + (8 * n_s if gp_rows else 0))
            key = f"model_step_{name}{'_gp' if gp_rows else ''}"
            out[key] = {"us": round(us, 2), "GBs": round(nbytes / us / 1e3, 1)}
            print(key, out[key], flush=True)
        x = obs[:, :n_s].contiguous()
        us = time_graph(lambda: lib.rcbf_predict_next_state(ctypes.byref(prm), B, _lib.ptr(x), _lib.ptr(act),
                                                            _lib.ptr(t), _lib.ptr(mean), _lib.ptr(std), 1,
                                                            _lib.ptr(nx), _lib.ptr(so), _lib.ptr(nt), _lib.stream_of(dev)))
        nbytes = B * (8 * (3 * n_s + n_u + 2) + 8 * n_s)
        out[f"predict_next_state_{name}_gp"] = {"us": round(us, 2), "GBs": round(nbytes / us / 1e3, 1)}
        print(f"predict_next_state_{name}_gp", out[f"predict_next_state_{name}_gp"], flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
