"""Diagnostic: PDIPM vs the exact solver on SURVEY 8(d) unicycle states
(status histogram, max |u_pdipm - u_exact|)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sac-rcbf_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import oracle as O  # noqa: E402
from rcbf_amd import _lib  # noqa: E402
from rcbf_amd.diff_cbf_qp import CBFQPLayer  # noqa: E402
from rcbf_amd.envs import BatchedUnicycleEnv, BatchedSimulatedCarsEnv  # noqa: E402


class A:
    cuda = True


rng = np.random.default_rng(0)
B = 65536
for mode in ("Unicycle", "SimulatedCars"):
    if mode == "Unicycle":
        hz = O.UNI["hazards"][:3]
        env = BatchedUnicycleEnv(4, hazards_locations=hz)
        x = np.stack([rng.uniform(-3, 3, B), rng.uniform(-3, 3, B), rng.uniform(-np.pi, np.pi, B)], 1)
        s32 = O.get_state_f32(mode, O.uni_obs(x).astype(np.float32))
        mu, sg = np.zeros((B, 3), np.float32), np.full((B, 3), 0.2, np.float32)
    else:
        env = BatchedSimulatedCarsEnv(4)
        xs, t, st = O.cars_reset(rng.normal(0, 0.5, B))
        n = rng.integers(0, 300, B)
        for k in range(300):
            a = rng.uniform(-1, 1, (B, 1)).astype(np.float32)
            live = k < n
            x2, t2, st2, *_ = O.cars_step(xs, t, st, a)
            xs[live], t[live], st[live] = x2[live], t2[live], st2[live]
        s32 = O.get_state_f32(mode, O.cars_obs(xs).astype(np.float32))
        m, sgd = O.predict_disturbance_prior(mode, B)
        mu, sg = m.astype(np.float32), sgd.astype(np.float32)
    u = rng.uniform(-1, 1, (B, env.n_u)).astype(np.float32)
    res = {}
    for solver in (0, 1):
        layer = CBFQPLayer(env, A(), gamma_b=20.0, solver=solver)
        X, U, M, S = (torch.as_tensor(v, device="cuda") for v in (s32, u, mu, sg))
        out = torch.empty_like(U)
        st_ = torch.zeros(B, dtype=torch.int32, device="cuda")
        fl = torch.zeros(1, dtype=torch.int32, device="cuda")
        rc = _lib.load().rcbf_safe_action(ctypes.byref(layer._prm), B, _lib.ptr(X), _lib.ptr(U), _lib.ptr(M),
                                          _lib.ptr(S), _lib.ptr(out), _lib.ptr(st_), _lib.ptr(fl),
                                          _lib.stream_of(torch.device("cuda")))
        torch.cuda.synchronize()
        res[solver] = (out.cpu().numpy(), np.bincount(st_.cpu().numpy(), minlength=4), int(fl.item()))
    d = np.abs(res[0][0] - res[1][0]).max(1)
    print(mode, "status exact", res[0][1], "pdipm", res[1][1], "flag bits", res[0][2], res[1][2],
          "max |du|", d.max(), "p99.9", np.quantile(d, 0.999), "n>1e-3", int((d > 1e-3).sum()))
    bad = np.nonzero(d > 1e-3)[0]
    if len(bad):
        np.savez(os.path.join(ROOT, "gpurun_out", f"pdipm_bad_{mode}.npz"), x=s32[bad], u=u[bad], mu=mu[bad],
                 sg=sg[bad], z_exact=res[0][0][bad], z_pdipm=res[1][0][bad])
