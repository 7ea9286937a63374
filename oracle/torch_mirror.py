"""CPU BASELINE MIRROR of the reference's own CPU mode -- TEST / BENCH
INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg and tests/ import it; the
product path never does).

The reference runs the safety layer on the CPU when `--cuda` is off: the
batched fp32 constraint builder (rcbf_sac/diff_cbf_qp.py:146-379, restated
by oracle.cars_build_diff / unicycle_build_diff), the row normaliser
(:103-106), qpth's batched primal-dual interior-point solve in fp64 (:139,
solver args eps = 1e-4, notImprovedLim = 10 from :107), the clamp (:77) and
the numpy env step.  qpth is not installed here, so its PDIPM is
restated from its published algorithm (OptNet, Amos & Kolter 2017; qpth
solvers/pdipm/batch.py): Mehrotra predictor-corrector on the KKT system,
initial point from one KKT solve with d = 1 shifted to s, z >= 1, 0.999 step
to the boundary, sigma = (mu_aff / mu)^3, batch-global stop (all residuals <
eps, or notImprovedLim iterations without any element improving) returning
each element's best iterate (also when a KKT factorisation fails).  The KKT
solves use the n x n normal equations (P + G' D G) dx = -rx + G' rs - G' D rz,
as torch batched solves.
"""
import numpy as np
import torch

from . import oracle as O


def _step(v, dv):
    """Largest a <= 1 with v + a dv >= 0, per batch element (qpth get_step)."""
    a = torch.where(dv < -1e-300, -v / torch.where(dv < -1e-300, dv, torch.ones_like(dv)), torch.full_like(v, np.inf))
    return torch.clamp(a.min(dim=1).values, max=1.0)


def _solve_kkt(P, G, d, rx, rs, rz):
    GtD = G.transpose(1, 2) * d[:, None, :]
    H = P + GtD @ G
    rhs = -rx + (G.transpose(1, 2) @ rs[..., None])[..., 0] - (GtD @ rz[..., None])[..., 0]
    dx, info = torch.linalg.solve_ex(H, rhs)
    ds = -rz - (G @ dx[..., None])[..., 0]
    dz = -rs - d * ds
    return dx, ds, dz, bool((info != 0).any())


def pdipm(P, q, G, h, eps=1e-4, not_improved_lim=10, max_iter=100):
    """Batched qpth-style PDIPM (fp64).  P (B,n,n), q (B,n), G (B,m,n),
    h (B,m) -> (z (B,n), iterations)."""
    B, m, n = G.shape
    d = torch.ones(B, m, dtype=G.dtype)
    x, s, z, _ = _solve_kkt(P, G, d, q, torch.zeros(B, m, dtype=G.dtype), -h)
    ms = s.min(dim=1, keepdim=True).values
    s = torch.where(ms < 0, s - ms + 1, s)
    mz = z.min(dim=1, keepdim=True).values
    z = torch.where(mz < 0, z - mz + 1, z)
    best_r, best_x = None, x.clone()
    n_not = 0
    it = 0
    for it in range(max_iter):
        rx = (G.transpose(1, 2) @ z[..., None])[..., 0] + (P @ x[..., None])[..., 0] + q
        rs = z
        rz = (G @ x[..., None])[..., 0] + s - h
        mu = (s * z).sum(1).abs() / m
        resid = rz.norm(dim=1) + rx.norm(dim=1) + m * mu
        if best_r is None:
            best_r, best_x = resid.clone(), x.clone()
        else:
            imp = resid < best_r
            n_not = 0 if bool(imp.any()) else n_not + 1
            best_r = torch.where(imp, resid, best_r)
            best_x = torch.where(imp[:, None], x, best_x)
        if n_not == not_improved_lim or float(best_r.max()) < eps:
            break
        d = z / s
        dx_a, ds_a, dz_a, bad = _solve_kkt(P, G, d, rx, rs, rz)
        if bad:  # qpth returns the best iterates when a KKT factorisation fails
            break
        a = torch.minimum(_step(z, dz_a), _step(s, ds_a))[:, None]
        sig = (((s + a * ds_a) * (z + a * dz_a)).sum(1) / (s * z).sum(1)) ** 3
        rs_c = ((-mu * sig)[:, None] + ds_a * dz_a) / s
        zero_n, zero_m = torch.zeros_like(rx), torch.zeros_like(rz)
        dx_c, ds_c, dz_c, bad = _solve_kkt(P, G, d, zero_n, rs_c, zero_m)
        if bad:
            break
        dx, ds, dz = dx_a + dx_c, ds_a + ds_c, dz_a + dz_c
        a = torch.clamp(0.999 * torch.minimum(_step(s, ds), _step(z, dz)), max=1.0)[:, None]
        x, s, z = x + a * dx, s + a * ds, z + a * dz
    return best_x, it + 1


def cars_safe_step(x, t, step, u_rl, gamma_b):
    """One reference-CPU-mode safe step of B SimulatedCars envs: get_state
    from the fp32 obs, prior mean/sigma, fp32 rows, normaliser, PDIPM (fp64),
    clamp, numpy env step.  Returns (x, t, step, u_safe, iterations)."""
    B = x.shape[0]
    s32 = O.get_state_f32("SimulatedCars", O.cars_obs(x).astype(np.float32))
    mu = np.zeros((B, 10), np.float32)
    sg = np.tile(np.asarray(O.MAX_STD["SimulatedCars"], np.float32), (B, 1))
    P, q, G, h = O.cars_build_diff(s32, u_rl, mu, sg, gamma_b)
    Gn, hn, _ = O.normalize_rows(G, h)
    z, its = pdipm(torch.from_numpy(P.astype(np.float64)), torch.from_numpy(q.astype(np.float64)),
                   torch.from_numpy(Gn.astype(np.float64)), torch.from_numpy(hn.astype(np.float64)))
    u = np.clip(u_rl + z[:, :1].numpy().astype(np.float32), np.float32(-10.0), np.float32(10.0))
    x2, t2, st2, _, _, _, _ = O.cars_step(x, t, step, u)
    return x2, t2, st2, u, its


def uni_safe_step(x, last_dist, step, u_rl, gamma_b, hazards):
    """The same for B Unicycle envs (prior sigma 0.2, rows of
    diff_cbf_qp.py:202-266).  Returns (x, last_dist, step, u_safe, iterations)."""
    B = x.shape[0]
    s32 = O.get_state_f32("Unicycle", O.uni_obs(x).astype(np.float32))
    mu = np.zeros((B, 3), np.float32)
    sg = np.full((B, 3), 0.2, np.float32)
    P, q, G, h = O.unicycle_build_diff(s32, u_rl, mu, sg, gamma_b, hazards)
    Gn, hn, _ = O.normalize_rows(G, h)
    z, its = pdipm(torch.from_numpy(P.astype(np.float64)), torch.from_numpy(q.astype(np.float64)),
                   torch.from_numpy(Gn.astype(np.float64)), torch.from_numpy(hn.astype(np.float64)))
    u = np.clip(u_rl + z[:, :2].numpy().astype(np.float32), np.float32(-2.5), np.float32(2.5))
    x2, ld2, st2 = O.uni_step(x, last_dist, step, u, hazards=hazards)[:3]
    return x2, ld2, st2, u, its
