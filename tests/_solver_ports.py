"""numpy restatements of the two closed-form QP solvers the HIP kernels use
(sac-rcbf_amd/csrc/rcbf_device.hpp: cars_qp_1d, uni_qp_2d), vectorised over
the batch.  Test infrastructure only: they let the CPU suite check the solver
*algorithm* against oracle.qp_exact (the KKT enumeration that stands in for
qpth / quadprog, diff_cbf_qp.py:136, cbf_qp.py:231) on many random states
without a GPU.  The GPU kernels themselves are checked in test_gpu_parity.py.

Both exploit the structure of the CBF-QP: the slack variable eps (weight
P[-1,-1]) only appears in the CBF rows  G_j[:n_u] u - eps <= h_j  (G_j[-1]<0
after normalisation), so for fixed u the optimal eps is
max(0, max_j (a_j.u + b_j)), and the QP reduces to minimising the convex
piecewise quadratic  phi(u) = sum p_k u_k^2 + p_eps max(0, a_j.u + b_j)^2
over the box  u_min - u_rl <= u <= u_max - u_rl.
"""
import itertools

import numpy as np


def cars_qp_1d(Gn, hn, pd):
    """SimulatedCars diff QP: variables (u, eps), rows [cbf0, cbf1, u<=U, -u<=-L].
    The minimiser of the 1-D convex phi over [L, U] is the clamp of one of
    {0, stationary point of each piece, kink}; take the best.  Rows are
    (B,4,2) f32 after normalize_rows, pd = diag(P) in f64."""
    G = Gn.astype(np.float64)
    h = hn.astype(np.float64)
    p0, p1 = pd
    U = h[:, 2] / G[:, 2, 0]
    L = h[:, 3] / G[:, 3, 0]
    i0 = 1 / G[:, 0, 1]
    i1 = 1 / G[:, 1, 1]
    a0, b0 = -G[:, 0, 0] * i0, h[:, 0] * i0
    a1, b1 = -G[:, 1, 0] * i1, h[:, 1] * i1
    c1 = -(p1 * a0 * b0) / (p1 * a0 * a0 + p0)
    c2 = -(p1 * a1 * b1) / (p1 * a1 * a1 + p0)
    den = a0 - a1
    c3 = np.where(den != 0, (b1 - b0) / np.where(den != 0, den, 1), 0)

    def cl(u):
        return np.minimum(np.maximum(u, L), U)

    def eps(u):
        return np.maximum(0, np.maximum(a0 * u + b0, a1 * u + b1))

    def phi(u):
        return p0 * u * u + p1 * eps(u) ** 2

    C = np.stack([cl(np.zeros_like(U)), cl(c1), cl(c2), cl(c3)], 1)
    f = np.stack([phi(C[:, k]) for k in range(4)], 1)
    u = C[np.arange(len(U)), f.argmin(1)]
    return np.stack([u, eps(u)], 1)


def uni_qp_2d(Gn, hn, pd, K, prune=True, wave=64, stats=None):
    """Unicycle QP: variables (u0, u1, eps), rows [K cbf rows, 4 box rows].
    Pruning (as the kernel): per lane, only the rows whose a_j.u + b_j can
    exceed 0 somewhere in the box are kept, compacted into slots (unused
    slots repeat slot 0); lanes are grouped in waves of `wave` and each wave
    solves with KK = its largest live count (KK = 0: the clamped origin).
    Returns ((B,3) z, in-box mask of the stage-1 point, KK per lane); `stats`
    (a dict) receives per-lane `open` (no certificate after the pieces:
    the lane's wave runs the kink / triple stage)."""
    G = Gn.astype(np.float64)
    h = hn.astype(np.float64)
    B = G.shape[0]
    inv = 1 / G[:, :K, 2]
    a0 = -G[:, :K, 0] * inv
    a1 = -G[:, :K, 1] * inv
    b = h[:, :K] * inv
    U0 = h[:, K] / G[:, K, 0]
    L0 = h[:, K + 1] / G[:, K + 1, 0]
    U1 = h[:, K + 2] / G[:, K + 2, 1]
    L1 = h[:, K + 3] / G[:, K + 3, 1]
    if not prune:
        z, inb, opn = _pieces_solve(a0, a1, b, L0, U0, L1, U1, pd, stats)
        if stats is not None:
            stats["open"] = opn
        return _with_eps(z, a0, a1, b), inb, np.full(B, K)
    emax = b + np.maximum(a0 * L0[:, None], a0 * U0[:, None]) + np.maximum(a1 * L1[:, None], a1 * U1[:, None])
    live = ~(emax <= 0)
    cnt = live.sum(1)
    A0, A1, Bv = (np.repeat(v[:, :1], K, 1) for v in (a0, a1, b))
    pos = np.cumsum(live, 1) - 1
    for j in range(K):
        sel = live[:, j]
        r = np.nonzero(sel)[0]
        A0[r, pos[r, j]], A1[r, pos[r, j]], Bv[r, pos[r, j]] = a0[r, j], a1[r, j], b[r, j]
    for sl in range(1, K):
        unused = sl >= cnt
        A0[unused, sl], A1[unused, sl], Bv[unused, sl] = A0[unused, 0], A1[unused, 0], Bv[unused, 0]
    nw = (B + wave - 1) // wave
    kk = np.zeros(nw * wave, int)
    kk[:B] = cnt
    kk = np.repeat(kk.reshape(nw, wave).max(1), wave)[:B]
    z = np.zeros((B, 2))
    inb = np.ones(B, bool)
    opn = np.zeros(B, bool)
    st = {k: np.zeros(B, bool) for k in ("need_u0_edge", "need_u1_edge", "edge_open")}
    for KK in range(K + 1):
        r = np.nonzero(kk == KK)[0]
        if r.size == 0:
            continue
        if KK == 0:
            z[r, 0] = np.minimum(np.maximum(0.0, L0[r]), U0[r])
            z[r, 1] = np.minimum(np.maximum(0.0, L1[r]), U1[r])
            continue
        sr = {}
        zr, ir, orr = _pieces_solve(A0[r, :KK], A1[r, :KK], Bv[r, :KK], L0[r], U0[r], L1[r], U1[r], pd, sr)
        z[r], inb[r], opn[r] = zr, ir, orr
        for k in st:
            st[k][r] = sr[k]
    if stats is not None:
        stats["open"] = opn
        stats.update(st)
    return _with_eps(z, a0, a1, b), inb, kk


def _with_eps(z, a0, a1, b):
    e = np.maximum(0, (a0 * z[:, :1] + a1 * z[:, 1:2] + b).max(1))
    return np.concatenate([z, e[:, None]], 1)


def _pieces_solve(a0, a1, b, L0, U0, L1, U1, pd, stats=None):
    """Stage 1 + stage 2 of the kernel's uni_pieces_solve on K pieces.  A
    lane whose origin (every b_j <= 0) or piece stationary point u_j (e_j(u_j)
    > 0 and piece j attains the max there) is certified takes that point (the
    first certified one); the others take the argmin over all candidates.
    Returns (z, in-box mask, open mask)."""
    p0, p1, p2 = pd
    B, K = a0.shape

    def eps(u0, u1):
        return np.maximum(0, (a0 * u0[:, None] + a1 * u1[:, None] + b).max(1))

    def phi(u0, u1):
        e = eps(u0, u1)
        return p0 * u0 * u0 + p1 * u1 * u1 + p2 * e * e

    C = [(np.zeros(B), np.zeros(B))]
    cert_k = np.where((b <= 0).all(1), 0, -1)  # index into C of the certified candidate, -1: none
    for j in range(K):
        w0 = a0[:, j] / p0
        w1 = a1[:, j] / p1
        s = 1 + p2 * (a0[:, j] * w0 + a1[:, j] * w1)
        f = -p2 * b[:, j] / s
        C.append((f * w0, f * w1))
        ej = a0[:, j] * C[-1][0] + a1[:, j] * C[-1][1] + b[:, j]
        cj = (ej > 0) & (ej >= eps(*C[-1]))
        cert_k = np.where((cert_k < 0) & cj, len(C) - 1, cert_k)
    for i in range(K):
        for j in range(i + 1, K):
            d0 = a0[:, i] - a0[:, j]
            d1 = a1[:, i] - a1[:, j]
            c = b[:, j] - b[:, i]
            dd = d0 * d0 + d1 * d1
            ok = dd > 1e-300
            dd = np.where(ok, dd, 1)
            q0, q1 = c * d0 / dd, c * d1 / dd
            n0, n1 = -d1, d0
            ea = a0[:, i] * q0 + a1[:, i] * q1 + b[:, i]
            an = a0[:, i] * n0 + a1[:, i] * n1
            num = p0 * q0 * n0 + p1 * q1 * n1 + p2 * ea * an
            den = p0 * n0 * n0 + p1 * n1 * n1 + p2 * an * an
            t = -num / np.where(den != 0, den, 1)
            C.append((np.where(ok, q0 + t * n0, 0), np.where(ok, q1 + t * n1, 0)))
    for i, j, l in itertools.combinations(range(K), 3):
        m00 = a0[:, i] - a0[:, j]
        m01 = a1[:, i] - a1[:, j]
        r0 = b[:, j] - b[:, i]
        m10 = a0[:, i] - a0[:, l]
        m11 = a1[:, i] - a1[:, l]
        r1 = b[:, l] - b[:, i]
        det = m00 * m11 - m01 * m10
        ok = np.abs(det) > 1e-300
        det = np.where(ok, det, 1)
        C.append((np.where(ok, (r0 * m11 - r1 * m01) / det, 0), np.where(ok, (m00 * r1 - m10 * r0) / det, 0)))
    Fv = np.stack([phi(u0, u1) for u0, u1 in C], 1)
    k = np.where(cert_k >= 0, cert_k, np.nanargmin(Fv, 1))
    U0s = np.stack([c[0] for c in C], 1)[np.arange(B), k]
    U1s = np.stack([c[1] for c in C], 1)[np.arange(B), k]
    inb = (U0s >= L0) & (U0s <= U0) & (U1s >= L1) & (U1s <= U1)
    # stage 2: the facing edges of the out-of-box lanes -- the u0-edge (u0 fixed
    # at clamp(u_f0)) only where u_f0 leaves [L0, U0], the u1-edge only where
    # u_f1 leaves [L1, U1]; on each edge the origin / piece certificates as in
    # stage 1, else the argmin over the edge's candidates
    best = np.full(B, np.inf)
    bu0, bu1 = U0s.copy(), U1s.copy()
    v0 = np.minimum(np.maximum(U0s, L0), U0)
    v1 = np.minimum(np.maximum(U1s, L1), U1)
    need = [(U0s < L0) | (U0s > U0), (U1s < L1) | (U1s > U1)]
    edge_open = np.zeros(B, bool)
    for fix0, v, lo, hi, nd in [(True, v0, L1, U1, need[0]), (False, v1, L0, U0, need[1])]:
        al = a1 if fix0 else a0
        be = (a0 * v[:, None] + b) if fix0 else (a1 * v[:, None] + b)
        pf = p1 if fix0 else p0
        ys = [np.zeros(B)] + [-(p2 * al[:, j] * be[:, j]) / (p2 * al[:, j] ** 2 + pf) for j in range(K)]
        ecert = np.where((be <= 0).all(1), 0, -1)
        for j in range(K):
            ej = al[:, j] * ys[j + 1] + be[:, j]
            em = np.maximum(0, (al * ys[j + 1][:, None] + be).max(1))
            ecert = np.where((ecert < 0) & (ej > 0) & (ej >= em), j + 1, ecert)
        for i in range(K):
            for j in range(i + 1, K):
                den = al[:, i] - al[:, j]
                ys.append(np.where(den != 0, (be[:, j] - be[:, i]) / np.where(den != 0, den, 1), 0))
        edge_open |= nd & (ecert < 0)
        Y = np.stack([np.minimum(np.maximum(y, lo), hi) for y in ys], 1)
        Fe = np.stack([phi(v, Y[:, k]) if fix0 else phi(Y[:, k], v) for k in range(Y.shape[1])], 1)
        ke = np.where(ecert >= 0, ecert, np.nanargmin(np.where(np.isnan(Fe), np.inf, Fe), 1))
        y = Y[np.arange(B), ke]
        f = Fe[np.arange(B), ke]
        u0 = v if fix0 else y
        u1 = y if fix0 else v
        t = nd & (f < best)
        best = np.where(t, f, best)
        bu0 = np.where(t, u0, bu0)
        bu1 = np.where(t, u1, bu1)
    if stats is not None:
        stats["need_u0_edge"], stats["need_u1_edge"], stats["edge_open"] = need[0], need[1], edge_open
    return np.stack([bu0, bu1], 1), inb, cert_k < 0
