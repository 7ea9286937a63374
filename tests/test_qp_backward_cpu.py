"""CPU checks of the generic QP backward oracle (oracle.qp_backward), the
checker of rcbf_qp_backward (CBFQPLayer.cbf_layer / solve_qp under autograd,
rcbf_sac/diff_cbf_qp.py:81-144):

  * central finite differences of the exact fp64 QP (with and without the
    row normaliser) match its P, q, G, h gradients: <= 1e-5 relative;
  * composed with the closed-form dh/du of the CBF rows, its h gradient
    reproduces the reference-run golden d final / d u_RL (tests/golden,
    cars and unicycle k = 3, 5): <= 1e-5 relative, the bar of the
    safe-action gradient checks in test_oracle_golden.py.

qpth itself is not installed: against qpth's own backward this
is parity-unpinned; the pin is the implicit-function derivative it
approximates (FD) and the reference's own gradient fixtures.
"""
import numpy as np
import pytest

from oracle import oracle as O


def rel(a, b):
    a = np.asarray(a, np.float64); b = np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b) / np.maximum(1.0, np.abs(b)))) if a.size else 0.0


def random_qps(rng, B, n, m):
    """Feasible strictly convex QPs with a mix of active sets: full SPD P, q
    and rows through a strictly feasible point z0 (h = G z0 + slack), with the
    unconstrained minimiser often outside."""
    A = rng.normal(0, 1, (B, n, n))
    P = (A @ np.swapaxes(A, 1, 2) + n * np.eye(n)).astype(np.float32).astype(np.float64)
    q = rng.normal(0, 1, (B, n)).astype(np.float32)
    G = rng.normal(0, 1, (B, m, n)).astype(np.float32)
    z0 = rng.normal(0, 0.3, (B, n))
    h = (np.einsum("bmn,bn->bm", G, z0) + np.abs(rng.normal(0, 0.5, (B, m)))).astype(np.float32)
    return P, q, G, h


def _loss(P, q, G, h, w, normalize):
    G = np.asarray(G, np.float64); h = np.asarray(h, np.float64)
    if normalize:
        N = np.abs(np.concatenate([G, h[..., None]], -1)).max(-1)
        G, h = G / N[..., None], h / N
    z, _, act, st = O.qp_exact_general(P, q, G, h, tol=1e-12)
    return (w * z).sum(axis=1), (st, act)


@pytest.mark.parametrize("normalize", [False, True])
@pytest.mark.parametrize("n,m", [(2, 4), (3, 7), (3, 9)])
def test_qp_backward_matches_finite_differences(n, m, normalize):
    rng = np.random.default_rng(100 * n + m + normalize)
    B = 24
    P, q, G, h = random_qps(rng, B, n, m)
    w = rng.normal(0, 1, (B, n))
    g = O.qp_backward(P, q, G, h, normalize, w)
    assert (g["status"] == 0).all()
    eps = 1e-6
    G64, h64 = G.astype(np.float64), h.astype(np.float64)

    def fd(f):
        # samples whose active set changes inside +-eps sit on a kink: skipped
        lp, (sp, ap) = f(+eps)
        lm, (sm, am) = f(-eps)
        return (lp - lm) / (2 * eps), (sp == 0) & (sm == 0) & (ap == am).all(axis=1)

    # q
    for a in range(n):
        d, ok = fd(lambda e: _loss(P, q + e * np.eye(n)[a], G64, h64, w, normalize))
        assert rel(d[ok], g["q"][ok, a]) < 1e-5
    # P (symmetric perturbation: the pair (a,b),(b,a) together)
    for a in range(n):
        for b in range(a, n):
            E = np.zeros((n, n)); E[a, b] = 1.0; E[b, a] = 1.0
            d, ok = fd(lambda e: _loss(P + e * E, q, G64, h64, w, normalize))
            want = g["P"][:, a, b] + (g["P"][:, b, a] if a != b else 0.0)
            assert rel(d[ok], want[ok]) < 1e-5
    # G, h
    for r in range(m):
        for k in range(n):
            E = np.zeros((m, n)); E[r, k] = 1.0
            d, ok = fd(lambda e: _loss(P, q, G64 + e * E, h64, w, normalize))
            assert rel(d[ok], g["G"][ok, r, k]) < 1e-5, (r, k)
        d, ok = fd(lambda e: _loss(P, q, G64, h64 + e * np.eye(m)[r], w, normalize))
        assert rel(d[ok], g["h"][ok, r]) < 1e-5, r


def _dh_du(mode, G):
    """Closed-form d h / d u_RL of the CBFQPLayer rows (diff_cbf_qp.py:259-261,
    348-349, 362-377): CBF rows carry Lg . u = -G[r, :nu] . u, actuator rows
    u_max - u and -u_min + u."""
    B, m, n = G.shape
    nu = n - 1
    k = m - 2 * nu
    dh = np.zeros((B, m, nu))
    dh[:, :k, :] = -G[:, :k, :nu]
    for c in range(nu):
        dh[:, k + 2 * c, c] = -1.0
        dh[:, k + 2 * c + 1, c] = 1.0
    return dh


@pytest.mark.parametrize("fixture,mode", [("cars_layer", "SimulatedCars"), ("unicycle3_layer", "Unicycle"),
                                          ("unicycle5_layer", "Unicycle")])
@pytest.mark.parametrize("tag", ["prior", "rand"])
def test_solve_qp_backward_composes_to_reference_grad(golden, fixture, mode, tag):
    d = golden(fixture)
    G, h, P, u, w = d[tag + "_G"], d[tag + "_h"], d[tag + "_P"], d[tag + "_u"], d[tag + "_w"]
    B, m, n = G.shape
    nu = n - 1
    lo, hi = (-10.0, 10.0) if mode == "SimulatedCars" else (-2.5, 2.5)
    z = O.qp_exact_general(P.astype(np.float64), None, *O.normalize_rows(G, h)[:2])[0]
    v = np.asarray(u, np.float32) + z[:, :nu].astype(np.float32)
    mask = ((v >= lo) & (v <= hi)).astype(np.float64)
    gz = np.zeros((B, n))
    gz[:, :nu] = mask * w
    g = O.qp_backward(P, None, G, h, True, gz)
    assert (g["status"] == 0).all()
    grad = mask * w + np.einsum("bm,bmc->bc", g["h"], _dh_du(mode, G.astype(np.float64)))
    assert rel(grad, d[tag + "_grad_u"]) < 1e-5
