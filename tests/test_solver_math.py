"""CPU checks of the closed-form QP algorithms the kernels run
(tests/_solver_ports.py restates rcbf_device.hpp cars_qp_1d / uni_qp_2d)
against the oracle's KKT enumeration (oracle.qp_exact), on random states
near the hazards and across gamma_b.  Tolerance: 1e-7 relative on z (the
north-star bar on the safe action is 1e-4 relative), and the final fp32
safe action u_rl + z[:n_u] (diff_cbf_qp.py:146-150) must match in >= 99.99%
of lanes (the remaining lanes differ by an fp32 rounding of a ~1e-12
difference)."""
import numpy as np
import pytest

from oracle import oracle as O
from _solver_ports import cars_qp_1d, uni_qp_2d

F = np.float32


def _cars_states(rng, B):
    x, t, st = O.cars_reset(rng.normal(0, 0.5, B))
    n = rng.integers(0, 300, B)
    for k in range(300):
        a = rng.uniform(-3, 3, (B, 1)).astype(F)
        live = k < n
        x2, t2, st2, *_ = O.cars_step(x, t, st, a)
        x[live], t[live], st[live] = x2[live], t2[live], st2[live]
    return x.astype(F)


@pytest.mark.parametrize("gamma", [20.0, 1.0, 100.0])
def test_cars_qp_1d_matches_enumeration(gamma):
    rng = np.random.default_rng(0)
    B = 20000
    s32 = _cars_states(rng, B)
    u = rng.uniform(-1.5, 1.5, (B, 1)).astype(F)
    sg = np.tile(np.array(O.MAX_STD["SimulatedCars"], F), (B, 1)) * rng.uniform(0, 2, (B, 1)).astype(F)
    P, q, G, h = O.cars_build_diff(s32, u, None, sg, gamma)
    Gn, hn, _ = O.normalize_rows(G, h)
    pd = np.array([np.float64(F(0.1)), np.float64(F(10.0))])
    z, lam, act, stt = O.qp_exact(pd, Gn, hn)
    assert (stt == 0).all()
    z1 = cars_qp_1d(Gn, hn, pd)
    err = np.abs(z1 - z).max(1) / np.maximum(1, np.abs(z).max(1))
    assert err.max() < 1e-7
    fin_ref = np.clip(u[:, 0] + z[:, 0].astype(F), -10, 10)
    fin = np.clip(u[:, 0] + z1[:, 0].astype(F), -10, 10)
    assert (fin != fin_ref).mean() <= 1e-4
    assert act.any(1).mean() > 0.05  # the sample exercises active constraints


def test_cars_qp_1d_golden(golden):
    d = golden("cars_layer")
    pd = np.array([np.float64(F(0.1)), np.float64(F(10.0))])
    for tag in ["prior", "rand"]:
        z1 = cars_qp_1d(d[tag + "_Gn"], d[tag + "_hn"], pd)
        ref = d[tag + "_z"]
        assert (np.abs(z1 - ref).max(1) / np.maximum(1, np.abs(ref).max(1))).max() < 1e-7


def _uni_states(rng, B, K):
    hz = O.UNI["hazards"][:K]
    x = np.stack([rng.uniform(-3, 3, B), rng.uniform(-3, 3, B), rng.uniform(-np.pi, np.pi, B)], 1).astype(F)
    idx = rng.integers(0, K, B // 2)
    x[: B // 2, :2] = (hz[idx] + rng.normal(0, 0.5, (B // 2, 2))).astype(F)
    return x, hz


@pytest.mark.parametrize("K", [3, 5])
@pytest.mark.parametrize("gamma", [20.0, 1.0, 100.0])
def test_uni_qp_2d_matches_enumeration(K, gamma):
    rng = np.random.default_rng(1 + K)
    B = 20000
    x, hz = _uni_states(rng, B, K)
    u = rng.uniform(-1, 1, (B, 2)).astype(F)
    mu = rng.normal(0, 0.1, (B, 3)).astype(F)
    sg = rng.uniform(0, 0.3, (B, 3)).astype(F)
    P, q, G, h = O.unicycle_build_diff(x, u, mu, sg, gamma, hz)
    Gn, hn, _ = O.normalize_rows(G, h)
    pd = np.array([np.float64(F(1.0)), np.float64(F(1e-2)), np.float64(F(1e5))])
    z, lam, act, st = O.qp_exact(pd, Gn, hn)
    z2, inb, kk = uni_qp_2d(Gn, hn, pd, K)
    z3, _, _ = uni_qp_2d(Gn, hn, pd, K, prune=False)
    ok = st == 0
    assert ok.mean() > 0.999
    err = np.abs(z2 - z).max(1) / np.maximum(1, np.abs(z).max(1))
    assert err[ok].max() < 1e-6
    assert np.abs(z3 - z)[ok].max() / max(1, np.abs(z[ok]).max()) < 1e-6
    assert kk.min() < K  # pruning is exercised
    fin = np.clip(u + z[:, :2].astype(F), -2.5, 2.5)
    fin2 = np.clip(u + z2[:, :2].astype(F), -2.5, 2.5)
    assert (fin[ok] != fin2[ok]).any(1).mean() <= 1e-3
    assert (~inb).mean() > 0.001  # the box (stage 2) is exercised


@pytest.mark.parametrize("K", [3, 5])
def test_uni_qp_2d_cascade(K):
    rng = np.random.default_rng(7)
    B = 20000
    x, hz = _uni_states(rng, B, K)
    u = rng.uniform(-1, 1, (B, 2)).astype(F)
    mu = rng.normal(0, 0.1, (B, 3)).astype(F)
    sg = rng.uniform(0, 0.3, (B, 3)).astype(F)
    P, G, h = O.unicycle_build_cascade(x.astype(np.float64), u, mu, sg, 40.0, 3.0, hz)
    Gn, hn, _ = O.normalize_rows(G, h)
    pd = np.array([10.0, 1e-4, 1e7])
    z, lam, act, st = O.qp_exact(pd, Gn, hn)
    z2, _, _ = uni_qp_2d(Gn, hn, pd, K)
    ok = st == 0
    err = np.abs(z2[:, :2] - z[:, :2]).max(1) / np.maximum(1, np.abs(z[:, :2]).max(1))
    assert err[ok].max() < 1e-6


@pytest.mark.parametrize("K", [3, 5])
def test_uni_pruning_on_the_bench_distribution(K):
    """SURVEY 8(d) config-3 states (x, y ~ U[-3, 3], theta ~ U[-pi, pi]): the
    pruned solver (waves of 64 lanes) equals the exhaustive enumeration, and
    almost every wave needs at most 2 pieces (what makes the kernel cheap)."""
    rng = np.random.default_rng(30 + K)
    B = 64 * 600
    hz = O.UNI["hazards"][:K]
    x = np.stack([rng.uniform(-3, 3, B), rng.uniform(-3, 3, B), rng.uniform(-np.pi, np.pi, B)], 1).astype(F)
    u = rng.uniform(-1, 1, (B, 2)).astype(F)
    P, q, G, h = O.unicycle_build_diff(x, u, np.zeros((B, 3), F), np.full((B, 3), 0.2, F), 20.0, hz)
    Gn, hn, _ = O.normalize_rows(G, h)
    pd = np.array([np.float64(F(1.0)), np.float64(F(1e-2)), np.float64(F(1e5))])
    z, lam, act, st = O.qp_exact(pd, Gn, hn)
    z2, _, kk = uni_qp_2d(Gn, hn, pd, K)
    ok = st == 0
    err = np.abs(z2 - z).max(1) / np.maximum(1, np.abs(z).max(1))
    assert err[ok].max() < 1e-6
    waves = kk[::64]
    assert (waves <= 2).mean() > 0.9, np.bincount(waves)
