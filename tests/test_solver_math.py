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
    stats = {}
    z2, inb, kk = uni_qp_2d(Gn, hn, pd, K, stats=stats)
    ok = st == 0
    err = np.abs(z2 - z).max(1) / np.maximum(1, np.abs(z).max(1))
    assert err[ok].max() < 1e-6
    waves = kk[::64]
    assert (waves <= 2).mean() > 0.9, np.bincount(waves)
    # the certificates: what fraction of waves runs each optional stage
    w = {k: stats[k].reshape(-1, 64).any(1).mean() for k in ("open", "need_u0_edge", "need_u1_edge", "edge_open")}
    print(K, w, (~inb).reshape(-1, 64).any(1).mean())
    assert w["open"] < 0.5 and w["edge_open"] < 0.5, w


def _fma(a, b, c):
    """fma emulated in x87 extended precision (64-bit significand): within
    an ulp of the fused result, enough for a statistics test."""
    L = np.longdouble
    return (L(a) * L(b) + L(c)).astype(np.float64)


def test_uni_theta32_from_cos_sin():
    """rcbf_device.hpp uni_state32_from_cs restated: theta32 and the rows'
    fp32 cos/sin(theta32) from the fp64 cos/sin of the state's theta (no
    atan2, no second sincos) equal the reference chain get_state(float(obs))
    -> RN32(arctan2) -> RN32(cos/sin(theta32)) on >= 99.999 % of states and
    are within 1 fp32 ulp on the rest; covers |theta| up to 200 rad, the
    +-pi seam and multiples of pi/2."""
    rng = np.random.default_rng(5)
    th = np.concatenate([rng.uniform(-np.pi, np.pi, 200000), rng.uniform(-200, 200, 200000),
                         np.pi + rng.normal(0, 1e-6, 20000), -np.pi + rng.normal(0, 1e-6, 20000),
                         np.arange(-64, 65) * (np.pi / 2), [0.0, -0.0, np.pi, -np.pi]])
    c, s = np.cos(th), np.sin(th)
    c32, s32 = c.astype(F), s.astype(F)
    ref_th = np.arctan2(s32.astype(np.float64), c32.astype(np.float64)).astype(F)
    ref_c, ref_s = np.cos(ref_th.astype(np.float64)).astype(F), np.sin(ref_th.astype(np.float64)).astype(F)
    hi, lo = 6.28318530717958623200, 2.44929359829470635e-16
    k = np.rint(th * (1.0 / hi))
    t0 = _fma(-k, lo, _fma(-k, hi, th))
    dc, ds = c32.astype(np.float64) - c, s32.astype(np.float64) - s
    t = t0 + _fma(c, ds, -s * dc)  # c^2 + s^2 = 1 to a few ulps: the kernel does not divide by it
    wrap = np.where((s32 > 0) & (t < 0), hi, np.where((s32 < 0) & (t > 0), -hi, 0.0))
    t, t0 = t + wrap, t0 + wrap
    tz = np.where(c32 < 0, np.copysign(np.pi, s32), np.copysign(0.0, s32))
    t, t0 = np.where(s32 == 0, tz, t), np.where(s32 == 0, tz, t0)
    th32 = t.astype(F)
    D = th32.astype(np.float64) - t0
    D2 = D * D
    cD = _fma(D2, _fma(D2, 1.0 / 24.0, -0.5), 1.0)
    sD = D * _fma(D2, -1.0 / 6.0, 1.0)
    cr, sr = _fma(c, cD, -(s * sD)).astype(F), _fma(s, cD, c * sD).astype(F)
    n_rand = 400000  # the random angles; the rest are seams and exact multiples of pi/2
    for got, want in ((th32, ref_th), (cr, ref_c), (sr, ref_s)):
        bad = got != want
        assert bad[:n_rand].mean() < 1e-5, bad[:n_rand].mean()
        # exact multiples of pi/2 of large magnitude: cos/sin ~ 4e-8 there, so the ~1e-16 absolute
        # error of the reduction is ~2e-9 relative -- a 1-ulp fp32 difference on a few of them
        assert bad.sum() <= 32
        ulps = np.abs(got.view(np.int32).astype(np.int64) - want.view(np.int32).astype(np.int64))
        assert ulps[bad].max(initial=0) <= 1
