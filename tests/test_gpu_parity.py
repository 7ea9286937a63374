"""GPU parity: the HIP path (through the C-ABI) against the golden vectors the
reference produced and against the CPU oracle on seeded inputs.

Tolerances (north star: safe action within 1e-4 relative):
  * safe action vs reference fixtures: <= 1e-5 relative to max(1,|u|)
  * cars CBF rows: bit-exact vs the reference (same fp32 op order, no FMA)
  * unicycle CBF rows: <= 2e-6 relative (fp32 cos/sin: 1 ulp vs torch SLEEF)
  * gradients d final / d u_RL: <= 1e-5 relative
  * cars env trajectories: <= 1e-12 relative (device sin vs glibc), rewards
    <= 2 fp32 ulp, cost/done exact; unicycle states <= 1e-12 relative
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = np.asarray(a, np.float64); b = np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b) / np.maximum(1.0, np.abs(b)))) if a.size else 0.0


class Args:
    cuda = True


def dev(a, dtype=torch.float32):
    return torch.as_tensor(np.asarray(a), dtype=dtype, device="cuda")


def _env(mode, hazards=None, B=4):
    from rcbf_amd.envs import BatchedSimulatedCarsEnv, BatchedUnicycleEnv
    if mode == "SimulatedCars":
        return BatchedSimulatedCarsEnv(B)
    return BatchedUnicycleEnv(B, hazards_locations=hazards)


def _layer(env, gamma_b, solver=0):
    from rcbf_amd.diff_cbf_qp import CBFQPLayer
    return CBFQPLayer(env, Args(), gamma_b=gamma_b, solver=solver)


# ----------------------------------------------------------------------------
# CBFQPLayer vs reference fixtures
# ----------------------------------------------------------------------------
@pytest.mark.parametrize("solver", [0, 1, 2])
@pytest.mark.parametrize("tag", ["prior", "rand"])
def test_cars_layer_golden(golden, tag, solver):
    d = golden("cars_layer")
    layer = _layer(_env("SimulatedCars"), float(d["gamma_b"]), solver)
    x, u, mu, sg = (dev(d[tag + k]) for k in ("_x", "_u", "_mu", "_sigma"))
    P, q, G, h = layer.get_cbf_qp_constraints(x, u, mu, sg)
    assert np.array_equal(G.cpu().numpy(), d[tag + "_G"])
    assert np.array_equal(h.cpu().numpy(), d[tag + "_h"])
    assert np.array_equal(P.cpu().numpy(), d[tag + "_P"])
    fin = layer.get_safe_action(x, u, mu, sg).cpu().numpy()
    assert rel(fin, d[tag + "_final"]) <= 1e-5
    uu = u.clone().requires_grad_(True)
    out = layer.get_safe_action(x, uu, mu, sg)
    (out * dev(d[tag + "_w"])).sum().backward()
    assert rel(uu.grad.cpu().numpy(), d[tag + "_grad_u"]) <= 1e-5


@pytest.mark.parametrize("solver", [0, 1])
@pytest.mark.parametrize("k", [3, 5])
@pytest.mark.parametrize("tag", ["prior", "rand"])
def test_unicycle_layer_golden(golden, k, tag, solver):
    d = golden(f"unicycle{k}_layer")
    layer = _layer(_env("Unicycle", d["hazards"]), float(d["gamma_b"]), solver)
    x, u, mu, sg = (dev(d[tag + s]) for s in ("_x", "_u", "_mu", "_sigma"))
    P, q, G, h = layer.get_cbf_qp_constraints(x, u, mu, sg)
    assert rel(h.cpu().numpy(), d[tag + "_h"]) <= 2e-6
    assert rel(G.cpu().numpy(), d[tag + "_G"]) <= 1e-6
    # the kernel computes exactly what the oracle computes (same cos/sin rounding)
    Po, qo, Go, ho = O.unicycle_build_diff(d[tag + "_x"], d[tag + "_u"], d[tag + "_mu"], d[tag + "_sigma"],
                                           float(d["gamma_b"]), d["hazards"])
    assert np.array_equal(h.cpu().numpy(), ho) and np.array_equal(G.cpu().numpy(), Go)
    fin = layer.get_safe_action(x, u, mu, sg).cpu().numpy()
    assert rel(fin, d[tag + "_final"]) <= 1e-5
    uu = u.clone().requires_grad_(True)
    out = layer.get_safe_action(x, uu, mu, sg)
    (out * dev(d[tag + "_w"])).sum().backward()
    assert rel(uu.grad.cpu().numpy(), d[tag + "_grad_u"]) <= 1e-5


@pytest.mark.parametrize("mode", ["SimulatedCars", "Unicycle"])
@pytest.mark.parametrize("B", [256, 512])
def test_sac_update_safe_action_from_obs(mode, B):
    """RCBF_SAC.get_safe_action(obs, action, dynamics_model)
    (sac_cbf.py:218-238) as the SAC update calls it on replay batches: the
    fused obs-input kernel == get_state (oracle) -> prior -> CBFQPLayer, the
    state-input kernel bit for bit, and its gradient w.r.t. the action ==
    the oracle's implicit-KKT derivative."""
    from rcbf_amd.dynamics import DynamicsModel
    from rcbf_amd.sac_cbf import get_safe_action
    rng = np.random.default_rng(B)
    if mode == "SimulatedCars":
        x, _, _ = _cars_states(B, 21)
        obs = O.cars_obs(x).astype(np.float32)
        hz = None
        env = _env(mode)
    else:
        hz = O.UNI["hazards"][:3]
        x = np.stack([rng.uniform(-3, 3, B), rng.uniform(-3, 3, B), rng.uniform(-np.pi, np.pi, B)], 1)
        obs = O.uni_obs(x).astype(np.float32)
        env = _env(mode, hz)
    layer = _layer(env, 20.0)
    dyn = DynamicsModel(env, Args())
    n_u = env.n_u
    u = rng.uniform(-1, 1, (B, n_u)).astype(np.float32)
    w = rng.normal(0, 1, (B, n_u)).astype(np.float32)
    uu = dev(u).requires_grad_(True)
    out = get_safe_action(layer, dev(obs), uu, dyn)
    (out * dev(w)).sum().backward()
    s32 = O.get_state_f32(mode, obs)
    mu, sg = O.predict_disturbance_prior(mode, B)
    mu, sg = mu.astype(np.float32), sg.astype(np.float32)
    fin, _ = O.safe_action_diff(mode, s32, u, mu, sg, 20.0, hazards=hz)
    assert rel(out.detach().cpu().numpy(), fin) <= 1e-5
    g, _ = O.safe_action_diff_grad(mode, s32, u, mu, sg, 20.0, w, hazards=hz)
    assert rel(uu.grad.cpu().numpy(), g) <= 1e-5
    # same numbers as the state-input kernel on the oracle's get_state
    u2 = dev(u).requires_grad_(True)
    out2 = layer.get_safe_action(dev(s32), u2, dev(mu), dev(sg))
    (out2 * dev(w)).sum().backward()
    assert torch.equal(out.detach(), out2.detach()) and torch.equal(uu.grad, u2.grad)


@pytest.mark.parametrize("mode,k", [("SimulatedCars", 0), ("Unicycle", 3), ("Unicycle", 5)])
@pytest.mark.parametrize("from_obs", [False, True])
def test_jacobian_forward_equals_resolving_backward(mode, k, from_obs):
    """rcbf_[obs_]safe_action_jac (the forward the autograd op runs when the
    action needs a gradient) writes the plain forward's u bit for bit, and
    rcbf_safe_action_apply_jac on its Jacobian gives the re-solving backward
    (rcbf_[obs_]safe_action_backward) bit for bit, clamped actions included;
    B = 4096 + 37 (small-batch workgroups, ragged tail), per-env mean/sigma."""
    import ctypes
    from rcbf_amd import _lib
    lib = _lib.load()
    rng = np.random.default_rng(17 + k + 100 * from_obs)
    B = 4096 + 37
    hz = O.UNI["hazards"][:k] if mode == "Unicycle" else None
    env = _env(mode, hz)
    layer = _layer(env, 20.0)
    if mode == "SimulatedCars":
        x, _, _ = _cars_states(B, 5)
        obs = O.cars_obs(x).astype(np.float32)
    else:
        x = np.stack([rng.uniform(-3, 3, B), rng.uniform(-3, 3, B), rng.uniform(-np.pi, np.pi, B)], 1)
        obs = O.uni_obs(x).astype(np.float32)
    s32 = O.get_state_f32(mode, obs)
    inp = dev(obs if from_obs else s32)
    n_u = env.n_u
    u = dev(rng.uniform(-3, 3, (B, n_u)))  # beyond the box: some actions saturate the clamp
    mu = dev(0.01 * rng.normal(0, 1, (B, env.n_s)))
    sg = dev(0.2 * rng.uniform(0, 1, (B, env.n_s)) + 0.05)
    g = dev(rng.normal(0, 1, (B, n_u)))
    out_a, out_b = torch.empty_like(u), torch.empty_like(u)
    jac = torch.empty(B, n_u, n_u, dtype=torch.float64, device="cuda")
    ga, gb = torch.empty_like(u), torch.empty_like(u)
    prm, s = ctypes.byref(layer._prm), _lib.stream_of(u.device)
    p = _lib.ptr
    pre = "rcbf_obs_safe_action" if from_obs else "rcbf_safe_action"
    assert getattr(lib, pre)(prm, B, p(inp), p(u), p(mu), p(sg), p(out_a), None, None, s) == 0
    assert getattr(lib, pre + "_jac")(prm, B, p(inp), p(u), p(mu), p(sg), p(out_b), p(jac), None, None, s) == 0
    assert getattr(lib, pre + "_backward")(prm, B, p(inp), p(u), p(mu), p(sg), p(g), p(ga), s) == 0
    assert lib.rcbf_safe_action_apply_jac(B, n_u, p(jac), p(g), p(gb), s) == 0
    torch.cuda.synchronize()
    def same(a, b):  # bit-equal values, NaN where the other has NaN
        return torch.equal(a.isnan(), b.isnan()) and torch.equal(a.nan_to_num(7.0), b.nan_to_num(7.0))
    assert same(out_a, out_b)
    assert same(ga, gb)
    # a saturated action's row holds the RCBF_JAC_NO_GRAD payload, and no other NaN occurs
    bits = jac.view(torch.int64)
    saturated = (bits == _lib.JAC_NO_GRAD).any(2).any(1)
    assert 0 < int(saturated.sum()) < B  # both kinds of rows occur
    assert torch.equal(jac.isnan(), bits == _lib.JAC_NO_GRAD)
    # a degenerate lane (a NaN the solve itself produced, any payload but the marker) reaches the gradient,
    # as in the re-solving backward; the marker alone reads as "no gradient"
    jd = jac.clone()
    jd[0, 0, :] = float("nan")
    jd.view(torch.int64)[1, 0, :] = _lib.JAC_NO_GRAD
    gd = torch.empty_like(u)
    assert lib.rcbf_safe_action_apply_jac(B, n_u, p(jd), p(g), p(gd), s) == 0
    torch.cuda.synchronize()
    assert bool(gd[0].isnan().all()) and not bool(gd[1].isnan().any())
    assert torch.equal(gd[2:], gb[2:])


@pytest.mark.parametrize("mode,k", [("SimulatedCars", 0), ("Unicycle", 3)])
def test_config5_workload_vs_c_oracle(mode, k):
    """Config 5 as bench.py runs it (SURVEY states, MAX_STD
    materialised per env as (B, n_s) rows, upstream gradient w ~ N(0, 1)):
    the autograd op's forward (rcbf_obs_safe_action_jac) and backward
    (rcbf_safe_action_apply_jac) against the C oracle's forward and implicit-
    KKT gradient (oracle_safe_action_grad), B = 4096."""
    from oracle import c_oracle as C
    from rcbf_amd.dynamics import MAX_STD
    from rcbf_amd.sac_cbf import get_safe_action
    from rcbf_amd.dynamics import DynamicsModel
    B = 4096
    rng = np.random.default_rng(55 + k)
    hz = O.UNI["hazards"][:k] if mode == "Unicycle" else None
    env = _env(mode, hz)
    layer = _layer(env, 20.0)
    if mode == "SimulatedCars":
        x, _, _ = _cars_states(B, 9)
        obs = O.cars_obs(x).astype(np.float32)
    else:
        x = np.stack([rng.uniform(-3, 3, B), rng.uniform(-3, 3, B), rng.uniform(-np.pi, np.pi, B)], 1)
        obs = O.uni_obs(x).astype(np.float32)
    u = rng.uniform(-1, 1, (B, env.n_u)).astype(np.float32)
    w = rng.normal(0, 1, (B, env.n_u)).astype(np.float32)
    mu = np.zeros((B, env.n_s), np.float32)
    sg = np.tile(np.asarray(MAX_STD[mode], np.float32), (B, 1))
    uu = dev(u).requires_grad_(True)
    out = layer.get_safe_action(dev(O.get_state_f32(mode, obs)), uu, dev(mu), dev(sg))
    (out * dev(w)).sum().backward()
    ref, g, fails = C.safe_action_grad(mode, O.get_state_f32(mode, obs), u, mu, sg, 20.0, w, hazards=hz, threads=4)
    assert fails == 0
    assert rel(out.detach().cpu().numpy(), ref) <= 1e-5
    assert rel(uu.grad.cpu().numpy(), g) <= 1e-5
    # the obs-input path of RCBF_SAC.get_safe_action gives the same numbers
    u2 = dev(u).requires_grad_(True)
    out2 = get_safe_action(layer, dev(obs), u2, DynamicsModel(env, Args()))
    (out2 * dev(w)).sum().backward()
    assert torch.equal(out2.detach(), out.detach()) and torch.equal(u2.grad, uu.grad)


def test_solve_qp_and_cbf_layer_surface(golden):
    d = golden("cars_layer")
    layer = _layer(_env("SimulatedCars"), float(d["gamma_b"]))
    P, q, G, h = (dev(d["prior_" + k]) for k in ("P", "q", "G", "h"))
    sol = layer.solve_qp(P, q, G, h).cpu().numpy()
    assert rel(sol, d["prior_z"][:, :1]) <= 1e-6
    z = layer.cbf_layer(P, q, dev(d["prior_Gn"]), dev(d["prior_hn"])).cpu().numpy()
    assert rel(z, d["prior_z"]) <= 1e-6


def test_layer_surfaces_by_keyword(golden):
    """Every layer surface called with the reference's keyword names
    (diff_cbf_qp.py:12,44,81,111,146; cbf_qp.py:7,29,55,242) gives the
    positional result, and solve_qp divides the caller's Gs in place like
    `Gs /= Ghs_norm` (diff_cbf_qp.py:105): bit for bit the reference's rows."""
    from rcbf_amd.cbf_qp import CascadeCBFLayer
    from rcbf_amd.diff_cbf_qp import CBFQPLayer
    from rcbf_amd.envs import SimulatedCarsEnv
    d = golden("cars_layer")
    layer = CBFQPLayer(env=_env("SimulatedCars"), args=Args(), gamma_b=float(d["gamma_b"]), k_d=1.5, l_p=0.03)
    x, u, mu, sg = (dev(d["rand" + k]) for k in ("_x", "_u", "_mu", "_sigma"))
    fin = layer.get_safe_action(state_batch=x, action_batch=u, mean_pred_batch=mu, sigma_batch=sg)
    assert torch.equal(fin, layer.get_safe_action(x, u, mu, sg))
    assert rel(fin.cpu().numpy(), d["rand_final"]) <= 1e-5
    P, q, G, h = layer.get_cbf_qp_constraints(state_batch=x, action_batch=u, mean_pred_batch=mu,
                                              sigma_pred_batch=sg)
    assert np.array_equal(G.cpu().numpy(), d["rand_G"])
    Gpos = G.clone()
    sol_pos = layer.solve_qp(P, q, Gpos, h)
    sol = layer.solve_qp(Ps=P, qs=q, Gs=G, hs=h)
    assert torch.equal(sol, sol_pos)
    assert np.array_equal(G.cpu().numpy(), d["rand_Gn"]) and torch.equal(G, Gpos)  # divided in place
    z = layer.cbf_layer(Qs=P, ps=q, Gs=dev(d["rand_Gn"]), hs=dev(d["rand_hn"]), As=None, bs=None,
                        solver_args={"eps": 1e-4})
    assert rel(z.cpu().numpy(), d["rand_z"]) <= 1e-6
    # autograd: a leaf that requires grad refuses the in-place division, as in the reference
    Gl = dev(d["rand_G"]).requires_grad_(True)
    with pytest.raises(RuntimeError):
        layer.solve_qp(P, q, Gl, h)
    # a non-leaf is divided with the division recorded; d sol / d G flows to the leaf
    G0 = dev(d["rand_G"]).requires_grad_(True)
    Gn = G0 * 1.0
    s2 = layer.solve_qp(P, q, Gn, h)
    assert torch.equal(Gn.detach(), dev(d["rand_Gn"])) and rel(s2.detach().cpu().numpy(), d["rand_z"][:, :1]) <= 1e-6
    s2.sum().backward()
    assert G0.grad is not None and torch.isfinite(G0.grad).all()
    # Cascade surfaces by keyword
    c = golden("cascade")
    cl = CascadeCBFLayer(env=SimulatedCarsEnv(), gamma_b=20.0, k_d=3.0, l_p=0.03)
    us = cl.get_u_safe(u_nom=c["cars_u"], s=c["cars_x"], mean_pred=c["cars_mu"], sigma=c["cars_sigma"])
    assert np.array_equal(np.asarray(us), np.asarray(cl.get_u_safe(c["cars_u"], c["cars_x"], c["cars_mu"],
                                                                   c["cars_sigma"])))
    Pc, qc, Gc, hc = cl.get_cbf_qp_constraints(u_nom=c["cars_u"][0], state=c["cars_x"][0],
                                              mean_pred=c["cars_mu"][0], sigma_pred=c["cars_sigma"][0])
    uc = cl.solve_qp(P=Pc, q=qc, G=np.array(Gc, copy=True), h=hc)
    assert rel(uc, cl.solve_qp(Pc, qc, np.array(Gc, copy=True), hc)) == 0.0


def test_single_sample_and_empty_batch(golden):
    d = golden("cars_layer")
    layer = _layer(_env("SimulatedCars"), float(d["gamma_b"]))
    x, u, mu, sg = (dev(d["prior" + k]) for k in ("_x", "_u", "_mu", "_sigma"))
    one = layer.get_safe_action(x[7], u[7], mu[7], sg[7])
    assert one.shape == (1,)
    assert rel(one.cpu().numpy(), d["prior_final"][7]) <= 1e-5
    empty = layer.get_safe_action(x[:0], u[:0], mu[:0], sg[:0])
    assert empty.shape == (0, 1)


def test_cpu_tensors_round_trip(golden):
    """args.cuda=False callers hand CPU tensors: computed on the device, returned on the CPU."""
    from rcbf_amd.diff_cbf_qp import CBFQPLayer

    class A:
        cuda = False

    d = golden("cars_layer")
    layer = CBFQPLayer(_env("SimulatedCars"), A(), gamma_b=float(d["gamma_b"]))
    fin = layer.get_safe_action(*(torch.tensor(d["prior" + k]) for k in ("_x", "_u", "_mu", "_sigma")))
    assert fin.device.type == "cpu"
    assert rel(fin.numpy(), d["prior_final"]) <= 1e-5


def test_cascade_golden(golden):
    from rcbf_amd.cbf_qp import CascadeCBFLayer
    from rcbf_amd.envs import SimulatedCarsEnv, UnicycleEnv
    c = golden("cascade")
    cl = CascadeCBFLayer(SimulatedCarsEnv(), gamma_b=20.0, k_d=3.0)
    us = cl.get_u_safe(c["cars_u"], c["cars_x"], c["cars_mu"], c["cars_sigma"])
    assert rel(us, c["cars_usafe"]) <= 1e-9
    P, q, G, h = cl.get_cbf_qp_constraints(c["cars_u"], c["cars_x"], c["cars_mu"], c["cars_sigma"])
    assert rel(G, c["cars_G"]) < 1e-14 and rel(h, c["cars_h"]) < 1e-13
    ul = CascadeCBFLayer(UnicycleEnv(), gamma_b=40.0, k_d=3.0, l_p=0.03)
    us = ul.get_u_safe(c["uni_u"], c["uni_x"], c["uni_mu"], c["uni_sigma"])
    assert rel(us, c["uni_usafe"]) <= 1e-7
    one = ul.get_u_safe(c["uni_u"][0], c["uni_x"][0], c["uni_mu"][0], c["uni_sigma"][0])
    assert one.shape == (2,) and rel(one, c["uni_usafe"][0]) <= 1e-7


def test_cascade_config_size_golden(golden):
    """rcbf_cascade_u_safe at config size: 4096 cars rows (config-2 start
    states) and 4096 unicycle rows with the config-3 hazard set (k = 3),
    against the reference's own CascadeCBFLayer.get_u_safe (cbf_qp.py:29-53)
    with the exact QP at cbf_qp.py:276."""
    from rcbf_amd.cbf_qp import CascadeCBFLayer
    from rcbf_amd.envs import SimulatedCarsEnv, UnicycleEnv
    c = golden("cascade_config")
    cl = CascadeCBFLayer(SimulatedCarsEnv(), gamma_b=20.0, k_d=3.0)
    us = cl.get_u_safe(c["cars_u"], c["cars_x"], c["cars_mu"], c["cars_sigma"])
    assert us.shape == (4096, 1) and rel(us, c["cars_usafe"]) <= 1e-9
    env = UnicycleEnv()
    env.hazards_locations = np.asarray(c["uni3_hazards"])
    ul = CascadeCBFLayer(env, gamma_b=40.0, k_d=3.0, l_p=0.03)
    us = ul.get_u_safe(c["uni3_u"], c["uni3_x"], c["uni3_mu"], c["uni3_sigma"])
    assert us.shape == (4096, 2) and rel(us, c["uni3_usafe"]) <= 1e-7


def test_cascade_slack_and_violation_warning(golden, capsys):
    """get_u_safe returns the QP's slack epsilon
    (rcbf_cascade_u_safe eps_out) and prints the reference's warning for every
    row with |epsilon| > 0.1 (cbf_qp.py:283-284).  The slack is checked
    against the exact QP on the normalised fp64 rows (oracle), on the 4096
    config-size cars rows plus unicycle states placed inside a hazard (which
    need a large slack)."""
    from rcbf_amd.cbf_qp import CascadeCBFLayer
    from rcbf_amd.envs import SimulatedCarsEnv, UnicycleEnv
    c = golden("cascade_config")
    cl = CascadeCBFLayer(SimulatedCarsEnv(), gamma_b=20.0, k_d=3.0)
    env = UnicycleEnv()
    ul = CascadeCBFLayer(env, gamma_b=40.0, k_d=3.0, l_p=0.03)
    rng = np.random.default_rng(3)
    hz = np.asarray(env.hazards_locations)
    ux = np.concatenate([hz[:, :2] + rng.normal(0, 0.05, hz.shape), rng.uniform(-np.pi, np.pi, (len(hz), 1))], 1)
    ux = np.concatenate([ux, np.stack([rng.uniform(-3, 3, 64), rng.uniform(-3, 3, 64),
                                       rng.uniform(-np.pi, np.pi, 64)], 1)], 0)
    uu = rng.uniform(-1, 1, (len(ux), 2))
    um, us_ = np.zeros_like(ux), np.full_like(ux, 0.2)
    for layer, args in ((cl, (c["cars_u"], c["cars_x"], c["cars_mu"], c["cars_sigma"])), (ul, (uu, ux, um, us_))):
        capsys.readouterr()
        layer.get_u_safe(*args)
        printed = [ln for ln in capsys.readouterr().out.splitlines() if ln.startswith("CBF indicates")]
        eps = layer.last_eps
        P, q, G, h = layer.get_cbf_qp_constraints(*args)
        Gn, hn, _ = O.normalize_rows(G, h)
        z, _, _, st = O.qp_exact_general(P, q, Gn, hn)
        assert (st == 0).all()
        assert np.max(np.abs(eps - z[:, -1]) / np.maximum(1.0, np.abs(z[:, -1]))) <= 1e-7
        assert len(printed) == int((np.abs(eps) > 0.1).sum())
    assert len(printed) >= 1  # the states inside a hazard need the slack


def test_cascade_solve_qp_golden(golden):
    """CascadeCBFLayer.solve_qp (cbf_qp.py:242-286) on the reference's own
    rows: the exact fp64 solution (quadprog's), the caller's G normalised in
    place, and quadprog's ValueError on an infeasible QP."""
    from rcbf_amd.cbf_qp import CascadeCBFLayer
    from rcbf_amd.envs import SimulatedCarsEnv, UnicycleEnv
    c = golden("cascade")
    for layer, nm, tol in ((CascadeCBFLayer(SimulatedCarsEnv(), gamma_b=20.0, k_d=3.0), "cars", 1e-9),
                           (CascadeCBFLayer(UnicycleEnv(), gamma_b=40.0, k_d=3.0, l_p=0.03), "uni", 1e-7)):
        P = c[nm + "_P"]
        for b in range(0, 256, 8):
            G, h = c[nm + "_G"][b].copy(), c[nm + "_h"][b]
            u = layer.solve_qp(P, np.zeros(P.shape[0]), G, h)
            assert u.shape == (P.shape[0] - 1,)
            assert rel(u, c[nm + "_usafe"][b]) <= tol
            Gn, _, _ = O.normalize_rows(c[nm + "_G"][b][None], h[None])
            assert np.array_equal(G, Gn[0])
    G = np.array([[1.0, 0.0], [-1.0, 0.0]])
    with pytest.raises(ValueError):
        layer.solve_qp(np.eye(2), np.zeros(2), G, np.array([-1.0, -1.0]))


# ----------------------------------------------------------------------------
# environments vs reference trajectories
# ----------------------------------------------------------------------------
def test_cars_env_traj(golden):
    from rcbf_amd.envs import BatchedSimulatedCarsEnv
    d = golden("env_traj")
    E = d["cars_noise"].shape[0]
    env = BatchedSimulatedCarsEnv(E)
    env.reset(noise=d["cars_noise"])
    assert np.array_equal(env.state_numpy(), d["cars_state"][:, 0])
    for k in range(300):
        obs, r, done, info = env.step(dev(d["cars_actions"][:, k]), auto_reset=False, obs64=True)
        assert rel(env.state_numpy(), d["cars_state"][:, k + 1]) <= 1e-12
        assert rel(info["obs64"].cpu().numpy(), d["cars_obs"][:, k + 1]) <= 1e-12
        rr = r.cpu().numpy()
        assert np.all(np.abs(rr - d["cars_reward"][:, k]) <= 2 * np.spacing(np.abs(rr).astype(np.float32)))
        assert np.array_equal(info["cost"].cpu().numpy(), d["cars_cost"][:, k])
        assert np.array_equal(done.cpu().numpy(), d["cars_done"][:, k])
        assert np.allclose(env.aux.cpu().numpy(), d["cars_t"][:, k + 1], rtol=0, atol=1e-12)


def test_unicycle_env_traj(golden):
    from rcbf_amd.envs import BatchedUnicycleEnv
    d = golden("env_traj")
    env = BatchedUnicycleEnv(1)
    for k in range(1000):
        obs, r, done, info = env.step(dev(d["uni_actions"][k][None]), auto_reset=False, obs64=True)
        assert rel(env.state_numpy()[0], d["uni_state"][k + 1]) <= 1e-12
        assert rel(info["obs64"].cpu().numpy()[0], d["uni_obs"][k + 1]) <= 1e-12
        assert abs(r.item() - d["uni_reward"][k]) <= 1e-12
        assert info["cost"].item() == d["uni_cost"][k] and bool(done.item()) == bool(d["uni_done"][k])
    # random starts: hazard contacts, goal hits, time limit
    E, T = d["unir_x0"].shape[0], d["unir_actions"].shape[1]
    env = BatchedUnicycleEnv(E)
    env.load_state(d["unir_x0"], d["unir_lastdist"][:, 0], d["unir_step0"])
    alive = np.ones(E, bool)
    for k in range(T):
        obs, r, done, info = env.step(dev(d["unir_actions"][:, k]), auto_reset=False, obs64=True)
        xs = env.state_numpy()
        assert rel(xs[alive], d["unir_state"][alive, k + 1]) <= 1e-11
        assert np.array_equal(info["cost"].cpu().numpy()[alive], d["unir_cost"][alive, k])
        assert np.array_equal(done.cpu().numpy()[alive], d["unir_done"][alive, k])
        assert np.array_equal(info["goal_met"].cpu().numpy()[alive], d["unir_goal"][alive, k])
        alive &= ~d["unir_done"][:, k]


def test_single_env_gym_api(golden):
    from rcbf_amd.envs import SimulatedCarsEnv, UnicycleEnv
    d = golden("env_traj")
    env = SimulatedCarsEnv()
    np.random.seed(100)
    obs = env.reset()
    assert rel(obs, d["cars_obs"][0, 0]) == 0.0
    for k in range(300):
        obs, r, done, info = env.step(d["cars_actions"][0, k])
        assert rel(obs, d["cars_obs"][0, k + 1]) <= 1e-12
        assert isinstance(r, np.float32) and set(info) == {"cost", "goal_met"}
    assert done and env.episode_step == 300
    u = UnicycleEnv()
    o = u.reset()
    assert rel(o, d["uni_obs"][0]) <= 1e-15
    o, r, dn, info = u.step(d["uni_actions"][0])
    assert rel(o, d["uni_obs"][1]) <= 1e-12


def test_closed_loop_config1(golden):
    """Config 1 on the device: hand controller + CascadeCBFLayer + cars env."""
    from rcbf_amd.cbf_qp import CascadeCBFLayer
    from rcbf_amd.dynamics import DynamicsModel
    from rcbf_amd.envs import SimulatedCarsEnv
    cl = golden("closed_loop_cars")
    env = SimulatedCarsEnv()

    class A:
        gp_model_size = 2000
        cuda = False

    dm = DynamicsModel(env, A())
    layer = CascadeCBFLayer(env, gamma_b=20.0, k_d=3.0)
    env._b.reset(noise=np.array([cl["noise"]]))
    obs = env._get_obs()
    for k in range(300):
        state = dm.get_state(obs)
        s = state
        u = np.array([(s[4] - s[6] - 0.4) * (s[4] - s[6] - 0.4 < 0)])
        u += np.array([(s[8] - s[6] + 0.4) * (s[8] - s[6] + 0.4 > 0)])
        assert rel(u, cl["u_nom"][k]) <= 1e-8
        m, sg = dm.predict_disturbance(state)
        us = layer.get_u_safe(u, state, m, sg)
        assert rel(us, cl["u_safe"][k]) <= 1e-6
        obs, r, done, info = env.step(u + us)
        assert rel(env.state, cl["state"][k + 1]) <= 1e-8
    assert done


# ----------------------------------------------------------------------------
# the fused safe step vs the oracle (seeded, config-2/3 style inputs)
# ----------------------------------------------------------------------------
def _cars_states(B, seed):
    rng = np.random.default_rng(seed)
    x, t, st = O.cars_reset(rng.normal(0, 0.5, B))
    n = rng.integers(0, 300, B)
    for k in range(300):
        a = rng.uniform(-1, 1, (B, 1)).astype(np.float32)
        live = k < n
        x2, t2, st2, *_ = O.cars_step(x, t, st, a)
        x[live], t[live], st[live] = x2[live], t2[live], st2[live]
    return x, t, st


@pytest.mark.parametrize("solver", [0, 1, 2])
def test_fused_safe_step_cars(solver):
    from rcbf_amd.envs import BatchedSimulatedCarsEnv
    B = 4096
    x, t, st = _cars_states(B, 5)
    env = BatchedSimulatedCarsEnv(B)
    env.load_state(x, t, st)
    layer = _layer(env, 20.0, solver)
    rng = np.random.default_rng(6)
    for k in range(3):
        u = rng.uniform(-1, 1, (B, 1)).astype(np.float32)
        obs, rew, done, out = env.safe_step(dev(u), layer, auto_reset=False)
        s32 = O.get_state_f32("SimulatedCars", O.cars_obs(x).astype(np.float32))
        mu, sg = O.predict_disturbance_prior("SimulatedCars", B)
        fin, aux = O.safe_action_diff("SimulatedCars", s32, u, mu.astype(np.float32), sg.astype(np.float32), 20.0)
        ug = out["u"].cpu().numpy()
        assert rel(ug, fin) <= 1e-4
        x, t, st, o, r, c, dn = O.cars_step(x, t, st, ug)  # the env physics, given the device's action
        assert rel(env.state_numpy(), x) <= 1e-9
        assert rel(obs.cpu().numpy(), o.astype(np.float32)) <= 1e-6
        assert rel(rew.cpu().numpy(), r) <= 1e-6
        assert np.array_equal(out["cost"].cpu().numpy(), c.astype(np.float32))
        assert np.array_equal(done.cpu().numpy().astype(bool), dn)
    env.check_failures()


@pytest.mark.parametrize("k", [1, 2, 3, 5, 8])
def test_fused_safe_step_unicycle(k):
    from rcbf_amd.envs import BatchedUnicycleEnv
    B = 4096
    rng = np.random.default_rng(7 + k)
    hz = O.UNI["hazards"][:k]
    if k > len(hz):  # up to RCBF_MAX_HAZARDS = 8: extra hazards at seeded positions
        hz = np.concatenate([hz, rng.uniform(-2.5, 2.5, (k - len(hz), 2))])
    env = BatchedUnicycleEnv(B, hazards_locations=hz)
    x = np.stack([rng.uniform(-3, 3, B), rng.uniform(-3, 3, B), rng.uniform(-np.pi, np.pi, B)], 1)
    ld = O.uni_goal_dist(x); st = np.zeros(B, np.int64)
    env.load_state(x, ld, np.zeros(B))
    layer = _layer(env, 20.0)
    for it in range(3):
        u = rng.uniform(-1, 1, (B, 2)).astype(np.float32)
        obs, rew, done, out = env.safe_step(dev(u), layer, auto_reset=False)
        s32 = O.get_state_f32("Unicycle", O.uni_obs(x).astype(np.float32))
        fin, aux = O.safe_action_diff("Unicycle", s32, u, np.zeros((B, 3), np.float32),
                                      np.full((B, 3), 0.2, np.float32), 20.0, hazards=hz)
        ug = out["u"].cpu().numpy()
        assert rel(ug, fin) <= 1e-4
        x, ld, st, o, r, c, dn, gm = O.uni_step(x, ld, st, ug, hazards=hz)  # the env physics, given the device's action
        assert rel(env.state_numpy(), x) <= 1e-9
        assert rel(rew.cpu().numpy(), r) <= 1e-5
    env.check_failures()


@pytest.mark.parametrize("mode", ["SimulatedCars", "Unicycle"])
def test_fused_step_ragged_batches_match_full_batch(mode):
    """Ragged batches (a partial last wave, which stores its observations per
    lane instead of through LDS) give bit-identical outputs to the same envs
    inside a batch of whole waves; auto-resets included (episodes end here)."""
    from rcbf_amd.envs import BatchedSimulatedCarsEnv, BatchedUnicycleEnv
    Bf = 4160
    rng = np.random.default_rng(31)
    if mode == "SimulatedCars":
        x, t, st = _cars_states(Bf, 32)
        st = np.where(rng.random(Bf) < 0.3, 297, st)  # some episodes end during the test

        def make(B):
            e = BatchedSimulatedCarsEnv(B, seed=4)
            e.load_state(x[:B], t[:B], st[:B])
            return e
    else:
        hz = O.UNI["hazards"][:3]
        x = np.stack([rng.uniform(-3, 3, Bf), rng.uniform(-3, 3, Bf), rng.uniform(-np.pi, np.pi, Bf)], 1)
        st = np.where(rng.random(Bf) < 0.3, 997, 0)

        def make(B):
            e = BatchedUnicycleEnv(B, seed=4, hazards_locations=hz)
            e.load_state(x[:B], O.uni_goal_dist(x[:B]), st[:B])
            return e
    full = make(Bf)
    lf = _layer(full, 20.0)
    us = [dev(rng.uniform(-1, 1, (Bf, full.n_u))) for _ in range(5)]
    ref = []
    for u in us:
        obs, r, d, out = full.safe_step(u, lf)
        ref.append([obs.clone(), r.clone(), d.clone(), out["u"].clone(), out["cost"].clone()])
    for B in (1, 63, 65, 4133):
        e = make(B)
        le = _layer(e, 20.0)
        for k, u in enumerate(us):
            obs, r, d, out = e.safe_step(u[:B].contiguous(), le)
            got = [obs, r, d, out["u"], out["cost"]]
            for g, w in zip(got, ref[k]):
                assert torch.equal(g, w[:B]), (B, k)
        assert torch.equal(e.state, full.state[:B]) and torch.equal(e.step_count, full.step_count[:B])
        e.check_failures()
    assert int(full.episode.max().item()) >= 2  # auto-resets happened (construction counts as episode 1)


@pytest.mark.parametrize("mode", ["SimulatedCars", "Unicycle"])
def test_fast_binding_matches_ctypes_path(mode, monkeypatch):
    """safe_step through the CPython binding (csrc/rcbf_pyfast.cpp) and through
    ctypes launch the same C-ABI entry point: bit-identical trajectories, with
    and without a disturbance prior, auto-resets included, on a side stream."""
    import rcbf_amd.envs as E
    from rcbf_amd import _lib
    assert _lib.fast() is not None, "_rcbf_fast extension not built (run __graft_entry__.build())"
    B = 1000
    rng = np.random.default_rng(5)
    us = [dev(rng.uniform(-1, 1, (B, 1 if mode == "SimulatedCars" else 2))) for _ in range(12)]

    def run(fast):
        monkeypatch.setattr(E, "_fast", fast)
        if mode == "SimulatedCars":
            e = E.BatchedSimulatedCarsEnv(B, seed=8)
        else:
            e = E.BatchedUnicycleEnv(B, seed=8, hazards_locations=O.UNI["hazards"][:3])
        lay = _layer(e, 20.0)
        mu = torch.full((B, e.n_s), 0.01, device="cuda")
        sg = torch.full((B, e.n_s), 0.2, device="cuda")
        got = []
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for k, u in enumerate(us):
                obs, r, d, out = e.safe_step(u, lay, mean=mu if k % 2 else None, sigma=sg if k % 2 else None)
                got += [obs.clone(), r.clone(), d.clone(), out["u"].clone()]
        torch.cuda.synchronize()
        e.check_failures()
        return got + [e.state.clone(), e.step_count.clone()]

    fast = E._fast
    a, b = run(fast), run(None)
    for g, w in zip(a, b):
        assert torch.equal(g, w)
    # malformed inputs are refused on the host, before any launch
    monkeypatch.setattr(E, "_fast", fast)
    e = E.BatchedSimulatedCarsEnv(8, seed=1)
    lay = _layer(e, 20.0)
    u = torch.zeros(8, 1, device="cuda")
    with pytest.raises(ValueError):
        e.safe_step(u, lay, mean=torch.zeros(8, 3, device="cuda"))
    with pytest.raises(ValueError):
        e.safe_step(torch.zeros(4, 1, device="cuda"), lay)
    e.safe_step(u, lay, mean=torch.zeros(8, 10, dtype=torch.float64, device="cuda"))  # converted to fp32
    e.check_failures()
    # a layer built for another env is refused (the kernel runs the env physics with the layer's params)
    uni = E.BatchedUnicycleEnv(8, seed=1, hazards_locations=O.UNI["hazards"][:3])
    with pytest.raises(ValueError, match="different env"):
        uni.safe_step(torch.zeros(8, 2, device="cuda"), lay)
    uni5 = E.BatchedUnicycleEnv(8, seed=1)
    with pytest.raises(ValueError, match="different env"):
        uni.safe_step(torch.zeros(8, 2, device="cuda"), _layer(uni5, 20.0))
    # malformed caller-supplied outputs are refused when the argument cache is built
    bad = e.make_outputs()
    bad["reward"] = torch.empty(8, dtype=torch.float64, device="cuda")
    with pytest.raises(ValueError, match="outputs"):
        e.safe_step(u, lay, outputs=bad)
    small = E.BatchedSimulatedCarsEnv(4, seed=1).make_outputs()
    with pytest.raises(ValueError, match="outputs"):
        e.safe_step(u, lay, outputs=small)


def test_rollout_matches_single_steps():
    """K fused steps in one launch == K launches of the fused step."""
    from rcbf_amd.envs import BatchedSimulatedCarsEnv
    B, K = 2048, 40
    a = BatchedSimulatedCarsEnv(B, seed=3)
    b = BatchedSimulatedCarsEnv(B, seed=3)
    la, lb = _layer(a, 20.0), _layer(b, 20.0)
    u = torch.rand(K, B, 1, device="cuda") * 2 - 1
    rs, cs, nd = a.rollout(u, la)
    tot_r = torch.zeros(B, device="cuda"); tot_c = torch.zeros(B, device="cuda")
    for k in range(K):
        _, r, d, out = b.safe_step(u[k], lb)
        tot_r += r; tot_c += out["cost"]
    assert torch.equal(a.x, b.x) and torch.equal(a.step_count, b.step_count)
    assert torch.allclose(rs, tot_r, rtol=1e-5, atol=1e-6) and torch.allclose(cs, tot_c, atol=1e-5)


def test_auto_reset_and_rng_sharding_invariance():
    """Episodes roll over at 300 steps; the reset draw depends only on
    (seed, global env index, episode) so a 2-way shard reproduces the whole."""
    from rcbf_amd.envs import BatchedSimulatedCarsEnv
    B = 512
    full = BatchedSimulatedCarsEnv(B, seed=9)
    lo = BatchedSimulatedCarsEnv(B // 2, seed=9, env_offset=0)
    hi = BatchedSimulatedCarsEnv(B // 2, seed=9, env_offset=B // 2)
    assert torch.equal(full.state[:B // 2], lo.state) and torch.equal(full.state[B // 2:], hi.state)
    lf = _layer(full, 20.0)
    u = torch.zeros(B, 1, device="cuda")
    nd = 0
    for k in range(300):
        _, _, d, _ = full.safe_step(u, lf)
        nd += int(d.sum().item()) if k == 299 else 0
    assert nd == B and int(full.step_count.max().item()) == 0 and int(full.episode.min().item()) == 2
    v = full.state[:, 1].cpu().numpy() - 30.0
    assert 0.3 < v.std() < 0.7  # N(0, 0.5) reset draw
    # the draw itself: 0.5 * Box-Muller(Philox4x32-10(seed, env, episode)), oracle restatement
    ref = 0.5 * O.normal_draw(9, np.arange(B), 2)
    assert np.max(np.abs(v - ref)) < 1e-5  # hardware fp32 log2/cos vs numpy fp32


def test_large_batch_properties():
    """Full-size batch (262144 = config 4): every QP solved, KKT conditions hold
    on the normalised rows, the safe action is inside the safe box."""
    from rcbf_amd import _lib
    B = 262144
    rng = np.random.default_rng(11)
    x, t, st = _cars_states(4096, 12)
    x = np.tile(x, (B // 4096, 1)) + rng.normal(0, 0.05, (B, 10))
    env = _env("SimulatedCars")
    layer = _layer(env, 20.0)
    xs, u = dev(x), dev(rng.uniform(-1, 1, (B, 1)))
    sg = dev(np.tile(np.array(O.MAX_STD["SimulatedCars"]), (B, 1)))
    mu = torch.zeros_like(sg)
    fin = layer.get_safe_action(xs, u, mu, sg)
    assert torch.isfinite(fin).all() and fin.abs().max() <= 10.0
    P, q, G, h = layer.get_cbf_qp_constraints(xs, u, mu, sg)
    Gn, hn, _ = O.normalize_rows(G.cpu().numpy(), h.cpu().numpy())
    zb = torch.empty(B, 2, device="cuda")
    lam = torch.empty(B, 4, dtype=torch.float64, device="cuda")
    stt = torch.empty(B, dtype=torch.int32, device="cuda")
    import ctypes
    Gd, hd = dev(Gn), dev(hn)  # keep the device copies alive until the kernel has run
    rc = _lib.load().rcbf_qp_solve(ctypes.byref(layer._prm), B, 2, 4, _lib.ptr(P), _lib.ptr(q), _lib.ptr(Gd),
                                   _lib.ptr(hd), 0, _lib.ptr(zb), _lib.ptr(lam), _lib.ptr(stt), None,
                                   _lib.stream_of(torch.device("cuda")))
    torch.cuda.synchronize()
    assert rc == 0 and int(stt.max().item()) == 0
    z = zb.double().cpu().numpy(); lm = lam.cpu().numpy()
    Pd = np.array([np.float32(0.1), np.float32(10.0)], np.float64)
    viol = np.einsum("bmn,bn->bm", Gn.astype(np.float64), z) - hn
    assert viol.max() <= 1e-5                                  # primal feasibility (fp32 z)
    assert lm.min() >= 0                                       # dual feasibility
    stat = Pd * z + np.einsum("bmn,bm->bn", Gn.astype(np.float64), lm)
    assert np.abs(stat).max() <= 1e-4 * (1 + np.abs(lm).max())  # stationarity
    assert np.abs(lm * viol).max() <= 1e-4                      # complementarity


# ----------------------------------------------------------------------------
# failure paths (diff_cbf_qp.py:141-143, cbf_qp.py:279-281)
# ----------------------------------------------------------------------------
@pytest.mark.parametrize("solver", [0, 1, 2])
def test_nan_input_raises_qp_failed(golden, solver):
    d = golden("cars_layer")
    layer = _layer(_env("SimulatedCars"), float(d["gamma_b"]), solver)
    x, u, mu, sg = (dev(d["prior" + k][:64]) for k in ("_x", "_u", "_mu", "_sigma"))
    x[5, 4] = float("nan")
    with pytest.raises(Exception, match="QP Failed to solve"):
        layer.get_safe_action(x, u, mu, sg)
    P, q, G, h = layer.get_cbf_qp_constraints(x, u, mu, sg)
    with pytest.raises(Exception, match="QP Failed to solve"):
        layer.solve_qp(P, q, G, h)
    x[5, 4] = 1.0  # a clean batch solves again on the same layer
    assert torch.isfinite(layer.get_safe_action(x, u, mu, sg)).all()


def test_fused_step_failure_flag_and_status():
    from rcbf_amd.envs import BatchedSimulatedCarsEnv
    B = 256
    x, t, st = _cars_states(B, 31)
    x[17, 6] = np.nan
    env = BatchedSimulatedCarsEnv(B)
    env.load_state(x, t, st)
    layer = _layer(env, 20.0)
    outs = env.make_outputs()
    env.safe_step(dev(np.zeros((B, 1))), layer, auto_reset=False, outputs=outs)
    with pytest.raises(Exception, match="QP Failed to solve"):
        env.check_failures()
    env.check_failures()  # the flag was cleared by the raise
    u = outs["u"].cpu().numpy()
    assert np.isfinite(np.delete(u, 17, axis=0)).all()


def test_cascade_nan_raises_value_error():
    from rcbf_amd.cbf_qp import CascadeCBFLayer
    env = _env("SimulatedCars")
    layer = CascadeCBFLayer(env, gamma_b=20.0, k_d=3.0)
    s = np.array([34.0, 30.0, 28.0, 30.0, 22.0, 30.0, 16.0, 35.0, 10.0, 30.0])
    assert np.all(np.isfinite(layer.get_u_safe(np.array([0.5]), s, np.zeros(10), np.zeros(10))))
    s[3] = np.nan  # car 1's velocity does not enter the cars CBF rows (cbf_qp.py:155-240): no failure
    assert np.all(np.isfinite(layer.get_u_safe(np.array([0.5]), s, np.zeros(10), np.zeros(10))))
    s[6] = np.nan  # car 3's position does
    with pytest.raises(ValueError):
        layer.get_u_safe(np.array([0.5]), s, np.zeros(10), np.zeros(10))


@pytest.mark.parametrize("mode", ["SimulatedCars", "Unicycle"])
def test_pdipm_agrees_with_exact_solver_at_scale(mode):
    """The qpth-style IPM (solver 1) returns the exact optimum on 65536
    SURVEY 8(d) states: stalled iterates (qpth's notImprovedLim exit) that fail
    the KKT certificate are re-solved exactly (found at x = (-1.45, -1.35,
    3.0): the stalled iterate was 3.0 off)."""
    rng = np.random.default_rng(0)
    B = 65536
    if mode == "Unicycle":
        hz = O.UNI["hazards"][:3]
        env = _env(mode, hz)
        x = np.stack([rng.uniform(-3, 3, B), rng.uniform(-3, 3, B), rng.uniform(-np.pi, np.pi, B)], 1)
        s32 = O.get_state_f32(mode, O.uni_obs(x).astype(np.float32))
    else:
        env = _env(mode)
        xs, _, _ = _cars_states(B, 40)
        s32 = O.get_state_f32(mode, O.cars_obs(xs).astype(np.float32))
    mu, sg = O.predict_disturbance_prior(mode, B)
    u = rng.uniform(-1, 1, (B, env.n_u)).astype(np.float32)
    args = [dev(v) for v in (s32, u, mu.astype(np.float32), sg.astype(np.float32))]
    a = _layer(env, 20.0, 0).get_safe_action(*args)
    b = _layer(env, 20.0, 1).get_safe_action(*args)
    assert float((a - b).abs().max()) <= 1e-5


@pytest.mark.parametrize("name,mode", [("cars", "SimulatedCars"), ("uni3", "Unicycle")])
def test_sac_update_config5_golden(golden, name, mode):
    """Config 5 (B = 4096, forward + backward) against the reference's own
    RCBF_SAC.get_safe_action (sac_cbf.py:218-238) run on the same fp32
    observations: safe action and d final / d action <= 1e-5."""
    from rcbf_amd.dynamics import DynamicsModel
    from rcbf_amd.sac_cbf import get_safe_action
    d = golden("sac_update_config5")
    env = _env(mode, d.get(f"{name}_hazards"))
    layer = _layer(env, float(d["gamma_b"]))
    dyn = DynamicsModel(env, Args())
    a = dev(d[f"{name}_action"]).requires_grad_(True)
    out = get_safe_action(layer, dev(d[f"{name}_obs32"]), a, dyn)
    (out * dev(d[f"{name}_w"])).sum().backward()
    assert rel(out.detach().cpu().numpy(), d[f"{name}_final"]) <= 1e-5
    assert rel(a.grad.cpu().numpy(), d[f"{name}_grad_action"]) <= 1e-5


@pytest.mark.parametrize("name,mode", [("cars", "SimulatedCars"), ("uni3", "Unicycle"), ("uni5", "Unicycle")])
def test_f64_build_variant_golden(golden, name, mode):
    """The fp32-built HIP layer against the reference built in fp64
    (torch.set_default_dtype(float64)), B = 4096: within 1e-4 (the build
    precision alone moves the action by up to ~1e-4), and equal to
    the fp32 oracle on the same inputs within 1e-5."""
    d = golden("layer_f64_build")
    g = lambda k: d[f"{name}_{k}"]  # noqa: E731
    env = _env(mode, d.get(f"{name}_hazards"))
    layer = _layer(env, float(d["gamma_b"]))
    x, u, mu, sg = (g(k).astype(np.float32) for k in ("x", "u", "mu", "sigma"))
    fin = layer.get_safe_action(dev(x), dev(u), dev(mu), dev(sg)).cpu().numpy()
    assert rel(fin, g("final")) <= 1e-4
    ref32, _ = O.safe_action_diff(mode, x, u, mu, sg, float(d["gamma_b"]), hazards=d.get(f"{name}_hazards"))
    assert rel(fin, ref32) <= 1e-5


@pytest.mark.parametrize("mode", ["SimulatedCars", "Unicycle"])
def test_torch_op_matches_python_function(mode, monkeypatch):
    """The C++ autograd op (csrc/rcbf_torch_op.cpp) and the Python
    autograd.Function launch the same kernels: bit-identical safe actions and
    d/d action, through RCBF_SAC.get_safe_action (obs input) and
    CBFQPLayer.get_safe_action (state input); both raise the reference's
    Exception('QP Failed to solve') on a NaN state and recover after it."""
    from rcbf_amd import _lib
    from rcbf_amd.dynamics import DynamicsModel
    from rcbf_amd.sac_cbf import get_safe_action
    assert _lib.torch_op() is not None, "_rcbf_torch not built (run __graft_entry__.build())"
    rng = np.random.default_rng(9)
    B = 512
    hz = O.UNI["hazards"][:3] if mode == "Unicycle" else None
    env = _env(mode, hz)
    layer = _layer(env, 20.0)
    dyn = DynamicsModel(env, Args())
    if mode == "SimulatedCars":
        x, _, _ = _cars_states(B, 4)
        obs = O.cars_obs(x).astype(np.float32)
    else:
        x = np.stack([rng.uniform(-3, 3, B), rng.uniform(-3, 3, B), rng.uniform(-np.pi, np.pi, B)], 1)
        obs = O.uni_obs(x).astype(np.float32)
    s32 = O.get_state_f32(mode, obs)
    mu, sg = (v.astype(np.float32) for v in O.predict_disturbance_prior(mode, B))
    u = rng.uniform(-1, 1, (B, env.n_u)).astype(np.float32)
    w = dev(rng.normal(0, 1, (B, env.n_u)))

    def run():
        a = dev(u).requires_grad_(True)
        o1 = get_safe_action(layer, dev(obs), a, dyn)
        (o1 * w).sum().backward()
        b = dev(u).requires_grad_(True)
        o2 = layer.get_safe_action(dev(s32), b, dev(mu), dev(sg))
        (o2 * w).sum().backward()
        return [o1.detach(), a.grad, o2.detach(), b.grad]

    cpp = run()
    monkeypatch.setattr(_lib, "_torch_op", None)
    py = run()
    monkeypatch.undo()
    for p, q in zip(cpp, py):
        assert torch.equal(p, q)
    bad = s32.copy()
    bad[3, 2] = np.nan
    with pytest.raises(Exception, match="QP Failed to solve"):
        layer.get_safe_action(dev(bad), dev(u), dev(mu), dev(sg))
    assert torch.equal(layer.get_safe_action(dev(s32), dev(u), dev(mu), dev(sg)), cpp[2])


@pytest.mark.parametrize("mode", ["SimulatedCars", "Unicycle"])
def test_torch_op_backward_outlives_the_layer(mode):
    """The autograd graph keeps its own copy of the layer's parameter block
    (csrc/rcbf_torch_op.cpp): a loss built with a temporary CBFQPLayer that is
    dropped (and its memory reused) before loss.backward() still gives the
    gradient of a live layer, bit for bit."""
    import ctypes
    import gc
    from rcbf_amd import _lib
    assert _lib.torch_op() is not None, "_rcbf_torch not built (run __graft_entry__.build())"
    rng = np.random.default_rng(21)
    B = 1024
    hz = O.UNI["hazards"][:3] if mode == "Unicycle" else None
    env = _env(mode, hz)
    if mode == "SimulatedCars":
        x, _, _ = _cars_states(B, 6)
        s32 = O.get_state_f32(mode, O.cars_obs(x).astype(np.float32))
    else:
        x = np.stack([rng.uniform(-3, 3, B), rng.uniform(-3, 3, B), rng.uniform(-np.pi, np.pi, B)], 1)
        s32 = O.get_state_f32(mode, O.uni_obs(x).astype(np.float32))
    mu, sg = (dev(v.astype(np.float32)) for v in O.predict_disturbance_prior(mode, B))
    u = rng.uniform(-1, 1, (B, env.n_u)).astype(np.float32)
    w = dev(rng.normal(0, 1, (B, env.n_u)))
    keep = _layer(env, 20.0)
    a = dev(u).requires_grad_(True)
    (keep.get_safe_action(dev(s32), a, mu, sg) * w).sum().backward()
    tmp = _layer(env, 20.0)
    b = dev(u).requires_grad_(True)
    loss = (tmp.get_safe_action(dev(s32), b, mu, sg) * w).sum()
    del tmp
    gc.collect()
    junk = [(ctypes.c_ubyte * ctypes.sizeof(_lib.RcbfParams))(*([0xFF] * ctypes.sizeof(_lib.RcbfParams)))
            for _ in range(64)]
    loss.backward()
    del junk
    assert torch.equal(a.grad, b.grad)


@pytest.mark.parametrize("mode", ["SimulatedCars", "Unicycle"])
@pytest.mark.parametrize("B", [1, 7, 256, 300])
def test_env_step_sync_matches_device_step(mode, B):
    """rcbf_env_step_sync (the gym env.step path, main.py:95): action read
    from and results written to pinned host memory; for B <= 256 the call
    returns on the kernel's completion word, above that on the stream.  Its
    packed obs64 / reward / cost / done / goal equal rcbf_env_step on device
    buffers from the same state, and the completion word holds the call's
    sequence number afterwards (so the outputs were complete when it returned)."""
    import ctypes
    from rcbf_amd import _lib
    from rcbf_amd.envs import BatchedSimulatedCarsEnv, BatchedUnicycleEnv
    lib = _lib.load()
    mk = BatchedSimulatedCarsEnv if mode == "SimulatedCars" else BatchedUnicycleEnv
    a_env, b_env = mk(B, seed=5), mk(B, seed=5)
    rng = np.random.default_rng(B)
    if mode == "SimulatedCars":
        st = rng.integers(250, 300, B).astype(np.int32)
        st[0] = 299  # env 0's episode ends (auto-reset on)
        a_env.reset(noise=rng.normal(0, 0.5, B)); a_env.step_count.copy_(torch.as_tensor(st, device="cuda"))
    else:
        x0 = np.stack([rng.uniform(-3, 3, B), rng.uniform(-3, 3, B), rng.uniform(-np.pi, np.pi, B)], 1)
        st = rng.integers(990, 1000, B).astype(np.int32)
        st[0] = 999  # env 0's episode ends (auto-reset on)
        a_env.load_state(x0, np.linalg.norm(x0[:, :2] - 2.5, axis=1), st)
    b_env.load_state(a_env.state_numpy(), a_env.aux.cpu().numpy(), a_env.step_count.cpu().numpy().astype(np.int32))
    b_env.episode.copy_(a_env.episode)
    n_o, n_u = a_env.n_o, a_env.n_u
    act = rng.uniform(-1, 1, (B, n_u)).astype(np.float32)
    W = (B * (8 * (n_o + 2) + 2) + 7) & ~7
    pk, ah = ctypes.c_void_p(), ctypes.c_void_p()
    assert lib.rcbf_host_alloc(W + 8, ctypes.byref(pk)) == 0 and lib.rcbf_host_alloc(4 * B * n_u, ctypes.byref(ah)) == 0
    try:
        ctypes.memmove(ah.value, act.ctypes.data, act.nbytes)
        word = ctypes.c_uint32.from_address(pk.value + W)
        word.value = 0
        rc = lib.rcbf_env_step_sync(ctypes.byref(a_env._prm_env), B, _lib.ptr(a_env.x), _lib.ptr(a_env.aux),
                                    _lib.ptr(a_env.step_count), _lib.ptr(a_env.episode), ah, 0, pk, 1,
                                    a_env._rng_seed(), a_env.env_offset, _lib.stream_of(torch.device("cuda")))
        assert rc == 0
        raw = (ctypes.c_char * W).from_address(pk.value).raw
        seq = word.value
        obs = np.frombuffer(raw, np.float64, B * n_o).reshape(B, n_o)
        rew = np.frombuffer(raw, np.float64, B, 8 * B * n_o)
        cost = np.frombuffer(raw, np.float64, B, 8 * B * (n_o + 1))
        done = np.frombuffer(raw, np.uint8, B, 8 * B * (n_o + 2))
        goal = np.frombuffer(raw, np.uint8, B, 8 * B * (n_o + 2) + B)
    finally:
        torch.cuda.synchronize()
        lib.rcbf_host_free(pk)
        lib.rcbf_host_free(ah)
    _, r2, d2, info = b_env.step(dev(act), auto_reset=True, obs64=True)
    torch.cuda.synchronize()
    assert B > 256 or seq != 0
    assert np.array_equal(obs, info["obs64"].cpu().numpy())
    assert np.array_equal(rew, r2.cpu().numpy()) and np.array_equal(cost, info["cost"].cpu().numpy())
    assert np.array_equal(done.astype(bool), d2.cpu().numpy()) and np.array_equal(goal.astype(bool),
                                                                                     info["goal_met"].cpu().numpy())
    assert np.array_equal(a_env.state_numpy(), b_env.state_numpy())
    assert done[0]
