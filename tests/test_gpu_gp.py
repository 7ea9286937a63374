"""GP disturbance posterior on the GPU through the C-ABI
(rcbf_gp_predict) vs the numpy oracle's exact posterior (oracle.gp_predict).
Tolerances (fp32 MFMA products and accumulation, as the reference's fp32
gpytorch model): mean |err| <= 2e-4 max|mean|; predictive std relative
<= 1e-4 (the latent variance s - k'C^-1 k cancels in fp32; measured r01:
mean <= 4e-5, std <= 3e-6 at N = 3000)."""
import types

import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _data(rng, N, n_s):
    tx = rng.normal(0, 1, (N, n_s)) * rng.uniform(0.5, 2.0, n_s)
    ty = 0.1 * np.sin(tx @ rng.normal(0, 1, (n_s, n_s))) + rng.normal(0, 0.05, (N, n_s))
    return tx, ty


def _check(m, s, mo, so):
    assert np.all(np.isfinite(m)) and np.all(np.isfinite(s))
    assert np.max(np.abs(m - mo)) <= 2e-4 * np.max(np.abs(mo)) + 1e-7
    assert np.max(np.abs(s - so) / so) <= 1e-4


@pytest.mark.parametrize("n_s,N,B", [(3, 300, 1), (3, 1100, 4096), (10, 1000, 200), (10, 3000, 257),
                                     (10, 3000, 1), (10, 1000, 5), (3, 300, 8), (3, 1100, 2),
                                     (3, 40, 1), (10, 64, 1), (3, 33, 8), (10, 65, 1)])
def test_gp_predict_vs_oracle(n_s, N, B):
    from rcbf_amd import gp
    rng = np.random.default_rng(n_s * N + B)
    tx, ty = _data(rng, N, n_s)
    hyper = [(rng.uniform(0.8, 2.5), rng.uniform(0.05, 0.5), rng.uniform(0.01, 0.2)) for _ in range(n_s)]
    model = gp.GPDisturbanceModel(tx, ty, hyper)
    q = (rng.normal(0, 1, (B, n_s)) * tx.std(0)).astype(np.float32)
    mean, std = model.predict(torch.as_tensor(q, device="cuda"))
    mo, so = O.gp_predict(q, tx, ty, hyper)
    _check(mean.cpu().numpy(), std.cpu().numpy(), mo, so)


def test_gp_predict_low_rank():
    """A Lanczos inverse root of size 64 (LOVE's algorithm, forced size) vs
    the oracle's restatement on the same start vectors."""
    from rcbf_amd import gp
    rng = np.random.default_rng(5)
    tx, ty = _data(rng, 500, 3)
    hyper = [(1.2, 0.3, 0.05)] * 3
    model = gp.GPDisturbanceModel(tx, ty, hyper, rank=64)
    q = (rng.normal(0, 1, (1000, 3)) * tx.std(0)).astype(np.float32)
    mean, std = model.predict(torch.as_tensor(q, device="cuda"))
    mo, so = O.gp_predict(q, tx, ty, hyper, rank=64, love_init=model.love_init.numpy())
    _check(mean.cpu().numpy(), std.cpu().numpy(), mo, so)


def test_gp_predict_love_default_vs_oracle():
    """The reference's own prediction algorithm at its gp_model_size (3000,
    main.py:247): gpytorch's fast_pred_var takes a rank-100 Lanczos inverse
    root above 800 points (gp_model.py:97-99, restated in oracle.love_inv_root;
    parity vs gpytorch unpinned).  The device factor from the same start
    vectors, through every path (GEMV B <= 8, split-K, single pass), meets
    the oracle at the same bars as the exact posterior; and LOVE's std is the
    one-sided approximation (never below exact, by more than the fp32 bar)."""
    from rcbf_amd import gp
    rng = np.random.default_rng(31)
    tx, ty = _data(rng, 3000, 10)
    hyper = [(rng.uniform(0.8, 2.5), rng.uniform(0.05, 0.5), rng.uniform(0.01, 0.2)) for _ in range(10)]
    assert gp.love_rank(3000) == 100
    model = gp.GPDisturbanceModel(tx, ty, hyper, rank=gp.love_rank(3000))
    assert model.r == 100 and model._m.C_pad == 128
    sizes = [1, 3, 8, 256, 1000]
    q = (rng.normal(0, 1, (sum(sizes), 10)) * tx.std(0)).astype(np.float32)
    mo, so = O.gp_predict(q, tx, ty, hyper, rank=100, love_init=model.love_init.numpy())
    _, se = O.gp_predict(q, tx, ty, hyper)
    b0 = 0
    for B in sizes:
        sl = slice(b0, b0 + B)
        mean, std = model.predict(torch.as_tensor(q[sl], device="cuda"))
        _check(mean.cpu().numpy(), std.cpu().numpy(), mo[sl], so[sl])
        assert np.all(std.cpu().numpy() >= se[sl] * (1 - 1e-4)), B
        b0 += B


def test_dynamics_model_love_fit_and_predict():
    """DynamicsModel's default variance setting above 800 points: the fit
    builds LOVE's rank-100 factor and predict_disturbance runs it on the
    device (vs the oracle on the model's own start vectors)."""
    from rcbf_amd.dynamics import DynamicsModel
    env = types.SimpleNamespace(dynamics_mode="Unicycle", dt=0.02)
    dm = DynamicsModel(env, types.SimpleNamespace(cuda=True, gp_model_size=1000))
    rng = np.random.default_rng(12)
    x = np.stack([rng.uniform(-3, 3, 1000), rng.uniform(-3, 3, 1000), rng.uniform(-np.pi, np.pi, 1000)], 1)
    u = rng.uniform(-1, 1, (1000, 2))
    nx = O.predict_next_state_prior("Unicycle", x, u) + 0.02 * (0.05 * np.sin(x) + rng.normal(0, 0.02, x.shape))
    dm.append_transition(x, u, nx)
    gpm = dm.disturb_estimators
    assert gpm.rank == 100 and gpm.love_init is not None and gpm.r <= 100
    qs = rng.normal(0, 1, (257, 3)).astype(np.float32)
    mean, std = dm.predict_disturbance(torch.as_tensor(qs, device="cuda"))
    # the mean weights are gpytorch's eval-mode CG iterate (DynamicsModel's default, checked against the
    # oracle's restatement on the CPU in tests/test_gp_host.py): the posterior kernels are checked on them
    assert dm.gp_mean == "cg" and gpm.mean_solve == "cg"
    mo, so = O.gp_predict(qs, dm.train_x, dm.train_y, gpm.hyper, rank=100, love_init=gpm.love_init.numpy(),
                          alpha=gpm.alpha.cpu().numpy())
    _check(mean.cpu().numpy(), std.cpu().numpy(), mo, so)


def test_dynamics_model_gp_fit_and_safe_action():
    """The reference configuration end to end: DynamicsModel.append_transition
    fills the history and fits the GPs (gpytorch-style training restated,
    oracle.gp_fit), predict_disturbance runs the kernel, and the SAC-update
    safe action (rcbf_amd.sac_cbf.get_safe_action) consumes the GP mean/std."""
    from rcbf_amd.dynamics import DynamicsModel
    from rcbf_amd.diff_cbf_qp import CBFQPLayer
    from rcbf_amd.envs import BatchedUnicycleEnv
    from rcbf_amd.sac_cbf import get_safe_action
    hz = O.UNI["hazards"][:3]
    env = BatchedUnicycleEnv(4, hazards_locations=hz)
    args = types.SimpleNamespace(cuda=True, gp_model_size=300)
    dm = DynamicsModel(env, args)
    rng = np.random.default_rng(9)
    x = np.stack([rng.uniform(-3, 3, 300), rng.uniform(-3, 3, 300), rng.uniform(-np.pi, np.pi, 300)], 1)
    u = rng.uniform(-1, 1, (300, 2))
    nx = O.predict_next_state_prior("Unicycle", x, u) + 0.02 * (0.05 * np.sin(x) + rng.normal(0, 0.02, x.shape))
    dm.append_transition(x, u, nx)
    assert dm.disturb_estimators is not None and dm.history_counter == 300
    hyper_o = O.gp_fit(dm.train_x, dm.train_y, O.MAX_STD["Unicycle"])
    assert np.allclose(np.array(dm.disturb_estimators.hyper), np.array(hyper_o), rtol=1e-6)
    B = 256
    xs = np.stack([rng.uniform(-3, 3, B), rng.uniform(-3, 3, B), rng.uniform(-np.pi, np.pi, B)], 1)
    obs = O.uni_obs(xs).astype(np.float32)
    s32 = O.get_state_f32("Unicycle", obs)
    mean, std = dm.predict_disturbance(torch.as_tensor(s32, device="cuda"))
    mo, so = O.gp_predict(s32, dm.train_x, dm.train_y, dm.disturb_estimators.hyper)
    _check(mean.cpu().numpy(), std.cpu().numpy(), mo, so)
    layer = CBFQPLayer(env, args, gamma_b=20.0)
    ua = rng.uniform(-1, 1, (B, 2)).astype(np.float32)
    out = get_safe_action(layer, torch.as_tensor(obs, device="cuda"), torch.as_tensor(ua, device="cuda"), dm)
    fin, _ = O.safe_action_diff("Unicycle", s32, ua, mean.cpu().numpy(), std.cpu().numpy(), 20.0, hazards=hz)
    assert np.max(np.abs(out.cpu().numpy() - fin)) <= 1e-4


def test_save_load_disturbance_models_round_trip(tmp_path):
    """main.py:136,183: save_disturbance_models then load_disturbance_models in
    a fresh DynamicsModel restores the same GP posterior (bit-equal)."""
    from rcbf_amd.dynamics import DynamicsModel
    env = types.SimpleNamespace(dynamics_mode="Unicycle", dt=0.02)
    args = types.SimpleNamespace(cuda=True, gp_model_size=200)
    dm = DynamicsModel(env, args)
    rng = np.random.default_rng(4)
    x = rng.normal(0, 1, (200, 3)); u = rng.uniform(-1, 1, (200, 2))
    nx = O.predict_next_state_prior("Unicycle", x, u) + 0.02 * (0.05 * np.sin(x) + rng.normal(0, 0.02, x.shape))
    dm.append_transition(x, u, nx)
    q = torch.as_tensor(rng.normal(0, 1, (64, 3)), dtype=torch.float32, device="cuda")
    m0, s0 = dm.predict_disturbance(q)
    dm.save_disturbance_models(str(tmp_path))
    dm2 = DynamicsModel(env, args)
    dm2.load_disturbance_models(str(tmp_path))
    m1, s1 = dm2.predict_disturbance(q)
    assert torch.equal(m0, m1) and torch.equal(s0, s1)
    assert dm2.disturb_estimators.hyper == dm.disturb_estimators.hyper


def test_gp_split_k_matches_single_pass():
    """Small grids take the split-K path (training rows split over workgroups,
    raw Q tiles summed in fixed order by k_gp_combine); a large batch of the
    same queries (B = 8192) takes the single-pass path.  Both meet the oracle
    bar (mean 2e-4 max|mean|, std 1e-4)."""
    from rcbf_amd import gp
    rng = np.random.default_rng(21)
    tx, ty = _data(rng, 3000, 10)
    hyper = [(rng.uniform(0.8, 2.5), rng.uniform(0.05, 0.5), rng.uniform(0.01, 0.2)) for _ in range(10)]
    model = gp.GPDisturbanceModel(tx, ty, hyper)
    qn = (rng.normal(0, 1, (8192, 10)) * tx.std(0)).astype(np.float32)
    q = torch.as_tensor(qn, device="cuda")
    m_big, s_big = model.predict(q)
    mo, so = O.gp_predict(qn[:256], tx, ty, hyper)
    # This random fit is ill-conditioned (small noise, N = 3000 in 10-D: large
    # alternating alpha).  The single pass takes the mean from a per-lane fp64
    # sum of A x alpha (r04; one fp32 MFMA accumulator over 1 500 k-steps lost
    # 3.2e-4 max|mean| here), so it meets the same bar as every other path.
    m_bg, s_bg = m_big[:256].cpu().numpy(), s_big[:256].cpu().numpy()
    _check(m_bg, s_bg, mo, so)
    m_s, s_s = model.predict(q[:256].contiguous())
    _check(m_s.cpu().numpy(), s_s.cpu().numpy(), mo, so)
    m_1, s_1 = model.predict(q[:1].contiguous())  # B = 1: the most splits
    assert np.max(np.abs(m_1.cpu().numpy() - mo[:1])) <= 2e-4 * np.max(np.abs(mo))
    assert np.max(np.abs(s_1.cpu().numpy() - so[:1]) / so[:1]) <= 1e-4


@pytest.mark.parametrize("B", [1, 5, 256, 1000, 4096])
def test_gp_upper_triangular_skip_is_exact(B):
    """The exact posterior's factor R = L^-T is upper triangular, so the
    kernels skip the training rows past each column block (rcbf_gp_model
    flags RCBF_GP_RT_UPPER): the skipped terms are exact zeros, so the single
    pass (B = 4096) and the GEMV path (B <= 8) equal the dense product's
    outputs bit for bit.  Split-K (B = 256, 1000) splits each block's own row
    range evenly, so its fp32 partial sums group differently: within 1e-6."""
    from rcbf_amd import _lib, gp
    rng = np.random.default_rng(B)
    tx, ty = _data(rng, 1100, 10)
    model = gp.GPDisturbanceModel(tx, ty, [(1.3, 0.2, 0.05)] * 10)
    assert model._m.flags == _lib.GP_RT_UPPER
    lR = model.logical_Rt()[:, :, :model.r].cpu().numpy()
    assert not np.any(np.tril(np.ones(lR.shape[1:], bool), -1)[None] & (lR != 0))  # zero below the diagonal
    q = torch.as_tensor((rng.normal(0, 1, (B, 10)) * tx.std(0)).astype(np.float32), device="cuda")
    m_t, s_t = model.predict(q)
    model._m.flags = 0
    m_d, s_d = model.predict(q)
    if B in (256, 1000):
        assert torch.allclose(m_t, m_d, rtol=1e-6, atol=1e-6 * m_d.abs().max().item())
        assert torch.allclose(s_t, s_d, rtol=1e-6, atol=0)
    else:
        assert torch.equal(m_t, m_d) and torch.equal(s_t, s_d)


def test_gp_predict_low_rank_split_k():
    """rank 100 (the root-decomposition size of gpytorch's fast_pred_var,
    gp_model.py:97): one 128-column block per GP, so B = 256 runs split-K."""
    from rcbf_amd import gp
    rng = np.random.default_rng(8)
    tx, ty = _data(rng, 1200, 3)
    hyper = [(1.1, 0.25, 0.04), (1.6, 0.4, 0.08), (0.9, 0.2, 0.02)]
    model = gp.GPDisturbanceModel(tx, ty, hyper, rank=100)
    q = (rng.normal(0, 1, (256, 3)) * tx.std(0)).astype(np.float32)
    mean, std = model.predict(torch.as_tensor(q, device="cuda"))
    mo, so = O.gp_predict(q, tx, ty, hyper, rank=100, love_init=model.love_init.numpy())
    _check(mean.cpu().numpy(), std.cpu().numpy(), mo, so)


@pytest.mark.parametrize("n_s,cols,B", [(10, (5, 7, 9), 4096), (10, (5, 7, 9), 3), (3, (0, 1, 2), 1000)])
def test_gp_predict_cols_equals_rows(n_s, cols, B):
    """rcbf_gp_predict_cols writes, in the column layout the fused step reads
    (rcbf_safe_step_cols), exactly the values rcbf_gp_predict writes as rows;
    the rows outputs are optional; and a fused step fed the columns equals one
    fed the rows, bit for bit."""
    from rcbf_amd import gp
    rng = np.random.default_rng(B + n_s)
    tx, ty = _data(rng, 600, n_s)
    model = gp.GPDisturbanceModel(tx, ty, [(1.3, 0.2, 0.05)] * n_s)
    q = torch.as_tensor((rng.normal(0, 1, (B, n_s)) * tx.std(0)).astype(np.float32), device="cuda")
    mean, std = model.predict(q)
    mc, sc, mr, sr = model.predict_cols(q, cols, rows=True)
    assert torch.equal(mr, mean) and torch.equal(sr, std)
    assert torch.equal(sc, std[:, list(cols)].t()) and torch.equal(mc, mean[:, list(cols)].t())
    mc2, sc2 = model.predict_cols(q, cols, mean=False)
    assert mc2 is None and torch.equal(sc2, sc)
    if B < 64:
        return
    from rcbf_amd.diff_cbf_qp import CBFQPLayer
    from rcbf_amd.envs import BatchedSimulatedCarsEnv, BatchedUnicycleEnv

    class A:
        cuda = True
    runs = []
    for layout in ("rows", "cols"):
        if n_s == 10:
            env = BatchedSimulatedCarsEnv(B, seed=3)
        else:
            env = BatchedUnicycleEnv(B, seed=3, hazards_locations=O.UNI["hazards"][:3])
            env.load_state(np.stack([rng.uniform(-3, 3, B) * 0 + np.linspace(-3, 3, B), np.linspace(3, -3, B),
                                     np.linspace(-3, 3, B)], 1), np.ones(B), np.zeros(B))
        lay = CBFQPLayer(env, A(), gamma_b=20.0)
        u = torch.linspace(-1, 1, B * env.n_u, device="cuda").reshape(B, env.n_u).contiguous()
        if layout == "rows":
            obs, r, d, o = env.safe_step(u, lay, mean=mean, sigma=std)
        else:
            obs, r, d, o = env.safe_step(u, lay, mean=None if n_s == 10 else mc, sigma=sc, prior_layout="cols")
        env.check_failures()
        runs.append([obs.clone(), r.clone(), o["u"].clone(), env.state.clone()])
    for a, b in zip(*runs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("rank", [100, None])
def test_gp_gemv_handoff_across_calls(rank):
    """The one-launch GEMV (B <= 8) hands its tile partials to the last
    arriving workgroup through write-through stores and arrival counters that
    the consumers reset: 48 back-to-back calls on one workspace, each with
    its own queries (B cycling 1, 2, 3, 8), captured in one hipGraph and
    replayed three times (the third beside GEMMs on another stream, so the
    workgroups arrive unevenly), every output against the oracle -- a stale
    partial or a counter left non-zero would reuse an earlier call's values.
    The counters are zero afterwards."""
    from rcbf_amd import gp
    rng = np.random.default_rng(77 + (rank or 0))
    tx, ty = _data(rng, 1500, 10)
    hyper = [(rng.uniform(0.8, 2.5), rng.uniform(0.05, 0.5), rng.uniform(0.01, 0.2)) for _ in range(10)]
    model = gp.GPDisturbanceModel(tx, ty, hyper, rank=rank)
    sizes = [(1, 2, 3, 8)[j % 4] for j in range(48)]
    q = (rng.normal(0, 1, (sum(sizes), 10)) * tx.std(0)).astype(np.float32)
    qd = torch.as_tensor(q, device="cuda")
    offs = np.concatenate([[0], np.cumsum(sizes)])
    model.predict(qd[:8].contiguous())  # size the workspace for B = 8 before the capture
    ws = model._workspace(8)[0]
    xs = [qd[offs[j]:offs[j + 1]].clone() for j in range(48)]
    outs = [(torch.empty(sizes[j], 10, device="cuda"), torch.empty(sizes[j], 10, device="cuda")) for j in range(48)]
    import ctypes
    from rcbf_amd import _lib
    lib = _lib.load()
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for j in range(48):
            rc = lib.rcbf_gp_predict(ctypes.byref(model._m), sizes[j], _lib.ptr(xs[j]), _lib.ptr(outs[j][0]),
                                     _lib.ptr(outs[j][1]), _lib.ptr(ws), _lib.stream_of(torch.device("cuda")))
            assert rc == 0
    mo, so = O.gp_predict(q, tx, ty, hyper, rank=rank, love_init=None if rank is None else model.love_init.numpy())
    side = torch.cuda.Stream()
    a = torch.randn(4096, 4096, device="cuda")
    for rep in range(3):
        for o in outs:
            o[0].zero_()
            o[1].zero_()
        torch.cuda.synchronize()
        if rep == 2:  # uneven load (G16): GEMMs on a second stream hold CUs while the 48 calls run
            with torch.cuda.stream(side):
                for _ in range(6):
                    a = (a @ a).clamp_(-1, 1)
        g.replay()
        torch.cuda.synchronize()
        for j in range(48):
            _check(outs[j][0].cpu().numpy(), outs[j][1].cpu().numpy(), mo[offs[j]:offs[j + 1]], so[offs[j]:offs[j + 1]])
    # the arrival counters (one per 128-B line: n_s (n_cb + 1) of them) and the fail word's line lead the
    # workspace and are zero again
    n_ctr = model.n_s * (model._m.C_pad // 128 + 1) * 32 + 64
    assert int(ws.view(torch.int32)[:n_ctr].abs().sum()) == 0
    model.check_failures()


@pytest.mark.parametrize("rank", [100, None])
def test_gp_gemv_poisoned_counter_is_detected_and_reset(rank):
    """a GEMV call that finds a non-zero arrival counter
    (a workspace not zero-filled, an aborted call, two calls sharing one
    workspace) sets the workspace's fail word; check_failures
    (rcbf_gp_workspace_check) raises and zeroes the counters, and the next
    call is correct again (bit-equal to the clean call before the poison)."""
    from rcbf_amd import gp
    rng = np.random.default_rng(5 + (rank or 0))
    tx, ty = _data(rng, 1500, 10)
    hyper = [(rng.uniform(0.8, 2.5), rng.uniform(0.05, 0.5), rng.uniform(0.01, 0.2)) for _ in range(10)]
    model = gp.GPDisturbanceModel(tx, ty, hyper, rank=rank)
    q = torch.as_tensor((rng.normal(0, 1, (1, 10)) * tx.std(0)).astype(np.float32), device="cuda")
    m1, s1 = model.predict(q)
    model.check_failures()
    ws = model._workspace(1)[0]
    n_cb = model._m.C_pad // 128
    # GP 0's first block counter; GP 3's counter (used only by a multi-block factor: the exact posterior)
    for word in [0] + ([(model.n_s * n_cb + 3) * 32] if n_cb > 1 else []):
        ws.view(torch.int32)[word] = 5
        model.predict(q)
        with pytest.raises(RuntimeError, match="arrival counter"):
            model.check_failures()
        m2, s2 = model.predict(q)
        model.check_failures()
        assert torch.equal(m1, m2) and torch.equal(s1, s2)


def test_one_launch_safe_action_reports_a_poisoned_counter():
    """The one-launch select_action call (rcbf_gp_obs_safe_action) on a
    workspace whose first arrival counter is far from zero: no workgroup draws
    the last ticket, the kernel completes without publishing, and the call
    returns RCBF_E_GP_HANDOFF instead of a stale action.  (A counter off by
    less than the block's tile count makes an early arrival the "last" one:
    that call's action is not valid, and only the fail word tells --
    check_failures, run below after both kinds.)  check_failures reports the
    fail word and zeroes the counters; the next call returns the clean action."""
    import types
    from rcbf_amd import gp
    from rcbf_amd.diff_cbf_qp import CBFQPLayer
    from rcbf_amd.envs import SimulatedCarsEnv
    from rcbf_amd.sac_cbf import get_safe_action_host
    rng = np.random.default_rng(21)
    env = SimulatedCarsEnv()
    layer = CBFQPLayer(env, types.SimpleNamespace(cuda=True), gamma_b=20.0)
    tx, ty = _data(rng, 1500, 10)
    hyper = [(rng.uniform(0.8, 2.5), rng.uniform(0.05, 0.5), rng.uniform(0.01, 0.2)) for _ in range(10)]
    dm = types.SimpleNamespace(disturb_estimators=gp.GPDisturbanceModel(tx, ty, hyper, rank=100))
    obs = torch.as_tensor(env.reset(), dtype=torch.float32, device="cuda")
    u = torch.tensor([0.3], device="cuda")
    clean = get_safe_action_host(layer, obs, u, dm)
    gpm = dm.disturb_estimators
    ws = gpm._sa_ws[2]
    ws.view(torch.int32)[0] = 1 << 20
    with pytest.raises(RuntimeError, match="RCBF_E_GP_HANDOFF"):
        get_safe_action_host(layer, obs, u, dm)
    with pytest.raises(RuntimeError, match="arrival counter"):
        gpm.check_failures()
    assert np.array_equal(get_safe_action_host(layer, obs, u, dm), clean)
    ws.view(torch.int32)[0] = 3  # off by a few tiles: a premature "last" arrival, flagged by the fail word
    get_safe_action_host(layer, obs, u, dm)
    with pytest.raises(RuntimeError, match="arrival counter"):
        gpm.check_failures()
    assert np.array_equal(get_safe_action_host(layer, obs, u, dm), clean)
    gpm.check_failures()


def test_gp_workspace_per_stream():
    """GEMV calls on two streams at once use two
    workspaces (GPDisturbanceModel._workspace keys them by stream), so their
    arrival counters never meet: 64 interleaved B = 1 calls on two streams,
    no GPU-side sync between them, each bit-equal to the same query on the
    default stream, and no fail word set."""
    from rcbf_amd import gp
    rng = np.random.default_rng(9)
    tx, ty = _data(rng, 1500, 10)
    hyper = [(rng.uniform(0.8, 2.5), rng.uniform(0.05, 0.5), rng.uniform(0.01, 0.2)) for _ in range(10)]
    model = gp.GPDisturbanceModel(tx, ty, hyper, rank=100)
    q = torch.as_tensor((rng.normal(0, 1, (64, 10)) * tx.std(0)).astype(np.float32), device="cuda")
    want = [model.predict(q[j:j + 1].contiguous()) for j in range(64)]
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    for s in streams:
        s.wait_stream(torch.cuda.current_stream())
    got = []
    for j in range(64):
        with torch.cuda.stream(streams[j % 2]):
            got.append(model.predict(q[j:j + 1].contiguous()))
    torch.cuda.synchronize()
    keys = {k for k in model._ws}
    assert len(keys) == 3  # the default stream's and one per side stream
    for (m1, s1), (m2, s2) in zip(want, got):
        assert torch.equal(m1, m2) and torch.equal(s1, s2)
    model.check_failures()


def test_state_from_obs_kernel_matches_reference_get_state(golden):
    """DynamicsModel.get_state on device fp32 observations is one launch
    (rcbf_state_from_obs); it returns the reference's own torch get_state
    output (dynamics.py:190-232, the committed golden) bit for bit, and the
    torch path on the same rows, for 4 096 random unicycle angles too."""
    from rcbf_amd.dynamics import DynamicsModel
    d = golden("dynamics")
    for nm, mode in (("cars", "SimulatedCars"), ("uni", "Unicycle")):
        dm = DynamicsModel(types.SimpleNamespace(dynamics_mode=mode, dt=0.02), types.SimpleNamespace(cuda=True))
        s = dm.get_state(torch.as_tensor(d[nm + "_obs32"], device="cuda"))
        assert s.dtype == torch.float32 and np.array_equal(s.cpu().numpy(), d[nm + "_state_t"])
        s1 = dm.get_state(torch.as_tensor(d[nm + "_obs32"][0], device="cuda"))  # 1-D in, 1-D out
        assert s1.shape == (dm.n_s,) and np.array_equal(s1.cpu().numpy(), d[nm + "_state_t"][0])
    rng = np.random.default_rng(3)
    th = rng.uniform(-np.pi, np.pi, 4096)
    obs = O.uni_obs(np.stack([rng.uniform(-3, 3, 4096), rng.uniform(-3, 3, 4096), th], 1)).astype(np.float32)
    dm = DynamicsModel(types.SimpleNamespace(dynamics_mode="Unicycle", dt=0.02), types.SimpleNamespace(cuda=True))
    got = dm.get_state(torch.as_tensor(obs, device="cuda")).cpu().numpy()
    assert np.array_equal(got, O.get_state_f32("Unicycle", obs))


@pytest.mark.parametrize("mode,k", [("SimulatedCars", 0), ("Unicycle", 3)])
def test_sac_safe_action_with_gp_is_the_reference_three_calls(mode, k):
    """RCBF_SAC.get_safe_action with a fitted GP (sac_cbf.py:233-236) through
    rcbf_amd.sac_cbf.get_safe_action -- state kernel, GP kernel, one safe-action
    launch reading the posterior rows -- equals the reference's three calls on
    rcbf_amd's surfaces (get_state -> predict_disturbance ->
    CBFQPLayer.get_safe_action) bit for bit, forward and d final / d action,
    at B = 1 (the env step) and B = 256 (the SAC update)."""
    from rcbf_amd import gp
    from rcbf_amd.diff_cbf_qp import CBFQPLayer
    from rcbf_amd.dynamics import DynamicsModel
    from rcbf_amd.envs import BatchedSimulatedCarsEnv, BatchedUnicycleEnv
    from rcbf_amd.sac_cbf import get_safe_action
    rng = np.random.default_rng(19 + k)
    if mode == "SimulatedCars":
        env = BatchedSimulatedCarsEnv(4)
        x = np.tile(np.array([34.0, 30, 28, 30, 22, 30, 16, 35, 10, 30]), (1100, 1)) + rng.normal(0, 1.5, (1100, 10))
    else:
        env = BatchedUnicycleEnv(4, hazards_locations=O.UNI["hazards"][:k])
        x = np.stack([rng.uniform(-3, 3, 1100), rng.uniform(-3, 3, 1100), rng.uniform(-np.pi, np.pi, 1100)], 1)
    n_s = x.shape[1]
    dm = DynamicsModel(env, types.SimpleNamespace(cuda=True, gp_model_size=1100))
    hyper = [(1.3, 0.2, 0.05)] * n_s
    dm.disturb_estimators = gp.GPDisturbanceModel(x, 0.05 * np.sin(x) + rng.normal(0, 0.02, x.shape), hyper,
                                                  rank=gp.love_rank(1100))
    layer = CBFQPLayer(env, types.SimpleNamespace(cuda=True), gamma_b=20.0)
    for B in (1, 256):
        idx = rng.integers(0, 1100, B)
        obs = (O.cars_obs(x[idx]) if mode == "SimulatedCars" else O.uni_obs(x[idx])).astype(np.float32)
        ob = torch.as_tensor(obs, device="cuda")
        ua = torch.as_tensor(rng.uniform(-1, 1, (B, env.n_u)).astype(np.float32), device="cuda")
        w = torch.as_tensor(rng.normal(0, 1, (B, env.n_u)).astype(np.float32), device="cuda")
        u1 = ua.clone().requires_grad_(True)
        out1 = get_safe_action(layer, ob, u1, dm)
        (out1 * w).sum().backward()
        state = dm.get_state(ob)
        mean, sigma = dm.predict_disturbance(state)
        u2 = ua.clone().requires_grad_(True)
        out2 = layer.get_safe_action(state, u2, mean, sigma)
        (out2 * w).sum().backward()
        assert torch.equal(out1.detach(), out2.detach()) and torch.equal(u1.grad, u2.grad), B
        assert bool((out1.detach() != ua).any()) or B == 1  # the filter is active on part of the batch


@pytest.mark.parametrize("mode,k,rank", [("SimulatedCars", 1, "love"), ("Unicycle", 3, "love"), ("Unicycle", 5, "love"),
                                         ("SimulatedCars", 1, "exact"), ("Unicycle", 5, "exact")])
def test_one_launch_safe_action_with_gp_equals_three_launches(mode, k, rank):
    """rcbf_gp_obs_safe_action -- get_state(obs), the GP
    posterior GEMV and the safe action in ONE launch, the action written to
    pinned host memory behind a completion word (sac_cbf.get_safe_action_host)
    -- equals the three-launch path (rcbf_state_from_obs -> rcbf_gp_predict ->
    rcbf_obs_safe_action, itself bit-equal to the reference's three calls)
    bit for bit, over 64 single observations with states spread so the filter
    is active on part of them, for a Lanczos (one column block) and an exact
    (multi-block: the second hand-off level) factor; the posterior rows and
    the counters are checked too."""
    from rcbf_amd import gp
    from rcbf_amd.diff_cbf_qp import CBFQPLayer
    from rcbf_amd.dynamics import DynamicsModel
    from rcbf_amd.envs import BatchedSimulatedCarsEnv, BatchedUnicycleEnv
    from rcbf_amd.sac_cbf import get_safe_action, get_safe_action_host
    rng = np.random.default_rng(31 + k)
    N = 1100
    if mode == "SimulatedCars":
        env = BatchedSimulatedCarsEnv(4)
        x = np.tile(np.array([34.0, 30, 28, 30, 22, 30, 16, 35, 10, 30]), (N, 1)) + rng.normal(0, 1.5, (N, 10))
    else:
        env = BatchedUnicycleEnv(4, hazards_locations=O.UNI["hazards"][:k])
        x = np.stack([rng.uniform(-3, 3, N), rng.uniform(-3, 3, N), rng.uniform(-np.pi, np.pi, N)], 1)
    n_s = x.shape[1]
    dm = DynamicsModel(env, types.SimpleNamespace(cuda=True, gp_model_size=N))
    hyper = [(1.3, 0.2, 0.05)] * n_s
    dm.disturb_estimators = gp.GPDisturbanceModel(x, 0.05 * np.sin(x) + rng.normal(0, 0.02, x.shape), hyper,
                                                  rank=gp.love_rank(N) if rank == "love" else None)
    gpm = dm.disturb_estimators
    layer = CBFQPLayer(env, types.SimpleNamespace(cuda=True), gamma_b=20.0)
    active = 0
    for j in range(64):
        idx = rng.integers(0, N)
        obs = (O.cars_obs(x[idx:idx + 1]) if mode == "SimulatedCars" else O.uni_obs(x[idx:idx + 1])).astype(np.float32)
        ob = torch.as_tensor(obs[0], device="cuda")
        ua = torch.as_tensor(rng.uniform(-1, 1, env.n_u).astype(np.float32), device="cuda")
        ref = get_safe_action(layer, ob, ua, dm).cpu().numpy()
        got = get_safe_action_host(layer, ob, ua, dm)
        assert got.shape == ref.shape and np.array_equal(got, ref), (j, got, ref)
        active += int(not np.array_equal(ref, ua.cpu().numpy()))
    assert active > 0
    # the posterior rows the fused kernel hands to its last stage equal rcbf_gp_predict's
    import ctypes
    from rcbf_amd import _lib
    ob = torch.as_tensor(obs, device="cuda")
    ua = torch.as_tensor(rng.uniform(-1, 1, (1, env.n_u)).astype(np.float32), device="cuda")
    mo, so, uo = torch.empty(1, n_s, device="cuda"), torch.empty(1, n_s, device="cuda"), torch.empty(1, env.n_u, device="cuda")
    ws, stream = gpm._workspace(1)
    rc = _lib.load().rcbf_gp_obs_safe_action(ctypes.byref(layer._prm), ctypes.byref(gpm._m), 1, _lib.ptr(ob), _lib.ptr(ua),
                                             _lib.ptr(mo), _lib.ptr(so), _lib.ptr(uo), None, None, 0, None, None,
                                             _lib.ptr(ws), stream)
    assert rc == 0
    m2, s2 = gpm.predict(dm.get_state(ob))
    torch.cuda.synchronize()
    assert torch.equal(mo, m2) and torch.equal(so, s2)
    assert torch.equal(uo, get_safe_action(layer, ob, ua, dm))
    gpm.check_failures()
    n_ctr = gpm.n_s * (gpm._m.C_pad // 128 + 1) * 32 + 64
    assert int(ws.view(torch.int32)[:n_ctr].abs().sum()) == 0
    # B != 1 and another solver are refused (the wrapper then takes the three launches)
    assert _lib.load().rcbf_gp_obs_safe_action(ctypes.byref(layer._prm), ctypes.byref(gpm._m), 2, _lib.ptr(ob),
                                               _lib.ptr(ua), None, None, _lib.ptr(uo), None, None, 0, None, None,
                                               _lib.ptr(ws), stream) == 1002
