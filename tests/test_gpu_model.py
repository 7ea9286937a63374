"""SURVEY 8f rows 3-4 on the GPU: the model-rollout step kernel against the
reference's own generate_model_rollouts outputs (tests/golden/model_rollouts.npz,
recorded N(0,1) draws replayed), and the device ReplayMemory against the
reference's list semantics."""
import types

import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _env(mode):
    from rcbf_amd.envs import BatchedSimulatedCarsEnv, BatchedUnicycleEnv
    return BatchedSimulatedCarsEnv(4) if mode == "SimulatedCars" else BatchedUnicycleEnv(4)


@pytest.mark.parametrize("nm,mode", [("cars", "SimulatedCars"), ("uni", "Unicycle")])
def test_model_step_vs_reference(golden, nm, mode):
    from rcbf_amd.generate_rollouts import model_step
    d = golden("model_rollouts")
    nobs, r, mask, nt = model_step(_env(mode), d[nm + "_obs"], d[nm + "_act"], d[nm + "_t"], z=d[nm + "_z"])
    assert np.max(np.abs(nobs.cpu().numpy() - d[nm + "_next_obs"])) <= 1e-12
    assert np.max(np.abs(r.cpu().numpy() - d[nm + "_reward"])) <= 1e-12
    assert np.array_equal(mask.cpu().numpy(), d[nm + "_mask"])
    assert np.array_equal(nt.cpu().numpy(), d[nm + "_next_t"])


def test_model_step_philox_noise_and_gp_mean():
    """In-kernel N(0,1) draws are standard normal and keyed by the counter;
    a GP mean/std enters as mu + dt mean, std dt std (oracle)."""
    from rcbf_amd.generate_rollouts import model_step
    rng = np.random.default_rng(4)
    B = 65536
    x = np.stack([rng.uniform(-3, 3, B), rng.uniform(-3, 3, B), rng.uniform(-np.pi, np.pi, B)], 1)
    obs = O.uni_obs(x)
    act = rng.uniform(-1, 1, (B, 2))
    env = _env("Unicycle")
    n1, *_ = model_step(env, obs, act, z=None, seed=5, counter=0)
    n2, *_ = model_step(env, obs, act, z=None, seed=5, counter=0)
    n3, *_ = model_step(env, obs, act, z=None, seed=5, counter=1)
    assert torch.equal(n1, n2) and not torch.equal(n1, n3)
    base, *_ = model_step(env, obs, act, z=np.zeros((B, 3)))
    zhat = ((n1 - base)[:, :2].cpu().numpy()) / (0.02 * 0.2)
    assert abs(zhat.mean()) < 0.02 and abs(zhat.std() - 1.0) < 0.02
    mean = rng.normal(0, 0.1, (B, 3)).astype(np.float32)
    std = rng.uniform(0.01, 0.3, (B, 3)).astype(np.float32)
    z = rng.normal(0, 1, (B, 3))
    nobs, r, mask, nt = model_step(env, obs, act, mean=mean, std=std, z=z)
    on, orr, om, ot = O.model_rollout_step("Unicycle", obs, act, None, z, mean=mean, std=std)
    assert np.max(np.abs(nobs.cpu().numpy() - on)) <= 1e-12 and np.max(np.abs(r.cpu().numpy() - orr)) <= 1e-12


def _assert_standard_normal(st, n):
    """Moment and tail bounds at about 6 standard errors for n samples."""
    se = 1.0 / np.sqrt(n)
    assert abs(st["mean"]) < 6 * se and abs(st["var"] - 1.0) < 6 * np.sqrt(2) * se, st
    assert abs(st["skew"]) < 6 * np.sqrt(6) * se and abs(st["exkurt"]) < 6 * np.sqrt(24) * se, st
    p3, p4 = 2.699796e-3, 6.334248e-5  # P(|z| > 3), P(|z| > 4) of N(0, 1)
    assert abs(st["p3"] - p3) < 6 * np.sqrt(p3 / n) and abs(st["p4"] - p4) < 6 * np.sqrt(p4 / n), st
    assert st["max"] <= np.sqrt(48 * np.log(2)) + 1e-6, st  # 24-bit uniforms: |z| <= 5.768


def test_model_step_draw_moments_tails_and_key():
    """The in-kernel N(0, 1) draws of rcbf_model_step (fp32 Box-Muller on
    24-bit Philox uniforms, hardware log2 / cos / sin) against the reference's
    np.random.normal (generate_rollouts.py:31; fp64, values unpinned): over
    2^20 rows x 4 counters x 2 recoverable components (8.4 M samples) the mean,
    variance, skewness, excess kurtosis and the P(|z| > 3), P(|z| > 4) tails
    sit within 6 standard errors of N(0, 1), and |z| never exceeds the
    truncation bound sqrt(48 ln 2) = 5.768.  The first 4096
    rows equal the oracle's restatement of the keyed draw
    (oracle.model_step_normal) to 2e-5."""
    from rcbf_amd.generate_rollouts import model_step
    rng = np.random.default_rng(6)
    B = 1 << 20
    x = np.stack([rng.uniform(-3, 3, B), rng.uniform(-3, 3, B), rng.uniform(-np.pi, np.pi, B)], 1)
    obs = O.uni_obs(x)
    act = rng.uniform(-1, 1, (B, 2))
    env = _env("Unicycle")
    base, *_ = model_step(env, obs, act, z=np.zeros((B, 3)))
    zs = []
    for counter in range(4):
        n1, *_ = model_step(env, obs, act, z=None, seed=11, counter=counter)
        z = ((n1 - base)[:, :2] / (0.02 * 0.2)).cpu().numpy()  # obs[:, :2] = next x, y = mu + dt sd z
        zs.append(z)
        if counter == 1:
            want = O.model_step_normal(11, np.arange(4096), counter, 3)[:, :2]
            assert np.max(np.abs(z[:4096] - want)) <= 2e-5
    zs = np.concatenate(zs)
    _assert_standard_normal(O.normal_moments(zs), zs.size)


def test_replay_memory_ring_and_sample():
    from rcbf_amd.replay_memory import ReplayMemory
    rng = np.random.default_rng(0)
    mem = ReplayMemory(100, seed=1)
    ref = []  # the reference's list semantics (replay_memory.py:12-21)
    pos = 0
    for n in (30, 50, 45, 7, 130):
        s = rng.normal(size=(n, 10)); a = rng.normal(size=(n, 1)); r = rng.normal(size=n)
        ns = rng.normal(size=(n, 10)); m = rng.integers(0, 2, n).astype(bool); t = rng.normal(size=n)
        mem.batch_push(s, a, r, ns, m, t, t + 0.02)
        for i in range(n):
            rec = np.concatenate([s[i], a[i], [r[i]], ns[i], [float(m[i])], [t[i]], [t[i] + 0.02]])
            if len(ref) < 100:
                ref.append(None)
            ref[pos] = rec
            pos = (pos + 1) % 100
        assert len(mem) == len(ref) and mem.position == pos
    ring = mem._ring.cpu().numpy()
    assert np.array_equal(ring, np.stack(ref))
    S, A, R, NS, M, T, NT = mem.sample(64)
    rows = np.hstack([S, A, R[:, None], NS, M[:, None], T[:, None], NT[:, None]])
    keys = {r.tobytes() for r in np.stack(ref)}
    assert all(r.tobytes() in keys for r in rows) and len({r.tobytes() for r in rows}) == 64  # no replacement
    with pytest.raises(ValueError):
        mem.sample(101)
    mem.push(s[0], a[0], r[0], ns[0], m[0])  # single push without t
    assert len(mem) == 100


def test_generate_model_rollouts_end_to_end():
    """generate_model_rollouts with device memories and a host policy:
    every pushed transition equals the oracle step on the sampled batch."""
    from rcbf_amd.dynamics import DynamicsModel
    from rcbf_amd.generate_rollouts import generate_model_rollouts
    from rcbf_amd.replay_memory import ReplayMemory
    env = _env("SimulatedCars")
    rng = np.random.default_rng(2)
    mem = ReplayMemory(1000, seed=3)
    B = 500
    st = np.tile(np.array([34.0, 30.0, 28.0, 30.0, 22.0, 30.0, 16.0, 35.0, 10.0, 30.0]), (B, 1)) + rng.normal(0, 1, (B, 10))
    obs = st.copy(); obs[:, ::2] /= 100.0; obs[:, 1::2] /= 30.0
    t = np.round(rng.uniform(0, 6, B) / 0.02) * 0.02
    mem.batch_push(obs, rng.uniform(-1, 1, (B, 1)), np.zeros(B), obs, np.ones(B), t, t + 0.02)

    class Agent:
        def select_action(self, o, dm, warmup=False, evaluate=False):
            return np.clip(o[:, 7:8] * 2 - 2, -1, 1)

    mm = ReplayMemory(1000, seed=4)
    dm = DynamicsModel(env, types.SimpleNamespace(cuda=True, gp_model_size=100))
    generate_model_rollouts(env, mm, mem, Agent(), dm, k_horizon=1, batch_size=200)
    assert len(mm) == 200
    S, A, R, NS, M, T, NT = (v.cpu().numpy() for v in mm.sample_tensors(200))
    assert np.allclose(A, np.clip(S[:, 7:8] * 2 - 2, -1, 1))
    # replay each transition through the oracle with the kernel's own draws recovered from NS
    base, rb, mb, tb = O.model_rollout_step("SimulatedCars", S, A, T, np.zeros((200, 10)))
    assert np.max(np.abs(R - rb)) <= 1e-12 and np.array_equal(M, mb) and np.array_equal(NT, tb)
    zh = (NS - base)[:, 1::2] * 30.0 / (0.02 * 0.2)
    assert np.all(np.abs(zh) < 7) and np.array_equal(NS[:, ::2], base[:, ::2])


@pytest.mark.parametrize("nm,mode", [("cars", "SimulatedCars"), ("uni", "Unicycle")])
def test_predict_next_state_device_vs_reference(golden, nm, mode):
    """DynamicsModel.predict_next_state on device tensors (the
    rcbf_predict_next_state kernel) against the reference's own outputs
    (tests/golden/dynamics.npz, use_gps=False: bit-exact), the MAX_STD prior
    (use_gps=True before a fit: dt * MAX_STD, mean 0), a GP posterior's
    (mean, std) entering as next + dt * mean, dt * std, and the 1-D form."""
    from rcbf_amd.dynamics import DynamicsModel
    from rcbf_amd.envs import SimulatedCarsEnv, UnicycleEnv
    d = golden("dynamics")
    env = SimulatedCarsEnv() if mode == "SimulatedCars" else UnicycleEnv()
    dm = DynamicsModel(env, types.SimpleNamespace(cuda=True, gp_model_size=2000))
    dev = torch.device("cuda", 0)
    x = torch.as_tensor(d[nm + "_state_np"], device=dev)
    u = torch.as_tensor(d[nm + "_u"], device=dev)
    t = torch.as_tensor(d[nm + "_t"], device=dev) if nm + "_t" in d else None
    nx, sd, nt = dm.predict_next_state(x, u, t_batch=t, use_gps=False)
    assert nx.is_cuda and np.array_equal(nx.cpu().numpy(), d[nm + "_next"])
    assert not sd.cpu().numpy().any()
    if t is not None:
        assert np.array_equal(nt.cpu().numpy(), d[nm + "_t"] + 0.02)
    # the prior: mean 0, std dt * MAX_STD (the numpy path of the same class agrees)
    nx2, sd2, _ = dm.predict_next_state(x, u, t_batch=t, use_gps=True)
    ref_nx, ref_sd, _ = dm.predict_next_state(d[nm + "_state_np"], d[nm + "_u"],
                                              t_batch=d.get(nm + "_t"), use_gps=True)
    assert np.array_equal(nx2.cpu().numpy(), ref_nx) and np.array_equal(sd2.cpu().numpy(), ref_sd)
    _, s_prior = O.predict_disturbance_prior(mode, x.shape[0])
    assert np.array_equal(sd2.cpu().numpy(), 0.02 * s_prior)
    # a fitted GP's posterior (stand-in estimator returning fixed f32 mean / std)
    rng = np.random.default_rng(11)
    m32 = rng.normal(0, 0.05, x.shape).astype(np.float32)
    s32 = rng.uniform(0.01, 0.3, x.shape).astype(np.float32)

    class _GP:
        def predict(self, xq):
            return torch.as_tensor(m32, device=xq.device), torch.as_tensor(s32, device=xq.device)
    dm.disturb_estimators = _GP()
    nx3, sd3, _ = dm.predict_next_state(x, u, t_batch=t, use_gps=True)
    assert np.array_equal(nx3.cpu().numpy(), d[nm + "_next"] + 0.02 * m32.astype(np.float64))
    assert np.array_equal(sd3.cpu().numpy(), 0.02 * s32.astype(np.float64))
    # 1-D state: squeezed outputs, like the reference's expand_dims handling
    dm.disturb_estimators = None
    n1, s1, t1 = dm.predict_next_state(x[3], u[3], t_batch=None if t is None else t[3], use_gps=False)
    assert n1.shape == (x.shape[1],) and np.array_equal(n1.cpu().numpy(), d[nm + "_next"][3])


def test_predict_next_obs_device(golden):
    """predict_next_obs (dynamics.py:107-123) on device tensors stays on the
    device and equals the numpy path (cars: bit-exact; unicycle: the device
    cos/sin within 1e-15)."""
    from rcbf_amd.dynamics import DynamicsModel
    from rcbf_amd.envs import UnicycleEnv
    d = golden("dynamics")
    dm = DynamicsModel(UnicycleEnv(), types.SimpleNamespace(cuda=True))
    x = torch.as_tensor(d["uni_state_np"], device="cuda")
    u = torch.as_tensor(d["uni_u"], device="cuda")
    o = dm.predict_next_obs(x, u)
    ref = dm.predict_next_obs(d["uni_state_np"], d["uni_u"])
    assert o.is_cuda and o.shape == ref.shape
    assert np.max(np.abs(o.cpu().numpy() - ref)) <= 1e-15


def test_predict_next_state_device_edge_cases():
    """Cars rows without t are refused (the model prior needs t, as the
    reference's numpy path fails without it); an empty batch is a no-op."""
    from rcbf_amd.dynamics import DynamicsModel
    from rcbf_amd.envs import SimulatedCarsEnv
    dm = DynamicsModel(SimulatedCarsEnv(), types.SimpleNamespace(cuda=True))
    x = torch.zeros(4, 10, dtype=torch.float64, device="cuda")
    u = torch.zeros(4, 1, dtype=torch.float64, device="cuda")
    with pytest.raises(Exception):
        dm.predict_next_state(x, u, t_batch=None, use_gps=False)
    nx, sd, nt = dm.predict_next_state(x[:0], u[:0], t_batch=torch.zeros(0, dtype=torch.float64, device="cuda"))
    assert nx.shape == (0, 10) and sd.shape == (0, 10) and nt.shape == (0,)


def test_predict_next_state_staged_rows_ragged_and_unaligned():
    """The cars kernel stages its 80-B rows through LDS (16-B accesses when
    the block's rows start 16-B aligned, element accesses otherwise): a
    ragged batch (B = 777: three full workgroups and a partial one) from an
    aligned buffer and from a view 8 bytes into one (the unaligned path)
    gives the same values bit for bit, the numpy path's within the device
    fp64 sin's ulps (car 0's v_des = 30 - 10 sin(0.2 t); random t here, the
    golden rows of test_predict_next_state_device_vs_reference are
    bit-exact), with the GP mean / std rows too."""
    from rcbf_amd.dynamics import DynamicsModel
    from rcbf_amd.envs import SimulatedCarsEnv
    dm = DynamicsModel(SimulatedCarsEnv(), types.SimpleNamespace(cuda=True))
    rng = np.random.default_rng(5)
    B = 777
    st = np.tile(np.array([34.0, 30.0, 28.0, 30.0, 22.0, 30.0, 16.0, 35.0, 10.0, 30.0]), (B, 1)) + rng.normal(0, 1, (B, 10))
    u = rng.uniform(-1, 1, (B, 1))
    t = np.round(rng.uniform(0, 6, B) / 0.02) * 0.02
    ref_nx, ref_sd, _ = dm.predict_next_state(st, u, t_batch=t, use_gps=False)
    ud, td = torch.as_tensor(u, device="cuda"), torch.as_tensor(t, device="cuda")
    buf = torch.zeros(B * 10 + 1, dtype=torch.float64, device="cuda")
    outs = []
    for x in (torch.as_tensor(st, device="cuda"), buf[1:].view(B, 10)):
        x.copy_(torch.as_tensor(st, device="cuda"))
        assert (x.data_ptr() % 16 == 0) == (x.storage_offset() == 0)
        nx, sd, nt = dm.predict_next_state(x, ud, t_batch=td, use_gps=False)
        assert np.max(np.abs(nx.cpu().numpy() - ref_nx)) <= 1e-13 * np.max(np.abs(ref_nx))
        assert not sd.cpu().numpy().any() and np.array_equal(nt.cpu().numpy(), t + 0.02)
        outs.append(nx.cpu().numpy())
    assert np.array_equal(outs[0], outs[1])
    m32 = rng.normal(0, 0.05, (B, 10)).astype(np.float32)
    s32 = rng.uniform(0.01, 0.3, (B, 10)).astype(np.float32)

    class _GP:
        def predict(self, xq):
            return torch.as_tensor(m32, device=xq.device), torch.as_tensor(s32, device=xq.device)
    dm.disturb_estimators = _GP()
    nx, sd, _ = dm.predict_next_state(buf[1:].view(B, 10), ud, t_batch=td, use_gps=True)
    assert np.array_equal(nx.cpu().numpy(), outs[0] + 0.02 * m32.astype(np.float64))
    assert np.array_equal(sd.cpu().numpy(), 0.02 * s32.astype(np.float64))
