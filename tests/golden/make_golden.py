#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the reference itself.

CONTAINER-ONLY. This script imports the read-only reference at /root/reference
(SAC-RCBF, pure Python) and runs its own code unmodified on seeded inputs.  The
reference never travels: only the .npz vectors this script writes are committed
and used by tests on the GPU box.

Four reference dependencies are absent from the image and are replaced by
import-time stubs written to a scratch dir (they carry no arithmetic of the
path):
  * gym       -- only `Env` and `spaces.Box` shapes are used
                 (envs/simulated_cars_env.py:6,18-20, envs/unicycle_env.py:8,21-23)
  * gpytorch  -- only the class statement at rcbf_sac/gp_model.py:12 runs
  * qpth      -- QPFunction is replaced by an EXACT fp64 QP (below), patched in
                 as CBFQPLayer.cbf_layer (rcbf_sac/diff_cbf_qp.py:111-144)
  * quadprog  -- solve_qp is replaced by the same exact QP
                 (rcbf_sac/cbf_qp.py:3,276)
qpth/quadprog are un-vendored third-party solvers whose versions are unpinned
(no requirements file).  The QP is strictly convex (P diagonal > 0), so its
optimum is unique; both solvers converge to it (quadprog exactly, qpth to
eps=1e-4).  The exact optimum is what the fixtures pin.

Exact QP used here: brute-force active-set enumeration in torch float64 over
all row subsets of size <= n (independent of both the numpy oracle's solver and
the HIP kernel's Goldfarb-Idnani solver).  Gradients come from autograd
through the reference's own normaliser/clamp code plus a differentiable KKT
solve on the identified active set (the implicit-function derivative that
qpth's backward approximates).

Usage:  python tests/golden/make_golden.py   (writes tests/golden/*.npz)
"""
import contextlib
import io
import itertools
import os
import sys
import tempfile
import types

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True  # never write __pycache__ into the read-only reference


# ----------------------------------------------------------------------------
# import stubs (no arithmetic on the path lives in them)
# ----------------------------------------------------------------------------
def _install_stubs():
    gym = types.ModuleType("gym")

    class Env:
        def seed(self, s=None):
            return [s]

        @property
        def unwrapped(self):
            return self

        def close(self):
            pass

    class Box:
        def __init__(self, low, high, shape=None, dtype=np.float32):
            shape = tuple(shape) if shape is not None else np.shape(low)
            self.low = np.full(shape, low, dtype=np.float32)
            self.high = np.full(shape, high, dtype=np.float32)
            self.shape = shape
            self.dtype = np.float32
            self._rng = np.random.RandomState(0)

        def seed(self, s):
            self._rng = np.random.RandomState(s)

        def sample(self):
            return self._rng.uniform(self.low, self.high).astype(np.float32)

        def contains(self, x):
            x = np.asarray(x)
            return x.shape == self.shape and np.all(x >= self.low) and np.all(x <= self.high)

    spaces = types.ModuleType("gym.spaces")
    spaces.Box = Box
    error = types.ModuleType("gym.error")
    gym.Env = Env
    gym.spaces = spaces
    gym.error = error
    sys.modules["gym"] = gym
    sys.modules["gym.spaces"] = spaces
    sys.modules["gym.error"] = error

    class _NS(types.ModuleType):
        def __getattr__(self, item):
            if item.startswith("__"):
                raise AttributeError(item)
            sub = _NS(self.__name__ + "." + item)
            setattr(self, item, sub)
            return sub

    gp = _NS("gpytorch")
    gp.models = _NS("gpytorch.models")
    gp.models.ExactGP = type("ExactGP", (torch.nn.Module,), {})
    sys.modules["gpytorch"] = gp

    qpth = types.ModuleType("qpth")
    qpth_qp = types.ModuleType("qpth.qp")

    def _qpfunction(*a, **k):
        raise RuntimeError("qpth is not installed; cbf_layer must be patched")

    qpth_qp.QPFunction = _qpfunction
    qpth.qp = qpth_qp
    sys.modules["qpth"] = qpth
    sys.modules["qpth.qp"] = qpth_qp

    quadprog = types.ModuleType("quadprog")

    def _solve_qp(P, q, C, b, meq=0):
        # quadprog.solve_qp(G, a, C, b): min 1/2 x'Gx - a'x  s.t.  C'x >= b.
        # Called as solve_qp(P, q, -G.T, -h)  <=>  G x <= h  (cbf_qp.py:276).
        Gm = -np.asarray(C).T
        hm = -np.asarray(b)
        Pt = torch.tensor(np.asarray(P), dtype=torch.float64)[None]
        qt = -torch.tensor(np.asarray(q), dtype=torch.float64)[None]
        z, _ = exact_qp(Pt, qt, torch.tensor(Gm)[None], torch.tensor(hm)[None])
        return (z[0].numpy(),)

    quadprog.solve_qp = _solve_qp
    sys.modules["quadprog"] = quadprog


# ----------------------------------------------------------------------------
# exact strictly-convex QP by active-set enumeration (fp64, differentiable)
# ----------------------------------------------------------------------------
def _kkt_subset(P, p, G, h, S):
    """Solve the equality-constrained KKT for rows S for every batch element.
    Returns z (B,n), lam_S (B,|S|), ok (B,) [non-singular]."""
    B, n = p.shape
    k = len(S)
    if k == 0:
        z = -torch.linalg.solve(P, p.unsqueeze(-1)).squeeze(-1)
        return z, p.new_zeros(B, 0), torch.ones(B, dtype=torch.bool)
    GS = G[:, list(S), :]
    K = torch.zeros(B, n + k, n + k, dtype=P.dtype)
    K[:, :n, :n] = P
    K[:, :n, n:] = GS.transpose(1, 2)
    K[:, n:, :n] = GS
    rhs = torch.cat([-p, h[:, list(S)]], dim=1).unsqueeze(-1)
    det = torch.linalg.det(K)
    ok = det.abs() > 1e-14
    Ksafe = torch.where(ok[:, None, None], K, torch.eye(n + k, dtype=P.dtype).expand(B, -1, -1))
    sol = torch.linalg.solve(Ksafe, rhs).squeeze(-1)
    return sol[:, :n], sol[:, n:], ok


def exact_qp(P, p, G, h, tol=1e-9):
    """min 1/2 z'Pz + p'z  s.t.  G z <= h   (batched, fp64).
    Returns z and an (B,) int64 index of the chosen active subset in the
    enumeration order (for the differentiable re-solve)."""
    P, p, G, h = (t.double() for t in (P, p, G, h))
    B, m, n = G.shape
    subsets = [S for k in range(0, n + 1) for S in itertools.combinations(range(m), k)]
    z_best = torch.full((B, n), float("nan"), dtype=torch.float64)
    chosen = torch.full((B,), -1, dtype=torch.int64)
    with torch.no_grad():
        for si, S in enumerate(subsets):
            z, lam, ok = _kkt_subset(P, p, G, h, S)
            scale = 1.0 + h.abs().amax(dim=1) + G.abs().amax(dim=(1, 2))
            prim = ((G @ z.unsqueeze(-1)).squeeze(-1) - h).amax(dim=1) <= tol * scale
            dual = (lam >= -tol * scale[:, None]).all(dim=1) if lam.shape[1] else torch.ones(B, dtype=torch.bool)
            take = ok & prim & dual & (chosen < 0)
            z_best[take] = z[take]
            chosen[take] = si
    return z_best, chosen


def exact_qp_diff(P, p, G, h):
    """Differentiable exact QP (autograd flows into G and h through the KKT
    solve on the identified active set)."""
    B, m, n = G.shape
    subsets = [S for k in range(0, n + 1) for S in itertools.combinations(range(m), k)]
    z0, chosen = exact_qp(P.detach(), p.detach(), G.detach(), h.detach())
    if (chosen < 0).any():
        raise RuntimeError("exact QP found no KKT point")
    out = [None] * B
    for si in torch.unique(chosen).tolist():
        idx = (chosen == si).nonzero().squeeze(-1)
        z, _, _ = _kkt_subset(P[idx].double(), p[idx].double(), G[idx].double(), h[idx].double(), subsets[si])
        for j, b in enumerate(idx.tolist()):
            out[b] = z[j]
    return torch.stack(out), chosen


# ----------------------------------------------------------------------------
def _import_reference():
    _install_stubs()
    sys.path.insert(0, REF)
    from envs.simulated_cars_env import SimulatedCarsEnv
    from envs.unicycle_env import UnicycleEnv
    from rcbf_sac import diff_cbf_qp, cbf_qp, dynamics
    return SimulatedCarsEnv, UnicycleEnv, diff_cbf_qp, cbf_qp, dynamics


class _Args:
    cuda = False
    gp_model_size = 2000
    l_p = 0.03


def _patch_layer(layer):
    """Replace the qpth call (diff_cbf_qp.py:139) by the exact QP, keeping the
    reference's fp64 cast / .float() / NaN check semantics."""

    def cbf_layer(Qs, ps, Gs, hs, As=None, bs=None, solver_args=None):
        z, chosen = exact_qp_diff(Qs.double(), ps.double(), Gs.double(), hs.double())
        layer._last_active = chosen
        result = z.float()
        if torch.any(torch.isnan(result)):
            raise Exception("QP Failed to solve")
        return result

    layer.cbf_layer = cbf_layer
    # capture the normalised rows solve_qp hands to the solver (diff_cbf_qp.py:103-107)
    orig = layer.cbf_layer

    def capturing(Qs, ps, Gs, hs, As=None, bs=None, solver_args=None):
        layer._last_norm = (Gs.detach().clone(), hs.detach().clone())
        return orig(Qs, ps, Gs, hs, As, bs, solver_args)

    layer.cbf_layer = capturing
    return layer


def _rollout_cars_states(SimulatedCarsEnv, B, rng, max_steps=300):
    env = SimulatedCarsEnv()
    states = np.zeros((B, 10))
    ts = np.zeros(B)
    for i in range(B):
        np.random.seed(int(rng.integers(1 << 30)))
        env.reset()
        k = int(rng.integers(0, max_steps))
        for _ in range(k):
            env.step(rng.uniform(-1, 1, size=(1,)).astype(np.float32))
        states[i] = env.state
        ts[i] = env.t
    return states, ts


def _layer_fixture(layer, x32, u32, mu32, sig32, w32):
    x = torch.tensor(x32)
    u = torch.tensor(u32, requires_grad=True)
    mu = torch.tensor(mu32)
    sig = torch.tensor(sig32)
    P, q, G, h = layer.get_cbf_qp_constraints(x, u.detach(), mu, sig)
    final = layer.get_safe_action(x, u, mu, sig)
    (final * torch.tensor(w32)).sum().backward()
    Gn, hn = layer._last_norm
    z, _ = exact_qp(P.double(), q.double(), Gn.double(), hn.double())
    return dict(x=x32, u=u32, mu=mu32, sigma=sig32, w=w32,
                P=P.numpy(), q=q.numpy(), G=G.numpy(), h=h.numpy(),
                Gn=Gn.numpy(), hn=hn.numpy(), z=z.numpy(),
                active=layer._last_active.numpy(),
                final=final.detach().numpy(), grad_u=u.grad.numpy())


def make_cars_layer(SimulatedCarsEnv, diff_cbf_qp, B=4096, seed=2, gamma_b=20.0):
    rng = np.random.default_rng(seed)
    env = SimulatedCarsEnv()
    layer = _patch_layer(diff_cbf_qp.CBFQPLayer(env, _Args(), gamma_b=gamma_b, k_d=3.0, l_p=0.03))
    states, _ = _rollout_cars_states(SimulatedCarsEnv, B, rng)
    x32 = states.astype(np.float32)
    u32 = rng.uniform(-1, 1, size=(B, 1)).astype(np.float32)
    # edge rows: Lg = 0 (p2 == p3), u at the box corners, very tight gaps
    x32[0, 6] = x32[0, 4]
    u32[1] = 1.0
    u32[2] = -1.0
    x32[3, 6] = x32[3, 4] - 2.0
    x32[4, 8] = x32[4, 6] - 1.0
    mu_prior = np.zeros((B, 10), np.float32)
    sig_prior = np.tile(np.array([0, .2, 0, .2, 0, .2, 0, .2, 0, .2], np.float32), (B, 1))
    w = rng.standard_normal((B, 1)).astype(np.float32)
    out = {}
    for tag, (mu, sig) in {
        "prior": (mu_prior, sig_prior),
        "rand": (rng.normal(0, 0.1, (B, 10)).astype(np.float32),
                 rng.uniform(0, 0.3, (B, 10)).astype(np.float32)),
    }.items():
        d = _layer_fixture(layer, x32, u32, mu, sig, w)
        out.update({f"{tag}_{k}": v for k, v in d.items()})
    out["gamma_b"] = np.float64(gamma_b)
    return out


def make_unicycle_layer(UnicycleEnv, diff_cbf_qp, n_hazards, B=4096, seed=3, gamma_b=20.0, l_p=0.03):
    rng = np.random.default_rng(seed + n_hazards)
    env = UnicycleEnv()
    env.hazards_locations = env.hazards_locations[:n_hazards]
    layer = _patch_layer(diff_cbf_qp.CBFQPLayer(env, _Args(), gamma_b=gamma_b, k_d=1.5, l_p=l_p))
    x32 = np.stack([rng.uniform(-3, 3, B), rng.uniform(-3, 3, B), rng.uniform(-np.pi, np.pi, B)], 1).astype(np.float32)
    u32 = rng.uniform(-1, 1, size=(B, 2)).astype(np.float32)
    x32[0, :2] = env.hazards_locations[0]  # on a hazard centre
    u32[1] = [1.0, -1.0]
    w = rng.standard_normal((B, 2)).astype(np.float32)
    out = {}
    for tag, (mu, sig) in {
        "prior": (np.zeros((B, 3), np.float32), np.full((B, 3), 0.2, np.float32)),
        "rand": (rng.normal(0, 0.1, (B, 3)).astype(np.float32), rng.uniform(0, 0.3, (B, 3)).astype(np.float32)),
    }.items():
        d = _layer_fixture(layer, x32, u32, mu, sig, w)
        out.update({f"{tag}_{k}": v for k, v in d.items()})
    out["hazards"] = env.hazards_locations.astype(np.float64)
    out["gamma_b"] = np.float64(gamma_b)
    out["l_p"] = np.float64(l_p)
    return out


def make_f64_build(SimulatedCarsEnv, UnicycleEnv, diff_cbf_qp, B=4096, seed=17, gamma_b=20.0):
    """SURVEY 8(c)(i) fp64 variant: the reference's CBFQPLayer with
    torch.set_default_dtype(torch.float64) and fp64 inputs (the rows are then
    built in fp64), on the config-2 / config-3 input distributions.  The HIP
    layer builds rows in fp32 like the shipped reference; this fixture bounds
    how far the fp32 build sits from an fp64 build (up to ~1e-4)."""
    rng = np.random.default_rng(seed)
    out = {}
    old = torch.get_default_dtype()
    torch.set_default_dtype(torch.float64)
    try:
        env = SimulatedCarsEnv()
        layer = _patch_layer(diff_cbf_qp.CBFQPLayer(env, _Args(), gamma_b=gamma_b, k_d=3.0, l_p=0.03))
        states, _ = _rollout_cars_states(SimulatedCarsEnv, B, rng)
        x = states.astype(np.float32).astype(np.float64)  # the fp32 state the policy path hands over, widened
        u = rng.uniform(-1, 1, size=(B, 1)).astype(np.float32).astype(np.float64)
        mu = np.zeros((B, 10))
        sig = np.tile(np.array([0, .2, 0, .2, 0, .2, 0, .2, 0, .2]), (B, 1))
        w = rng.standard_normal((B, 1))
        d = _layer_fixture(layer, x, u, mu, sig, w)
        out.update({f"cars_{k}": v for k, v in d.items()})
        for k in (3, 5):
            env = UnicycleEnv()
            env.hazards_locations = env.hazards_locations[:k]
            layer = _patch_layer(diff_cbf_qp.CBFQPLayer(env, _Args(), gamma_b=gamma_b, k_d=1.5, l_p=0.03))
            xs = np.stack([rng.uniform(-3, 3, B), rng.uniform(-3, 3, B), rng.uniform(-np.pi, np.pi, B)], 1)
            xs = xs.astype(np.float32).astype(np.float64)
            uu = rng.uniform(-1, 1, size=(B, 2)).astype(np.float32).astype(np.float64)
            d = _layer_fixture(layer, xs, uu, np.zeros((B, 3)), np.full((B, 3), 0.2), rng.standard_normal((B, 2)))
            out.update({f"uni{k}_{kk}": v for kk, v in d.items()})
            out[f"uni{k}_hazards"] = env.hazards_locations.astype(np.float64)
    finally:
        torch.set_default_dtype(old)
    out["gamma_b"] = np.float64(gamma_b)
    return out


def make_sac_update(SimulatedCarsEnv, UnicycleEnv, diff_cbf_qp, dynamics, B=4096, seed=19, gamma_b=20.0):
    """Config 5 (SimulatedCars batch 4096, diff CBF-QP forward + backward) as
    the SAC update runs it: the reference's own RCBF_SAC.get_safe_action
    (rcbf_sac/sac_cbf.py:218-238: DynamicsModel.get_state -> predict_disturbance
    prior -> CBFQPLayer.get_safe_action) on an fp32 observation batch, then
    d(sum(w * safe_action)) / d action with w ~ N(0, 1) -- the gradient
    policy_loss.backward() sends into the policy (sac_cbf.py:147-158).  Also
    unicycle (3 hazards) at the same size."""
    from rcbf_sac import sac_cbf
    rng = np.random.default_rng(seed)
    out = {}

    class A:
        gp_model_size = 2000
        cuda = False

    class Agent:  # the two attributes RCBF_SAC.get_safe_action touches
        pass

    for name, Env in (("cars", SimulatedCarsEnv), ("uni3", UnicycleEnv)):
        env = Env()
        if name == "cars":
            st, _ = _rollout_cars_states(SimulatedCarsEnv, B, rng)
            obs = st.copy(); obs[:, ::2] /= 100.0; obs[:, 1::2] /= 30.0
            n_u = 1
        else:
            env.hazards_locations = env.hazards_locations[:3]
            x = np.stack([rng.uniform(-3, 3, B), rng.uniform(-3, 3, B), rng.uniform(-np.pi, np.pi, B)], 1)
            rel = np.array([2.5, 2.5]) - x[:, :2]
            c, s_ = np.cos(x[:, 2]), np.sin(x[:, 2])
            comp = np.stack([rel[:, 0] * c + rel[:, 1] * s_, -rel[:, 0] * s_ + rel[:, 1] * c], 1)
            comp /= np.linalg.norm(comp, axis=1, keepdims=True) + 0.001
            obs = np.hstack([x[:, :2], c[:, None], s_[:, None], comp, np.exp(-np.linalg.norm(rel, axis=1))[:, None]])
            n_u = 2
        agent = Agent()
        agent.cbf_layer = _patch_layer(diff_cbf_qp.CBFQPLayer(env, A(), gamma_b=gamma_b, k_d=1.5, l_p=0.03))
        dm = dynamics.DynamicsModel(env, A())
        obs32 = obs.astype(np.float32)
        act = rng.uniform(-1, 1, (B, n_u)).astype(np.float32)
        w = rng.standard_normal((B, n_u)).astype(np.float32)
        a_t = torch.tensor(act, requires_grad=True)
        safe = sac_cbf.RCBF_SAC.get_safe_action(agent, torch.tensor(obs32), a_t, dm)
        (safe * torch.tensor(w)).sum().backward()
        out.update({f"{name}_obs32": obs32, f"{name}_action": act, f"{name}_w": w,
                    f"{name}_final": safe.detach().numpy(), f"{name}_grad_action": a_t.grad.numpy()})
        if name == "uni3":
            out["uni3_hazards"] = env.hazards_locations.astype(np.float64)
    out["gamma_b"] = np.float64(gamma_b)
    return out


def make_cascade(SimulatedCarsEnv, UnicycleEnv, cbf_qp, B=256, seed=5):
    rng = np.random.default_rng(seed)
    out = {}
    # cars, gamma_b=20, k_d=3 (simulated_cars_env.py:170-177)
    env = SimulatedCarsEnv()
    layer = cbf_qp.CascadeCBFLayer(env, gamma_b=20.0, k_d=3.0)
    states, _ = _rollout_cars_states(SimulatedCarsEnv, B, rng)
    un = rng.uniform(-1, 1, (B, 1))
    mu = np.zeros((B, 10))
    sig = np.tile(np.array([0, .2, 0, .2, 0, .2, 0, .2, 0, .2]), (B, 1))
    G_, h_, us = [], [], []
    for i in range(B):
        P, q, G, h = layer.get_cbf_qp_constraints(un[i], states[i], mu[i], sig[i])
        G_.append(G.copy()); h_.append(h.copy())
        with contextlib.redirect_stdout(io.StringIO()):
            us.append(layer.get_u_safe(un[i], states[i], mu[i], sig[i]))
    out.update(cars_x=states, cars_u=un, cars_mu=mu, cars_sigma=sig, cars_G=np.array(G_),
               cars_h=np.array(h_), cars_P=P, cars_usafe=np.array(us))
    # unicycle (5 hazards), gamma_b=40, k_d=3 (unicycle_env.py:334-340)
    env = UnicycleEnv()
    layer = cbf_qp.CascadeCBFLayer(env, gamma_b=40.0, k_d=3.0, l_p=0.03)
    xs = np.stack([rng.uniform(-3, 3, B), rng.uniform(-3, 3, B), rng.uniform(-np.pi, np.pi, B)], 1)
    un = rng.uniform(-1, 1, (B, 2))
    mu = rng.normal(0, 0.1, (B, 3))
    sig = rng.uniform(0, 0.3, (B, 3))
    G_, h_, us = [], [], []
    for i in range(B):
        P, q, G, h = layer.get_cbf_qp_constraints(un[i], xs[i], mu[i], sig[i])
        G_.append(G.copy()); h_.append(h.copy())
        with contextlib.redirect_stdout(io.StringIO()):
            us.append(layer.get_u_safe(un[i], xs[i], mu[i], sig[i]))
    out.update(uni_x=xs, uni_u=un, uni_mu=mu, uni_sigma=sig, uni_G=np.array(G_),
               uni_h=np.array(h_), uni_P=P, uni_usafe=np.array(us))
    return out


def make_cascade_config(SimulatedCarsEnv, UnicycleEnv, cbf_qp, B=4096, seed=23):
    """Cascade rows at config size (SURVEY 8(c)(ii) per config): cars B = 4096
    from the config-2 start-state distribution (gamma_b = 20, k_d = 3,
    simulated_cars_env.py:170-171) and unicycle with the config-3 hazard set
    (the first 3 hazards, gamma_b = 40, k_d = 3, unicycle_env.py:334-340),
    through the reference's own CascadeCBFLayer.get_u_safe with the exact QP
    in place of quadprog (cbf_qp.py:276)."""
    rng = np.random.default_rng(seed)
    out = {}
    env = SimulatedCarsEnv()
    layer = cbf_qp.CascadeCBFLayer(env, gamma_b=20.0, k_d=3.0)
    states, _ = _rollout_cars_states(SimulatedCarsEnv, B, rng)
    un = rng.uniform(-1, 1, (B, 1))
    mu = np.zeros((B, 10))
    sig = np.tile(np.array([0, .2, 0, .2, 0, .2, 0, .2, 0, .2]), (B, 1))
    us = []
    for i in range(B):
        with contextlib.redirect_stdout(io.StringIO()):
            us.append(layer.get_u_safe(un[i], states[i], mu[i], sig[i]))
    out.update(cars_x=states, cars_u=un, cars_mu=mu, cars_sigma=sig, cars_usafe=np.array(us))
    env = UnicycleEnv()
    env.hazards_locations = env.hazards_locations[:3]
    layer = cbf_qp.CascadeCBFLayer(env, gamma_b=40.0, k_d=3.0, l_p=0.03)
    xs = np.stack([rng.uniform(-3, 3, B), rng.uniform(-3, 3, B), rng.uniform(-np.pi, np.pi, B)], 1)
    un = rng.uniform(-1, 1, (B, 2))
    mu = rng.normal(0, 0.1, (B, 3))
    sig = rng.uniform(0, 0.3, (B, 3))
    us = []
    for i in range(B):
        with contextlib.redirect_stdout(io.StringIO()):
            us.append(layer.get_u_safe(un[i], xs[i], mu[i], sig[i]))
    out.update(uni3_x=xs, uni3_u=un, uni3_mu=mu, uni3_sigma=sig, uni3_usafe=np.array(us),
               uni3_hazards=np.asarray(env.hazards_locations, np.float64))
    return out


def make_env_traj(SimulatedCarsEnv, UnicycleEnv, seed=7):
    rng = np.random.default_rng(seed)
    out = {}
    # cars: 3 episodes of 300 steps; the reset's N(0,0.5) draw is recorded so
    # the device env can inject it (simulated_cars_env.py:120)
    env = SimulatedCarsEnv()
    E, T = 3, 300
    noise = np.zeros(E); acts = np.zeros((E, T, 1), np.float32)
    obs = np.zeros((E, T + 1, 10)); rew = np.zeros((E, T)); cost = np.zeros((E, T)); done = np.zeros((E, T), bool)
    st = np.zeros((E, T + 1, 10)); tt = np.zeros((E, T + 1))
    for e in range(E):
        np.random.seed(100 + e)
        obs[e, 0] = env.reset()
        noise[e] = env.state[1] - 30.0
        st[e, 0] = env.state; tt[e, 0] = env.t
        scale = [1.0, 3.0, 8.0][e]
        for k in range(T):
            a = rng.uniform(-scale, scale, (1,)).astype(np.float32)
            acts[e, k] = a
            o, r, d, info = env.step(a)
            obs[e, k + 1] = o; rew[e, k] = r; cost[e, k] = info["cost"]; done[e, k] = d
            st[e, k + 1] = env.state; tt[e, k + 1] = env.t
    out.update(cars_noise=noise, cars_actions=acts, cars_obs=obs, cars_reward=rew, cars_cost=cost,
               cars_done=done, cars_state=st, cars_t=tt)
    # unicycle: 1 full 1000-step episode from reset with clipped random actions,
    # plus 64 short episodes from random starts (hazard contacts, goal hits)
    env = UnicycleEnv()
    T = 1000
    env.reset()
    acts = rng.uniform(-1.5, 1.5, (T, 2)).astype(np.float32)
    o_, r_, c_, d_, s_ = [env.get_obs()], [], [], [], [env.state.copy()]
    for k in range(T):
        o, r, d, info = env.step(acts[k])
        o_.append(o); r_.append(r); c_.append(info.get("cost", 0.0)); d_.append(d); s_.append(env.state.copy())
    out.update(uni_actions=acts, uni_obs=np.array(o_), uni_reward=np.array(r_), uni_cost=np.array(c_),
               uni_done=np.array(d_), uni_state=np.array(s_))
    E, T = 32, 100
    x0 = np.stack([rng.uniform(-3, 3, E), rng.uniform(-3, 3, E), rng.uniform(-np.pi, np.pi, E)], 1)
    step0 = rng.integers(0, 1000, E)
    x0[0, :2] = [2.3, 2.3]  # starts next to the goal
    step0[1] = 995          # hits the time limit
    acts = np.zeros((E, T, 2), np.float32)
    S = np.zeros((E, T + 1, 3)); O = np.zeros((E, T + 1, 7)); R = np.zeros((E, T)); C = np.zeros((E, T))
    D = np.zeros((E, T), bool); GM = np.zeros((E, T), bool); LD = np.zeros((E, T + 1))
    for e in range(E):
        env.reset()
        env.state = x0[e].copy(); env.last_goal_dist = env._goal_dist(); env.episode_step = int(step0[e])
        S[e, 0] = env.state; O[e, 0] = env.get_obs(); LD[e, 0] = env.last_goal_dist
        for k in range(T):
            # steer toward the goal with noise: produces hazard contacts and goal hits
            rel = env.goal_pos - env.state[:2]
            ang = np.arctan2(rel[1], rel[0]) - env.state[2]
            ang = np.arctan2(np.sin(ang), np.cos(ang))
            a = np.array([1.0, 3.0 * ang]) + rng.normal(0, 0.5, 2)
            a = a.astype(np.float32)
            acts[e, k] = a
            o, r, d, info = env.step(a)
            S[e, k + 1] = env.state; O[e, k + 1] = o; R[e, k] = r; C[e, k] = info.get("cost", 0.0)
            D[e, k] = d; GM[e, k] = info.get("goal_met", False); LD[e, k + 1] = env.last_goal_dist
            if d:
                break
    out.update(unir_x0=x0, unir_step0=step0, unir_actions=acts, unir_state=S, unir_obs=O, unir_reward=R,
               unir_cost=C, unir_done=D, unir_goal=GM, unir_lastdist=LD)
    return out


def make_closed_loop(SimulatedCarsEnv, cbf_qp, dynamics):
    """Config 1: hand controller (simulated_cars_env.py:195-199) + Cascade layer
    (gamma_b=20, k_d=3) + cars env, one 300-step episode, seed 12345."""
    env = SimulatedCarsEnv()

    class A:
        gp_model_size = 2000
        cuda = False

    dm = dynamics.DynamicsModel(env, A())
    layer = cbf_qp.CascadeCBFLayer(env, gamma_b=20.0, k_d=3.0)

    def controller(state):
        gain = 1.0
        a = np.array([gain * (state[4] - state[6] - 0.4) * (state[4] - state[6] - 0.4 < 0)])
        a += np.array([gain * (state[8] - state[6] + 0.4) * (state[8] - state[6] + 0.4 > 0)])
        return a

    np.random.seed(12345)
    obs = env.reset()
    noise = env.state[1] - 30.0
    done = False
    S, O, UN, US, R, C = [env.state.copy()], [obs], [], [], [], []
    while not done:
        state = dm.get_state(obs)
        u = controller(state)
        m, s = dm.predict_disturbance(state)
        with contextlib.redirect_stdout(io.StringIO()):
            us = layer.get_u_safe(u, state, m, s)
        obs, r, done, info = env.step(u + us)
        S.append(env.state.copy()); O.append(obs); UN.append(u); US.append(us); R.append(r); C.append(info["cost"])
    return dict(noise=noise, state=np.array(S), obs=np.array(O), u_nom=np.array(UN), u_safe=np.array(US),
                reward=np.array(R), cost=np.array(C))


def make_dynamics(SimulatedCarsEnv, UnicycleEnv, dynamics, seed=11):
    rng = np.random.default_rng(seed)
    out = {}

    class A:
        gp_model_size = 2000
        cuda = False

    for name, Env, n_o in (("cars", SimulatedCarsEnv, 10), ("uni", UnicycleEnv, 7)):
        env = Env()
        dm = dynamics.DynamicsModel(env, A())
        B = 64
        if name == "cars":
            st, _ = _rollout_cars_states(SimulatedCarsEnv, B, rng, 100)
            obs = st.copy(); obs[:, ::2] /= 100.0; obs[:, 1::2] /= 30.0
            t = rng.uniform(0, 6, (B,))
            u = rng.uniform(-1, 1, (B, 1))
        else:
            th = rng.uniform(-np.pi, np.pi, B)
            obs = np.stack([rng.uniform(-3, 3, B), rng.uniform(-3, 3, B), np.cos(th), np.sin(th),
                            rng.uniform(-1, 1, B), rng.uniform(-1, 1, B), rng.uniform(0, 1, B)], 1)
            t = None
            u = rng.uniform(-1, 1, (B, 2))
        obs32 = obs.astype(np.float32)
        s_np = dm.get_state(obs)
        s_t = dm.get_state(torch.tensor(obs32)).numpy()
        m_t, sg_t = dm.predict_disturbance(torch.tensor(s_t))
        nxt, nstd, _ = dm.predict_next_state(s_np, u, t_batch=t, use_gps=False)
        out.update({f"{name}_obs": obs, f"{name}_obs32": obs32, f"{name}_state_np": s_np,
                    f"{name}_state_t": s_t, f"{name}_mean": m_t.numpy(), f"{name}_sigma": sg_t.numpy(),
                    f"{name}_u": u, f"{name}_next": nxt, f"{name}_obs_back": dm.get_obs(s_np)})
        if t is not None:
            out[f"{name}_t"] = t
    return out


def make_model_rollouts(SimulatedCarsEnv, UnicycleEnv, dynamics, seed=13):
    """rcbf_sac/generate_rollouts.py:6-81 run unmodified
    with k_horizon=1 on fixed (obs, action, t) batches (a stub memory and agent
    supply them) and the model prior (no GP fitted); np.random.normal is
    routed through recorded N(0,1) draws z so the device kernel can replay
    next = mu + std * z.  The transitions come out of the reference's own
    ReplayMemory.batch_push (rcbf_sac/replay_memory.py:23-29)."""
    from rcbf_sac import generate_rollouts, replay_memory
    rng = np.random.default_rng(seed)
    out = {}

    class A:
        gp_model_size = 2000
        cuda = False

    B = 256
    for name, Env, n_u in (("cars", SimulatedCarsEnv, 1), ("uni", UnicycleEnv, 2)):
        env = Env()
        dm = dynamics.DynamicsModel(env, A())
        if name == "cars":
            st, _ = _rollout_cars_states(SimulatedCarsEnv, B, rng, 300)
            obs = st.copy(); obs[:, ::2] /= 100.0; obs[:, 1::2] /= 30.0
            t = np.round(rng.uniform(0, 6.0, B) / 0.02) * 0.02
            t[:8] = 6.0 - 0.02  # episodes that end in this model step
        else:
            x = np.stack([rng.uniform(-3, 3, B), rng.uniform(-3, 3, B), rng.uniform(-np.pi, np.pi, B)], 1)
            x[:8, :2] = np.array([2.5, 2.5]) + rng.normal(0, 0.1, (8, 2))  # near the goal
            rel = np.array([2.5, 2.5]) - x[:, :2]
            d = np.linalg.norm(rel, axis=1)
            c, s_ = np.cos(x[:, 2]), np.sin(x[:, 2])
            comp = np.stack([rel[:, 0] * c + rel[:, 1] * s_, -rel[:, 0] * s_ + rel[:, 1] * c], 1)
            comp /= np.linalg.norm(comp, axis=1, keepdims=True) + 0.001
            obs = np.hstack([x[:, :2], c[:, None], s_[:, None], comp, np.exp(-d)[:, None]])
            t = np.zeros(B)
        act = rng.uniform(-1, 1, (B, n_u))
        z = rng.normal(0, 1, (B, obs.shape[1] if name == "cars" else 3))

        class Mem:
            def sample(self, batch_size):
                return obs.copy(), act.copy(), np.zeros(B), obs.copy(), np.ones(B), t.copy(), t + 0.02

        class Agent:
            def select_action(self, o, dm_, warmup=False, evaluate=False):
                return act.copy()

        mm = replay_memory.ReplayMemory(10 * B, 0)
        saved = generate_rollouts.np.random.normal
        generate_rollouts.np.random.normal = lambda mu, sd: mu + sd * z
        try:
            generate_rollouts.generate_model_rollouts(env, mm, Mem(), Agent(), dm, k_horizon=1, batch_size=B)
        finally:
            generate_rollouts.np.random.normal = saved
        tr = list(zip(*mm.buffer))
        out.update({f"{name}_obs": obs, f"{name}_act": act, f"{name}_t": t, f"{name}_z": z,
                    f"{name}_next_obs": np.stack(tr[3]), f"{name}_reward": np.asarray(tr[2], np.float64),
                    f"{name}_mask": np.asarray(tr[4]).astype(np.float64), f"{name}_next_t": np.asarray(tr[6], np.float64)})
    return out


def main():
    torch.set_num_threads(8)
    SimulatedCarsEnv, UnicycleEnv, diff_cbf_qp, cbf_qp, dynamics = _import_reference()
    jobs = {
        "cars_layer.npz": lambda: make_cars_layer(SimulatedCarsEnv, diff_cbf_qp),
        "unicycle3_layer.npz": lambda: make_unicycle_layer(UnicycleEnv, diff_cbf_qp, 3),
        "unicycle5_layer.npz": lambda: make_unicycle_layer(UnicycleEnv, diff_cbf_qp, 5),
        "cascade.npz": lambda: make_cascade(SimulatedCarsEnv, UnicycleEnv, cbf_qp),
        "cascade_config.npz": lambda: make_cascade_config(SimulatedCarsEnv, UnicycleEnv, cbf_qp),
        "env_traj.npz": lambda: make_env_traj(SimulatedCarsEnv, UnicycleEnv),
        "closed_loop_cars.npz": lambda: make_closed_loop(SimulatedCarsEnv, cbf_qp, dynamics),
        "dynamics.npz": lambda: make_dynamics(SimulatedCarsEnv, UnicycleEnv, dynamics),
        "model_rollouts.npz": lambda: make_model_rollouts(SimulatedCarsEnv, UnicycleEnv, dynamics),
        "layer_f64_build.npz": lambda: make_f64_build(SimulatedCarsEnv, UnicycleEnv, diff_cbf_qp),
        "sac_update_config5.npz": lambda: make_sac_update(SimulatedCarsEnv, UnicycleEnv, diff_cbf_qp, dynamics),
    }
    only = set(sys.argv[1:])
    for fname, fn in jobs.items():
        if only and fname not in only:
            continue
        d = fn()
        np.savez_compressed(os.path.join(OUT, fname), **d)
        print("wrote", fname, sum(v.nbytes for v in d.values()), "bytes raw")


if __name__ == "__main__":
    main()
