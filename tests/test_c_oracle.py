"""The C oracle (oracle/rcbf_oracle.c, CPU baseline of bench.py) agrees with
the numpy oracle pinned to the reference fixtures."""
import numpy as np
import pytest

from oracle import c_oracle as C
from oracle import oracle as O


def rel(a, b):
    a = np.asarray(a, np.float64); b = np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b) / np.maximum(1.0, np.abs(b))))


@pytest.mark.parametrize("tag", ["prior", "rand"])
def test_c_oracle_layer_cars(golden, tag):
    d = golden("cars_layer")
    out, fails = C.safe_action("SimulatedCars", d[tag + "_x"], d[tag + "_u"], d[tag + "_mu"], d[tag + "_sigma"],
                               float(d["gamma_b"]), threads=2)
    assert fails == 0 and rel(out, d[tag + "_final"]) <= 1e-5


@pytest.mark.parametrize("k", [3, 5])
def test_c_oracle_layer_unicycle(golden, k):
    d = golden(f"unicycle{k}_layer")
    out, fails = C.safe_action("Unicycle", d["rand_x"], d["rand_u"], d["rand_mu"], d["rand_sigma"],
                               float(d["gamma_b"]), hazards=d["hazards"], threads=2)
    assert fails == 0 and rel(out, d["rand_final"]) <= 1e-5


def test_c_oracle_fused_step_matches_numpy():
    rng = np.random.default_rng(3)
    B = 2048
    x, t, st = O.cars_reset(rng.normal(0, 0.5, B))
    xc, tc, sc = x.copy(), t.copy(), st.astype(np.int32)
    for k in range(20):
        u = rng.uniform(-1, 1, (B, 1)).astype(np.float32)
        s32 = O.get_state_f32("SimulatedCars", O.cars_obs(x).astype(np.float32))
        mu, sg = O.predict_disturbance_prior("SimulatedCars", B)
        fin, _ = O.safe_action_diff("SimulatedCars", s32, u, mu.astype(np.float32), sg.astype(np.float32), 20.0)
        x, t, st, o, r, c, dn = O.cars_step(x, t, st, fin)
        uo, rew, cost, done, fails = C.safe_step("SimulatedCars", xc, tc, sc, u, 20.0, threads=2)
        assert fails == 0 and rel(uo, fin) <= 1e-6
        assert rel(xc, x) <= 1e-12 and np.array_equal(cost, c.astype(np.float32))
        assert np.array_equal(rew, r.astype(np.float32))
    hz = O.UNI["hazards"][:3]
    x = np.stack([rng.uniform(-3, 3, B), rng.uniform(-3, 3, B), rng.uniform(-np.pi, np.pi, B)], 1)
    ld = O.uni_goal_dist(x); st = np.zeros(B, np.int64)
    xc, lc, sc = x.copy(), ld.copy(), st.astype(np.int32)
    for k in range(10):
        u = rng.uniform(-1, 1, (B, 2)).astype(np.float32)
        s32 = O.get_state_f32("Unicycle", O.uni_obs(x).astype(np.float32))
        fin, _ = O.safe_action_diff("Unicycle", s32, u, np.zeros((B, 3), np.float32),
                                    np.full((B, 3), 0.2, np.float32), 20.0, hazards=hz)
        x, ld, st, o, r, c, dn, gm = O.uni_step(x, ld, st, fin, hazards=hz)
        uo, rew, cost, done, fails = C.safe_step("Unicycle", xc, lc, sc, u, 20.0, hazards=hz, threads=2)
        assert fails == 0 and rel(uo, fin) <= 1e-5
        assert rel(xc, x) <= 1e-9


@pytest.mark.parametrize("mode", ["SimulatedCars", "Unicycle"])
def test_c_oracle_fused_step_with_mean_sigma_matches_numpy(mode):
    """The C oracle's fused step with per-env mean/sigma (what the GPU parity
    test of the post-GP-fit regime checks against) equals the numpy oracle,
    which the reference fixtures pin with random mean/sigma."""
    rng = np.random.default_rng(11)
    B = 2048
    hz = O.UNI["hazards"][:5] if mode == "Unicycle" else None
    n_s = 10 if mode == "SimulatedCars" else 3
    if mode == "SimulatedCars":
        x, aux, st = O.cars_reset(rng.normal(0, 0.5, B))
        st = rng.integers(0, 299, B)
    else:
        x = np.stack([rng.uniform(-3, 3, B), rng.uniform(-3, 3, B), rng.uniform(-np.pi, np.pi, B)], 1)
        aux, st = O.uni_goal_dist(x), rng.integers(0, 999, B)
    xc, ac, sc = x.copy(), aux.copy(), st.astype(np.int32)
    for k in range(12):
        u = rng.uniform(-1, 1, (B, 1 if mode == "SimulatedCars" else 2)).astype(np.float32)
        mu = (0.01 * rng.normal(0, 1, (B, n_s))).astype(np.float32)
        sg = (0.2 * rng.uniform(0, 1, (B, n_s)) + 0.05).astype(np.float32)
        obs = O.cars_obs(x) if mode == "SimulatedCars" else O.uni_obs(x)
        s32 = O.get_state_f32(mode, obs.astype(np.float32))
        fin, _ = O.safe_action_diff(mode, s32, u, mu, sg, 20.0, hazards=hz)
        if mode == "SimulatedCars":
            x, aux, st, o, r, c, dn = O.cars_step(x, aux, st, fin)
        else:
            x, aux, st, o, r, c, dn, gm = O.uni_step(x, aux, st, fin, hazards=hz)
        ref = C.safe_step_ex(mode, xc, ac, sc, u, 20.0, hazards=hz, mean=mu, sigma=sg, threads=2)
        assert ref["fails"] == 0 and rel(ref["u"], fin) <= 1e-5
        assert rel(xc, x) <= 1e-9 and np.array_equal(ref["cost"], np.asarray(c, np.float32))


@pytest.mark.parametrize("name,mode", [("cars_layer", "SimulatedCars"), ("unicycle3_layer", "Unicycle"),
                                       ("unicycle5_layer", "Unicycle")])
@pytest.mark.parametrize("tag", ["prior", "rand"])
def test_c_oracle_gradient_matches_reference_fixtures(golden, name, mode, tag):
    """oracle_safe_action_grad (config 5's CPU baseline) vs the reference's
    own d final / d u_RL (fixtures made by autograd through the reference's
    normaliser and clamp) and the numpy oracle's restatement."""
    d = golden(name)
    hz = d["hazards"] if mode == "Unicycle" else None
    x, u, mu, sg, w = (d[tag + k] for k in ("_x", "_u", "_mu", "_sigma", "_w"))
    out, grad, fails = C.safe_action_grad(mode, x, u, mu, sg, float(d["gamma_b"]), w, hazards=hz, threads=2)
    assert fails == 0
    assert rel(out, d[tag + "_final"]) <= 1e-5
    assert rel(grad, d[tag + "_grad_u"]) <= 1e-5
    g_np, _ = O.safe_action_diff_grad(mode, x[:300], u[:300], mu[:300], sg[:300], float(d["gamma_b"]), w[:300],
                                      hazards=hz)
    assert rel(grad[:300], g_np) <= 1e-9


def test_c_closed_loop_config1_matches_the_reference_loop(golden):
    """BASELINE config 1 in C (oracle_cars_cascade_loop, bench.py --config 1's
    CPU baseline): the hand controller, the Cascade QP and the env over the
    golden 300-step episode equal the reference's own closed loop."""
    cl = golden("closed_loop_cars")
    un, us, xs = C.cars_cascade_loop(float(cl["noise"]), 300)
    assert np.max(np.abs(un - cl["u_nom"][:, 0]) / np.maximum(1, np.abs(cl["u_nom"][:, 0]))) <= 1e-12
    assert np.max(np.abs(us - cl["u_safe"][:, 0]) / np.maximum(1, np.abs(cl["u_safe"][:, 0]))) <= 1e-7
    assert np.max(np.abs(xs - cl["state"]) / np.maximum(1, np.abs(cl["state"]))) <= 1e-9
