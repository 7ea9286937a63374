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
