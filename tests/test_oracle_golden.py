"""Pin the CPU oracle (oracle/oracle.py) against the golden vectors that
tests/golden/make_golden.py produced by running the reference's own code.

Tolerances (written per check):
  * cars CBF rows: bit-exact (same fp32 op order as rcbf_sac/diff_cbf_qp.py:268-357)
  * unicycle CBF rows: <= 2e-6 relative -- the only difference is torch's SLEEF
    fp32 cos/sin vs the oracle's correctly rounded cos/sin (1 ulp on theta;
    with torch's cos/sin substituted the oracle rows are bit-exact)
  * safe action: <= 1e-5 relative to max(1,|u|) (north-star bar is 1e-4)
  * gradients: <= 1e-5 relative (the reference's grad runs through fp32 rows)
  * env states: bit-exact for cars; unicycle <= 1e-14 relative (BLAS ddot FMA)
"""
import numpy as np
import pytest

from oracle import oracle as O


def rel(a, b):
    a = np.asarray(a, np.float64); b = np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b) / np.maximum(1.0, np.abs(b)))) if a.size else 0.0


@pytest.mark.parametrize("tag", ["prior", "rand"])
def test_cars_layer(golden, tag):
    d = golden("cars_layer")
    g = float(d["gamma_b"])
    P, q, G, h = O.cars_build_diff(d[tag + "_x"], d[tag + "_u"], d[tag + "_mu"], d[tag + "_sigma"], g)
    assert np.array_equal(G, d[tag + "_G"]) and np.array_equal(h, d[tag + "_h"])
    assert np.array_equal(P, d[tag + "_P"])
    fin, aux = O.safe_action_diff("SimulatedCars", d[tag + "_x"], d[tag + "_u"], d[tag + "_mu"], d[tag + "_sigma"], g)
    assert np.array_equal(aux["Gn"], d[tag + "_Gn"]) and np.array_equal(aux["hn"], d[tag + "_hn"])
    assert (aux["status"] == 0).all()
    assert rel(aux["z"], d[tag + "_z"]) < 1e-10
    assert rel(fin, d[tag + "_final"]) < 1e-5
    grad, _ = O.safe_action_diff_grad("SimulatedCars", d[tag + "_x"], d[tag + "_u"], d[tag + "_mu"],
                                      d[tag + "_sigma"], g, d[tag + "_w"])
    assert rel(grad, d[tag + "_grad_u"]) < 1e-5


@pytest.mark.parametrize("k", [3, 5])
@pytest.mark.parametrize("tag", ["prior", "rand"])
def test_unicycle_layer(golden, k, tag):
    d = golden(f"unicycle{k}_layer")
    g = float(d["gamma_b"])
    args = (d[tag + "_x"], d[tag + "_u"], d[tag + "_mu"], d[tag + "_sigma"], g)
    P, q, G, h = O.unicycle_build_diff(*args, d["hazards"], l_p=float(d["l_p"]))
    # a 1-ulp cos/sin difference moves h through gamma*h_s^3 by ~1e-6 relative
    assert rel(h, d[tag + "_h"]) < 2e-6
    assert rel(G, d[tag + "_G"]) < 1e-6
    fin, aux = O.safe_action_diff("Unicycle", *args, hazards=d["hazards"], l_p=float(d["l_p"]))
    assert (aux["status"] == 0).all()
    assert rel(fin, d[tag + "_final"]) < 1e-5
    grad, _ = O.safe_action_diff_grad("Unicycle", *args, d[tag + "_w"], hazards=d["hazards"], l_p=float(d["l_p"]))
    assert rel(grad, d[tag + "_grad_u"]) < 1e-5


def test_cascade(golden):
    c = golden("cascade")
    P, G, h = O.cars_build_cascade(c["cars_x"], c["cars_u"], 20.0)
    assert rel(G, c["cars_G"]) < 1e-15 and rel(h, c["cars_h"]) < 1e-14
    Gn, hn, _ = O.normalize_rows(G, h)
    z, lam, act, st = O.qp_exact(np.diag(P), Gn, hn)
    assert (st == 0).all() and rel(z[:, :1], c["cars_usafe"]) < 1e-9
    P, G, h = O.unicycle_build_cascade(c["uni_x"], c["uni_u"], c["uni_mu"], c["uni_sigma"], 40.0, 3.0, O.UNI["hazards"])
    assert rel(G, c["uni_G"]) < 1e-14 and rel(h, c["uni_h"]) < 1e-14
    Gn, hn, _ = O.normalize_rows(G, h)
    z, lam, act, st = O.qp_exact(np.diag(P), Gn, hn)
    assert (st == 0).all() and rel(z[:, :2], c["uni_usafe"]) < 1e-8


def test_cascade_config_size(golden):
    """The Cascade layer at config size (4096 rows each): cars from the
    config-2 start states, unicycle with the config-3 hazard set (k = 3)."""
    c = golden("cascade_config")
    P, G, h = O.cars_build_cascade(c["cars_x"], c["cars_u"], 20.0)
    Gn, hn, _ = O.normalize_rows(G, h)
    z, lam, act, st = O.qp_exact(np.diag(P), Gn, hn)
    assert (st == 0).all() and rel(z[:, :1], c["cars_usafe"]) < 1e-9
    P, G, h = O.unicycle_build_cascade(c["uni3_x"], c["uni3_u"], c["uni3_mu"], c["uni3_sigma"], 40.0, 3.0,
                                       c["uni3_hazards"])
    Gn, hn, _ = O.normalize_rows(G, h)
    z, lam, act, st = O.qp_exact(np.diag(P), Gn, hn)
    assert (st == 0).all() and rel(z[:, :2], c["uni3_usafe"]) < 1e-8


def test_cars_env_traj(golden):
    d = golden("env_traj")
    for e in range(d["cars_noise"].shape[0]):
        x, t, st = O.cars_reset(d["cars_noise"][e:e + 1])
        assert np.array_equal(x[0], d["cars_state"][e, 0])
        for k in range(300):
            x, t, st, obs, r, c, dn = O.cars_step(x, t, st, d["cars_actions"][e, k][None])
            assert np.array_equal(x[0], d["cars_state"][e, k + 1])
            assert np.array_equal(obs[0], d["cars_obs"][e, k + 1])
            assert t[0] == d["cars_t"][e, k + 1]
            # reference squares an np.float32 SCALAR (powf): <= 1 fp32 ulp from a*a
            assert abs(r[0] - d["cars_reward"][e, k]) <= 2 * np.spacing(np.float32(abs(r[0])))
            assert c[0] == d["cars_cost"][e, k] and dn[0] == d["cars_done"][e, k]


def test_unicycle_env_traj(golden):
    d = golden("env_traj")
    x, ld, st = O.uni_reset(1)
    assert np.array_equal(O.uni_obs(x)[0], d["uni_obs"][0])
    for k in range(1000):
        x, ld, st, obs, r, c, dn, gm = O.uni_step(x, ld, st, d["uni_actions"][k][None])
        assert rel(x[0], d["uni_state"][k + 1]) < 1e-14
        assert rel(obs[0], d["uni_obs"][k + 1]) < 1e-13
        assert abs(r[0] - d["uni_reward"][k]) < 1e-13
        assert c[0] == d["uni_cost"][k] and dn[0] == d["uni_done"][k]
    n_goal = 0
    for e in range(d["unir_x0"].shape[0]):
        x = d["unir_x0"][e:e + 1].copy(); ld = O.uni_goal_dist(x); st = d["unir_step0"][e:e + 1]
        for k in range(d["unir_actions"].shape[1]):
            x, ld, st, obs, r, c, dn, gm = O.uni_step(x, ld, st, d["unir_actions"][e, k][None])
            assert rel(x[0], d["unir_state"][e, k + 1]) < 1e-13
            assert rel(obs[0], d["unir_obs"][e, k + 1]) < 1e-12
            assert c[0] == d["unir_cost"][e, k] and dn[0] == d["unir_done"][e, k] and gm[0] == d["unir_goal"][e, k]
            n_goal += int(gm[0])
            if dn[0]:
                break
    assert n_goal >= 1 and d["unir_cost"].sum() > 0


def test_dynamics_glue(golden):
    d = golden("dynamics")
    for nm, mode in (("cars", "SimulatedCars"), ("uni", "Unicycle")):
        assert np.array_equal(O.get_state(mode, d[nm + "_obs"]), d[nm + "_state_np"])
        assert np.array_equal(O.get_state_f32(mode, d[nm + "_obs32"]), d[nm + "_state_t"])
        m, s = O.predict_disturbance_prior(mode, d[nm + "_obs"].shape[0])
        assert np.array_equal(m.astype(np.float32), d[nm + "_mean"])
        assert np.array_equal(s.astype(np.float32), d[nm + "_sigma"])
        nx = O.predict_next_state_prior(mode, d[nm + "_state_np"], d[nm + "_u"], d.get(nm + "_t"))
        assert np.array_equal(nx, d[nm + "_next"])


def test_closed_loop_config1(golden):
    """Config 1: hand controller + CascadeCBFLayer(gamma_b=20,k_d=3) + cars env,
    300 steps (envs/simulated_cars_env.py:161-228 without the plotting)."""
    cl = golden("closed_loop_cars")
    x, t, st = O.cars_reset(cl["noise"])
    for k in range(300):
        s = O.get_state("SimulatedCars", O.cars_obs(x))
        un = cl["u_nom"][k]
        P, G, h = O.cars_build_cascade(s, un[None], 20.0)
        Gn, hn, _ = O.normalize_rows(G, h)
        z, lam, act, stt = O.qp_exact(np.diag(P), Gn, hn)
        assert rel(z[:, :1], cl["u_safe"][k]) < 1e-8
        x, t, st, obs, r, c, dn = O.cars_step(x, t, st, un[None] + cl["u_safe"][k][None])
        assert np.array_equal(x[0], cl["state"][k + 1])


def test_philox_known_answer():
    """Philox4x32-10 known-answer vectors (Random123 kat_vectors, the
    published test vectors of Salmon et al.): counter/key all zero and all
    ones.  Pins the oracle restatement of the batched envs' reset RNG."""
    c = O.philox4x32_10([np.uint64(0)] * 4, 0)
    assert [int(v) for v in c] == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    ff = np.uint64(0xFFFFFFFF)
    c = O.philox4x32_10([ff] * 4, 0xFFFFFFFFFFFFFFFF)
    assert [int(v) for v in c] == [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]


def test_normal_draw_distribution():
    z = O.normal_draw(1234, np.arange(200000), 1)
    assert abs(z.mean()) < 0.01 and abs(z.std() - 1.0) < 0.01
    z2 = O.normal_draw(1234, np.arange(200000), 2)
    assert abs(np.corrcoef(z, z2)[0, 1]) < 0.01


def test_model_rollout_step_vs_reference(golden):
    """the oracle's model-rollout step == the reference's
    generate_model_rollouts (k_horizon = 1) on recorded N(0,1) draws."""
    d = golden("model_rollouts")
    for nm, mode in (("cars", "SimulatedCars"), ("uni", "Unicycle")):
        nobs, r, mask, tn = O.model_rollout_step(mode, d[nm + "_obs"], d[nm + "_act"], d[nm + "_t"], d[nm + "_z"])
        assert np.max(np.abs(nobs - d[nm + "_next_obs"])) <= 1e-13
        assert np.max(np.abs(r - d[nm + "_reward"])) <= 1e-13
        assert np.array_equal(mask, d[nm + "_mask"]) and np.array_equal(tn, d[nm + "_next_t"])
        assert (mask == 0).sum() >= 8  # the fixture exercises episode ends / goals


@pytest.mark.parametrize("name,mode", [("cars", "SimulatedCars"), ("uni3", "Unicycle")])
def test_sac_update_config5(golden, name, mode):
    """Config 5 through the reference's own RCBF_SAC.get_safe_action
    (sac_cbf.py:218-238) at B = 4096: the oracle's get_state(obs32) -> prior
    -> safe action and its d final / d action equal the reference's."""
    d = golden("sac_update_config5")
    obs = d[f"{name}_obs32"]
    hz = d.get(f"{name}_hazards")
    s32 = O.get_state_f32(mode, obs)
    mu, sg = O.predict_disturbance_prior(mode, obs.shape[0])
    mu, sg = mu.astype(np.float32), sg.astype(np.float32)
    fin, _ = O.safe_action_diff(mode, s32, d[f"{name}_action"], mu, sg, float(d["gamma_b"]), hazards=hz)
    assert rel(fin, d[f"{name}_final"]) <= 1e-5
    g, _ = O.safe_action_diff_grad(mode, s32, d[f"{name}_action"], mu, sg, float(d["gamma_b"]), d[f"{name}_w"],
                                   hazards=hz)
    assert rel(g, d[f"{name}_grad_action"]) <= 1e-5


@pytest.mark.parametrize("name,mode", [("cars", "SimulatedCars"), ("uni3", "Unicycle"), ("uni5", "Unicycle")])
def test_f64_build_variant(golden, name, mode):
    """The reference built in fp64 (torch.set_default_dtype(float64)): the
    exact QP on its fp64 normalised rows reproduces its z, and the shipped
    fp32 build (what the oracle and the kernel compute) lands within 1e-4 of
    its safe action -- the precision sensitivity SURVEY 7 measured."""
    d = golden("layer_f64_build")
    g = lambda k: d[f"{name}_{k}"]  # noqa: E731
    Pd = np.diagonal(g("P"), axis1=1, axis2=2).astype(np.float64)
    z, _, _, st = O.qp_exact(Pd, g("Gn"), g("hn"))
    ok = st == 0
    assert ok.mean() > 0.999 and rel(z[ok], g("z")[ok]) <= 1e-9
    f32 = lambda k: g(k).astype(np.float32)  # noqa: E731
    fin, _ = O.safe_action_diff(mode, f32("x"), f32("u"), f32("mu"), f32("sigma"), float(d["gamma_b"]),
                                hazards=d.get(f"{name}_hazards"))
    assert rel(fin, g("final")) <= 1e-4
