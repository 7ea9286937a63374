"""The CPU-baseline mirror of the reference's own CPU mode
(oracle/torch_mirror.py: fp32 rows, normaliser, qpth-style batched PDIPM in
torch fp64, clamp, numpy env step) reproduces the exact safe action: its
PDIPM stops at qpth's eps = 1e-4 residual (or its notImprovedLim, capped at
100 iterations where the reference allows 100 000), and the actions agree
with the exact solver to <= 1e-4 relative (the north-star bar) on SURVEY 8(d)
states -- every cars QP, and all but qpth's rare stalled unicycle QPs."""
import numpy as np

from oracle import oracle as O
from oracle import torch_mirror as M


def test_cars_mirror_matches_exact():
    rng = np.random.default_rng(3)
    B = 2048
    x, t, st = O.cars_reset(rng.normal(0, 0.5, B))
    k_stop = rng.integers(0, 300, B)
    snap, ts, sts = x.copy(), t.copy(), st.copy()
    for k in range(1, 300):
        x, t, st = O.cars_step(x, t, st, rng.uniform(-1, 1, (B, 1)).astype(np.float32))[:3]
        sel = k_stop == k
        snap[sel], ts[sel], sts[sel] = x[sel], t[sel], st[sel]
    u = rng.uniform(-1, 1, (B, 1)).astype(np.float32)
    s32 = O.get_state_f32("SimulatedCars", O.cars_obs(snap).astype(np.float32))
    sg = np.tile(np.asarray(O.MAX_STD["SimulatedCars"], np.float32), (B, 1))
    fin, _ = O.safe_action_diff("SimulatedCars", s32, u, np.zeros((B, 10), np.float32), sg, 20.0)
    x2, t2, st2, us, its = M.cars_safe_step(snap, ts, sts, u, 20.0)
    assert its < 100
    assert np.max(np.abs(us - fin) / np.maximum(1.0, np.abs(fin))) <= 1e-4
    xe, te, ste = O.cars_step(snap, ts, sts, fin)[:3]
    assert np.max(np.abs(x2 - xe) / np.maximum(1.0, np.abs(xe))) <= 1e-5


def test_unicycle_mirror_matches_exact():
    rng = np.random.default_rng(4)
    B = 2048
    hz = O.UNI["hazards"][:3]
    x = np.stack([rng.uniform(-3, 3, B), rng.uniform(-3, 3, B), rng.uniform(-np.pi, np.pi, B)], 1)
    ld = O.uni_goal_dist(x)
    st = np.zeros(B, np.int64)
    u = rng.uniform(-1, 1, (B, 2)).astype(np.float32)
    s32 = O.get_state_f32("Unicycle", O.uni_obs(x).astype(np.float32))
    fin, _ = O.safe_action_diff("Unicycle", s32, u, np.zeros((B, 3), np.float32), np.full((B, 3), 0.2, np.float32),
                                20.0, hazards=hz)
    _, _, _, us, its = M.uni_safe_step(x, ld, st, u, 20.0, hz)
    # qpth's algorithm stalls on rare unicycle QPs (its best iterate is then
    # far off: 1 of 2048 here, 0.12 away; the product's PDIPM certifies and
    # re-solves such points exactly), and one element that keeps
    # improving holds the batch-global loop to the mirror's 100-iteration cap
    err = (np.abs(us - fin) / np.maximum(1.0, np.abs(fin))).max(axis=1)
    assert its <= 100
    assert (err <= 1e-4).mean() >= 0.999
