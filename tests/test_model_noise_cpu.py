"""The model-rollout step's N(0, 1) draw as restated in the oracle
(oracle.model_step_normal: fp32 Box-Muller on 24-bit Philox4x32-10 uniforms,
the arithmetic of k_model_step in rcbf_model.hip) is standard normal by its
moments and tails; the reference draws np.random.normal in fp64
(generate_rollouts.py:31), so values are unpinned and the statistics are the
check.  The device draw is checked against this restatement and by the same
bounds in tests/test_gpu_model.py."""
import numpy as np

from oracle import oracle as O


def test_model_step_normal_restatement_is_standard_normal():
    z = np.concatenate([O.model_step_normal(3, np.arange(1 << 19), c, 10)[:, [0, 1, 2, 3, 8, 9]]
                        for c in range(2)])
    n = z.size  # 6.3 M samples over both Philox calls of a cars row (components 0-3 and 8-9)
    st = O.normal_moments(z)
    se = 1.0 / np.sqrt(n)
    assert abs(st["mean"]) < 6 * se and abs(st["var"] - 1.0) < 6 * np.sqrt(2) * se, st
    assert abs(st["skew"]) < 6 * np.sqrt(6) * se and abs(st["exkurt"]) < 6 * np.sqrt(24) * se, st
    p3, p4 = 2.699796e-3, 6.334248e-5
    assert abs(st["p3"] - p3) < 6 * np.sqrt(p3 / n) and abs(st["p4"] - p4) < 6 * np.sqrt(p4 / n), st
    assert st["max"] <= np.sqrt(48 * np.log(2)) + 1e-6


def test_model_step_normal_is_keyed():
    """Same (seed, row, counter) -> same draw; another counter or seed -> another."""
    a = O.model_step_normal(3, np.arange(64), 0, 3)
    assert np.array_equal(a, O.model_step_normal(3, np.arange(64), 0, 3))
    assert not np.any(a == O.model_step_normal(3, np.arange(64), 1, 3))
    assert not np.any(a == O.model_step_normal(4, np.arange(64), 0, 3))
    assert np.array_equal(O.model_step_normal(3, np.arange(10, 20), 0, 3), a[10:20])
