"""Per-call host latency of the B = 1 drop-in surfaces the reference's
training loop calls every env step (main.py:93-110): the gym env.step on a
numpy action, CBFQPLayer.get_safe_action on 1-D device tensors, and
RCBF_SAC.get_safe_action (rcbf_amd.sac_cbf) on one observation, without and
with a fitted GP (300 points, Lanczos rank 16, the training-loop test's
setting): back to back, and as select_action takes it (each call followed by
.cpu(), i.e. one host round trip), with its three launches timed apart;
and at the reference's N = 3000 (LOVE rank 100) the one-launch host-result
path (sac_cbf.get_safe_action_host) against the three launches + .cpu().
Prints one JSON line of microseconds per call (median of 5 runs of 200 calls)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "sac-rcbf_amd")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def gp_dynamics(env, rng):
    """A DynamicsModel with its GP fitted on 300 transitions around the prior."""
    import types
    from rcbf_amd.dynamics import DynamicsModel
    dm = DynamicsModel(env, types.SimpleNamespace(cuda=True, gp_model_size=300, gp_rank=16))
    n_u = env.action_space.shape[0]
    x = rng.uniform(-1, 1, (300, dm.n_s)) * (30.0 if dm.n_s == 10 else 3.0)
    u = rng.uniform(-1, 1, (300, n_u))
    nx = x + 0.02 * (np.sin(x) + rng.normal(0, 0.05, x.shape))
    dm.append_transition(x, u, nx, t_batch=rng.uniform(0, 15, 300))
    assert dm.disturb_estimators is not None
    return dm


def per_call_us(fn, n=200, reps=5):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e6 / n)
    return round(float(np.median(ts)), 1)


def main():
    from rcbf_amd.diff_cbf_qp import CBFQPLayer
    from rcbf_amd.dynamics import DynamicsModel
    from rcbf_amd.envs import SimulatedCarsEnv, UnicycleEnv
    from rcbf_amd.sac_cbf import get_safe_action

    class A:
        cuda = True

    out = {}
    rng = np.random.default_rng(0)
    for name, env in (("cars", SimulatedCarsEnv()), ("unicycle", UnicycleEnv())):
        n_u = env.action_space.shape[0]
        acts = rng.uniform(-1, 1, (64, n_u)).astype(np.float32)
        k = [0]

        def step():
            obs, r, done, info = env.step(acts[k[0] % 64])
            k[0] += 1
            if done:
                env.reset()
        out[f"{name}_env_step_us"] = per_call_us(step)
        layer = CBFQPLayer(env, A(), gamma_b=20.0)
        dm = DynamicsModel(env, A())
        obs = env.reset()
        st = torch.as_tensor(dm.get_state(obs), dtype=torch.float32, device="cuda")
        mu, sg = dm.predict_disturbance(st)
        u = torch.as_tensor(acts[0], device="cuda")
        out[f"{name}_layer_safe_action_us"] = per_call_us(lambda: layer.get_safe_action(st, u, mu, sg))
        ot = torch.as_tensor(obs, dtype=torch.float32, device="cuda")
        out[f"{name}_sac_get_safe_action_us"] = per_call_us(lambda: get_safe_action(layer, ot, u, dm))
        gdm = gp_dynamics(env, rng)
        gpm = gdm.disturb_estimators
        o2 = ot.unsqueeze(0)
        s2 = gdm.get_state(o2)
        out[f"{name}_gp_sac_get_safe_action_us"] = per_call_us(lambda: get_safe_action(layer, ot, u, gdm))
        out[f"{name}_gp_sac_get_safe_action_to_host_us"] = per_call_us(
            lambda: get_safe_action(layer, ot, u, gdm).cpu())
        out[f"{name}_gp_get_state_us"] = per_call_us(lambda: gdm.get_state(o2))
        out[f"{name}_gp_predict_us"] = per_call_us(lambda: gpm.predict(s2))
        out[f"{name}_to_host_us"] = per_call_us(lambda: u.cpu())
        # the one-launch host-result call on the 300-point fits: Lanczos rank 16 (above), and the exact factor the
        # training-loop test's DynamicsModel uses below 800 points (3 column blocks: one more hand-off level)
        from rcbf_amd.sac_cbf import get_safe_action_host
        out[f"{name}_gp300_rank16_one_launch_host_result_us"] = per_call_us(
            lambda: get_safe_action_host(layer, ot, u, gdm))
        from rcbf_amd import gp as _gp
        g16 = gdm.disturb_estimators
        gdm.disturb_estimators = _gp.GPDisturbanceModel(np.asarray(gdm.train_x), np.asarray(gdm.train_y),
                                                        g16.hyper, rank=None)
        if True:
            out[f"{name}_gp300_exact_one_launch_host_result_us"] = per_call_us(
                lambda: get_safe_action_host(layer, ot, u, gdm))

            def gapped():  # the training loop's pattern: the host busy ~0.3 ms between calls
                t_end = time.perf_counter() + 3e-4
                while time.perf_counter() < t_end:
                    pass
                t0 = time.perf_counter()
                get_safe_action_host(layer, ot, u, gdm)
                return time.perf_counter() - t0
            for _ in range(20):
                gapped()
            out[f"{name}_gp300_exact_one_launch_after_300us_idle_us"] = round(
                float(np.median([gapped() for _ in range(400)])) * 1e6, 1)
        gdm.disturb_estimators = g16
        # the reference's gp_model_size N = 3000 with LOVE rank 100, select_action's call
        # as ONE launch whose action lands in pinned host memory (get_safe_action_host) vs the three launches
        # + .cpu()
        from rcbf_amd import gp
        from rcbf_amd.sac_cbf import get_safe_action_host
        n_s = gdm.n_s
        xb = rng.uniform(-1, 1, (3000, n_s)) * (30.0 if n_s == 10 else 3.0)
        gdm.disturb_estimators = gp.GPDisturbanceModel(xb, 0.05 * np.sin(xb) + rng.normal(0, 0.02, xb.shape),
                                                       [(1.3, 0.2, 0.05)] * n_s, rank=gp.love_rank(3000))
        assert gdm.disturb_estimators.r <= 100 and gdm.disturb_estimators.rank == 100
        a = get_safe_action_host(layer, ot, u, gdm)
        b = get_safe_action(layer, ot, u, gdm).cpu().numpy()
        assert np.array_equal(a, b)
        out[f"{name}_gp3000_three_launches_to_host_us"] = per_call_us(
            lambda: get_safe_action(layer, ot, u, gdm).cpu())
        out[f"{name}_gp3000_one_launch_host_result_us"] = per_call_us(
            lambda: get_safe_action_host(layer, ot, u, gdm))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
