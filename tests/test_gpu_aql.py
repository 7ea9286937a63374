"""The fused safe step dispatched on the library's own AQL queue
(csrc/rcbf_aql.hip, rcbf_amd.aql) against the same steps launched through
HIP (rcbf_safe_step_seq): the kernels are the same machine code, so every
output must be bit-identical -- state, aux, step counters, episode counters,
observations, safe actions, reward, cost, done, goal -- across K steps with
auto-resets, at the headline batch, a small batch (64-thread workgroups), a
ragged batch, both envs, both prior layouts; plus the profiled plan's
dispatch timestamps and the span instantiation."""
import numpy as np
import pytest
import torch

import bench
from test_gpu_headline_parity import _make

pytestmark = pytest.mark.gpu


def _pair(mode, B, hazards=3, seed=77):
    """Two identical envs at the bench start states."""
    out = []
    for _ in range(2):
        env, layer = _make(mode, B, hazards=hazards, seed=seed)
        gen = torch.Generator(device="cuda")
        gen.manual_seed(5)
        bench.init_states(env, gen, mode)
        out.append((env, layer))
    return out


def _snapshot(env, o):
    t = {"x": env.x, "aux": env.aux, "step": env.step_count, "episode": env.episode, "obs": env.obs}
    t.update({k: v for k, v in o.items() if v is not None})
    return {k: v.clone() for k, v in t.items()}


def _assert_same(a, b):
    for k in a:
        assert torch.equal(a[k], b[k]), k


@pytest.fixture(scope="module")
def queue():
    from rcbf_amd.aql import AqlQueue
    q = AqlQueue(torch.device("cuda", 0), profile=True)
    yield q
    q.close()


def test_queue_loads_the_step_code_object(queue):
    assert queue.kernel_count() > 0


@pytest.mark.parametrize("mode,B,hazards,layout", [
    ("SimulatedCars", 65536, 0, "rows"),
    ("SimulatedCars", 4096, 0, "rows"),
    ("SimulatedCars", 1000, 0, "cols"),
    ("Unicycle", 65536, 5, "rows"),
    ("Unicycle", 4096, 3, "cols"),
])
def test_aql_steps_equal_hip_launches(queue, mode, B, hazards, layout):
    (e1, l1), (e2, l2) = _pair(mode, B, hazards=hazards or 3)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(9)
    pool = [(torch.rand(B, e1.n_u, device="cuda", generator=gen) * 2 - 1).contiguous() for _ in range(7)]
    mean = sigma = None
    if layout == "cols":
        cols = len(e1.PRIOR_COLS[mode])
        sigma = (0.2 * torch.rand(cols, B, device="cuda", generator=gen) + 0.05).contiguous()
        if mode == "Unicycle":
            mean = (0.01 * torch.randn(cols, B, device="cuda", generator=gen)).contiguous()
    K = 310 if mode == "SimulatedCars" else 40  # cars: every env passes its 300-step time limit and resets
    o1, o2 = e1.make_outputs(), e2.make_outputs()
    e1.safe_step_seq(pool, l1, mean=mean, sigma=sigma, outputs=o1, steps=K, prior_layout=layout)
    plan = queue.safe_step_plan(e2, pool, l2, steps=K, mean=mean, sigma=sigma, outputs=o2, prior_layout=layout)
    plan.run()
    torch.cuda.synchronize()
    _assert_same(_snapshot(e1, o1), _snapshot(e2, o2))
    # a second run of the same plan continues from the new state like K more launches
    e1.safe_step_seq(pool, l1, mean=mean, sigma=sigma, outputs=o1, steps=K, prior_layout=layout)
    plan.run()
    torch.cuda.synchronize()
    _assert_same(_snapshot(e1, o1), _snapshot(e2, o2))
    e1.check_failures()
    e2.check_failures()
    if mode == "SimulatedCars":
        assert int(e2.episode.min()) >= 1  # every env reset at least once inside the runs
    plan.free()


def test_plan_longer_than_the_ring(queue):
    """K = 5 000 steps through the 4 096-packet ring: rcbf_aql_run feeds the
    packets in as the packet processor frees slots; the result equals 5 000
    HIP launches bit for bit."""
    B, K = 512, 5000
    (e1, l1), (e2, l2) = _pair("SimulatedCars", B)
    pool = [(torch.rand(B, 1, device="cuda") * 2 - 1).contiguous() for _ in range(5)]
    o1, o2 = e1.make_outputs(), e2.make_outputs()
    plan = queue.safe_step_plan(e2, pool, l2, steps=K, outputs=o2)
    plan.run()
    e1.safe_step_seq(pool, l1, outputs=o1, steps=K)
    torch.cuda.synchronize()
    _assert_same(_snapshot(e1, o1), _snapshot(e2, o2))
    assert int(e2.episode.min()) >= 16  # 5 000 steps: every env through >= 16 time-limit resets
    plan.free()


def test_profiled_plan_times_and_span(queue):
    B = 65536
    (e1, l1), (e2, l2) = _pair("SimulatedCars", B)
    pool = [(torch.rand(B, 1, device="cuda") * 2 - 1).contiguous() for _ in range(3)]
    o1, o2 = e1.make_outputs(), e2.make_outputs()
    plan = queue.safe_step_plan(e2, pool, l2, steps=50, outputs=o2, profile=True)
    plan.run()
    t = plan.times_ns()
    dur = t[:, 1] - t[:, 0]
    assert (dur > 0).all() and (dur < 1_000_000).all()
    assert (np.diff(t[:, 0]) > 0).all()  # in order: each dispatch starts after the previous one started
    e1.safe_step_seq(pool, l1, outputs=o1, steps=50)
    torch.cuda.synchronize()
    _assert_same(_snapshot(e1, o1), _snapshot(e2, o2))
    # the span instantiation through the queue: the same step plus per-wave chip-clock stamps
    nw = B // 64
    span = torch.zeros(nw, 4, dtype=torch.int64, device="cuda")
    sp = queue.safe_step_plan(e2, pool[:1], l2, steps=1, outputs=o2, span=span)
    sp.run()
    e1.safe_step(pool[0], l1, outputs=o1)
    torch.cuda.synchronize()
    _assert_same(_snapshot(e1, o1), _snapshot(e2, o2))
    s = span.cpu().numpy()
    assert (s[:, 0] > 0).all() and (s[:, 1] >= s[:, 0]).all() and (s[:, 3] > s[:, 2]).all()
    assert (s[:, 1].max() - s[:, 0].min()) < 100_000  # < 1 ms of 100 MHz ticks
    clk = (s[:, 3] - s[:, 2]) / np.maximum(s[:, 1] - s[:, 0], 1) * 100.0  # MHz
    assert 500 < np.median(clk) < 3000
    e2.check_failures()


def test_one_step_plan_over_a_persistent_action_buffer(queue):
    """INTEGRATION.md's training-loop form: a one-step plan over a buffer the
    policy rewrites every step (torch writes it on its stream; run() waits for
    that work first).  30 steps equal 30 safe_step launches bit for bit."""
    B = 4096
    (e1, l1), (e2, l2) = _pair("Unicycle", B, hazards=5)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(4)
    acts = [(torch.rand(B, 2, device="cuda", generator=gen) * 2 - 1).contiguous() for _ in range(30)]
    o1, o2 = e1.make_outputs(), e2.make_outputs()
    u_buf = torch.zeros(B, 2, device="cuda")
    step1 = queue.safe_step_plan(e2, [u_buf], l2, steps=1, outputs=o2)
    for a in acts:
        e1.safe_step(a, l1, outputs=o1)
        u_buf.copy_(a)
        step1.run()
    torch.cuda.synchronize()
    _assert_same(_snapshot(e1, o1), _snapshot(e2, o2))
    step1.free()


def test_closing_the_queue_frees_its_plans():
    """A plan points into its queue: AqlQueue.close() frees the live plans
    first, and a freed plan (or one whose queue is closed) refuses to run
    instead of touching freed memory."""
    from rcbf_amd.aql import AqlQueue
    (e1, l1), _ = _pair("SimulatedCars", 256)
    q = AqlQueue(torch.device("cuda", 0))
    pool = [torch.zeros(256, 1, device="cuda")]
    p1 = q.safe_step_plan(e1, pool, l1, steps=2)
    p2 = q.safe_step_plan(e1, pool, l1, steps=3)
    p1.run()
    p2.free()
    with pytest.raises(RuntimeError, match="freed"):
        p2.run()
    q.close()
    with pytest.raises(RuntimeError, match="freed"):
        p1.run()


def test_plan_argument_errors(queue):
    (e1, l1), _ = _pair("SimulatedCars", 256)
    pool = [torch.zeros(256, 1, device="cuda")]
    with pytest.raises(RuntimeError, match="RCBF_E_BAD_SHAPE"):
        queue.safe_step_plan(e1, pool, l1, steps=0)
    with pytest.raises(ValueError):
        queue.safe_step_plan(e1, [], l1, steps=3)
    with pytest.raises(ValueError):  # a span plan needs K blocks of stamps
        queue.safe_step_plan(e1, pool, l1, steps=2, span=torch.zeros(4, 4, dtype=torch.int64, device="cuda"))
