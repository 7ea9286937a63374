"""Where a short run of fused steps spends its wall time (the driver's
20-step form): hipGraph replay vs the AQL plan, K = 1 ... 1000, wall per run
(synchronize -> launch -> synchronize, no events), and a span-stamped AQL run
of 20 steps (per step: first wave start, last wave end, chip clock), so the
start latency, the per-kernel span and the gaps of a cold 20-step run can be
read off.  Prints one JSON object."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "sac-rcbf_amd")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from rcbf_amd.aql import AqlQueue  # noqa: E402
from rcbf_amd.diff_cbf_qp import CBFQPLayer  # noqa: E402
from rcbf_amd.envs import BatchedSimulatedCarsEnv  # noqa: E402


class A:
    cuda = True


def main():
    dev = torch.device("cuda", 0)
    B = 65536
    env = BatchedSimulatedCarsEnv(B, device=dev, seed=1234)
    layer = CBFQPLayer(env, A(), gamma_b=20.0)
    gen = torch.Generator(device=dev)
    gen.manual_seed(1000)
    bench.init_states(env, gen, "SimulatedCars")
    pool = [(torch.rand(B, 1, device=dev, generator=gen) * 2 - 1).contiguous() for _ in range(50)]
    outs = env.make_outputs()
    outs["goal_met"] = None
    q = AqlQueue(dev, profile=True)
    res = {}
    Ks = [1, 2, 5, 10, 20, 50, 100, 1000]
    plans = {K: q.safe_step_plan(env, pool, layer, steps=K, outputs=outs) for K in Ks}
    graphs = {}
    for K in Ks:
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            env.safe_step(pool[0], layer, outputs=outs)
        torch.cuda.current_stream().wait_stream(s)
        with torch.cuda.graph(g):
            for j in range(min(K, 500)):
                env.safe_step(pool[j % 50], layer, outputs=outs)
        g.replay()
        graphs[K] = g
    torch.cuda.synchronize()
    plans[1000].run()

    def wall(fn, reps=30, gap_s=0.0):
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize()
            if gap_s:
                time.sleep(gap_s)
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts)) * 1e6

    for K in Ks:
        res[f"aql_K{K}_us"] = round(wall(lambda: plans[K].run(sync_hip=False)), 2)
        if K <= 500:
            res[f"graph_K{K}_us"] = round(wall(lambda: graphs[K].replay()), 2)
    # after an idle gap (the GPU drops its clock when idle?)
    for gap in (0.001, 0.01):
        res[f"aql_K20_after_{int(gap * 1e3)}ms_idle_us"] = round(wall(lambda: plans[20].run(sync_hip=False), 20, gap), 2)
        res[f"graph_K20_after_{int(gap * 1e3)}ms_idle_us"] = round(wall(lambda: graphs[20].replay(), 20, gap), 2)
    # the driver form's own sequence around the 20 steps: HIP events recorded before and after
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def ev_graph():
        e0.record()
        graphs[20].replay()
        e1.record()
    res["graph_K20_with_events_us"] = round(wall(ev_graph), 2)

    def ev_aql():
        e0.record()
        plans[20].run(sync_hip=False)
        e1.record()
    res["aql_K20_with_events_us"] = round(wall(ev_aql), 2)
    # host cost of the calls alone
    t0 = time.perf_counter()
    for _ in range(100):
        e0.record()
    torch.cuda.synchronize()
    res["event_record_host_us"] = round((time.perf_counter() - t0) * 1e4, 3)
    t0 = time.perf_counter()
    for _ in range(100):
        torch.cuda.synchronize()
    res["idle_synchronize_us"] = round((time.perf_counter() - t0) * 1e4, 3)
    # span-stamped AQL run of 20 steps: per step first start / last end (100 MHz chip clock)
    nw = B // 64
    span = torch.zeros(20, nw, 4, dtype=torch.int64, device=dev)
    sp = q.safe_step_plan(env, pool, layer, steps=20, outputs=outs, span=span)
    for rep in range(3):
        torch.cuda.synchronize()
        span.zero_()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sp.run(sync_hip=False)
        w = (time.perf_counter() - t0) * 1e6
        t = span.cpu().numpy().astype(np.float64)
        st, en = t[:, :, 0].min(1), t[:, :, 1].max(1)
        res[f"span20_rep{rep}"] = {"wall_us": round(w, 2), "first_start_to_last_end_us": round((en[-1] - st[0]) * .01, 2),
                                   "span_us": [round(v, 2) for v in (en - st) * .01],
                                   "gap_us": [round(v, 2) for v in (st[1:] - en[:-1]) * .01]}
    # the same with the graph path (span entry point through HIP)
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g2):
        for j in range(20):
            env.safe_step_span(pool[j], layer, span[j], outputs=outs)
    g2.replay()
    for rep in range(3):
        torch.cuda.synchronize()
        span.zero_()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g2.replay()
        torch.cuda.synchronize()
        w = (time.perf_counter() - t0) * 1e6
        t = span.cpu().numpy().astype(np.float64)
        st, en = t[:, :, 0].min(1), t[:, :, 1].max(1)
        res[f"graph_span20_rep{rep}"] = {"wall_us": round(w, 2),
                                         "first_start_to_last_end_us": round((en[-1] - st[0]) * .01, 2),
                                         "span_us": [round(v, 2) for v in (en - st) * .01],
                                         "gap_us": [round(v, 2) for v in (st[1:] - en[:-1]) * .01]}
    # fence-scope variants of the AQL plan (flags of rcbf_aql_safe_step_plan): wall of K = 1 / 20 and the
    # span-stamped 20-step run (first span, median gap)
    for fl in (0, 2, 16, 32, 8):
        p1 = q.safe_step_plan(env, pool, layer, steps=1, outputs=outs, fence_flags=fl)
        p20 = q.safe_step_plan(env, pool, layer, steps=20, outputs=outs, fence_flags=fl)
        s20 = q.safe_step_plan(env, pool, layer, steps=20, outputs=outs, span=span, fence_flags=fl)
        p20.run()
        r = {"K1_us": round(wall(lambda: p1.run(sync_hip=False)), 2),
             "K20_us": round(wall(lambda: p20.run(sync_hip=False)), 2)}
        firsts, gaps, f2l = [], [], []
        for rep in range(5):
            torch.cuda.synchronize()
            span.zero_()
            torch.cuda.synchronize()
            s20.run(sync_hip=False)
            t = span.cpu().numpy().astype(np.float64)
            st, en = t[:, :, 0].min(1), t[:, :, 1].max(1)
            firsts.append((en[0] - st[0]) * .01)
            gaps.append(float(np.median((st[1:] - en[:-1]) * .01)))
            f2l.append((en[-1] - st[0]) * .01)
        r.update({"first_span_us": round(float(np.median(firsts)), 2), "gap_us": round(float(np.median(gaps)), 2),
                  "first_start_to_last_end_us": round(float(np.median(f2l)), 2)})
        res[f"fence_flags_{fl}"] = r
        for pp in (p1, p20, s20):
            pp.free()
    env.check_failures()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
