#!/usr/bin/env python3
"""Where the fixed cost of a short timed region goes (the driver runs
`bench.py --steps 20`): host time of graph.replay(), GPU start latency
(event before replay -> first kernel), and the completion wait
(torch.cuda.synchronize vs spinning on an event query).  Cars B = 65536,
SURVEY start states, one hipGraph of K fused steps; prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sac-rcbf_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
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
    pool = [(torch.rand(B, 1, device=dev, generator=gen) * 2 - 1).contiguous() for _ in range(20)]
    outs = env.make_outputs()
    outs["goal_met"] = None
    res = {}
    for K in (20, 100, 500):
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            env.safe_step(pool[0], layer, outputs=outs)
        torch.cuda.current_stream(dev).wait_stream(s)
        with torch.cuda.graph(g):
            for j in range(K):
                env.safe_step(pool[j % 20], layer, outputs=outs)
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        rows = {"replay_host_us": [], "wall_sync_us": [], "wall_spin_us": [], "event_us": []}
        for rep in range(20):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e0.record()
            g.replay()
            t1 = time.perf_counter()
            e1.record()
            if rep % 2:
                while not e1.query():
                    pass
                rows["wall_spin_us"].append((time.perf_counter() - t0) * 1e6)
            else:
                torch.cuda.synchronize()
                rows["wall_sync_us"].append((time.perf_counter() - t0) * 1e6)
            torch.cuda.synchronize()
            rows["replay_host_us"].append((t1 - t0) * 1e6)
            rows["event_us"].append(e0.elapsed_time(e1) * 1e3)
        res[f"K{K}"] = {k: round(sorted(v)[len(v) // 2], 2) for k, v in rows.items()}
        res[f"K{K}"]["per_step_event_us"] = round(res[f"K{K}"]["event_us"] / K, 3)
    # eager K = 20 through the CPython binding
    rows = []
    for rep in range(10):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for j in range(20):
            env.safe_step(pool[j], layer, outputs=outs)
        torch.cuda.synchronize()
        rows.append((time.perf_counter() - t0) * 1e6)
    res["eager_K20_wall_us"] = round(sorted(rows)[5], 2)
    env.check_failures()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
