"""Does enabling HSA profiling on the AQL queue (hsa_amd_profiling_set_profiler_enabled,
AqlQueue(profile=True), which bench.py opens for its dispatch timestamps) slow the
timed run?  Two queues in one process, profiling on / off, the same plans (cars,
B = 65 536, K = 20 and K = 1 000, product fences), runs interleaved: median wall
per run.  Prints one JSON."""
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
    qs = {"profiled": AqlQueue(dev, profile=True), "plain": AqlQueue(dev, profile=False)}
    plans = {(n, K): q.safe_step_plan(env, pool, layer, steps=K, outputs=outs) for n, q in qs.items() for K in (20, 1000)}
    for p in plans.values():
        p.run()
    walls = {k: [] for k in plans}
    for rep in range(40):
        for k, p in plans.items():
            if k[1] == 1000 and rep % 4:
                continue
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            p.run(sync_hip=False)
            walls[k].append(time.perf_counter() - t0)
    res = {f"{n}_K{K}_us_per_step": round(float(np.median(v)) * 1e6 / K, 4) for (n, K), v in walls.items()}
    env.check_failures()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
