"""The training-loop form: one env step per host call with
the action buffer rewritten by torch before each step.  Per step, median
wall (host call to results complete) of: (a) a one-step AQL plan over the
persistent buffer (u_buf.copy_ + plan.run(), which waits for the copy), (b)
safe_step through HIP (u_buf.copy_ + env.safe_step + torch.cuda.synchronize).
Cars B = 65 536 and 4 096.  Prints one JSON."""
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
    q = AqlQueue(torch.device("cuda", 0))
    res = {}
    for B in (65536, 4096):
        env = BatchedSimulatedCarsEnv(B, device="cuda", seed=1)
        layer = CBFQPLayer(env, A(), gamma_b=20.0)
        gen = torch.Generator(device="cuda")
        gen.manual_seed(3)
        bench.init_states(env, gen, "SimulatedCars")
        acts = [(torch.rand(B, 1, device="cuda", generator=gen) * 2 - 1).contiguous() for _ in range(16)]
        outs = env.make_outputs()
        outs["goal_met"] = None
        u_buf = torch.zeros(B, 1, device="cuda")
        step1 = q.safe_step_plan(env, [u_buf], layer, steps=1, outputs=outs)

        def aql(j):
            u_buf.copy_(acts[j % 16])
            step1.run()

        def hip(j):
            u_buf.copy_(acts[j % 16])
            env.safe_step(u_buf, layer, outputs=outs)
            torch.cuda.synchronize()

        for name, fn in (("aql", aql), ("hip", hip), ("aql2", aql), ("hip2", hip)):
            for j in range(50):
                fn(j)
            ts = []
            for j in range(400):
                t0 = time.perf_counter()
                fn(j)
                ts.append(time.perf_counter() - t0)
            res[f"B{B}_{name}_us_per_step"] = round(float(np.median(ts)) * 1e6, 2)
        step1.free()
        env.check_failures()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
