"""Why the first dispatch of an AQL run is slower (span ~4.5 us against
~2.6 for the others, aql_timeline_r06c.json): a span-stamped 20-step plan
(rcbf_safe_step_span: per wave the chip clock and the shader clock at its
start and after its stores landed), run 10 times after a synchronize; per
dispatch: the spread of the wave starts (p50 / p90 / max - first start), the
median wave duration, the median shader clock.  Dispatch 0 against the median
of dispatches 1-19.  Prints one JSON."""
import json
import os
import sys

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
    B, K = 65536, 20
    env = BatchedSimulatedCarsEnv(B, device="cuda", seed=1)
    layer = CBFQPLayer(env, A(), gamma_b=20.0)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(3)
    bench.init_states(env, gen, "SimulatedCars")
    pool = [(torch.rand(B, 1, device="cuda", generator=gen) * 2 - 1).contiguous() for _ in range(K)]
    outs = env.make_outputs()
    outs["goal_met"] = None
    nw = B // 64
    span = torch.zeros(K, nw, 4, dtype=torch.int64, device="cuda")
    q = AqlQueue(torch.device("cuda", 0))
    plan = q.safe_step_plan(env, pool, layer, steps=K, outputs=outs, span=span)
    plan.run()
    per = []
    for _ in range(10):
        torch.cuda.synchronize()
        span.zero_()
        torch.cuda.synchronize()
        plan.run(sync_hip=False)
        t = span.cpu().numpy().astype(np.float64)
        rows = []
        for j in range(K):
            st, en, c0, c1 = t[j, :, 0], t[j, :, 1], t[j, :, 2], t[j, :, 3]
            s0 = st.min()
            rel = (st - s0) * 0.01
            clk = (c1 - c0) / np.maximum(en - st, 1) * 100.0
            rows.append([(en.max() - s0) * 0.01, np.percentile(rel, 50), np.percentile(rel, 90), rel.max(),
                         np.median((en - st) * 0.01), np.median(clk)])
        per.append(rows)
    a = np.median(np.array(per), 0)  # (K, 6) medians over runs
    names = ["span_us", "start_p50_us", "start_p90_us", "start_max_us", "wave_us_median", "shader_mhz"]
    res = {"dispatch0": {n: round(float(a[0, i]), 3) for i, n in enumerate(names)},
           "dispatch1_19_median": {n: round(float(np.median(a[1:, i])), 3) for i, n in enumerate(names)}}
    env.check_failures()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
