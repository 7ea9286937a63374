"""Where the driver form's ~10 us outside the GPU period go: a 20-step AQL
plan with timestamps on its first and last dispatch (RCBF_AQL_PROFILE_ENDS),
and the HSA system clock (the same clock, hsa_system_get_info TIMESTAMP) read
on the host just before the run call and just after it returns.  Per run:
host call -> first dispatch start, first start -> last end (the GPU period x
20), last end -> host return; median of 50 runs, cars B = 65 536.  Prints one
JSON."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "sac-rcbf_amd")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from rcbf_amd.aql import PROFILE_ENDS, AqlQueue  # noqa: E402
from rcbf_amd.diff_cbf_qp import CBFQPLayer  # noqa: E402
from rcbf_amd.envs import BatchedSimulatedCarsEnv  # noqa: E402


class A:
    cuda = True


def main():
    hsa = ctypes.CDLL("libhsa-runtime64.so.1")
    freq = ctypes.c_uint64()

    def now_ns():
        t = ctypes.c_uint64()
        hsa.hsa_system_get_info(2, ctypes.byref(t))
        return t.value * 1e9 / freq.value

    B = 65536
    env = BatchedSimulatedCarsEnv(B, device="cuda", seed=1)
    layer = CBFQPLayer(env, A(), gamma_b=20.0)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(3)
    bench.init_states(env, gen, "SimulatedCars")
    pool = [(torch.rand(B, 1, device="cuda", generator=gen) * 2 - 1).contiguous() for _ in range(20)]
    outs = env.make_outputs()
    outs["goal_met"] = None
    q = AqlQueue(torch.device("cuda", 0), profile=True)  # the library's hsa_init: the runtime is up from here
    hsa.hsa_system_get_info(3, ctypes.byref(freq))
    assert freq.value > 0
    p = q.safe_step_plan(env, pool, layer, steps=20, outputs=outs, fence_flags=PROFILE_ENDS)
    p.run()
    rows = []
    for _ in range(50):
        torch.cuda.synchronize()
        t0 = now_ns()
        p.run(sync_hip=False)
        t1 = now_ns()
        t = p.times_ns().astype(np.float64)
        rows.append((t[0, 0] - t0, t[-1, 1] - t[0, 0], t1 - t[-1, 1], t1 - t0))
    r = np.median(np.array(rows), 0) / 1e3
    res = {"host_call_to_first_start_us": round(r[0], 2), "first_start_to_last_end_us": round(r[1], 2),
           "last_end_to_host_return_us": round(r[2], 2), "host_call_to_return_us": round(r[3], 2),
           "period_us": round(r[1] / 20, 3)}
    env.check_failures()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
