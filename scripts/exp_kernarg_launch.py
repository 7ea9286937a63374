"""Does the kernel-argument size change the cost of replaying a 20-node
hipGraph?  Graph A: 20 launches of rcbf_safe_step at B = 256 (one
workgroup; rcbf_params by value + 20 pointers/scalars, ~400 B of kernel
arguments).  Graph B: 20 launches of rcbf_gather_rows_f64 with 256 rows
(6 arguments, ~48 B).  Both kernels take ~2 us.  Per graph: host time of the
replay call, wall time sync to sync and HIP events around it, median of 30
timed replays after 10.  Prints one JSON line."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sac-rcbf_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rcbf_amd import _lib  # noqa: E402
from rcbf_amd.diff_cbf_qp import CBFQPLayer  # noqa: E402
from rcbf_amd.envs import BatchedSimulatedCarsEnv  # noqa: E402


class A:
    cuda = True


def timed(graph, K):
    host, wall, ev = [], [], []
    for rep in range(40):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record()
        graph.replay()
        t1 = time.perf_counter()
        e1.record()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        if rep >= 10:
            host.append((t1 - t0) * 1e6)
            wall.append((t2 - t0) * 1e6)
            ev.append(e0.elapsed_time(e1) * 1e3)
    return {"host_us": round(float(np.median(host)), 2), "wall_us": round(float(np.median(wall)), 2),
            "event_us": round(float(np.median(ev)), 2)}


def capture(fn, K):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(K):
            fn()
    g.replay()
    torch.cuda.synchronize()
    return g


def main():
    K = 20
    dev = torch.device("cuda", 0)
    lib = _lib.load()
    env = BatchedSimulatedCarsEnv(256, device=dev)
    layer = CBFQPLayer(env, A(), gamma_b=20.0)
    u = torch.zeros(256, 1, device=dev)
    outs = env.make_outputs()
    outs["goal_met"] = None
    ga = capture(lambda: env.safe_step(u, layer, outputs=outs), K)
    ring = torch.zeros(1 << 16, 25, dtype=torch.float64, device=dev)
    idx = torch.randint(0, 1 << 16, (256,), device=dev)
    dst = torch.empty(256, 25, dtype=torch.float64, device=dev)
    gb = capture(lambda: lib.rcbf_gather_rows_f64(_lib.ptr(dst), _lib.ptr(ring), 25, _lib.ptr(idx), 256,
                                                  _lib.stream_of(dev)), K)
    print(json.dumps({"K": K, "safe_step_B256_400B_args": timed(ga, K), "gather_256_48B_args": timed(gb, K)}))


if __name__ == "__main__":
    main()
