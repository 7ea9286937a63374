"""Host cost of replaying the bench's 20-step hipGraph: torch's
CUDAGraph.replay() against hipGraphLaunch on the same instantiated graph
(CUDAGraph.raw_cuda_graph_exec(), through the HIP runtime torch loaded).
Cars fused step, B = 65536, SURVEY start states; per form: host time of the
launch call, wall time of the whole region (sync to sync) and HIP events
around it, median of 30 timed regions.  Prints one JSON line."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sac-rcbf_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    sys.argv = [sys.argv[0], "--steps", str(K), "--warmup", "5"]
    args = bench.parse()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    env, layer, graph, S, _ = bench.setup_gpu(args, dev, 0, args.batch)
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipGraphLaunch.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    exe = ctypes.c_void_p(graph.raw_cuda_graph_exec())
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)

    def direct():
        rc = hip.hipGraphLaunch(exe, stream)
        assert rc == 0, rc

    out = {}
    for name, fn in (("torch_replay", graph.replay), ("hipGraphLaunch", direct)):
        host, wall, ev = [], [], []
        for rep in range(35):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e0.record()
            fn()
            t1 = time.perf_counter()
            e1.record()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            if rep >= 5:
                host.append((t1 - t0) * 1e6)
                wall.append((t2 - t0) * 1e6)
                ev.append(e0.elapsed_time(e1) * 1e3)
        out[name] = {"host_us": round(float(np.median(host)), 2), "wall_us": round(float(np.median(wall)), 2),
                     "event_us": round(float(np.median(ev)), 2),
                     "wall_us_per_step": round(float(np.median(wall)) / K, 3)}
    env.check_failures()
    print(json.dumps({"K": K, **out}))


if __name__ == "__main__":
    main()
