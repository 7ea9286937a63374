"""Control for the kernel-trace vs untraced gap: what
rocprofv3 --kernel-trace does to kernels that are not ours.

Two torch kernels, each captured N times in one hipGraph and replayed, timed
by HIP events on the replay stream (per launch), exactly as bench.py times
the fused step:
  copy  -- dst.copy_(src) of 7.9 MB fp64 (read 7.9 + write 7.9 = 15.8 MB,
           the fused cars step's algorithmic bytes at B = 65 536);
  tiny  -- a 256-element add_ (the dependent-kernel boundary alone).
Run it plain (prints the events figures) and under
`rocprofv3 --kernel-trace --stats` (the trace gives each kernel's traced
duration); the difference is the tracer's, not the fused step's.
Usage: python scripts/tracer_control.py [N]"""
import json
import sys

import torch


def timed(fn, n, reps=3):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = []
    for _ in range(reps):
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best.append(e0.elapsed_time(e1) * 1e3 / n)
    return sorted(best)[len(best) // 2]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    src = torch.rand(65536 * 15, dtype=torch.float64, device="cuda")  # 7.86 MB
    dst = torch.empty_like(src)
    tiny = torch.zeros(256, device="cuda")
    copy_us = timed(lambda: dst.copy_(src), n)
    tiny_us = timed(lambda: tiny.add_(1.0), n)
    nbytes = 2 * src.numel() * 8
    print(json.dumps({"copy_bytes": nbytes, "copy_us_per_launch_events": round(copy_us, 3),
                      "copy_GBs_events": round(nbytes / copy_us / 1e3, 1),
                      "tiny_us_per_launch_events": round(tiny_us, 3), "launches": n}), flush=True)


if __name__ == "__main__":
    main()
