#!/usr/bin/env python3
"""Experiment: does splitting the B = 65 536 batch into S shards on S HIP
streams (one hipGraph chain each, replayed concurrently) hide the per-launch
floor of the fused step?  Also measures the graph-node floor of a trivial
kernel.  Prints one line per variant: µs per step of the WHOLE batch."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "sac-rcbf_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--shards", default="d1,m1,f2,m2,f4,m4,d1,f2,f4")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--reps", type=int, default=8)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from rcbf_amd.diff_cbf_qp import CBFQPLayer
    from rcbf_amd.envs import BatchedSimulatedCarsEnv

    class LArgs:
        cuda = True

    B, S = args.batch, args.steps
    full = BatchedSimulatedCarsEnv(B, device=dev, seed=1234)
    layer = CBFQPLayer(full, LArgs(), gamma_b=20.0)
    gen = torch.Generator(device=dev)
    gen.manual_seed(1000)
    bench.init_states(full, gen, "SimulatedCars")
    rows, aux, stc = full.state.clone(), full.aux.clone(), full.step_count.clone()
    pool = [(torch.rand(B, 1, device=dev, generator=gen) * 2 - 1).contiguous() for _ in range(S)]

    # graph-node floor: a one-element add per node
    t1 = torch.zeros(1, device=dev)
    s0 = torch.cuda.Stream(device=dev)
    with torch.cuda.stream(s0):
        t1.add_(1.0)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s0):
        for _ in range(S):
            t1.add_(1.0)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    print(f"floor add_(1 elem) per graph node: {e0.elapsed_time(e1) * 1e3 / (args.reps * S):.3f} us", flush=True)

    def make(ns):
        b = B // ns
        envs, outs = [], []
        for k in range(ns):
            e = BatchedSimulatedCarsEnv(b, device=dev, seed=1234, env_offset=k * b)
            e.load_state(rows[k * b:(k + 1) * b], aux[k * b:(k + 1) * b], stc[k * b:(k + 1) * b])
            o = e.make_outputs()
            o["goal_met"] = None
            envs.append(e)
            outs.append(o)
        torch.cuda.synchronize()
        return b, envs, outs

    def timed(replay, label, envs):
        replay()
        torch.cuda.synchronize()
        e0.record()
        for _ in range(args.reps):
            replay()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / (args.reps * S)
        for e in envs:
            e.check_failures()
        print(f"{label}: {us:.3f} us per step of {B} envs -> {B / us * 1e-3:.3f} G steps/s", flush=True)

    cur = torch.cuda.current_stream(dev)
    for spec in args.shards.split(","):
        kind, ns = spec[0], int(spec[1:])
        b, envs, outs = make(ns)
        for k in range(ns):
            for j in range(3):
                envs[k].safe_step(pool[j][k * b:(k + 1) * b], layer, outputs=outs[k])
        torch.cuda.synchronize()
        if kind == "d":  # bench.py style: capture on torch's capture stream, replay on the current stream
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for j in range(S):
                    for k in range(ns):
                        envs[k].safe_step(pool[j][k * b:(k + 1) * b], layer, outputs=outs[k])
            timed(g.replay, f"d{ns} one graph, one stream, shards interleaved, b={b}", envs)
        elif kind == "f":  # one graph, shard k's chain on forked stream k inside the capture
            g = torch.cuda.CUDAGraph()
            side = [torch.cuda.Stream(device=dev) for _ in range(ns)]
            with torch.cuda.graph(g):
                cap = torch.cuda.current_stream(dev)
                for k in range(ns):
                    side[k].wait_stream(cap)
                    with torch.cuda.stream(side[k]):
                        for j in range(S):
                            envs[k].safe_step(pool[j][k * b:(k + 1) * b], layer, outputs=outs[k])
                for k in range(ns):
                    cap.wait_stream(side[k])
            timed(g.replay, f"f{ns} one graph, {ns} forked branches, b={b}", envs)
        else:  # ns graphs replayed on ns streams
            streams = [torch.cuda.Stream(device=dev) for _ in range(ns)]
            graphs = []
            for k in range(ns):
                gk = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gk, stream=streams[k]):
                    for j in range(S):
                        envs[k].safe_step(pool[j][k * b:(k + 1) * b], layer, outputs=outs[k])
                graphs.append(gk)

            def replay_all():
                for k in range(ns):
                    streams[k].wait_stream(cur)
                for k in range(ns):
                    with torch.cuda.stream(streams[k]):
                        graphs[k].replay()
                for k in range(ns):
                    cur.wait_stream(streams[k])
            timed(replay_all, f"m{ns} {ns} graphs on {ns} streams, b={b}", envs)


if __name__ == "__main__":
    main()
