"""GP posterior timings (rcbf_gp_predict) at the reference's GP size
(gp_model_size = 3000, main.py:247; cars n_s = 10), hipGraph-timed like
bench.py --extra: the exact posterior and LOVE's rank-100 Lanczos factor
(gpytorch fast_pred_var above 800 points, the DynamicsModel default), per
query batch.  For B <= 8 the kernel streams [R | alpha]: `Rt_GBs` is the
factor's bytes read per call / time (exact: the upper triangle only).
Usage: python scripts/gp_graph_bench.py [reps_small] [reps_large]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sac-rcbf_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rcbf_amd import gp  # noqa: E402


def time_graph(fn, reps):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = None
    for _ in range(3):
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        best = ms if best is None else min(best, ms)
    return best


def main():
    rs = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    rl = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    rng = np.random.default_rng(0)
    tx = rng.normal(0, 1, (3000, 10))
    ty = 0.1 * np.sin(tx) + rng.normal(0, 0.05, (3000, 10))
    hyper = [(1.5, 0.2, 0.05)] * 10
    out = {}
    only = os.environ.get("GP_BENCH_ONLY", "")  # e.g. "love100:256" -- one model (and batch) for a clean trace
    om, _, ob = only.partition(":")
    for name, rank in (("love100", 100), ("exact", None)):
        if om and name != om:
            continue
        m = gp.GPDisturbanceModel(tx, ty, hyper, device="cuda", rank=rank)
        if rank is None:
            rows = sum(min(m.N, 128 * (cb + 1)) for cb in range(m._m.C_pad // 128))
            rt_bytes = rows * 128 * 4 * 10
        else:
            rt_bytes = m._m.N_pad * m._m.C_pad * 4 * 10
        for B in (1, 2, 8, 256, 4096):
            if ob and B != int(ob):
                continue
            x = torch.as_tensor(rng.normal(0, 1, (B, 10)), dtype=torch.float32, device="cuda")
            ms = time_graph(lambda: m.predict(x), rs if B <= 256 else rl)
            rec = {"us": round(ms * 1e3, 2), "tflops": round(m.flops_per_query() * B / ms / 1e9, 2)}
            if B <= 8:
                rec["Rt_GBs"] = round(rt_bytes / ms / 1e6, 1)
            out[f"{name}_B{B}"] = rec
            print(name, B, rec, flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
