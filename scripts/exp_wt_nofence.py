"""Write-through outputs + AQL packets without the per-step release (study).

The product AQL plan releases at agent scope after every step (the XCD L2
write-back), which costs ~1 us of the ~1.6 us step boundary
(profiles/r06/aql_fences_r06e/f.json).  A library built with -DRCBF_WT_OUT=1
stores every output write-through (`sc1`) and drains each wave's stores before
it ends, so nothing the step writes is dirty in an L2 when the dispatch
completes, and the next packet's agent-scope acquire is all the next step
needs.  This script measures, for the library it runs with (RCBF_HIP_LIB /
the code object given):

  parity: K AQL steps with fence_flags (0 = product fences, 32 = no release
          between steps) against K HIP launches of the same library, bit for
          bit, the tests' configurations plus a 1 000-step cars soak;
  timing: K = 20 and K = 1 000 wall per run and the span-stamped 20-step run
          (first span, median span, median gap) per fence setting, cars
          B = 65 536 and unicycle k = 5 B = 65 536.

Usage: python scripts/exp_wt_nofence.py LABEL [CODE_OBJECT]   (prints one JSON)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "sac-rcbf_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from rcbf_amd.aql import AqlQueue  # noqa: E402
from test_gpu_headline_parity import _make  # noqa: E402


def pair(mode, B, hazards=3, seed=77):
    out = []
    for _ in range(2):
        env, layer = _make(mode, B, hazards=hazards, seed=seed)
        gen = torch.Generator(device="cuda")
        gen.manual_seed(5)
        bench.init_states(env, gen, mode)
        out.append((env, layer))
    return out


def snap(env, o):
    t = {"x": env.x, "aux": env.aux, "step": env.step_count, "episode": env.episode, "obs": env.obs}
    t.update({k: v for k, v in o.items() if v is not None})
    return {k: v.clone() for k, v in t.items()}


def diff(a, b):
    return sorted(k for k in a if not torch.equal(a[k], b[k]))


def parity(q, mode, B, hazards, layout, K, fl, runs=2):
    (e1, l1), (e2, l2) = pair(mode, B, hazards=hazards or 3)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(9)
    pool = [(torch.rand(B, e1.n_u, device="cuda", generator=gen) * 2 - 1).contiguous() for _ in range(7)]
    mean = sigma = None
    if layout == "cols":
        cols = len(e1.PRIOR_COLS[mode])
        sigma = (0.2 * torch.rand(cols, B, device="cuda", generator=gen) + 0.05).contiguous()
        if mode == "Unicycle":
            mean = (0.01 * torch.randn(cols, B, device="cuda", generator=gen)).contiguous()
    o1, o2 = e1.make_outputs(), e2.make_outputs()
    plan = q.safe_step_plan(e2, pool, l2, steps=K, mean=mean, sigma=sigma, outputs=o2, prior_layout=layout,
                            fence_flags=fl)
    bad = []
    for r in range(runs):
        e1.safe_step_seq(pool, l1, mean=mean, sigma=sigma, outputs=o1, steps=K, prior_layout=layout)
        plan.run()
        torch.cuda.synchronize()
        bad.append(diff(snap(e1, o1), snap(e2, o2)))
    plan.free()
    e1.check_failures()
    e2.check_failures()
    return {"mode": mode, "B": B, "k": hazards, "layout": layout, "K": K, "fence_flags": fl,
            "mismatched_per_run": bad, "ok": not any(bad), "min_episode": int(e2.episode.min())}


def timing(q, mode, B, hazards, fl):
    (env, layer), _ = pair(mode, B, hazards=hazards or 3)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(1000)
    pool = [(torch.rand(B, env.n_u, device="cuda", generator=gen) * 2 - 1).contiguous() for _ in range(50)]
    outs = env.make_outputs()
    outs["goal_met"] = None
    p20 = q.safe_step_plan(env, pool, layer, steps=20, outputs=outs, fence_flags=fl)
    p1k = q.safe_step_plan(env, pool, layer, steps=1000, outputs=outs, fence_flags=fl)
    nw = (B + 63) // 64
    span = torch.zeros(20, nw, 4, dtype=torch.int64, device="cuda")
    s20 = q.safe_step_plan(env, pool, layer, steps=20, outputs=outs, span=span, fence_flags=fl)
    p1k.run()

    def wall(fn, reps):
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts)) * 1e6

    r = {"K20_us": round(wall(lambda: p20.run(sync_hip=False), 40), 2),
         "K1000_us_per_step": round(wall(lambda: p1k.run(sync_hip=False), 7) / 1000, 4)}
    firsts, spans, gaps = [], [], []
    for _ in range(7):
        torch.cuda.synchronize()
        span.zero_()
        torch.cuda.synchronize()
        s20.run(sync_hip=False)
        t = span.cpu().numpy().astype(np.float64)
        st, en = t[:, :, 0].min(1), t[:, :, 1].max(1)
        firsts.append((en[0] - st[0]) * .01)
        spans.append(float(np.median((en - st)[1:])) * .01)
        gaps.append(float(np.median((st[1:] - en[:-1]) * .01)))
    r.update({"first_span_us": round(float(np.median(firsts)), 3), "span_us": round(float(np.median(spans)), 3),
              "gap_us": round(float(np.median(gaps)), 3)})
    for pp in (p20, p1k, s20):
        pp.free()
    env.check_failures()
    return r


def ragged():
    """The product library, no release between steps, on grids whose workgroup count is NOT a multiple of the
    8 XCDs (B = 960: 15 workgroups of 64; B = 65 280: 510 of 128; B = 1 000: 16 of 64, a multiple, as the
    control): if the dispatcher's round-robin start moves from one dispatch to the next, a tile lands on another
    XCD than the one holding its dirty lines and reads stale state."""
    q = AqlQueue(torch.device("cuda", 0))
    out = []
    for B in (960, 65280, 1000):
        for fl in (32, 0):
            out.append(parity(q, "SimulatedCars", B, 0, "rows", 310, fl, runs=3))
            print(json.dumps(out[-1]), flush=True)
    print("RAGGED " + json.dumps(out), flush=True)


def main():
    if sys.argv[1] == "ragged":
        return ragged()
    label = sys.argv[1]
    co = sys.argv[2] if len(sys.argv) > 2 else None
    q = AqlQueue(torch.device("cuda", 0), code_object=co)
    res = {"label": label, "lib": os.environ.get("RCBF_HIP_LIB", "product"), "code_object": co or "product",
           "parity": [], "timing": {}}
    cases = [("SimulatedCars", 65536, 0, "rows", 310), ("SimulatedCars", 4096, 0, "rows", 310),
             ("SimulatedCars", 1000, 0, "cols", 310), ("Unicycle", 65536, 5, "rows", 40),
             ("Unicycle", 4096, 3, "cols", 40), ("SimulatedCars", 65536, 0, "rows", 1000)]
    for fl in (32, 0):
        for c in cases:
            res["parity"].append(parity(q, *c, fl))
            print(json.dumps(res["parity"][-1]), flush=True)
    for mode, k in (("SimulatedCars", 0), ("Unicycle", 5)):
        for fl in (0, 32, 8):
            res["timing"][f"{mode}_k{k}_flags{fl}"] = timing(q, mode, 65536, k, fl)
            print(mode, k, fl, json.dumps(res["timing"][f"{mode}_k{k}_flags{fl}"]), flush=True)
    print("RESULT " + json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
