"""Roofline of the GP disturbance posterior (rcbf_gp_predict)
at the reference's GP size (gp_model_size = 3000, main.py:247), exact
variance (r = N), for the SAC-update batch (256), config-2 batch (4096) and
the env batch (65536).  Algorithmic work: 2 N C_pad flops per query per GP
(the k(x, X) [R | alpha] product on the fp32 MFMA, peak 157.3 TFLOP/s) plus
N exps; timed with HIP events on the launch stream.
Usage: python scripts/gp_bench.py [n_s] [N] [rank]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sac-rcbf_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rcbf_amd import gp  # noqa: E402

n_s = int(sys.argv[1]) if len(sys.argv) > 1 else 10
N = int(sys.argv[2]) if len(sys.argv) > 2 else 3000
rank = int(sys.argv[3]) if len(sys.argv) > 3 else None
rng = np.random.default_rng(0)
tx = rng.normal(0, 1, (N, n_s))
ty = 0.1 * np.sin(tx) + rng.normal(0, 0.05, (N, n_s))
hyper = [(1.5, 0.2, 0.05)] * n_s
model = gp.GPDisturbanceModel(tx, ty, hyper, rank=rank)
PEAK = 157.3  # TFLOP/s dense fp32 MFMA (MI355X_MICROARCH.md)
out = {"n_s": n_s, "N": N, "rank": model.r, "C_pad": model._m.C_pad}
for B in (1, 8, 256, 4096, 65536):
    x = torch.as_tensor(rng.normal(0, 1, (B, n_s)), dtype=torch.float32, device="cuda")
    for _ in range(2):
        model.predict(x)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20 if B <= 4096 else 3
    e0.record()
    for _ in range(reps):
        model.predict(x)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    fl = model.flops_per_query() * B
    out[f"B{B}"] = {"ms": round(ms, 4), "queries_per_s": round(B / (ms * 1e-3), 1),
                    "tflops": round(fl / (ms * 1e-3) / 1e12, 2), "frac_fp32_mfma": round(fl / (ms * 1e-3) / 1e12 / PEAK, 4),
                    "Rt_stream_GBs": round(model.Rt.numel() * 4 / (ms * 1e-3) / 1e9, 1)}  # HBM-bound at B <= 8
print(json.dumps(out))
