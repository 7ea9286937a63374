"""One GP posterior batch size, for counter passes (rocprofv3 --pmc) and
A/B timing: N = 3000 training points, n_s GPs, exact variance, B queries,
`reps` predictions after two warm-up calls; prints ms per prediction (HIP
events on the launch stream).  GP_RANK=r: LOVE's rank-r Lanczos factor instead.
Usage: python scripts/gp_one.py B [reps] [n_s] [N]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sac-rcbf_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rcbf_amd import gp  # noqa: E402

B = int(sys.argv[1])
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
n_s = int(sys.argv[3]) if len(sys.argv) > 3 else 10
N = int(sys.argv[4]) if len(sys.argv) > 4 else 3000
rng = np.random.default_rng(0)
tx = rng.normal(0, 1, (N, n_s))
ty = 0.1 * np.sin(tx) + rng.normal(0, 0.05, (N, n_s))
rank = int(os.environ["GP_RANK"]) if os.environ.get("GP_RANK") else None  # e.g. 100: LOVE's Lanczos factor
model = gp.GPDisturbanceModel(tx, ty, [(1.5, 0.2, 0.05)] * n_s, rank=rank)
if os.environ.get("RCBF_GP_DENSE"):  # A/B: read the whole [R | alpha] (no upper-triangular skip)
    model._m.flags = 0
x = torch.as_tensor(rng.normal(0, 1, (B, n_s)), dtype=torch.float32, device="cuda")
for _ in range(2):
    model.predict(x)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    model.predict(x)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / reps
fl = model.flops_per_query() * B
print(f"B={B} ms={ms:.4f} tflops={fl / (ms * 1e-3) / 1e12:.1f} frac={fl / (ms * 1e-3) / 1e12 / 157.3:.3f}")
