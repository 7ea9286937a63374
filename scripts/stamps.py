"""Phase timing of the fused step from a -DRCBF_STAMPS=1 diagnostic build
(per-wave s_memtime at phase boundaries).  Usage:
  RCBF_HIP_LIB=build/variants/librcbf_stamps.so python scripts/stamps.py [B]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sac-rcbf_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rcbf_amd import _lib  # noqa: E402
from rcbf_amd.diff_cbf_qp import CBFQPLayer  # noqa: E402
from rcbf_amd.envs import BatchedSimulatedCarsEnv, BatchedUnicycleEnv  # noqa: E402


class A:
    cuda = True


B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
uni = "unicycle" in sys.argv[2:]
if uni:
    hz = np.array([[0., 0.], [-1., 1.], [-1., -1.]]) * 1.5
    env = BatchedUnicycleEnv(B, seed=3, hazards_locations=hz)
else:
    env = BatchedSimulatedCarsEnv(B, seed=3)
from bench import init_states  # noqa: E402  (SURVEY 8(d) start states, as the bench)
gen = torch.Generator(device="cuda")
gen.manual_seed(1000)
init_states(env, gen, "Unicycle" if uni else "SimulatedCars")
layer = CBFQPLayer(env, A(), gamma_b=20.0)
o = env.make_outputs()
nw = (B + 63) // 64
st = torch.zeros(nw * 16, dtype=torch.int64, device="cuda")
u = (torch.rand(B, env.n_u, device="cuda") * 2 - 1).contiguous()
lib = _lib.load()
names = ["load", "get_state", "rows+norm", "QP", "env step", "obs+stores issued", "stores drained"]
res = []
fbs = []
graph = "--eager" not in sys.argv  # default: steady state inside a hipGraph replay, like bench.py


def launch():
    rc = lib.rcbf_safe_step(ctypes.byref(layer._prm), B, _lib.ptr(env.x), _lib.ptr(env.aux), _lib.ptr(env.step_count),
                            _lib.ptr(env.episode), _lib.ptr(u), None, None, _lib.ptr(env.obs), _lib.ptr(o["u"]),
                            _lib.ptr(o["reward"]), _lib.ptr(o["cost"]), _lib.ptr(o["done"]), None, _lib.ptr(st),
                            None, 1, 1, 0, _lib.stream_of(torch.device("cuda")))
    assert rc == 0


if graph:
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        launch()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(20):
            launch()
for rep in range(30):
    if graph:
        g.replay()  # the stamps of the last of 20 back-to-back steps
    else:
        st.zero_()
        launch()
    torch.cuda.synchronize()
    if rep >= 10:
        t = st.view(nw, 16)[:, :8].cpu().numpy().astype(np.int64)
        res.append(np.diff(t, axis=1))
        fb = st.view(nw, 16)[:, 9].cpu().numpy()
        fbs = fbs + [fb] if rep > 10 else [fb]
d = np.concatenate(res)
print(f"B={B} ({'hipGraph replay' if graph else 'eager'}): per-phase s_memtime ticks per wave (median / p90), {d.shape[0]} wave samples")
for k, n in enumerate(names):
    print(f"  {n:20s} {np.median(d[:, k]):8.0f} {np.percentile(d[:, k], 90):8.0f}")
fbv = np.concatenate(fbs)
print(f"  waves with >=1 fp64-fallback lane: {(fbv > 0).mean():.4f}; lanes: {fbv.sum() / (64 * fbv.size):.5f}")
tot = d.sum(1)
print(f"  {'total':20s} {np.median(tot):8.0f} {np.percentile(tot, 90):8.0f}")
