"""Phase timing of the fused step from the study build
(sac-rcbf_amd/csrc/study/rcbf_stamps.hip: the same kernel template with
per-wave s_memtime stamps at phase boundaries).  Build it here (hipcc,
gfx950) with `python scripts/stamps.py --build`, then on the GPU:
  python scripts/stamps.py [B] [unicycle [K]] [--eager]"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sac-rcbf_amd")]
STUDY_LIB = os.path.join(ROOT, "build", "study", "librcbf_stamps.so")
if "--build" in sys.argv:
    os.makedirs(os.path.dirname(STUDY_LIB), exist_ok=True)
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-std=c++17",
           "-fhip-fp32-correctly-rounded-divide-sqrt", "-mllvm", "-amdgpu-kernarg-preload-count=16",
           "-I" + os.path.join(ROOT, "include"),
           "-I" + os.path.join(ROOT, "sac-rcbf_amd", "csrc"), "-o", STUDY_LIB,
           os.path.join(ROOT, "sac-rcbf_amd", "csrc", "study", "rcbf_stamps.hip")]
    subprocess.run(cmd, check=True)
    sys.exit(0)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rcbf_amd import _lib  # noqa: E402
from rcbf_amd.diff_cbf_qp import CBFQPLayer  # noqa: E402
from rcbf_amd.envs import BatchedSimulatedCarsEnv, BatchedUnicycleEnv  # noqa: E402


class A:
    cuda = True


args = [a for a in sys.argv[1:] if not a.startswith("--")]
B = int(args[0]) if args else 65536
uni = "unicycle" in args[1:]
if uni:
    k = int(args[2]) if len(args) > 2 else 3
    from rcbf_amd.envs import _EnvSpec
    hz = _EnvSpec("Unicycle").hazards_locations[:k]
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
slib = ctypes.CDLL(STUDY_LIB)
P = ctypes.c_void_p
slib.rcbf_study_safe_step_stamps.argtypes = [ctypes.POINTER(_lib.RcbfParams), ctypes.c_int64] + [P] * 11 + [
    ctypes.c_int32, ctypes.c_uint64, P]
# the unicycle QP's per-stage record (rcbf_device.hpp RCBF_QP_STAMP / RCBF_QP_COUNT)
qst = torch.zeros(nw * 16, dtype=torch.int64, device="cuda")
slib.rcbf_study_set_qp_stamps.argtypes = [P]
assert slib.rcbf_study_set_qp_stamps(_lib.ptr(qst) if uni else None) == 0
qres, qcnt = [], []
names = ["load", "get_state", "rows+norm", "QP", "env step", "obs+stores issued", "stores drained"]
res, real = [], []
fbs = []
graph = "--eager" not in sys.argv  # default: steady state inside a hipGraph replay, like bench.py


def launch():
    rc = slib.rcbf_study_safe_step_stamps(ctypes.byref(layer._prm), B, _lib.ptr(env.x), _lib.ptr(env.aux),
                                          _lib.ptr(env.step_count), _lib.ptr(env.episode), _lib.ptr(u),
                                          _lib.ptr(env.obs), _lib.ptr(o["u"]), _lib.ptr(o["reward"]),
                                          _lib.ptr(o["cost"]), _lib.ptr(o["done"]), _lib.ptr(st), 1, 1,
                                          _lib.stream_of(torch.device("cuda")))
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
        rt = st.view(nw, 16)[:, 10:12].cpu().numpy().astype(np.int64)
        rt = rt[(rt > 0).all(1)]
        real.append((rt[:, 1].max() - rt[:, 0].min(), np.percentile(rt[:, 0] - rt[:, 0].min(), 50),
                     rt[:, 0].max() - rt[:, 0].min(), np.percentile(rt[:, 1] - rt[:, 0], 50)))
        if uni:
            q = qst.view(nw, 16).cpu().numpy().astype(np.int64)
            qres.append(np.diff(q[:, [0, 1, 2, 3, 4, 9]], axis=1))
            qcnt.append(q[:, [5, 6, 7, 8, 10, 11]])
        fb = st.view(nw, 16)[:, 9].cpu().numpy()
        fbs = fbs + [fb] if rep > 10 else [fb]
d = np.concatenate(res)
print(f"B={B} ({'hipGraph replay' if graph else 'eager'}): per-phase s_memtime ticks per wave (median / p90), {d.shape[0]} wave samples")
for k, n in enumerate(names):
    print(f"  {n:20s} {np.median(d[:, k]):8.0f} {np.percentile(d[:, k], 90):8.0f}")
fbv = np.concatenate(fbs)
print(f"  lanes whose action the filter changed: {fbv.sum() / (64 * fbv.size):.4f}")
tot = d.sum(1)
print(f"  {'total':20s} {np.median(tot):8.0f} {np.percentile(tot, 90):8.0f}   p99 {np.percentile(tot, 99):.0f}  max {tot.max()}")
rl = np.array(real) * 0.01  # s_memrealtime ticks (100 MHz) -> us
print(f"  chip clock (s_memrealtime, us, median over launches): first wave start -> last wave end {np.median(rl[:, 0]):.2f}; "
      f"wave start offsets median {np.median(rl[:, 1]):.2f}, last {np.median(rl[:, 2]):.2f}; wave lifetime median "
      f"{np.median(rl[:, 3]):.2f}")
if uni:
    qd = np.concatenate(qres)
    qc = np.concatenate(qcnt)
    live = qc[:, 3] > 0  # waves that ran the piecewise solver (the others skip slots 1-7: stale in graph replays)
    print(f"  waves with a live hazard row: {live.mean():.4f}; with KK >= 2: {(qc[:, 4] > 0).mean():.4f}, KK >= 3: "
          f"{(qc[:, 5] > 0).mean():.4f}")
    qd, qc = qd[live], qc[live]
    qn = ["mask + wave max + slots", "stage 1a (u = 0, pieces)", "stage 1b (kinks, triples)", "stage 2 u0-edge",
          "stage 2 u1-edge"]
    print("  unicycle QP stages, waves with a live row (ticks per wave, median / p90 / mean; the stamps' scheduling barriers included):")
    for k, n in enumerate(qn):
        print(f"    {n:26s} {np.median(qd[:, k]):8.0f} {np.percentile(qd[:, k], 90):8.0f} {qd[:, k].mean():8.0f}")
    print(f"    {'QP total':26s} {np.median(qd.sum(1)):8.0f} {np.percentile(qd.sum(1), 90):8.0f} {qd.sum(1).mean():8.0f}")
    for j, n in ((0, "open after stage 1a (run 1b)"), (1, "need the u0-edge"), (2, "need the u1-edge")):
        print(f"  lanes {n}: {qc[:, j].sum() / (64 * qc.shape[0]):.4f} of lanes; waves with any: {(qc[:, j] > 0).mean():.4f}")
