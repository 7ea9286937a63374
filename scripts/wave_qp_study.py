"""One QP per wavefront vs one QP per lane (SURVEY 7 / the north star's
"one-QP-per-wavefront IPM"; the qpth call it would replace is
rcbf_sac/diff_cbf_qp.py:107,139).

Study build: sac-rcbf_amd/csrc/study/rcbf_wave_qp.hip (the product's
qpth-style interior point with the rows spread over 64 or 16 lanes and every
row sum / min a butterfly reduction).  Build it here with
  python scripts/wave_qp_study.py --build
then on the GPU:
  python scripts/wave_qp_study.py
On the layer's own rows (row-normalised, diagonal P, q = 0; cars n = 2,
m = 4 and unicycle k = 3, n = 3, m = 7) at B = 4096 and 65536, it times
(hipGraph, 20 launches) the wave-per-QP interior point (W = 64 and 16) against
the product's lane-per-QP solvers through rcbf_qp_solve (the same interior
point, solver=PDIPM, and the exact closed form), and checks every solution
against the exact one.  Prints one JSON line."""
import ctypes
import json
import math
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sac-rcbf_amd")]
STUDY_LIB = os.path.join(ROOT, "build", "study", "librcbf_wave_qp.so")
if "--build" in sys.argv:
    os.makedirs(os.path.dirname(STUDY_LIB), exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-std=c++17",
                    "-fhip-fp32-correctly-rounded-divide-sqrt", "-I" + os.path.join(ROOT, "include"),
                    "-I" + os.path.join(ROOT, "sac-rcbf_amd", "csrc"), "-o", STUDY_LIB,
                    os.path.join(ROOT, "sac-rcbf_amd", "csrc", "study", "rcbf_wave_qp.hip")], check=True)
    sys.exit(0)

import torch  # noqa: E402

import bench  # noqa: E402
from rcbf_amd import _lib  # noqa: E402
from rcbf_amd.diff_cbf_qp import CBFQPLayer  # noqa: E402
from rcbf_amd.envs import BatchedSimulatedCarsEnv, BatchedUnicycleEnv  # noqa: E402


class A:
    cuda = True


def rows(name, B, gen, dev):
    if name == "cars":
        env = BatchedSimulatedCarsEnv(4, device=dev)
        x = torch.tensor([34., 30., 28., 30., 22., 30., 16., 35., 10., 30.], device=dev).repeat(B, 1)
        x = x + torch.randn(B, 10, device=dev, generator=gen) * torch.tensor([3., 1.] * 5, device=dev)
    else:
        env = BatchedUnicycleEnv(4, device=dev, hazards_locations=bench.unicycle_hazards(3))
        x = torch.cat([torch.rand(B, 2, device=dev, generator=gen) * 6 - 3,
                       (torch.rand(B, 1, device=dev, generator=gen) * 2 - 1) * math.pi], 1)
    u = torch.rand(B, env.n_u, device=dev, generator=gen) * 2 - 1
    lay = CBFQPLayer(env, A(), gamma_b=20.0)
    mu = torch.zeros(B, env.n_s, device=dev)
    sg = torch.full((B, env.n_s), 0.2, device=dev)
    return lay, [t.contiguous() for t in lay.get_cbf_qp_constraints(x, u, mu, sg)]


def main():
    dev = torch.device("cuda", 0)
    lib = _lib.load()
    slib = ctypes.CDLL(STUDY_LIB)
    P_ = ctypes.c_void_p
    slib.rcbf_study_wave_pdipm.argtypes = [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, P_, P_, P_,
                                           ctypes.c_int32, ctypes.c_int32, ctypes.c_double, ctypes.c_int32,
                                           P_, P_, P_]
    gen = torch.Generator(device=dev)
    gen.manual_seed(9)
    out = {}
    for name in ("cars", "unicycle3"):
        for B in (4096, 65536):
            lay, (P, q, G, h) = rows(name, B, gen, dev)
            n, m = G.shape[2], G.shape[1]
            z_exact = torch.empty(B, n, device=dev)
            lay._prm.solver = _lib.SOLVER_ACTIVE_SET
            prm_exact = ctypes.byref(lay._prm)

            def exact():
                lib.rcbf_qp_solve(prm_exact, B, n, m, _lib.ptr(P), _lib.ptr(q), _lib.ptr(G), _lib.ptr(h), 1,
                                  _lib.ptr(z_exact), None, None, None, _lib.stream_of(dev))
            t_exact = bench._time_graph(exact, 20, dev)
            prm_ipm = _lib.RcbfParams.from_buffer_copy(lay._prm)
            prm_ipm.solver = _lib.SOLVER_PDIPM
            z_lane = torch.empty(B, n, device=dev)

            def lane_ipm():
                lib.rcbf_qp_solve(ctypes.byref(prm_ipm), B, n, m, _lib.ptr(P), _lib.ptr(q), _lib.ptr(G), _lib.ptr(h),
                                  1, _lib.ptr(z_lane), None, None, None, _lib.stream_of(dev))
            t_lane = bench._time_graph(lane_ipm, 20, dev)
            rec = {"lane_exact_us": round(t_exact * 1e3, 2), "lane_pdipm_us": round(t_lane * 1e3, 2)}
            torch.cuda.synchronize()
            scale = z_exact.abs().clamp_min(1.0)
            rec["lane_pdipm_max_rel_err"] = float(((z_lane - z_exact).abs() / scale).max())
            for W in (64, 16):
                z_w = torch.empty(B, n, device=dev)
                its = torch.zeros(B, dtype=torch.int32, device=dev)

                def wave_ipm():
                    rc = slib.rcbf_study_wave_pdipm(B, n, m, _lib.ptr(P), _lib.ptr(G), _lib.ptr(h), 1, 50, 1e-10, W,
                                                    _lib.ptr(z_w), _lib.ptr(its), _lib.stream_of(dev))
                    assert rc == 0, rc
                t_w = bench._time_graph(wave_ipm, 20, dev)
                torch.cuda.synchronize()
                rec[f"wave{W}_pdipm_us"] = round(t_w * 1e3, 2)
                err = ((z_w - z_exact).abs() / scale).max(1).values
                rec[f"wave{W}_max_rel_err"] = float(err.max())
                rec[f"wave{W}_frac_err_gt_1e-4"] = round(float((err > 1e-4).float().mean()), 6)
                rec[f"wave{W}_mean_iters"] = round(float(its.float().mean()), 2)
            out[f"{name}_n{n}_m{m}_B{B}"] = rec
            print(name, B, rec, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
