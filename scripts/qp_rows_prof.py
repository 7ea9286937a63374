"""Eager launches of the generic QP kernels on the layer's own rows
(rcbf_qp_solve_saved / rcbf_qp_backward_saved and the re-solving
rcbf_qp_backward, CBFQPLayer.solve_qp / cbf_layer under
autograd, diff_cbf_qp.py:81-144) for rocprofv3 passes: unicycle k = 3
(n = 3, m = 7) and cars (n = 2, m = 4) at B = 65536, 50 forward and 50
backward launches each.  Prints the mean event time per launch."""
import ctypes
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sac-rcbf_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from rcbf_amd import _lib  # noqa: E402
from rcbf_amd.diff_cbf_qp import CBFQPLayer  # noqa: E402
from rcbf_amd.envs import BatchedSimulatedCarsEnv, BatchedUnicycleEnv  # noqa: E402


class LArgs:
    cuda = True


def main():
    dev = torch.device("cuda", 0)
    lib = _lib.load()
    gen = torch.Generator(device=dev)
    gen.manual_seed(5)
    B = 65536
    for name, env in (("unicycle3", BatchedUnicycleEnv(4, device=dev, hazards_locations=bench.unicycle_hazards(3))),
                      ("cars", BatchedSimulatedCarsEnv(4, device=dev))):
        lay = CBFQPLayer(env, LArgs(), gamma_b=20.0)
        if name == "cars":
            x = torch.tensor([34., 30., 28., 30., 22., 30., 16., 35., 10., 30.], device=dev).repeat(B, 1)
            x = x + torch.randn(B, 10, device=dev, generator=gen) * torch.tensor([3., 1.] * 5, device=dev)
        else:
            x = torch.cat([torch.rand(B, 2, device=dev, generator=gen) * 6 - 3,
                           (torch.rand(B, 1, device=dev, generator=gen) * 2 - 1) * math.pi], 1)
        u = torch.rand(B, env.n_u, device=dev, generator=gen) * 2 - 1
        mu = torch.zeros(B, env.n_s, device=dev)
        sg = torch.full((B, env.n_s), 0.2, device=dev)
        P, q, G, h = (t.contiguous() for t in lay.get_cbf_qp_constraints(x, u, mu, sg))
        n, m = G.shape[2], G.shape[1]
        z = torch.empty(B, n, device=dev)
        z64 = torch.empty(B, n, dtype=torch.float64, device=dev)
        gz = torch.randn(B, n, device=dev, generator=gen)
        gP, gq, gG, gh = torch.empty_like(P), torch.empty_like(q), torch.empty_like(G), torch.empty_like(h)
        prm = ctypes.byref(lay._prm)

        ins = [_lib.ptr(P), _lib.ptr(q), _lib.ptr(G), _lib.ptr(h), 1]
        grads = [_lib.ptr(gP), _lib.ptr(gq), _lib.ptr(gG), _lib.ptr(gh)]

        def fwd():
            lib.rcbf_qp_solve_saved(prm, B, n, m, *ins, _lib.ptr(z), _lib.ptr(z64), None, None, _lib.stream_of(dev))

        def bwd():
            lib.rcbf_qp_backward_saved(prm, B, n, m, *ins, _lib.ptr(z64), _lib.ptr(gz), *grads, _lib.stream_of(dev))

        def bwd_resolve():
            lib.rcbf_qp_backward(prm, B, n, m, *ins, _lib.ptr(gz), *grads, _lib.stream_of(dev))
        for fn, tag in ((fwd, "fwd"), (bwd, "bwd (saved z)"), (bwd_resolve, "bwd (re-solve)")):
            for _ in range(5):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(50):
                fn()
            e1.record()
            torch.cuda.synchronize()
            print(f"{name} n={n} m={m} B={B} {tag}: {e0.elapsed_time(e1) * 1e3 / 50:.2f} us per eager launch",
                  flush=True)


if __name__ == "__main__":
    main()
