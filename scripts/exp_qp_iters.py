#!/usr/bin/env python3
"""Generic QP kernel study: time of rcbf_qp_solve (n = 3, m = 7, random
dense SPD P as bench.py's generic_qp_rows) versus the Goldfarb-Idnani
iteration cap, and the status mix at each cap.  Prints JSON lines."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sac-rcbf_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
from rcbf_amd import _lib  # noqa: E402
from rcbf_amd.diff_cbf_qp import CBFQPLayer  # noqa: E402
from rcbf_amd.envs import BatchedSimulatedCarsEnv  # noqa: E402


class A:
    cuda = True


dev = torch.device("cuda", 0)
lib = _lib.load()
layer = CBFQPLayer(BatchedSimulatedCarsEnv(4, device=dev), A(), gamma_b=20.0)
gen = torch.Generator(device=dev)
gen.manual_seed(5)
n, m = 3, 7
for B in (64, 4096, 65536):
    Am = torch.randn(B, n, n, device=dev, generator=gen)
    P = (Am @ Am.transpose(1, 2) + n * torch.eye(n, device=dev)).contiguous()
    q = torch.randn(B, n, device=dev, generator=gen)
    G = torch.randn(B, m, n, device=dev, generator=gen)
    z0 = 0.3 * torch.randn(B, n, device=dev, generator=gen)
    h = (torch.einsum("bmn,bn->bm", G, z0) + 0.5 * torch.randn(B, m, device=dev, generator=gen).abs()).contiguous()
    z = torch.empty(B, n, device=dev)
    st = torch.empty(B, dtype=torch.int32, device=dev)
    for cap in (1, 2, 3, 4, 6, 8, 12, 52):
        layer._prm.max_iter = cap

        def fwd():
            lib.rcbf_qp_solve(ctypes.byref(layer._prm), B, n, m, _lib.ptr(P), _lib.ptr(q), _lib.ptr(G), _lib.ptr(h),
                              1, _lib.ptr(z), None, _lib.ptr(st), None, _lib.stream_of(dev))
        ms = bench._time_graph(fwd, 20, dev)
        fwd()
        torch.cuda.synchronize()
        counts = torch.bincount(st.long(), minlength=4).tolist()
        print(json.dumps({"B": B, "cap": cap, "us": round(ms * 1e3, 2), "status_counts": counts}), flush=True)
