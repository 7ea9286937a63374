"""Lane-pair study of the unicycle fused step: the
study build sac-rcbf_amd/csrc/study/rcbf_uni_pair.hip (two lanes per env,
the hazard rows and live-row test split over the pair) against the product
k_safe_step on the same envs, start states (bench.init_states), actions and
reset stream.
  python scripts/uni_pair_study.py --build      (here: hipcc -> build/study/librcbf_uni_pair.so)
  python scripts/uni_pair_study.py [--sq]       (GPU: parity, then hipGraph timings; --sq: eager launches
                                                 only, for a rocprofv3 --pmc pass)
Parity: every output of 12 steps (auto-reset on) bit for bit equal to the
product's.  Timing: per step, a hipGraph of 200 steps replayed 3 times (best),
HIP events, B = 65 536 (k = 3, 5) and B = 4 096 (k = 3, config 3).
Kill criterion stated before the run: k = 5 at B = 65 536 at or
under 3.6 us by events, else the build stays a study."""
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sac-rcbf_amd")]
VARIANT = os.environ.get("RCBF_PAIR_VARIANT", "")  # "" (the masked solve) or "core" (the product's core)
STUDY_LIB = os.path.join(ROOT, "build", "study", f"librcbf_uni_pair{('_' + VARIANT) if VARIANT else ''}.so")
if "--build" in sys.argv:
    os.makedirs(os.path.dirname(STUDY_LIB), exist_ok=True)
    for var, defs in (("", []), ("core", ["-DRCBF_PAIR_CORE=1"])):
        out = os.path.join(ROOT, "build", "study", f"librcbf_uni_pair{('_' + var) if var else ''}.so")
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-std=c++17",
               "-fhip-fp32-correctly-rounded-divide-sqrt", "-mllvm", "-amdgpu-kernarg-preload-count=16", *defs,
               "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "sac-rcbf_amd", "csrc"), "-o", out,
               os.path.join(ROOT, "sac-rcbf_amd", "csrc", "study", "rcbf_uni_pair.hip")]
        subprocess.run(cmd, check=True)
    sys.exit(0)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rcbf_amd import _lib  # noqa: E402
from rcbf_amd.diff_cbf_qp import CBFQPLayer  # noqa: E402
from rcbf_amd.envs import BatchedUnicycleEnv, _EnvSpec  # noqa: E402

from bench import init_states  # noqa: E402


class _A:
    cuda = True


P = ctypes.c_void_p
slib = ctypes.CDLL(STUDY_LIB)
slib.rcbf_study_uni_pair_step.argtypes = [ctypes.POINTER(_lib.RcbfParams), ctypes.c_int64] + [P] * 12 + [
    ctypes.c_int32, ctypes.c_uint64, ctypes.c_int64, ctypes.c_int32, P]


def make(B, k, seed=3):
    env = BatchedUnicycleEnv(B, seed=seed, hazards_locations=_EnvSpec("Unicycle").hazards_locations[:k])
    gen = torch.Generator(device="cuda")
    gen.manual_seed(1000)
    init_states(env, gen, "Unicycle")
    return env, CBFQPLayer(env, _A(), gamma_b=20.0)


def pair_step(env, layer, u, o, flag):
    rc = slib.rcbf_study_uni_pair_step(ctypes.byref(layer._prm), env.num_envs, _lib.ptr(env.x), _lib.ptr(env.aux),
                                       _lib.ptr(env.step_count), _lib.ptr(env.episode), _lib.ptr(u),
                                       _lib.ptr(o["obs"]), _lib.ptr(o["u"]), _lib.ptr(o["reward"]),
                                       _lib.ptr(o["cost"]), _lib.ptr(o["done"]), _lib.ptr(o["goal_met"]),
                                       _lib.ptr(flag), 1, env._rng_seed(), env.env_offset, 0,
                                       _lib.stream_of(env.device))
    assert rc == 0


def outputs(env):
    o = env.make_outputs()
    o.setdefault("obs", env.obs)
    return o


def parity(B, k, steps=12):
    a, la = make(B, k)
    b, lb = make(B, k)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(7)
    oa, ob = outputs(a), outputs(b)
    flag = torch.zeros(1, dtype=torch.int32, device="cuda")
    for _ in range(steps):
        u = (torch.rand(B, 2, device="cuda", generator=gen) * 2 - 1).contiguous()
        a.safe_step(u, la, outputs=oa)
        pair_step(b, lb, u, ob, flag)
        torch.cuda.synchronize()
        for key in ("u", "reward", "cost", "done", "goal_met"):
            assert torch.equal(oa[key], ob[key]), key
        assert torch.equal(a.obs, b.obs), "obs"
        assert torch.equal(a.x, b.x) and torch.equal(a.aux, b.aux) and torch.equal(a.step_count, b.step_count)
        assert torch.equal(a.episode, b.episode)
    return True


def time_graph(fn, reps=200):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        fn(0)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for j in range(reps):
            fn(j)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = None
    for _ in range(3):
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / reps
        best = us if best is None else min(best, us)
    return best


def timing(B, k):
    out = {}
    for name in ("product", "pair"):
        env, layer = make(B, k)
        o = outputs(env)
        flag = torch.zeros(1, dtype=torch.int32, device="cuda")
        pool = [(torch.rand(B, 2, device="cuda") * 2 - 1).contiguous() for _ in range(16)]
        if name == "product":
            fn = lambda j: env.safe_step(pool[j % 16], layer, outputs=o)  # noqa: E731
        else:
            fn = lambda j: pair_step(env, layer, pool[j % 16], o, flag)  # noqa: E731
        out[name + "_us"] = round(time_graph(fn), 3)
    return out


def main():
    if "--sq" in sys.argv:  # eager launches only: rocprofv3 --pmc reads the two kernels' counters
        for B, k in ((65536, 5), (4096, 3)):
            for name in ("product", "pair"):
                env, layer = make(B, k)
                o = outputs(env)
                flag = torch.zeros(1, dtype=torch.int32, device="cuda")
                u = (torch.rand(B, 2, device="cuda") * 2 - 1).contiguous()
                for _ in range(30):
                    env.safe_step(u, layer, outputs=o) if name == "product" else pair_step(env, layer, u, o, flag)
        torch.cuda.synchronize()
        return
    res = {}
    for B, k in ((65536, 5), (65536, 3), (4096, 3), (4096, 5), (1000, 3)):
        assert parity(B, k), (B, k)
        res[f"uni{k}_B{B}"] = {"parity_12_steps": "bit-exact", **timing(B, k)}
        print(f"uni{k}_B{B}", res[f"uni{k}_B{B}"], flush=True)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
