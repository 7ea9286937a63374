#!/usr/bin/env python3
"""Headline benchmark: safe env steps/s (dynamics + CBF-QP) at batch 65536.

A "step" is one fused safe step of every env of the batch
(rcbf_safe_step: get_state(obs32) -> CBFQPLayer.get_safe_action (build,
row-normalise, fp64 QP, clamp) -> env.step -> obs/reward/cost/done,
auto-reset) with the env state, u_RL and outputs resident in HBM.  u_RL is
synthetic (uniform in the action box, like the reference's warm-up policy,
main.py:88-92), mean/sigma are the DynamicsModel prior (dynamics.py:381-384).

Multi-GPU: one process per GPU (torchrun), each GPU owns `--batch` envs
(weak scaling, no collective on the data path; RCCL only for the barrier and
the max-over-ranks time).  Rank 0 prints one JSON line.
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, os.path.join(ROOT, "sac-rcbf_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)

# Algorithmic HBM bytes of one env-step of rcbf_safe_step ("bytes per step"):
#   cars:     read  x 80 + t 8 + step 4 + u_RL 4                         =  96
#             write x 80 + t 8 + step 4 + obs 40 + u 4 + r 4 + c 4 + done 1 = 145
#   unicycle: read  x 24 + last_dist 8 + step 4 + u_RL 8                 =  44
#             write x 24 + ld 8 + step 4 + obs 28 + u 8 + r 4 + c 4 + done 1 + goal 1 = 82
BYTES_PER_STEP = {"SimulatedCars": 96 + 145, "Unicycle": 44 + 82}
# with per-env mean/sigma tensors (--prior tensor) the kernel also reads what
# the rows use: cars sigma[5], sigma[7], sigma[9] (the cars rows ignore mu,
# diff_cbf_qp.py:298-299) = 12 B; unicycle mu 12 + sigma 12 = 24 B
PRIOR_TENSOR_BYTES = {"SimulatedCars": 12, "Unicycle": 24}


def bytes_per_step(args):
    prior = PRIOR_TENSOR_BYTES[args.env] if args.prior in ("tensor", "rows") else 0
    if args.workload == "sac_update":
        return SAC_UPDATE_BYTES[args.env] + prior
    return BYTES_PER_STEP[args.env] + prior


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=65536,
                    help="envs per GPU (weak scaling) or in total (--scaling strong)")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="weak: --batch envs on every GPU; strong: --batch envs split over the GPUs")
    ap.add_argument("--env", default="SimulatedCars", choices=["SimulatedCars", "Unicycle"])
    ap.add_argument("--hazards", type=int, default=3, help="unicycle hazard count")
    ap.add_argument("--solver", default="active_set", choices=["active_set", "pdipm"])
    ap.add_argument("--graph-steps", type=int, default=500,
                    help="fused steps per captured hipGraph (fewer replays: less host launch overhead in the wall time)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="budget of the CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--extra", action="store_true", help="also time the K-step rollout kernel and big batches")
    ap.add_argument("--no-graph", action="store_true", help="eager launches (for PMC counter passes)")
    ap.add_argument("--prior", default="prior", choices=["prior", "tensor", "rows"],
                    help="prior: the DynamicsModel prior in-kernel (before any GP fit); tensor: per-env mean/sigma "
                         "read from HBM (after the GP fit) in the column layout the GP writes for the step "
                         "(rcbf_gp_predict_cols -> rcbf_safe_step_cols); rows: the same as (B, n_s) row tensors")
    ap.add_argument("--rccl", action="store_true",
                    help="bring up the RCCL process group even on one rank: the N > 1 path's init, barriers, "
                         "all_gather and MAX all_reduce then run on the device (world size 1)")
    ap.add_argument("--rehearse-shared-gpu", action="store_true",
                    help="rehearsal of the N > 1 path on a 1-GPU box: every rank runs on GPU 0 (its own AQL queue and "
                         "env shard), the process group is gloo; checks the multi-process launch, per-rank queues, "
                         "barriers and max-over-ranks on the device path -- NOT a scaling measurement")
    ap.add_argument("--cpu-dry-run", action="store_true",
                    help="CPU/gloo plumbing check of the launcher (no kernel, no measurement)")
    ap.add_argument("--launch", default=None, choices=["graph", "seq", "aql"],
                    help="aql (the default for the fused step): the K dispatches as pre-built AQL packets on the "
                         "library's own HSA queue (rcbf_aql_run, csrc/rcbf_aql.hip), one doorbell per run; graph "
                         "(the default for --workload sac_update): hipGraph replays of --graph-steps launches; seq: "
                         "the K launches issued from one host call (rcbf_safe_step_seq)")
    ap.add_argument("--cpu-baseline-only", action="store_true",
                    help="(internal) print the CPU baselines as JSON and exit; never touches the GPU")
    ap.add_argument("--host-cores", type=int, default=4,
                    help="host cores per rank for the launch threads (0: no pinning)")
    ap.add_argument("--config", type=int, default=0, choices=[0, 1, 2, 3, 4, 5],
                    help="a BASELINE.json config (0: the headline, cars B = 65536 per GPU): 1 cars, one env; "
                         "2 cars B = 4096; 3 unicycle (3 hazards) B = 4096; 4 cars B = 262144 split over the GPUs "
                         "(strong); 5 cars B = 4096 SAC-update safe action, forward + backward")
    ap.add_argument("--workload", default="step", choices=["step", "sac_update", "closed_loop"],
                    help="step: the fused safe step; sac_update: RCBF_SAC.get_safe_action on a replay batch "
                         "forward + backward (rcbf_obs_safe_action + its backward, config 5)")
    ap.add_argument("--no-span", action="store_true", help="skip the untimed in-kernel span measurement")
    ap.add_argument("--record", default=None,
                    help="write this run's roofline evidence (per-step GPU time, dispatch timestamps, span stamps, "
                         "shader clock) to this JSON file (committed under profiles/ as roofline_record_*.json)")
    ap.add_argument("--prior-values", default="posterior", choices=["posterior", "maxstd"],
                    help="values of the per-env mean/sigma tensors (--prior rows/tensor): posterior = a fitted GP's "
                         "stand-in (small mean, sigma near MAX_STD); maxstd = mean 0, sigma = MAX_STD materialised per "
                         "env, as predict_disturbance returns them before any fit (SURVEY 8(d) configs 2 and 5)")
    ap.add_argument("--sac-bwd", default="jac", choices=["jac", "resolve"],
                    help="config 5's backward: jac = the forward keeps d final / d u (rcbf_obs_safe_action_jac) and "
                         "the backward applies it (rcbf_safe_action_apply_jac), as the autograd op runs it; resolve "
                         "= the plain forward and the re-solving backward (rcbf_obs_safe_action_backward)")
    args = ap.parse_args()
    preset = {1: dict(env="SimulatedCars", batch=1, workload="closed_loop"),
              2: dict(env="SimulatedCars", batch=4096, workload="step", prior="rows", prior_values="maxstd"),
              3: dict(env="Unicycle", hazards=3, batch=4096, workload="step"),
              4: dict(env="SimulatedCars", batch=262144, scaling="strong", workload="step"),
              5: dict(env="SimulatedCars", batch=4096, workload="sac_update", prior="rows",
                      prior_values="maxstd")}.get(args.config, {})
    for k, v in preset.items():
        setattr(args, k, v)
    if args.launch is None:
        args.launch = "graph" if (args.workload == "sac_update" or args.no_graph) else "aql"
    if args.workload == "sac_update" and (args.prior == "tensor" or args.launch != "graph" or args.no_graph):
        raise SystemExit("--workload sac_update reads (B, n_s) rows or the in-kernel prior, hipGraph-launched")
    return args


AQL_MAX_STEPS = 4096  # dispatches per AQL plan (one ring's worth: csrc/rcbf_aql.hip kQueueSize)


def aql_dispatch_times(env, layer, ctx, graph, S):
    """Untimed, after the timed region (--launch aql): the same S steps as a
    profiled plan (a completion signal per dispatch on the same queue), so
    each dispatch's start / end comes from the packet processor's own
    timestamps (hsa_amd_profiling_get_dispatch_time, the source rocprofv3's
    kernel trace reads).  Returns the per-dispatch durations and the period."""
    from rcbf_amd.aql import PROFILE_ENDS
    kw = dict(steps=S, mean=ctx["mean"], sigma=ctx["sigma"], outputs=ctx["outs"], prior_layout=ctx["layout"])
    # end to end: timestamps on the first and the last dispatch only (a signal on every dispatch adds its
    # own cost to each step), three runs, the median
    ends = graph.queue.safe_step_plan(env, ctx["pool"], layer, fence_flags=PROFILE_ENDS, **kw)
    ends.run(sync_hip=True)
    runs = []
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ends.run(sync_hip=False)
        wall = time.perf_counter() - t0
        t = ends.times_ns().astype(np.float64)
        runs.append({"first_start_ns": int(t[0, 0]), "last_end_ns": int(t[-1, 1]), "wall_us": round(wall * 1e6, 2),
                     "period_us": round(float((t[-1, 1] - t[0, 0]) / 1e3 / S), 4)})
    ends.free()
    # per dispatch: a completion signal on every dispatch (each one's own duration, with the signal's cost)
    prof = graph.queue.safe_step_plan(env, ctx["pool"], layer, profile=True, **kw)
    prof.run(sync_hip=True)
    t = prof.times_ns().astype(np.float64)
    prof.free()
    dur = (t[:, 1] - t[:, 0]) / 1e3
    env.check_failures()
    period = float(np.median([r["period_us"] for r in runs]))
    return {"period_us": round(period, 4), "runs": runs,
            "signalled_dispatch_us_mean": round(float(dur.mean()), 4),
            "signalled_dispatch_us_median": round(float(np.median(dur)), 4), "dispatches": S,
            "how": "the timed plan's S dispatches re-run on the same AQL queue, untimed: period_us = (last dispatch "
                   "end - first dispatch start) / S from the packet processor's timestamps "
                   "(hsa_amd_profiling_get_dispatch_time) with a completion signal on the first and last dispatch "
                   "only, median of 3 runs; signalled_dispatch_us_* = each dispatch's own start-to-end with a "
                   "signal on every dispatch (the per-dispatch signal adds ~1.5 us, as rocprofv3's tracer does)"}


def largest_divisor_le(n, cap):
    for s in range(min(n, cap), 0, -1):
        if n % s == 0:
            return s
    return 1


def cpu_baseline(env_name, hazards, seconds, B=65536):
    """The C oracle's fused step (oracle/rcbf_oracle.c: build + exact QP +
    clamp + env step, OpenMP over envs) on this host's cores, on a bounded
    sample of the same workload (B envs, prior mean/sigma), ~`seconds` in
    total: first 1 thread, then all threads OMP_NUM_THREADS allows (1 thread
    below 1024 envs, where a parallel region costs more than the step)."""
    from oracle import c_oracle as C
    from oracle import oracle as O
    rng = np.random.default_rng(0)
    hz = O.UNI["hazards"][:hazards] if env_name == "Unicycle" else None
    threads_all = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    if B < 1024:
        threads_all = 1

    def run(threads, budget):
        if env_name == "SimulatedCars":
            x, aux, st = O.cars_reset(rng.normal(0, 0.5, B))
        else:
            x, aux, st = O.uni_reset(B)
        st = st.astype(np.int32)
        n_u = 1 if env_name == "SimulatedCars" else 2
        u = rng.uniform(-1, 1, (B, n_u)).astype(np.float32)
        n, t0 = 0, time.perf_counter()
        while True:
            C.safe_step(env_name, x, aux, st, u, 20.0, hazards=hz, threads=threads)
            n += 1
            el = time.perf_counter() - t0
            if el >= budget or n * B >= 100000 * 65536:
                return n * B / el, n, el

    v1, n1, e1 = run(1, seconds * 0.25)
    run(threads_all, min(1.0, seconds * 0.05))  # untimed: the OpenMP pool's start-up (tens of ms per step at first)
    samples = [run(threads_all, seconds * 0.25) for _ in range(3)]
    rates = sorted(v for v, _, _ in samples)
    nN, eN = sum(n for _, n, _ in samples), sum(e for _, _, e in samples)
    return {"value": round(rates[1], 1), "unit": "safe env steps/s", "cores": threads_all, "kind": "port",
            "sample": f"C oracle fused step (oracle/rcbf_oracle.c, exact QP, gcc -O3 -march=x86-64-v3), median of 3 "
                      f"samples on {threads_all} threads ({rates[0]:.4g} / {rates[1]:.4g} / {rates[2]:.4g} steps/s; "
                      f"{nN} steps x {B} envs in {eN:.1f} s); 1 thread: {v1:.4g} steps/s ({n1} steps)",
            "spread": [round(r, 1) for r in rates]}


def cpu_sac_update(env_name, hazards, seconds, B):
    """Config 5's CPU baseline: the C oracle's CBFQPLayer forward and its
    gradient w.r.t. the action (oracle/rcbf_oracle.c oracle_safe_action_grad,
    the restatement of oracle.safe_action_diff_grad: fp32 rows, normaliser,
    exact QP, clamp, implicit-KKT derivative on the active set, OpenMP over
    rows) on B observations' states of the SURVEY 8(d) distribution, prior
    mean/sigma; 1 thread, then the median of 3 samples on all threads."""
    from oracle import c_oracle as C
    from oracle import oracle as O
    rng = np.random.default_rng(3)
    hz = O.UNI["hazards"][:hazards] if env_name == "Unicycle" else None
    threads_all = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    if env_name == "SimulatedCars":  # SURVEY 8(d) states: seeded resets advanced 0-299 steps under u ~ U[-1, 1]
        x, t, st = O.cars_reset(rng.normal(0, 0.5, B))
        stop = rng.integers(0, 300, B)
        for k in range(int(stop.max())):
            xn, tn, sn, _, _, _, _ = O.cars_step(x, t, st, rng.uniform(-1, 1, (B, 1)).astype(np.float32))
            go = (k < stop)[:, None]
            x, t, st = np.where(go, xn, x), np.where(go[:, 0], tn, t), np.where(go[:, 0], sn, st)
        obs = O.cars_obs(x).astype(np.float32)
        n_u = 1
    else:
        x = np.stack([rng.uniform(-3, 3, B), rng.uniform(-3, 3, B), rng.uniform(-np.pi, np.pi, B)], 1)
        obs = O.uni_obs(x).astype(np.float32)
        n_u = 2
    s32 = O.get_state_f32(env_name, obs)
    mu, sg = O.predict_disturbance_prior(env_name, B)
    mu, sg = mu.astype(np.float32), sg.astype(np.float32)
    u = rng.uniform(-1, 1, (B, n_u)).astype(np.float32)
    w = rng.normal(0, 1, (B, n_u)).astype(np.float32)

    def run(threads, budget):
        n, t0 = 0, time.perf_counter()
        while True:
            C.safe_action_grad(env_name, s32, u, mu, sg, 20.0, w, hazards=hz, threads=threads)
            n += 1
            el = time.perf_counter() - t0
            if el >= budget:
                return n * B / el, n, el

    v1, n1, _ = run(1, seconds * 0.25)
    run(threads_all, min(1.0, seconds * 0.05))  # untimed: the OpenMP pool's start-up
    samples = [run(threads_all, seconds * 0.25) for _ in range(3)]
    rates = sorted(v for v, _, _ in samples)
    nN, eN = sum(n for _, n, _ in samples), sum(e for _, _, e in samples)
    return {"value": round(rates[1], 1), "unit": "safe actions/s (forward + backward)", "cores": threads_all,
            "kind": "port",
            "sample": f"C oracle CBFQPLayer forward + d/du backward (oracle/rcbf_oracle.c oracle_safe_action_grad, "
                      f"exact QP, implicit-KKT gradient), median of 3 samples on {threads_all} threads "
                      f"({rates[0]:.4g} / {rates[1]:.4g} / {rates[2]:.4g} actions/s; {nN} batches x {B} rows in "
                      f"{eN:.1f} s); 1 thread: {v1:.4g} actions/s ({n1} batches)",
            "spread": [round(r, 1) for r in rates]}


def cpu_baselines_in_child(args):
    """Both CPU baselines in a fresh child process that has never touched the
    GPU and starts with this process's full CPU mask (its OpenMP and torch
    thread pools are created there, so no pinning of this rank leaks into
    them).  The parent waits for the child's JSON line."""
    import subprocess
    cmd = [sys.executable, os.path.abspath(__file__), "--cpu-baseline-only", "--env", args.env,
           "--hazards", str(args.hazards), "--cpu-seconds", str(args.cpu_seconds), "--batch", str(args.batch),
           "--workload", args.workload]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        raise RuntimeError(f"CPU baseline child failed ({r.returncode}): {r.stderr[-2000:]}")
    return json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])


def cpu_reference_mode(env_name, hazards, seconds, B=65536):
    """The reference's own CPU mode restated (oracle/torch_mirror.py): fp32
    rows, normaliser, qpth-style batched PDIPM in torch fp64 (eps 1e-4,
    notImprovedLim 10, capped at 100 iterations), clamp, numpy env step, on
    the same B envs, on the torch threads of this host."""
    from oracle import oracle as O
    from oracle import torch_mirror as M
    rng = np.random.default_rng(1)
    threads = torch.get_num_threads()
    if env_name == "SimulatedCars":
        x, aux, st = O.cars_reset(rng.normal(0, 0.5, B))
    else:
        hz = O.UNI["hazards"][:hazards]
        x = np.stack([rng.uniform(-3, 3, B), rng.uniform(-3, 3, B), rng.uniform(-np.pi, np.pi, B)], 1)
        aux, st = O.uni_goal_dist(x), np.zeros(B, np.int64)
    n_u = 1 if env_name == "SimulatedCars" else 2
    n, its, t0 = 0, 0, time.perf_counter()
    while True:
        u = rng.uniform(-1, 1, (B, n_u)).astype(np.float32)
        if env_name == "SimulatedCars":
            x, aux, st, _, k = M.cars_safe_step(x, aux, st, u, 20.0)
        else:
            x, aux, st, _, k = M.uni_safe_step(x, aux, st, u, 20.0, hz)
        n, its = n + 1, its + k
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": round(n * B / el, 1), "unit": "safe env steps/s", "cores": threads, "kind": "port",
            "sample": f"reference CPU mode restated (oracle/torch_mirror.py: torch-CPU qpth-style PDIPM, from seeded resets, "
                      f"{its / n:.1f} iterations per step), {n} steps x {B} envs in {el:.1f} s on {threads} threads"}


def init_states(env, gen, env_name):
    """Untimed set-up: start the benchmark from the state distribution of
    SURVEY.md 8(d), not from B identical resets.
    Cars: seeded resets, each advanced a uniform-random 0-299 steps under
    u ~ U[-1, 1] (about 45 % of the QPs active).  Unicycle: x, y ~ U[-3, 3],
    theta ~ U[-pi, pi], episode step ~ U{0..999}."""
    B, dev = env.num_envs, env.device
    if env_name == "SimulatedCars":
        k_stop = torch.randint(0, 300, (B,), device=dev, generator=gen)
        snap, snap_t = env.state.clone(), env.aux.clone()
        for k in range(1, 300):
            u = torch.rand(B, 1, device=dev, generator=gen) * 2 - 1
            env.step(u, auto_reset=False)
            sel = k_stop == k
            snap[sel] = env.state[sel]
            snap_t[sel] = env.aux[sel]
        env.load_state(snap, snap_t, k_stop.to(torch.int32))
    else:
        xy = torch.rand(B, 2, device=dev, generator=gen, dtype=torch.float64) * 6 - 3
        th = (torch.rand(B, 1, device=dev, generator=gen, dtype=torch.float64) * 2 - 1) * math.pi
        gd = torch.linalg.norm(xy - 2.5, dim=1)
        st = torch.randint(0, 1000, (B,), device=dev, generator=gen, dtype=torch.int32)
        env.load_state(torch.cat([xy, th], 1), gd, st)
    torch.cuda.synchronize()


def one_rank_rendezvous(world):
    """--rccl on one rank: a rendezvous of its own on the loopback address."""
    if world == 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(free_port()))
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")


def free_port():
    """A free TCP port on the loopback address (the rendezvous of spawned or single ranks)."""
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def spawn_ranks(n):
    """`bench.py --gpus N` run as a plain process: start N rank processes of
    this same script BEFORE anything touches the GPU (this parent never
    initialises HIP), one per GPU, with the torchrun environment (RANK,
    LOCAL_RANK, WORLD_SIZE, MASTER_ADDR=127.0.0.1, a free MASTER_PORT).  Rank
    0 inherits stdout and prints the JSON line.  If a rank fails the others
    are stopped; returns the first non-zero exit status (0 if all succeed)."""
    import subprocess
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    rc = 0
    while procs:
        for p in list(procs):
            code = p.poll()
            if code is None:
                continue
            procs.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in procs:
                    q.terminate()
        time.sleep(0.05)
    return rc


class _DryRun:
    """--cpu-dry-run: the launcher, rendezvous, barrier / max-over-ranks and
    the JSON line, on the CPU with gloo and no kernel (the timed region is an
    empty loop).  For the multi-process CPU tests only; never a measurement."""

    def __init__(self, B, n_u):
        self.num_envs, self.n_u = B, n_u

    def replay(self):
        pass

    def check_failures(self):
        pass


def pin_host_cores(local, n):
    """Keep this rank's host threads (the replay calls and the HIP runtime's
    own threads, created after this) on n cores of their own, before anything
    touches the GPU (device counting included).  The replay call then takes
    14-16 us instead of 18-34 us of host time in the driver's 20-step form
    (profiles/r02/host_pinning_study_r02ag.txt).  The node's allowed CPUs are
    split evenly over LOCAL_WORLD_SIZE ranks, each on its GPU's NUMA node
    where the sysfs topology says which it is (rcbf_amd.shard.plan_host_cores:
    every rank pinned, or none).  Returns (the original mask, this rank's
    cores); the original mask is None when nothing was pinned.  The restore
    before the CPU baseline covers the calling thread; the baseline's OpenMP
    threads are created after it and inherit the full mask."""
    from rcbf_amd import shard
    allowed = sorted(os.sched_getaffinity(0))
    plan = shard.plan_host_cores(allowed, shard.local_world_size(), n, shard.gpu_numa_nodes(), shard.node_cpus())
    if plan is None or local >= len(plan):
        return None, None
    os.sched_setaffinity(0, set(plan[local]))
    return set(allowed), plan[local]


METRICS = {
    0: "safe env steps/sec (dynamics+CBF-QP) at batch 65536, 1/2/4/8 MI355X",
    1: "safe env steps/sec (dynamics+CBF-QP), config 1: SimulatedCars, 1 env, 300-step episode, the Cascade "
       "closed loop with the hand controller",
    2: "safe env steps/sec (dynamics+CBF-QP), config 2: SimulatedCars batch 4096, 1 MI355X",
    3: "safe env steps/sec (dynamics+CBF-QP), config 3: Unicycle (3 hazards) batch 4096, 1 MI355X",
    4: "safe env steps/sec (dynamics+CBF-QP), config 4: SimulatedCars batch 262144 over the GPUs",
    5: "safe actions/sec (diff CBF-QP forward + backward), config 5: SimulatedCars batch 4096, 1 MI355X",
}

# Algorithmic bytes of one forward + backward of the SAC-update safe action
# per row, prior mean/sigma (config 5): the op's own inputs and outputs --
# obs + u_RL in, u out (forward), grad_u in, grad_u_RL out (backward):
#   cars     40 + 4 + 4 + 4 + 4 = 56;   unicycle 28 + 8 + 8 + 8 + 8 = 60.
# What an implementation keeps between the two (the saved Jacobian, 8 / 32 B,
# or re-reading obs and u_RL) is traffic, not algorithmic bytes.
SAC_UPDATE_BYTES = {"SimulatedCars": 56, "Unicycle": 60}


def block_for_envs(B):
    """Workgroup size of the one-env-per-lane kernels (rcbf_common.hpp
    block_for_envs): 256 from 65 536 envs, 128 from 32 768, else 64."""
    return 256 if B >= 256 * 256 else 128 if B >= 256 * 128 else 64


def workload_short(args):
    """The workload's name in profiles/ file names."""
    base = ("sacupd_" if args.workload == "sac_update" else "") + ("cars" if args.env == "SimulatedCars"
                                                                  else f"uni{args.hazards}")
    return base + {"prior": "", "tensor": "_tensorprior", "rows": "_rowsprior"}[args.prior] + \
        ("_maxstd" if args.prior != "prior" and args.prior_values == "maxstd" else "")


def dominant_kernels(args, B):
    """The kernel(s) one timed step launches, as rocprofv3 names them."""
    solver = 1 if args.solver == "pdipm" else 0
    mode, K = (0, 1) if args.env == "SimulatedCars" else (1, args.hazards)
    bs = block_for_envs(B) if solver == 0 else 256  # the small workgroups are the exact solver's only
    if args.workload == "sac_update":
        if args.sac_bwd == "jac":
            return [f"k_safe_action_jac<{solver}, {mode}, {K}, true, {bs}>", f"k_apply_jac<{1 if mode == 0 else 2}, {bs}>"]
        return [f"k_safe_action<{solver}, {mode}, {K}, true, {bs}>", f"k_safe_action_bwd<{solver}, {mode}, {K}, true, {bs}>"]
    return [f"k_safe_step<{solver}, {mode}, {K}, false, {bs}, false>"]


def _profiles_newest(pattern):
    """profiles/r*/<pattern> files, newest round (then run tag) first."""
    import glob
    return sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", pattern)), reverse=True)


def pmc_traffic_file(short, B):
    """HBM bytes per launch of the dominant kernel from the committed
    rocprofv3 PMC passes (scripts/pmc_traffic.py: 2 x FETCH_SIZE +
    WRITE_SIZE, gfx950 corrections) of this exact workload, newest first;
    (None, None) if absent."""
    for path in _profiles_newest(f"pmc_traffic_{short}_B{B}.json"):
        try:
            return float(json.load(open(path))["traffic_bytes"]), os.path.relpath(path, ROOT)
        except Exception:
            continue
    return None, None


DRIVER_FORM = (20, 5)  # the driver's command: bench.py --gpus 1 --steps 20 --warmup 5


DEFAULT_FORM = (1000, 20)  # bench.py with no flags


def rocprof_form(steps, warmup):
    """Which committed traces / records are "the same command": the driver's
    20-step form (rocprofv3 of `bench.py --steps 20 --warmup 5`), the default
    form (`bench.py`, 1000 steps, 20 warm-up), or None for any other
    (steps, warmup) -- no committed file is evidence for those."""
    return {DRIVER_FORM: "driver", DEFAULT_FORM: "default"}.get((steps, warmup))


def _form_tag(form, launch):
    """The form part of a profiles/ file name: driver_form_[aql_] / [aql_]."""
    aql = "aql_" if launch == "aql" else ""
    return f"driver_form_{aql}" if form == "driver" else aql


def rocprof_kernel_us(short, B, kernels, form="default", launch="graph"):
    """Mean duration (us) of one timed step's kernels -- the sum of their
    AverageNs -- from the newest committed rocprofv3 --kernel-trace --stats
    summary of this workload in the given command form and launch path
    (kernel_stats_<form tag><workload>_B<B>_<tag>.csv); (None, None) if there
    is none.  A trace of another command is not evidence for the line."""
    import csv
    if form is None:
        return None, None
    pat = f"kernel_stats_{_form_tag(form, launch)}{short}_B{B}_*.csv"
    for path in _profiles_newest(pat):
        try:
            rows = list(csv.DictReader(open(path)))
            tot = 0.0
            for k in kernels:
                hit = [r for r in rows if k in r["Name"]]
                if len(hit) != 1:
                    raise KeyError(k)
                tot += float(hit[0]["AverageNs"]) / 1e3
            return round(tot, 4), os.path.relpath(path, ROOT)
        except Exception:
            continue
    return None, None


def roofline_record(short, B, form, launch):
    """The newest committed roofline record of the same command
    (profiles/r*/roofline_record_<form tag><workload>_B<B>_<tag>.json, written
    by `bench.py --record`): (per-step kernel us, path) or (None, None)."""
    if form is None:
        return None, None
    for path in _profiles_newest(f"roofline_record_{_form_tag(form, launch)}{short}_B{B}_*.json"):
        try:
            r = json.load(open(path))
            return float(r["kernel_us_per_step"]), os.path.relpath(path, ROOT)
        except Exception:
            continue
    return None, None


def measure_span(env, layer, ctx, dev, B, bps, n=100, queue=None):
    """Untimed, after the timed region: the kernel's own span, untraced.  n
    launches of rcbf_safe_step_span (the product kernel plus, per wave, the
    100 MHz chip clock and the shader clock at its start and after its stores
    have landed) -- a hipGraph replayed twice, or with `queue` (--launch aql)
    one AQL plan of n dispatches run twice; per launch, span = last wave end -
    first wave start, period = next launch's first start - this one's, gap =
    next launch's first start - this launch's last end (the dependent-kernel
    boundary).  The span run's own per-step time is reported beside it (the
    stamps and a drain per wave)."""
    nw = (B + 63) // 64
    buf = torch.zeros(n, nw, 4, dtype=torch.int64, device=dev)
    pool, mean, sigma, layout, outs = ctx["pool"], ctx["mean"], ctx["sigma"], ctx["layout"], ctx["outs"]
    if queue is not None:
        from rcbf_amd.aql import PROFILE_ENDS
        plan = queue.safe_step_plan(env, pool, layer, steps=n, mean=mean, sigma=sigma, outputs=outs,
                                    prior_layout=layout, span=buf, fence_flags=PROFILE_ENDS)
        plan.run()
        torch.cuda.synchronize()
        buf.zero_()
        torch.cuda.synchronize()
        plan.run(sync_hip=False)
        tt = plan.times_ns().astype(np.float64)
        plan.free()
        env.check_failures()
        return _span_summary(buf, (tt[-1, 1] - tt[0, 0]) / 1e3 / n, n, nw, B, bps,
                             f"one AQL plan of {n} dispatches (rcbf_aql_run)")

    def launches():
        for j in range(n):
            env.safe_step_span(pool[j % len(pool)], layer, buf[j], mean=mean, sigma=sigma, outputs=outs,
                               prior_layout=layout)
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        launches()
    torch.cuda.current_stream(dev).wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        launches()
    g.replay()
    torch.cuda.synchronize()
    buf.zero_()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    env.check_failures()
    return _span_summary(buf, e0.elapsed_time(e1) * 1e3 / n, n, nw, B, bps, f"a hipGraph of {n} launches")


def _span_summary(buf, per_step_us, n, nw, B, bps, how_run):
    t = buf.cpu().numpy().astype(np.float64)
    valid = t[:, :, 1] > 0
    start = np.where(valid, t[:, :, 0], np.inf).min(1)
    end = np.where(valid, t[:, :, 1], -np.inf).max(1)
    span = (end - start) * 0.01  # 100 MHz ticks -> us
    period = np.diff(start) * 0.01
    gap = (start[1:] - end[:-1]) * 0.01
    med = float(np.median(span))
    # the shader clock each wave ran at: delta(s_memtime) / delta(s_memrealtime) x 100 MHz
    dreal = np.where(valid, t[:, :, 1] - t[:, :, 0], 0)
    dmem = np.where(valid, t[:, :, 3] - t[:, :, 2], 0)
    clk = dmem[dreal > 0] / dreal[dreal > 0] * 100.0
    return {"kernel_span_us_median": round(med, 3), "kernel_span_us_mean": round(float(span.mean()), 3),
            "kernel_span_us_p10_p90": [round(float(np.percentile(span, 10)), 3),
                                       round(float(np.percentile(span, 90)), 3)],
            "period_us_median": round(float(np.median(period)), 3),
            "boundary_gap_us_median": round(float(np.median(gap)), 3),
            "span_run_us_per_step": round(per_step_us, 3), "launches": n, "waves_per_launch": nw,
            "shader_clock_mhz_median": round(float(np.median(clk)), 1) if clk.size else None,
            "frac_span": round(B * bps / (med * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
            "_stamps": {"first_start_ticks": start.astype(np.int64).tolist(),
                        "last_end_ticks": end.astype(np.int64).tolist()},
            "how": f"rcbf_safe_step_span, {how_run}, untraced: per launch the last wave's end (after its stores "
                   "landed) minus the first wave's start, s_memrealtime (100 MHz chip clock); frac_span = "
                   "bytes_per_launch / median span; shader clock = delta(s_memtime) / delta(s_memrealtime) x "
                   "100 MHz per wave, median"}


def main():
    args = parse()
    if args.cpu_baseline_only:
        if args.workload == "sac_update":
            out = {"cpu_baseline": cpu_sac_update(args.env, args.hazards, args.cpu_seconds, args.batch)}
        else:
            out = {"cpu_baseline": cpu_baseline(args.env, args.hazards, args.cpu_seconds, args.batch),
                   "cpu_reference_mode": cpu_reference_mode(args.env, args.hazards, args.cpu_seconds / 3,
                                                            args.batch)}
        print(json.dumps(out), flush=True)
        return
    if args.workload == "closed_loop":
        return bench_closed_loop(args)
    from rcbf_amd import shard
    rank, local, world = shard.world_info()
    if world == 1 and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    if args.gpus != world and args.gpus != 1:
        raise SystemExit(f"--gpus {args.gpus} but the launcher started {world} ranks")
    if args.scaling == "strong":
        if args.batch % world:
            raise SystemExit("--scaling strong needs --batch divisible by the GPU count")
        args.batch //= world
    B = args.batch
    host_mask = host_cores = None
    if args.cpu_dry_run:
        dev = torch.device("cpu")
        if world > 1 or args.rccl:  # --rccl on one rank: the same group code, over gloo
            one_rank_rendezvous(world)
            dist.init_process_group("gloo")
        S, reps = args.steps, 1
        graph = env = _DryRun(B, 1 if args.env == "SimulatedCars" else 2)
        active_frac, layer, untimed = 0.0, None, 0
        sync = lambda: None  # noqa: E731
    else:
        host_mask, host_cores = pin_host_cores(local, args.host_cores)
        gpu = 0 if args.rehearse_shared_gpu else local
        if gpu >= torch.cuda.device_count():
            raise SystemExit(f"rank {rank}: LOCAL_RANK {local}, but {torch.cuda.device_count()} HIP device(s) visible")
        torch.cuda.set_device(gpu)
        dev = torch.device("cuda", gpu)
        if world > 1 or args.rccl:
            one_rank_rendezvous(world)
            if args.rehearse_shared_gpu:  # RCCL refuses two ranks on one GPU: the host-side group instead
                dist.init_process_group("gloo")
            else:
                dist.init_process_group("nccl", device_id=dev)
        setup = setup_sac_update if args.workload == "sac_update" else setup_gpu
        env, layer, graph, S, active_frac, untimed, ctx = setup(args, dev, rank, B)
        reps = args.steps // S
        sync = torch.cuda.synchronize

    if not args.cpu_dry_run:
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        # untimed rehearsal of the timed sequence (sync, event, replays, event, sync): the first
        # such sequence after set-up spends ~35-50 us instead of ~15 us of host time in the replay
        # call (profiles/r02/bench_rehearsal_r02y.txt); part of the warm-up, not of the K timed steps
        sync()
        ev0.record()
        for _ in range(reps):
            graph.replay()
        ev1.record()
        sync()
        untimed += reps * S
    shard.barrier(world)
    sync()
    # HIP events bracket the HIP launches; the AQL dispatches run on no HIP stream (their per-launch time
    # comes from the packet processor's timestamps after the region, aql_dispatch_times), so no event there
    events = not args.cpu_dry_run and args.launch != "aql"
    t0 = time.perf_counter()
    if events:
        ev0.record()
    for _ in range(reps):
        graph.replay()
    t_sub = time.perf_counter() - t0
    if events:
        ev1.record()
    sync()
    # this rank's K steps end at its own synchronize; the closing barrier only brackets the region (an RCCL
    # barrier is a device collective of tens of us, r05y: 20 steps 5.3 -> 7.7 us per step with it inside)
    # and the MAX over ranks below makes the slowest rank's time the job's
    el = time.perf_counter() - t0
    shard.barrier(world)
    # per fused-step launch, HIP events on the launch stream (torch's current stream)
    kern_ms = ev0.elapsed_time(ev1) / args.steps if events else 0.0
    env.check_failures()
    aql_times = {}
    if args.launch == "aql" and not args.cpu_dry_run:
        # no HIP stream carries the AQL dispatches: the per-launch duration comes from the packet processor's
        # dispatch timestamps of the same S steps, re-run profiled right after the timed region
        aql_times = aql_dispatch_times(env, layer, ctx, graph, S)
        kern_ms = aql_times["period_us"] / 1e3
    red_dev = torch.device("cpu") if args.rehearse_shared_gpu else dev  # gloo reduces host tensors
    per_rank_s = shard.gather_over_ranks(el, world, red_dev)
    el = max(per_rank_s)
    kern_ms = shard.max_over_ranks(kern_ms, world, red_dev)
    value = shard.whole_job_rate(world, B, args.steps, el)
    bps = bytes_per_step(args)
    achieved = B * bps / (kern_ms * 1e-3) / 1e9 if kern_ms > 0 else 0.0
    short = workload_short(args)
    traffic, traffic_src = pmc_traffic_file(short, B)
    kernels = dominant_kernels(args, B)
    rp_form = rocprof_form(args.steps, args.warmup)
    k_us_rp, rp_src = rocprof_kernel_us(short, B, kernels, rp_form, args.launch)
    k_us_rec, rec_src = roofline_record(short, B, rp_form, args.launch)
    span = {}
    if world == 1 and not args.cpu_dry_run and not args.no_span and args.workload == "step":
        span = measure_span(env, layer, ctx, dev, B, bps, queue=getattr(graph, "queue", None))
    extra = {}
    if args.extra and rank == 0 and not args.cpu_dry_run and args.workload == "step":
        extra = extra_measurements(env, layer, dev, args)
    hz = f"{args.hazards}-hazard " if args.env == "Unicycle" else ""
    launch = ("no kernel (CPU dry run)" if args.cpu_dry_run else "eager launches" if args.no_graph
              else f"{S} launches from one host call" if args.launch == "seq"
              else f"{S} AQL dispatches per run on the library's HSA queue" if args.launch == "aql"
              else f"hipGraph of {S} steps")
    sac = args.workload == "sac_update"
    prior_text = {"prior": "prior mean/sigma in-kernel",
                  "tensor": "per-env mean/sigma, column layout of rcbf_gp_predict_cols",
                  "rows": "per-env mean/sigma (B, n_s) row tensors"}[args.prior] + (
        "" if args.prior == "prior" else
        " (mean 0, sigma = MAX_STD materialised, before the GP fit)" if args.prior_values == "maxstd" else
        " (post-GP-fit stand-in)")
    what = (("RCBF_SAC.get_safe_action forward + backward on a replay batch (" +
             ("rcbf_obs_safe_action_jac + rcbf_safe_action_apply_jac" if args.sac_bwd == "jac" else
              "rcbf_obs_safe_action + rcbf_obs_safe_action_backward") +
             ", diff CBF-QP, implicit-KKT grad)") if sac else
            "fused safe step (rcbf_safe_step), non-diff CBF-QP")
    rec = {
        "metric": METRICS.get(args.config, METRICS[0]),
        "value": round(value, 1),
        "unit": "safe actions/s (forward + backward)" if sac else "safe env steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "untimed_steps_executed": untimed,
        "ms_per_step": round(el / args.steps * 1e3, 5),
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "f32 rows / f64 QP" if sac else "f32 rows / f64 QP / f64 env",
        "data": ("dry run: launcher and collectives only, no kernel, not a measurement" if args.cpu_dry_run else
                 "synthetic (fp32 observations of SURVEY 8(d) states one env step on, policy actions ~ U[-1,1], "
                 "upstream gradient ~ N(0,1), " + prior_text + ")" if sac else
                 "synthetic (SURVEY 8(d) start states, u_RL ~ U[-1,1], " + prior_text + ", seeded auto-resets)"),
        "config": {"workload": f"{args.env} {what}, {hz}"
                               f"batch {B} envs per GPU, {args.solver} fp64 QP, {launch}",
                   "baseline_config": args.config or None,
                   "batch_per_gpu": B, "global_batch": B * world, "env": args.env,
                   "solver": args.solver, "parallelism": f"env-shard x{world} (no collective)",
                   "collectives": (f"{'gloo' if args.cpu_dry_run else 'RCCL'} process group, world {world}: "
                                   "barrier around the timed region, "
                                   "all_gather of per-rank times, MAX all_reduce of the per-launch time"
                                   if dist.is_available() and dist.is_initialized() else None),
                   "prior": args.prior, "qp_active_frac_at_start": round(active_frac, 4),
                   "host_cores_per_rank": len(host_cores) if host_cores else None},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "traffic_source": traffic_src,
                     "kernel": " + ".join(kernels), "bytes_per_env_step": bps, "bytes_per_launch": B * bps,
                     "kernel_ms": round(kern_ms, 5), "host_submit_ms": round(t_sub * 1e3, 4),
                     "kernel_us_rocprof": k_us_rp,
                     "frac_rocprof": round(B * bps / (k_us_rp * 1e-6) / 1e9 / HBM_PEAK_GBS, 4) if k_us_rp else None,
                     "rocprof_source": rp_src,
                     "rocprof_form": {"driver": f"driver: rocprofv3 of bench.py --steps {DRIVER_FORM[0]} --warmup "
                                                f"{DRIVER_FORM[1]} --launch {args.launch}",
                                      "default": f"default: rocprofv3 of bench.py --launch {args.launch}"}.get(rp_form),
                     "rocprof_same_command": bool(rp_src),
                     "frac_wall": round(B * bps / (el / args.steps) / 1e9 / HBM_PEAK_GBS, 4),
                     "record": rec_src, "kernel_us_record": k_us_rec,
                     "frac_record": round(B * bps / (k_us_rec * 1e-6) / 1e9 / HBM_PEAK_GBS, 4) if k_us_rec else None,
                     "timing": "achieved = bytes_per_launch / kernel_ms; kernel_ms = HIP events around the timed "
                               "region / steps (includes the graph launch and the inter-kernel gaps); host_submit_ms "
                               "= host time spent in the graph replay calls; kernel_us_rocprof = the AverageNs of "
                               "this kernel in rocprof_source (rocprofv3 --kernel-trace --stats of this command, a "
                               "traced run: each dispatch serialised with its own completion signal); frac_rocprof "
                               "= bytes_per_launch / kernel_us_rocprof"},
    }
    if k_us_rp and k_us_rp * 1e-3 > rec["ms_per_step"]:
        # flagged, not replaced: a traced dispatch carries the tracer's own per-dispatch cost (+2.2-2.5 us on
        # torch kernels of the same size, profiles/r04/tracer_control_r04b.txt), so its mean can exceed the
        # untraced wall time per step
        rec["roofline"]["rocprof_mean_above_wall_per_step"] = True
        rec["roofline"]["rocprof_note"] = ("the traced mean exceeds ms_per_step: rocprofv3 --kernel-trace serialises "
                                           "each dispatch with its own completion signal (tracer control: +2.2-2.5 us "
                                           "per dispatch); frac_rocprof is a traced figure, frac the untraced one")
    stamps = span.pop("_stamps", None) if span else None
    if span:
        rec["roofline"]["span"] = span
    if aql_times:
        rec["roofline"]["aql_dispatch_times"] = aql_times
        rec["roofline"]["timing"] = ("achieved = bytes_per_launch / kernel_ms; kernel_ms = the per-step GPU time of "
                                     "the timed plan's steps re-run on the same queue, (last dispatch end - first "
                                     "dispatch start) / steps from the packet processor's timestamps "
                                     "(aql_dispatch_times.period_us; the AQL counterpart of HIP events around the "
                                     "region); host_submit_ms = host time of the timed run call (submission AND the "
                                     "wait for completion)")
    if args.rehearse_shared_gpu:
        rec["rehearsal"] = (f"{world} ranks sharing GPU 0 over a gloo group: a check of the N > 1 launch path, "
                            "NOT a scaling measurement (the ranks contend for one GPU)")
        rec["config"]["collectives"] = rec["config"]["collectives"] and rec["config"]["collectives"].replace(
            "RCCL", "gloo")
    if world > 1:  # the spread of the timed region over ranks (value is set by the slowest)
        ms = sorted(v / args.steps * 1e3 for v in per_rank_s)
        rec["per_rank_ms"] = {"min": round(ms[0], 5), "median": round(float(np.median(ms)), 5),
                              "max": round(ms[-1], 5)}
    if extra:
        rec["extra"] = extra
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.cpu_dry_run:
        if host_mask:  # the child starts with every allowed core
            os.sched_setaffinity(0, host_mask)
        rec.update(cpu_baselines_in_child(args))
    if rank == 0 and args.record and not args.cpu_dry_run:
        write_record(args, rec, short, B, bps, kern_ms, aql_times, span, stamps)
    if rank == 0:
        print(json.dumps(rec), flush=True)
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()


def write_record(args, rec, short, B, bps, kern_ms, aql_times, span, stamps):
    """--record PATH: the roofline evidence of this run as one JSON file --
    the command, the per-step GPU time `frac` is computed from
    (kernel_us_per_step: AQL first-dispatch-start to last-dispatch-end per step,
    or HIP events), the raw per-run dispatch timestamps, the per-launch span
    stamps (first wave start, last wave end, 100 MHz ticks) and the shader
    clock.  Committed under profiles/ as roofline_record_<form tag><workload>
    _B<B>_<tag>.json, bench.py reads it back (roofline.record, frac_record)."""
    out = {"what": "roofline record of one bench.py run (bench.py --record)",
           "command": "bench.py " + " ".join(a for a in sys.argv[1:] if not a.startswith("--record")
                                             and a != args.record),
           "form": rocprof_form(args.steps, args.warmup), "launch": args.launch, "workload": short, "batch": B,
           "steps": args.steps, "warmup": args.warmup, "bytes_per_env_step": bps, "bytes_per_launch": B * bps,
           "ms_per_step": rec["ms_per_step"], "kernel_us_per_step": round(kern_ms * 1e3, 4),
           "peak_GBs": HBM_PEAK_GBS, "frac": rec["roofline"]["frac"], "frac_wall": rec["roofline"]["frac_wall"],
           "recompute": "frac = bytes_per_launch / (kernel_us_per_step * 1e-6) / 1e9 / peak_GBs; frac_wall the "
                        "same with ms_per_step; frac_span with span.kernel_span_us_median",
           "aql_dispatch_times": aql_times or None, "span": span or None, "span_stamps": stamps,
           "value": rec["value"]}
    os.makedirs(os.path.dirname(os.path.abspath(args.record)), exist_ok=True)
    with open(args.record, "w") as f:
        json.dump(out, f, indent=1)


def bench_closed_loop(args):
    """BASELINE config 1 as the reference runs it (envs/simulated_cars_env.py:161-228): ONE SimulatedCars env,
    the hand controller (:195-199), DynamicsModel.get_state / predict_disturbance (the prior) and
    CascadeCBFLayer(env, gamma_b=20, k_d=3).get_u_safe (cbf_qp.py:29-53) on rcbf_cascade_u_safe_sync, then
    env.step(u_nom + u_safe) on rcbf_env_step_sync -- every call the reference's own surface, per step.
    Timed: exactly --steps closed-loop steps (episodes of 300 from the golden reset, resetting when done),
    after --warmup untimed ones.  Then, untimed, one full episode is checked against the reference's own
    closed loop (tests/golden/closed_loop_cars.npz) and the C oracle's loop is timed on one core beside it.
    One process (the loop is single-env, host-driven: replicas only across GPUs)."""
    import types
    from rcbf_amd.cbf_qp import CascadeCBFLayer
    from rcbf_amd.dynamics import DynamicsModel
    from rcbf_amd.envs import SimulatedCarsEnv
    gold = np.load(os.path.join(ROOT, "tests", "golden", "closed_loop_cars.npz"))
    noise = float(gold["noise"])
    env = SimulatedCarsEnv()
    dm = DynamicsModel(env, types.SimpleNamespace(gp_model_size=2000, cuda=False))
    layer = CascadeCBFLayer(env, gamma_b=20.0, k_d=3.0)

    def reset():
        env._b.reset(noise=np.array([noise]))  # the golden episode's velocity draw (:120)
        return env._get_obs()

    def controller(s):  # simulated_cars_env.py:195-199
        a = np.array([1.0 * (s[4] - s[6] - 0.4) * (s[4] - s[6] - 0.4 < 0)])
        a += np.array([1.0 * (s[8] - s[6] + 0.4) * (s[8] - s[6] + 0.4 > 0)])
        return a

    def run(n, obs, record=None):
        for _ in range(n):
            state = dm.get_state(obs)
            u = controller(state)
            mean, std = dm.predict_disturbance(state)
            us = layer.get_u_safe(u, state, mean, std)
            obs, r, done, info = env.step(u + us)
            if record is not None:
                record.append((u[0], us[0], env.state.copy()))
            if done:
                obs = reset()
        return obs

    obs = run(max(args.warmup, 1), reset())
    obs = reset()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    obs = run(args.steps, obs)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    # parity, untimed: one whole episode against the reference's own loop
    rec = []
    run(300, reset(), rec)
    u_nom = np.array([r[0] for r in rec]); u_safe = np.array([r[1] for r in rec])
    xs = np.array([r[2] for r in rec])

    def rel(a, b):
        return float(np.max(np.abs(a - b) / np.maximum(1.0, np.abs(b))))
    parity = {"u_nom": rel(u_nom, gold["u_nom"][:, 0]), "u_safe": rel(u_safe, gold["u_safe"][:, 0]),
              "state": rel(xs, gold["state"][1:]), "steps": 300,
              "against": "tests/golden/closed_loop_cars.npz (the reference's own closed loop, exact QP)"}
    ok = parity["u_safe"] <= 1e-6 and parity["state"] <= 1e-8
    line = {"metric": METRICS.get(1, METRICS[0]), "value": round(args.steps / el, 1), "unit": "safe env steps/s",
            "n_gpus": 1, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 5),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64 rows / f64 QP / f64 env",
            "data": "the reference's config-1 episode: golden reset draw, the hand controller's actions",
            "config": {"workload": "SimulatedCars Cascade closed loop (config 1, envs/simulated_cars_env.py:161-228): "
                                   "1 env, hand controller + DynamicsModel prior + CascadeCBFLayer.get_u_safe "
                                   "(rcbf_cascade_u_safe_sync) + env.step (rcbf_env_step_sync), host-driven per step",
                       "baseline_config": 1, "batch_per_gpu": 1, "global_batch": 1, "env": "SimulatedCars",
                       "parallelism": "single env (replicas only)"},
            "parity": dict(parity, ok=ok)}
    if not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_closed_loop(noise, args.cpu_seconds)
    print(json.dumps(line), flush=True)
    if not ok:
        raise SystemExit(f"config-1 closed loop differs from the reference's: {parity}")


def cpu_closed_loop(noise, seconds):
    """The C oracle's config-1 closed loop (oracle_cars_cascade_loop: the same controller, Cascade QP and env
    in fp64 C) on ONE core, repeated for ~seconds / 5."""
    from oracle import c_oracle as C
    budget = max(1.0, seconds / 5)
    n, t0 = 0, time.perf_counter()
    while True:
        C.cars_cascade_loop(noise, 300)
        n += 1
        el = time.perf_counter() - t0
        if el >= budget:
            break
    return {"value": round(n * 300 / el, 1), "unit": "safe env steps/s", "cores": 1, "kind": "port",
            "sample": f"C oracle closed loop (oracle/rcbf_oracle.c oracle_cars_cascade_loop), {n} episodes of 300 "
                      f"steps in {el:.2f} s on one thread"}


def unicycle_hazards(k):
    """The reference's hazard list (unicycle_env.py:25-26), first k."""
    from rcbf_amd.envs import _EnvSpec
    return _EnvSpec("Unicycle").hazards_locations[:k]


def prior_tensors(args, env, gen):
    """Per-env (B, n_s) mean / sigma rows for --prior rows / tensor."""
    B, dev = env.num_envs, env.device
    if args.prior_values == "maxstd":  # predict_disturbance before any fit (dynamics.py:381-384), materialised
        from rcbf_amd.dynamics import MAX_STD
        sigma = torch.tensor(MAX_STD[args.env], dtype=torch.float32, device=dev).repeat(B, 1).contiguous()
        return torch.zeros(B, env.n_s, device=dev), sigma
    # a fitted GP's per-env posterior (dynamics.py:342-390): small mean, sigma near MAX_STD
    mean = (0.01 * torch.randn(B, env.n_s, device=dev, generator=gen)).contiguous()
    sigma = (0.2 * torch.rand(B, env.n_s, device=dev, generator=gen) + 0.05).contiguous()
    return mean, sigma


def setup_gpu(args, dev, rank, B):
    """Untimed set-up of the measured workload on this rank's GPU: envs at
    SURVEY start states, the layer, a pool of u_RL batches, warm-up, and the
    captured hipGraph (or the launch object of --launch seq / --no-graph)."""
    from rcbf_amd import _lib, shard
    from rcbf_amd.diff_cbf_qp import CBFQPLayer
    from rcbf_amd.envs import BatchedSimulatedCarsEnv, BatchedUnicycleEnv

    class LArgs:
        cuda = True

    solver = _lib.SOLVER_PDIPM if args.solver == "pdipm" else _lib.SOLVER_ACTIVE_SET
    if args.env == "SimulatedCars":
        env = BatchedSimulatedCarsEnv(B, device=dev, seed=1234, env_offset=shard.env_offset(rank, B))
    else:
        env = BatchedUnicycleEnv(B, device=dev, seed=1234, env_offset=shard.env_offset(rank, B),
                                 hazards_locations=unicycle_hazards(args.hazards))
    layer = CBFQPLayer(env, LArgs(), gamma_b=20.0, solver=solver)
    S = (args.steps if args.launch == "seq" or (args.launch == "aql" and args.steps <= AQL_MAX_STEPS)
         else largest_divisor_le(args.steps, AQL_MAX_STEPS if args.launch == "aql" else args.graph_steps))
    gen = torch.Generator(device=dev)
    gen.manual_seed(1000 + rank)
    init_states(env, gen, args.env)
    # 50 distinct u_RL batches, cycled through by the captured steps
    pool = [(torch.rand(B, env.n_u, device=dev, generator=gen) * 2 - 1).contiguous() for _ in range(min(S, 50))]
    mean = sigma = None
    layout = "cols" if args.prior == "tensor" else "rows"
    if args.prior in ("tensor", "rows"):  # a fitted GP's per-env posterior (dynamics.py:342-390): small mean, sigma near MAX_STD
        mean, sigma = prior_tensors(args, env, gen)
        if layout == "cols":  # what GPDisturbanceModel.predict_cols writes for the step
            cols = list(env.PRIOR_COLS[args.env])
            sigma = sigma[:, cols].t().contiguous()
            mean = None if args.env == "SimulatedCars" else mean[:, cols].t().contiguous()
    outs = env.make_outputs()
    if args.env == "SimulatedCars":
        outs["goal_met"] = None

    def steps(n, off=0):
        for j in range(n):
            env.safe_step(pool[(off + j) % len(pool)], layer, mean=mean, sigma=sigma, outputs=outs, prior_layout=layout)

    # fraction of envs whose safety filter changes the action at the start states
    steps(1)
    untimed = 1 + max(args.warmup, 1)
    active_frac = float((outs["u"] != pool[0]).any(1).float().mean().item())
    # warmup (eager), then capture S fused steps into one hipGraph
    steps(max(args.warmup, 1))
    torch.cuda.synchronize()
    if args.launch == "seq" and not args.no_graph:
        class _Seq:
            def replay(self):
                env.safe_step_seq(pool, layer, mean=mean, sigma=sigma, outputs=outs, steps=S, prior_layout=layout)
        graph = _Seq()
        graph.replay()
        untimed += S
    elif args.no_graph:
        class _Eager:
            def replay(self):
                steps(S)
        graph = _Eager()
    elif args.launch == "aql":
        from rcbf_amd.aql import AqlQueue
        queue = AqlQueue(dev, profile=True)
        plan = queue.safe_step_plan(env, pool, layer, steps=S, mean=mean, sigma=sigma, outputs=outs,
                                    prior_layout=layout)

        class _Aql:
            def replay(self):
                plan.run(sync_hip=False)  # the timed region synchronises the device before it starts
        graph = _Aql()
        graph.queue, graph.plan = queue, plan
        for _ in range(2):
            graph.replay()
        untimed += 2 * S
    else:
        graph = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            steps(2)  # warm the side stream before capture
        torch.cuda.current_stream(dev).wait_stream(s)
        with torch.cuda.graph(graph):
            steps(S)
        for _ in range(2):
            graph.replay()
        untimed += 2 + 2 * S
    torch.cuda.synchronize()
    env.check_failures()
    ctx = {"pool": pool, "mean": mean, "sigma": sigma, "layout": layout, "outs": outs}
    return env, layer, graph, S, active_frac, untimed, ctx


def setup_sac_update(args, dev, rank, B):
    """Untimed set-up of config 5: RCBF_SAC.get_safe_action as the SAC update
    calls it on a replay batch (sac_cbf.py:133,149 -> :218-238): fp32
    observations of SURVEY 8(d) start states, policy actions u ~ U[-1, 1]
    (50 batches cycled), the prior, and an upstream gradient; one timed step
    = rcbf_obs_safe_action + rcbf_obs_safe_action_backward over the batch,
    S of them captured in one hipGraph."""
    import ctypes
    from rcbf_amd import _lib, shard
    from rcbf_amd.diff_cbf_qp import CBFQPLayer
    from rcbf_amd.envs import BatchedSimulatedCarsEnv, BatchedUnicycleEnv

    class LArgs:
        cuda = True
    if args.env == "SimulatedCars":
        env = BatchedSimulatedCarsEnv(B, device=dev, seed=1234, env_offset=shard.env_offset(rank, B))
    else:
        env = BatchedUnicycleEnv(B, device=dev, seed=1234, env_offset=shard.env_offset(rank, B),
                                 hazards_locations=unicycle_hazards(args.hazards))
    layer = CBFQPLayer(env, LArgs(), gamma_b=20.0)
    lib = _lib.load()
    gen = torch.Generator(device=dev)
    gen.manual_seed(2000 + rank)
    init_states(env, gen, args.env)
    # a replay batch: the observations of SURVEY 8(d) states one env step on (load_state leaves obs as it was)
    env.step(torch.rand(B, env.n_u, device=dev, generator=gen) * 2 - 1, auto_reset=False)
    obs = env.obs.clone()
    S = largest_divisor_le(args.steps, args.graph_steps)
    npool = min(S, 50)
    us = [(torch.rand(B, env.n_u, device=dev, generator=gen) * 2 - 1).contiguous() for _ in range(npool)]
    ws = [torch.randn(B, env.n_u, device=dev, generator=gen).contiguous() for _ in range(npool)]
    mu = sg = None
    if args.prior == "rows":  # predict_disturbance's (B, n_s) outputs (sac_cbf.py:231-236)
        mu, sg = prior_tensors(args, env, gen)
    uo = torch.empty(B, env.n_u, device=dev)
    gu = torch.empty(B, env.n_u, device=dev)
    jac = torch.empty(B, env.n_u, env.n_u, dtype=torch.float64, device=dev)
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    prm = ctypes.byref(layer._prm)
    p = _lib.ptr

    def steps(n, off=0):
        s = _lib.stream_of(dev)
        for j in range(n):
            k = (off + j) % npool
            if args.sac_bwd == "jac":
                _lib.check(lib.rcbf_obs_safe_action_jac(prm, B, p(obs), p(us[k]), p(mu), p(sg), p(uo), p(jac), None,
                                                        p(flag), s), "rcbf_obs_safe_action_jac")
                _lib.check(lib.rcbf_safe_action_apply_jac(B, env.n_u, p(jac), p(ws[k]), p(gu), s),
                           "rcbf_safe_action_apply_jac")
            else:
                _lib.check(lib.rcbf_obs_safe_action(prm, B, p(obs), p(us[k]), p(mu), p(sg), p(uo), None, p(flag), s),
                           "rcbf_obs_safe_action")
                _lib.check(lib.rcbf_obs_safe_action_backward(prm, B, p(obs), p(us[k]), p(mu), p(sg), p(ws[k]), p(gu),
                                                             s), "rcbf_obs_safe_action_backward")
    steps(1)
    torch.cuda.synchronize()
    active_frac = float((uo != us[0]).any(1).float().mean().item())
    steps(max(args.warmup, 1))
    side = torch.cuda.Stream(device=dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        steps(2)
    torch.cuda.current_stream(dev).wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        steps(S)
    for _ in range(2):
        graph.replay()
    torch.cuda.synchronize()

    class _Fails:
        def check_failures(self):
            if int(flag.item()):
                raise Exception("QP Failed to solve")
    _Fails().check_failures()
    untimed = 1 + max(args.warmup, 1) + 2 + 2 * S
    return _Fails(), layer, graph, S, active_frac, untimed, {}


def sac_update_safe_action(env, layer, dev):
    """RCBF_SAC.get_safe_action on a replay batch as the SAC
    update calls it (obs -> get_state -> prior -> CBF-QP layer, forward and
    backward w.r.t. the policy action), B = 256 / 512 / 4096 (config 5).
    kernel_us: rcbf_obs_safe_action + its backward captured in a hipGraph;
    autograd_us: the Python surface (rcbf_amd.sac_cbf.get_safe_action +
    .backward) eagerly, including the host fail-flag check."""
    import ctypes
    from rcbf_amd import _lib
    from rcbf_amd.dynamics import DynamicsModel
    from rcbf_amd.sac_cbf import get_safe_action

    class A:
        cuda = True

    lib = _lib.load()
    dyn = DynamicsModel(env, A())
    res = {}
    gen = torch.Generator(device=dev)
    gen.manual_seed(77)
    for B in (256, 512, 4096):
        obs = env.obs[:B].clone()
        u = (torch.rand(B, env.n_u, device=dev, generator=gen) * 2 - 1).contiguous()
        w = torch.randn(B, env.n_u, device=dev, generator=gen)
        uo = torch.empty_like(u)
        gu = torch.empty_like(u)
        flag = torch.zeros(1, dtype=torch.int32, device=dev)
        stream = torch.cuda.Stream(device=dev)
        reps = 50

        def launch():
            s = _lib.stream_of(dev)
            lib.rcbf_obs_safe_action(ctypes.byref(layer._prm), B, _lib.ptr(obs), _lib.ptr(u), None, None,
                                     _lib.ptr(uo), None, _lib.ptr(flag), s)
            lib.rcbf_obs_safe_action_backward(ctypes.byref(layer._prm), B, _lib.ptr(obs), _lib.ptr(u), None, None,
                                              _lib.ptr(w), _lib.ptr(gu), s)

        with torch.cuda.stream(stream):
            launch()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=stream):
            for _ in range(reps):
                launch()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(4):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        k_us = e0.elapsed_time(e1) * 1e3 / (4 * reps)

        def eager():
            uu = u.clone().requires_grad_(True)
            out = get_safe_action(layer, obs, uu, dyn)
            (out * w).sum().backward()
            return uu.grad

        def torch_floor():  # the same loss around a torch-only stand-in op: torch's own autograd cost
            uu = u.clone().requires_grad_(True)
            (torch.clamp(uu + 0.1, -10.0, 10.0) * w).sum().backward()
            return uu.grad

        def per_call(fn, n=50):
            for _ in range(5):
                fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(n):
                fn()
            torch.cuda.synchronize()
            return (time.perf_counter() - t0) * 1e6 / n

        a_us = per_call(eager)
        op, _lib._torch_op = _lib._torch_op, None  # the Python autograd.Function path, for comparison
        try:
            p_us = per_call(eager)
        finally:
            _lib._torch_op = op
        res[f"sac_safe_action_fwd_bwd_B{B}"] = {"kernel_us": round(k_us, 2), "autograd_us": round(a_us, 1),
                                                "python_function_us": round(p_us, 1),
                                                "torch_only_floor_us": round(per_call(torch_floor), 1)}
    return res


def generic_qp_rows(layer, dev):
    """CBFQPLayer.solve_qp / cbf_layer under autograd (rcbf_qp_solve +
    rcbf_qp_backward, diff_cbf_qp.py:81-144) on the layer's own rows:
    cars-shaped (n = 2, m = 4) and unicycle-shaped (n = 3, m = 7) QPs, full
    P, row-normalised; forward and backward launch times from one hipGraph,
    with the algorithmic bytes per QP (fwd: P, q, G, h in + z out; bwd: the
    same in + grad_z in + grad_P, grad_q, grad_G, grad_h out)."""
    import ctypes
    from rcbf_amd import _lib
    lib = _lib.load()
    out = {}
    gen = torch.Generator(device=dev)
    gen.manual_seed(5)
    for n, m in ((2, 4), (3, 7)):
        for B in (4096, 65536):
            A = torch.randn(B, n, n, device=dev, generator=gen)
            P = (A @ A.transpose(1, 2) + n * torch.eye(n, device=dev)).contiguous()
            q = torch.randn(B, n, device=dev, generator=gen)
            G = torch.randn(B, m, n, device=dev, generator=gen)
            z0 = 0.3 * torch.randn(B, n, device=dev, generator=gen)
            h = (torch.einsum("bmn,bn->bm", G, z0) + 0.5 * torch.randn(B, m, device=dev, generator=gen).abs()).contiguous()
            out[f"qp_n{n}_m{m}_B{B}"] = _qp_pair_times(lib, layer._prm, P, q, G, h, gen, dev)
    # the layer's own rows (diagonal P, q = 0, slack/actuator structure): solve_qp as
    # get_safe_action calls it -- the closed-form path
    from rcbf_amd.diff_cbf_qp import CBFQPLayer
    from rcbf_amd.envs import BatchedSimulatedCarsEnv, BatchedUnicycleEnv

    class LArgs:
        cuda = True
    B = 65536
    for name, env in (("cars", BatchedSimulatedCarsEnv(4, device=dev)),
                      ("unicycle3", BatchedUnicycleEnv(4, device=dev, hazards_locations=unicycle_hazards(3)))):
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
        out[f"qp_layer_rows_{name}_B{B}"] = _qp_pair_times(lib, lay._prm, P, q, G, h, gen, dev)
    return out


def _qp_pair_times(lib, prm_struct, P, q, G, h, gen, dev):
    """Forward and backward launch times of one batch of QPs, row-normalised,
    as the autograd surface runs them: rcbf_qp_solve_saved (z and the saved
    fp64 solution) then rcbf_qp_backward_saved from it; plus the backward
    that re-solves (rcbf_qp_backward).  Algorithmic bytes per QP: fwd P, q,
    G, h in + z out (+ the saved z64), bwd the same in + z64 + grad_z in +
    grad_P, grad_q, grad_G, grad_h out."""
    import ctypes
    from rcbf_amd import _lib
    B, m, n = G.shape
    z = torch.empty(B, n, device=dev)
    z64 = torch.empty(B, n, dtype=torch.float64, device=dev)
    gz = torch.randn(B, n, device=dev, generator=gen)
    gP, gq, gG, gh = torch.empty_like(P), torch.empty_like(q), torch.empty_like(G), torch.empty_like(h)
    prm = ctypes.byref(prm_struct)
    ins = [_lib.ptr(P), _lib.ptr(q), _lib.ptr(G), _lib.ptr(h), 1]
    grads = [_lib.ptr(gP), _lib.ptr(gq), _lib.ptr(gG), _lib.ptr(gh)]

    def fwd():
        lib.rcbf_qp_solve_saved(prm, B, n, m, *ins, _lib.ptr(z), _lib.ptr(z64), None, None, _lib.stream_of(dev))

    def bwd():
        lib.rcbf_qp_backward_saved(prm, B, n, m, *ins, _lib.ptr(z64), _lib.ptr(gz), *grads, _lib.stream_of(dev))

    def bwd_resolve():
        lib.rcbf_qp_backward(prm, B, n, m, *ins, _lib.ptr(gz), *grads, _lib.stream_of(dev))
    fms = _time_graph(fwd, 200, dev)
    bms, rms = _time_graph(bwd, 200, dev), _time_graph(bwd_resolve, 200, dev)
    by_in = 4 * (n * n + n + m * n + m)
    return {"fwd_us": round(fms * 1e3, 2), "bwd_us": round(bms * 1e3, 2), "bwd_resolve_us": round(rms * 1e3, 2),
            "fwd_GBs": round(B * (by_in + 12 * n) / fms / 1e6, 1),
            "bwd_GBs": round(B * (2 * by_in + 12 * n) / bms / 1e6, 1)}


def _time_graph(fn, reps, dev):
    """Mean ms per fn() call, fn captured `reps` times in one hipGraph, the best of 3 replays (each
    replay's events also hold the graph's start, ~15 us: keep reps * per-call time well above it)."""
    s = torch.cuda.Stream(device=dev)
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


def next_rows(dev):
    """SURVEY 8f rows 1, 3, 4 (secondary numbers, not `value`): GP posterior
    (rcbf_gp_predict, N = gp_model_size = 3000, exact variance, cars n_s = 10)
    as TFLOP/s of the fp32 MFMA; the model-rollout step (rcbf_model_step) and
    the replay ring push / sample (rcbf_ring_scatter_f64 / rcbf_gather_rows_f64)
    as rows/s and algorithmic GB/s."""
    import ctypes
    from rcbf_amd import _lib, gp
    from rcbf_amd.envs import BatchedSimulatedCarsEnv
    from rcbf_amd.params import make_params
    lib = _lib.load()
    out = {}
    rng = np.random.default_rng(0)
    tx = rng.normal(0, 1, (3000, 10))
    ty = 0.1 * np.sin(tx) + rng.normal(0, 0.05, (3000, 10))
    model = gp.GPDisturbanceModel(tx, ty, [(1.5, 0.2, 0.05)] * 10, device=dev)
    for B in (1, 256, 4096):
        x = torch.as_tensor(rng.normal(0, 1, (B, 10)), dtype=torch.float32, device=dev)
        ms = _time_graph(lambda: model.predict(x), 20 if B <= 256 else 5, dev)
        out[f"gp_predict_N3000_B{B}"] = {"ms": round(ms, 4), "tflops": round(model.flops_per_query() * B / ms / 1e9, 1),
                                          "frac_fp32_mfma_157TF": round(model.flops_per_query() * B / ms / 1e9 / 157.3, 3)}
    lr = gp.GPDisturbanceModel(tx, ty, [(1.5, 0.2, 0.05)] * 10, device=dev, rank=100)
    for B in (1, 256, 4096):  # rank 100: the root-decomposition size of gpytorch's fast_pred_var
        x = torch.as_tensor(rng.normal(0, 1, (B, 10)), dtype=torch.float32, device=dev)
        ms = _time_graph(lambda: lr.predict(x), 20 if B <= 256 else 5, dev)
        out[f"gp_predict_N3000_rank100_B{B}"] = {"us": round(ms * 1e3, 2),
                                                  "tflops": round(lr.flops_per_query() * B / ms / 1e9, 2)}
    B = 65536
    env = BatchedSimulatedCarsEnv(4, device=dev)
    prm = make_params(env, 1.0)
    obs = torch.rand(B, 10, dtype=torch.float64, device=dev)
    act = torch.rand(B, 1, dtype=torch.float64, device=dev)
    t = torch.rand(B, dtype=torch.float64, device=dev)
    nobs = torch.empty_like(obs)
    r, m, nt = (torch.empty(B, dtype=torch.float64, device=dev) for _ in range(3))

    def step():
        lib.rcbf_model_step(ctypes.byref(prm), B, _lib.ptr(obs), _lib.ptr(act), _lib.ptr(t), None, None, None, 1, 0,
                            _lib.ptr(nobs), _lib.ptr(r), _lib.ptr(m), _lib.ptr(nt), _lib.stream_of(dev))
    ms = _time_graph(step, 20, dev)
    out["model_step_cars_B65536"] = {"us": round(ms * 1e3, 2), "rows_per_s": round(B / ms * 1e3, 1),
                                     "GBs": round(B * 200 / ms / 1e6, 1)}
    # DynamicsModel.predict_next_state on device rows with the GP mean / std (f32): x, act, t, mean, std in;
    # next_x, std_out, next_t out = 80 + 8 + 8 + 40 + 40 + 80 + 80 + 8 = 344 B per row
    mean, std = (torch.rand(B, 10, dtype=torch.float32, device=dev) for _ in range(2))
    nx, so = torch.empty_like(obs), torch.empty_like(obs)
    ms = _time_graph(lambda: lib.rcbf_predict_next_state(ctypes.byref(prm), B, _lib.ptr(obs), _lib.ptr(act),
                                                         _lib.ptr(t), _lib.ptr(mean), _lib.ptr(std), 1, _lib.ptr(nx),
                                                         _lib.ptr(so), _lib.ptr(nt), _lib.stream_of(dev)), 20, dev)
    out["predict_next_state_gp_cars_B65536"] = {"us": round(ms * 1e3, 2), "GBs": round(B * 344 / ms / 1e6, 1)}
    W, cap = 25, 1 << 20
    ring = torch.zeros(cap, W, dtype=torch.float64, device=dev)
    src = torch.rand(B, W, dtype=torch.float64, device=dev)
    ms = _time_graph(lambda: lib.rcbf_ring_scatter_f64(_lib.ptr(ring), cap, W, cap - 100, _lib.ptr(src), B,
                                                        _lib.stream_of(dev)), 20, dev)
    out["replay_push_B65536"] = {"us": round(ms * 1e3, 2), "GBs": round(2 * B * W * 8 / ms / 1e6, 1)}
    for n in (256, 65536):
        idx = torch.randint(0, cap, (n,), device=dev)
        dst = torch.empty(n, W, dtype=torch.float64, device=dev)
        ms = _time_graph(lambda: lib.rcbf_gather_rows_f64(_lib.ptr(dst), _lib.ptr(ring), W, _lib.ptr(idx), n,
                                                           _lib.stream_of(dev)), 20, dev)
        out[f"replay_sample_B{n}"] = {"us": round(ms * 1e3, 2), "GBs": round(n * (2 * W * 8 + 8) / ms / 1e6, 1)}
    return out


def cascade_rows(dev):
    """SURVEY 8(a) row a12 at config size: CascadeCBFLayer.get_u_safe
    (rcbf_cascade_u_safe: fp64 rows, normalisation, exact QP) on 4096 cars
    rows (config-2 start states, gamma_b 20, k_d 3) and 4096 unicycle rows
    (k = 3 hazards, gamma_b 40, k_d 3), one launch each, hipGraph-timed; the
    algorithmic bytes per QP are the fp64 inputs and the fp64 u_safe."""
    import ctypes
    from rcbf_amd import _lib
    from rcbf_amd.cbf_qp import CascadeCBFLayer
    from rcbf_amd.envs import SimulatedCarsEnv, UnicycleEnv
    lib = _lib.load()
    out = {}
    gen = torch.Generator(device=dev)
    gen.manual_seed(23)
    B = 4096
    cars = BatchedStartStates.cars(B, dev, gen)
    uni = UnicycleEnv()
    uni.hazards_locations = uni.hazards_locations[:3]
    for name, layer, X, n_u, n_s in (("cars", CascadeCBFLayer(SimulatedCarsEnv(), gamma_b=20.0, k_d=3.0), cars, 1, 10),
                                     ("unicycle3", CascadeCBFLayer(uni, gamma_b=40.0, k_d=3.0, l_p=0.03),
                                      torch.cat([torch.rand(B, 2, device=dev, generator=gen, dtype=torch.float64) * 6 - 3,
                                                 (torch.rand(B, 1, device=dev, generator=gen, dtype=torch.float64) * 2 - 1)
                                                 * math.pi], 1).contiguous(), 2, 3)):
        U = (torch.rand(B, n_u, device=dev, generator=gen, dtype=torch.float64) * 2 - 1).contiguous()
        M = torch.zeros(B, n_s, dtype=torch.float64, device=dev)
        S = torch.full((B, n_s), 0.2, dtype=torch.float64, device=dev)
        if name == "cars":
            S[:, 0::2] = 0.0
        o = torch.empty(B, n_u, dtype=torch.float64, device=dev)
        flag = torch.zeros(1, dtype=torch.int32, device=dev)

        def launch():
            lib.rcbf_cascade_u_safe(ctypes.byref(layer._prm), B, _lib.ptr(U), _lib.ptr(X), _lib.ptr(M), _lib.ptr(S),
                                    _lib.ptr(o), None, _lib.ptr(flag), None, _lib.stream_of(dev))
        ms = _time_graph(launch, 50, dev)
        nbytes = B * 8 * (n_u + 3 * n_s + n_u)
        out[f"cascade_u_safe_{name}_B{B}"] = {"us": round(ms * 1e3, 2), "qps_per_s": round(B / ms * 1e3, 1),
                                              "GBs": round(nbytes / ms / 1e6, 1)}
    return out


class BatchedStartStates:
    @staticmethod
    def cars(B, dev, gen):
        """Config-2 start states (bench.init_states), as an fp64 (B, 10) tensor."""
        from rcbf_amd.envs import BatchedSimulatedCarsEnv
        env = BatchedSimulatedCarsEnv(B, device=dev, seed=77)
        init_states(env, gen, "SimulatedCars")
        return env.state.double().contiguous()


def extra_measurements(env, layer, dev, args):
    """Secondary numbers (not `value`): the K-step rollout kernel (state in
    registers across steps) and the fused step at a batch beyond the 256 MiB
    Infinity Cache."""
    from rcbf_amd.envs import BatchedSimulatedCarsEnv
    out = {}
    K = 100
    u = (torch.rand(K, env.num_envs, env.n_u, device=dev) * 2 - 1).contiguous()
    env.rollout(u, layer)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    env.rollout(u, layer)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    out["rollout_K100_steps_per_s"] = round(env.num_envs * K / (ms * 1e-3), 1)
    out.update(sac_update_safe_action(env, layer, dev))
    out.update(generic_qp_rows(layer, dev))
    out.update(cascade_rows(dev))
    out.update(next_rows(dev))
    if args.env == "SimulatedCars":
        Bb = 4 * 1024 * 1024
        big = BatchedSimulatedCarsEnv(Bb, device=dev, seed=5)
        ub = (torch.rand(Bb, 1, device=dev) * 2 - 1).contiguous()
        o = big.make_outputs()
        o["goal_met"] = None
        for _ in range(3):
            big.safe_step(ub, layer, outputs=o)
        torch.cuda.synchronize()
        e0.record()
        n = 20
        for _ in range(n):
            big.safe_step(ub, layer, outputs=o)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / n
        out["batch_4M_steps_per_s"] = round(Bb / (ms * 1e-3), 1)
        out["batch_4M_hbm_GBs"] = round(Bb * BYTES_PER_STEP["SimulatedCars"] / (ms * 1e-3) / 1e9, 1)
    return out


if __name__ == "__main__":
    main()
