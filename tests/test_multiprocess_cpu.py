"""The N > 1 path on CPU (gloo, world_size 2): the shard layout, barrier and
max-over-ranks reduction bench.py uses (rcbf_amd.shard), and sharding
invariance of the batched episode stream -- each rank steps its contiguous
shard with auto-resets whose N(0, 0.5) draw is keyed by the GLOBAL env index
(the device RNG restated by the oracle), and the gathered result equals the
unsharded run bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import oracle as O

B_TOTAL, STEPS, SEED = 64, 310, 9


def _run_shard(x, t, st, ep, offset, u_seq):
    """Oracle cars episodes with auto-reset for envs [offset, offset + len(x))."""
    x, t, st, ep = x.copy(), t.copy(), st.copy(), ep.copy()
    for k in range(STEPS):
        u = u_seq[k, offset:offset + x.shape[0]]
        x, t, st, obs, r, c, done = O.cars_step(x, t, st, u)
        if done.any():
            idx = np.nonzero(done)[0]
            ep[idx] += 1
            nz = 0.5 * O.normal_draw(SEED, offset + idx, ep[idx])
            xr, tr, sr = O.cars_reset(nz)
            x[idx], t[idx], st[idx] = xr, tr, sr
    return x, ep


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from rcbf_amd import shard
    dist.init_process_group("gloo", rank=rank, world_size=world)
    r, lr, w = shard.world_info()
    per = B_TOTAL // w
    off = shard.env_offset(r, per)
    rng = np.random.default_rng(0)
    u_seq = rng.uniform(-1, 1, (STEPS, B_TOTAL, 1)).astype(np.float32)
    ep = np.ones(per, np.int64)
    x0, t0, st0 = O.cars_reset(0.5 * O.normal_draw(SEED, off + np.arange(per), ep))
    shard.barrier(w)
    xs, eps = _run_shard(x0, t0, st0, ep, off, u_seq)
    shard.barrier(w)
    el = shard.max_over_ranks(0.5 + r, w, "cpu")  # rank 1 is "slower"
    gx = [torch.zeros(per, 10, dtype=torch.float64) for _ in range(w)]
    dist.all_gather(gx, torch.as_tensor(xs))
    if r == 0:
        q.put((torch.cat(gx).numpy(), el, shard.whole_job_rate(w, per, STEPS, el)))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_gloo_shards_reproduce_unsharded_run():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    x_sharded, el, rate = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # unsharded reference run
    rng = np.random.default_rng(0)
    u_seq = rng.uniform(-1, 1, (STEPS, B_TOTAL, 1)).astype(np.float32)
    ep = np.ones(B_TOTAL, np.int64)
    x0, t0, st0 = O.cars_reset(0.5 * O.normal_draw(SEED, np.arange(B_TOTAL), ep))
    x_full, _ = _run_shard(x0, t0, st0, ep, 0, u_seq)
    assert np.array_equal(x_sharded, x_full)
    assert el == 1.5  # max over ranks
    assert rate == pytest.approx(2 * (B_TOTAL // 2) * STEPS / 1.5)


def test_bench_gpus_flag_launches_ranks():
    """`python bench.py --gpus 2` (no torchrun) starts 2 rank processes before
    any GPU call; they rendezvous on 127.0.0.1, run the barrier / max-over-
    ranks timing and rank 0 prints ONE JSON line for the whole job.  Here on
    the CPU with gloo and no kernel (--cpu-dry-run)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--cpu-dry-run",
                        "--steps", "5", "--warmup", "1", "--batch", "1024"],
                       capture_output=True, text=True, timeout=300, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["config"]["global_batch"] == 2 * 1024
    assert rec["config"]["parallelism"] == "env-shard x2 (no collective)" and rec["steps"] == 5
    assert rec["value"] > 0 and "dry run" in rec["data"]


@pytest.mark.parametrize("n", [2, 8])
def test_bench_under_torchrun_launcher(n):
    """The driver's N > 1 launch form: python -m torch.distributed.run
    --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N
    (ranks from the torchrun environment, no second spawn), CPU dry run; N = 8
    rehearses the driver's full-node scaling run."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(root, "bench.py"),
                        "--gpus", str(n), "--cpu-dry-run", "--steps", "4", "--warmup", "1", "--batch", "512"],
                       capture_output=True, text=True, timeout=300, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == n and rec["config"]["global_batch"] == n * 512
    assert rec["config"]["parallelism"] == f"env-shard x{n} (no collective)"
    spread = rec["per_rank_ms"]  # the slowest rank sets value; the spread shows a straggler
    assert spread["min"] <= spread["median"] <= spread["max"] == rec["ms_per_step"]


def _check_plan(plan, world, cpus):
    assert plan is not None and len(plan) == world
    sizes = {len(m) for m in plan}
    assert len(sizes) == 1 and sizes.pop() >= 1  # equal-sized
    flat = [c for m in plan for c in m]
    assert len(flat) == len(set(flat))  # disjoint
    assert set(flat) <= set(cpus)


@pytest.mark.parametrize("ncpu", [16, 64])
@pytest.mark.parametrize("numa", [False, True])
def test_host_core_plan_eight_ranks(ncpu, numa):
    """bench.py --host-cores on an 8-GPU node: the allowed CPUs are split into
    disjoint, equal-sized masks over the 8 local ranks (every rank pinned, or
    none); with a 2-socket topology (GPUs 0-3 on node 0, 4-7 on node 1) each
    rank's cores sit on its GPU's node."""
    from rcbf_amd import shard
    cpus = list(range(ncpu))
    gpu_numa = [0, 0, 0, 0, 1, 1, 1, 1] if numa else []
    node_cpus = {0: cpus[:ncpu // 2], 1: cpus[ncpu // 2:]} if numa else {}
    plan = shard.plan_host_cores(cpus, 8, 4, gpu_numa, node_cpus)
    _check_plan(plan, 8, cpus)
    assert len(plan[0]) == min(4, ncpu // 8)
    if numa:
        for r in range(8):
            assert set(plan[r]) <= set(node_cpus[gpu_numa[r]])
    # a rank's GPU on a node with no allowed CPUs: fall back to the plain split, still equal and disjoint
    plan = shard.plan_host_cores(cpus, 8, 4, [0] * 7 + [3], {0: cpus})
    _check_plan(plan, 8, cpus)
    # fewer CPUs than ranks: nobody is pinned
    assert shard.plan_host_cores(cpus[:7], 8, 4) is None
    assert shard.plan_host_cores(cpus, 8, 0) is None


def test_gpu_numa_nodes_from_a_sysfs_tree(tmp_path, monkeypatch):
    """The GPU -> NUMA node map is read from the KFD topology and the PCI
    devices' numa_node (no GPU call), CPU nodes skipped, visible-device masks
    applied."""
    from rcbf_amd import shard
    topo = tmp_path / "class/kfd/kfd/topology/nodes"
    gpus = [(0x0300, 0), (0x8300, 1)]  # (location_id, numa node): bus 03 and bus 83
    (topo / "0").mkdir(parents=True)
    (topo / "0/properties").write_text("cpu_cores_count 64\nsimd_count 0\n")
    for k, (loc, node) in enumerate(gpus, 1):
        (topo / str(k)).mkdir()
        (topo / str(k) / "properties").write_text(f"simd_count 1024\nlocation_id {loc}\ndomain 0\n")
        bdf = tmp_path / "bus/pci/devices" / f"0000:{loc >> 8:02x}:00.0"
        bdf.mkdir(parents=True)
        (bdf / "numa_node").write_text(f"{node}\n")
    for n, cl in ((0, "0-3,8-11"), (1, "4-7,12-15")):
        (tmp_path / f"devices/system/node/node{n}").mkdir(parents=True)
        (tmp_path / f"devices/system/node/node{n}/cpulist").write_text(cl + "\n")
    monkeypatch.delenv("ROCR_VISIBLE_DEVICES", raising=False)
    monkeypatch.delenv("HIP_VISIBLE_DEVICES", raising=False)
    assert shard.gpu_numa_nodes(str(tmp_path)) == [0, 1]
    assert shard.node_cpus(str(tmp_path)) == {0: [0, 1, 2, 3, 8, 9, 10, 11], 1: [4, 5, 6, 7, 12, 13, 14, 15]}
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "1")
    assert shard.gpu_numa_nodes(str(tmp_path)) == [1]
    assert shard.gpu_numa_nodes(str(tmp_path / "nowhere")) == []
