"""Multi-GPU layout of the batched safe step: one process per GPU,
each owning a contiguous shard of the global env batch; nothing crosses GPUs
on the data path.  The only collectives are the measurement's barrier and
max-over-ranks time (bench.py).  Backend-agnostic (RCCL on the GPU box, gloo
in the CPU tests), so the code the tests exercise is the code bench.py runs.
"""
import os

import torch
import torch.distributed as dist


def local_world_size():
    """Ranks on this node (torchrun's LOCAL_WORLD_SIZE; WORLD_SIZE if unset)."""
    return int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1")))


def world_info():
    """(rank, local_rank, world) from the torchrun environment (1 process if unset)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def env_offset(rank, per_rank):
    """Global index of this rank's env 0 under weak scaling (per_rank envs each):
    the reset RNG is keyed by (seed, env_offset + i, episode), so any sharding
    reproduces the unsharded run (test_auto_reset_and_rng_sharding_invariance)."""
    return rank * per_rank


def _group_on():
    """A process group is up (world > 1, or bench.py --rccl on one rank)."""
    return dist.is_available() and dist.is_initialized()


def barrier(world):
    if world > 1 or _group_on():
        dist.barrier()


def max_over_ranks(x, world, device):
    """The slowest rank's value (elapsed time, per-launch time)."""
    if world <= 1 and not _group_on():
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def whole_job_rate(world, per_rank, steps, elapsed_max):
    """Aggregate safe env steps/s of the whole job: all ranks' env-steps over
    the slowest rank's time."""
    return world * per_rank * steps / elapsed_max


def gather_over_ranks(x, world, device):
    """Every rank's value, in rank order (for the per-rank spread of the
    timed region in bench.py's N > 1 line)."""
    if world <= 1 and not _group_on():
        return [float(x)]
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    out = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return [float(v.item()) for v in out]


# ---------------------------------------------------------------------------
# host-core placement of the rank processes (bench.py --host-cores)
# ---------------------------------------------------------------------------
def parse_cpulist(s):
    """'0-3,8,10-11' -> [0, 1, 2, 3, 8, 10, 11]."""
    out = []
    for part in s.strip().split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        out.extend(range(int(a), int(b or a) + 1))
    return out


def _read(path):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def gpu_numa_nodes(sysfs="/sys"):
    """NUMA node of every GPU in HIP's device order (KFD topology order, then
    ROCR_/HIP_VISIBLE_DEVICES applied in that order), read from sysfs WITHOUT
    touching the GPU; -1 where unknown, [] if the topology is unreadable."""
    base = os.path.join(sysfs, "class/kfd/kfd/topology/nodes")
    try:
        nodes = sorted(int(n) for n in os.listdir(base) if n.isdigit())
    except OSError:
        return []
    out = []
    for n in nodes:
        props = {}
        for line in (_read(os.path.join(base, str(n), "properties")) or "").splitlines():
            kv = line.split()
            if len(kv) == 2 and kv[1].lstrip("-").isdigit():
                props[kv[0]] = int(kv[1])
        if props.get("simd_count", 0) == 0:  # a CPU node
            continue
        loc, dom = props.get("location_id", 0), props.get("domain", 0)
        bdf = f"{dom:04x}:{(loc >> 8) & 0xff:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 7:x}"
        numa = _read(os.path.join(sysfs, "bus/pci/devices", bdf, "numa_node"))
        out.append(int(numa) if numa is not None and numa.lstrip("-").isdigit() else -1)
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v:
            try:
                out = [out[int(i)] for i in v.split(",") if i.strip()]
            except (ValueError, IndexError):
                return []
    return out


def node_cpus(sysfs="/sys"):
    """{numa node: [cpus]} from sysfs ({} if unreadable)."""
    base = os.path.join(sysfs, "devices/system/node")
    out = {}
    try:
        names = os.listdir(base)
    except OSError:
        return out
    for name in names:
        if name.startswith("node") and name[4:].isdigit():
            cl = _read(os.path.join(base, name, "cpulist"))
            if cl is not None:
                out[int(name[4:])] = parse_cpulist(cl)
    return out


def plan_host_cores(allowed, local_world, per_rank, gpu_numa=None, numa_cpus=None):
    """Host-core masks of all `local_world` ranks of this node, or None (no
    rank pinned).  Every rank computes the same plan from the same inputs, so
    either all ranks are pinned or none is; the masks are disjoint and of
    equal size n = min(per_rank, len(allowed) // local_world).  Ranks are
    placed on the allowed cores of their GPU's NUMA node when every node has
    room for its ranks, else over the allowed cores in order."""
    allowed = sorted(set(allowed))
    if per_rank <= 0 or local_world <= 0:
        return None
    n = min(per_rank, len(allowed) // local_world)
    if n < 1:
        return None
    if gpu_numa and len(gpu_numa) >= local_world and numa_cpus:
        groups = {}
        for r in range(local_world):
            groups.setdefault(gpu_numa[r], []).append(r)
        masks, ok = {}, True
        for node, ranks in groups.items():
            mine = set(numa_cpus.get(node, ())) if node >= 0 else set()
            cpus = [c for c in allowed if c in mine]
            if len(cpus) < n * len(ranks):
                ok = False
                break
            for j, r in enumerate(ranks):
                masks[r] = cpus[n * j:n * (j + 1)]
        if ok:
            return [masks[r] for r in range(local_world)]
    return [allowed[n * r:n * (r + 1)] for r in range(local_world)]
