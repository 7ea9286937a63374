"""Multi-GPU layout of the batched safe step: one process per GPU,
each owning a contiguous shard of the global env batch; nothing crosses GPUs
on the data path.  The only collectives are the measurement's barrier and
max-over-ranks time (bench.py).  Backend-agnostic (RCCL on the GPU box, gloo
in the CPU tests), so the code the tests exercise is the code bench.py runs.
"""
import os

import torch
import torch.distributed as dist


def world_info():
    """(rank, local_rank, world) from the torchrun environment (1 process if unset)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def env_offset(rank, per_rank):
    """Global index of this rank's env 0 under weak scaling (per_rank envs each):
    the reset RNG is keyed by (seed, env_offset + i, episode), so any sharding
    reproduces the unsharded run (test_auto_reset_and_rng_sharding_invariance)."""
    return rank * per_rank


def barrier(world):
    if world > 1:
        dist.barrier()


def max_over_ranks(x, world, device):
    """The slowest rank's value (elapsed time, per-launch time)."""
    if world <= 1:
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def whole_job_rate(world, per_rank, steps, elapsed_max):
    """Aggregate safe env steps/s of the whole job: all ranks' env-steps over
    the slowest rank's time."""
    return world * per_rank * steps / elapsed_max
