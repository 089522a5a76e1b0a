"""Candidate sharding across GPUs: one process per GPU, each
evaluates a contiguous slice [r*N/W, (r+1)*N/W) of the candidate batch with the
model replicated; the only exchange is the final gather of the per-candidate
results, after which the order-dependent `enough_stable` prefix rule of the
reference (gravityless_object_grasping.py:151-156) is applied once, globally.
No data-path collective: candidates are independent.

The CLIs (filter_to_stable, gen_grasps, eval_grasps, ...) run sharded when
started under a launcher that sets WORLD_SIZE > 1 (`torchrun --nproc-per-node
N -m mgs.cli.filter_to_stable ...`): every rank evaluates its slice on its
own GPU, the results are gathered over a gloo group (host arrays), and rank 0
writes the reference's files."""
from __future__ import annotations

import os

import numpy as np


def shard_bounds(n: int, world: int, rank: int):
    """Contiguous, balanced slice of n candidates for `rank` of `world`."""
    base, rem = divmod(n, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def gather_results(local: dict, group=None) -> dict:
    """Concatenate per-rank result dicts (numpy arrays, rank order) on every rank."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    parts = [None] * world
    dist.all_gather_object(parts, {k: np.asarray(v) for k, v in local.items()}, group=group)
    return {k: np.concatenate([p[k] for p in parts]) for k in local}


def evaluate_sharded(env, poses, joints, horizon="h200", enough_stable=None, group=None, evaluate=None):
    """filter_to_stable over a batch sharded across the ranks of `group`
    (each rank drives its own GPU through `env.engine`).  `evaluate(poses,
    joints) -> (mask, stable)` is the per-rank evaluator, default
    `env.evaluate(..., horizon=horizon)`; the CPU tests pass the oracle's."""
    import torch.distributed as dist
    from mgs.env.gravityless_object_grasping import apply_enough_stable
    if evaluate is None:
        def evaluate(p, j):
            return env.evaluate(p, j, horizon=horizon)
    lo, hi = shard_bounds(len(poses), dist.get_world_size(group), dist.get_rank(group))
    mask, stable = evaluate(poses[lo:hi], joints[lo:hi])
    out = gather_results({"mask": np.asarray(mask, bool), "stable": np.asarray(stable, bool)}, group)
    out["stable"] = apply_enough_stable(out["stable"], enough_stable)
    return out["mask"], out["stable"]


# ---------------------------------------------------------------------------
# CLI launch helpers
def launch_world():
    """(rank, world size) from the launcher environment (1 process: (0, 1))."""
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))


def init_cli_group():
    """The CLI's process group when WORLD_SIZE > 1: gloo (only host result
    arrays are exchanged); returns (rank, world)."""
    rank, world = launch_world()
    if world > 1:
        import torch.distributed as dist
        if not dist.is_initialized():
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo", rank=rank, world_size=world)
    return rank, world


def cli_device() -> int:
    """This rank's GPU: LOCAL_RANK, shared round-robin when there are more ranks
    than visible GPUs (device counting does not start the HIP runtime)."""
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if int(os.environ.get("WORLD_SIZE", "1")) <= 1:
        return 0
    import torch
    n = torch.cuda.device_count()
    return local % n if n else local


def broadcast_from_rank0(obj):
    """rank 0's object on every rank (identity with one process)."""
    if launch_world()[1] <= 1:
        return obj
    import torch.distributed as dist
    box = [obj]
    dist.broadcast_object_list(box, src=0)
    return box[0]


def filter_sharded(collision_mask, stable_mask, poses, joints, enough_stable=None):
    """The filter_to_stable pipeline (reference mgs/cli/filter_to_stable.py:
    39-50) sharded over the launch's ranks: `collision_mask(poses, joints)` of
    every candidate, then `stable_mask(poses, joints)` of the collision-free
    ones, each rank on its contiguous slice; the gathered per-candidate results
    keep the global order, so the enough_stable first-K prefix over the
    collision-free list is the single-process one.  Returns (mask over all
    candidates, stable over the collision-free candidates) on every rank."""
    from mgs.env.gravityless_object_grasping import apply_enough_stable
    rank, world = launch_world()
    lo, hi = shard_bounds(len(poses), world, rank)
    p, j = poses[lo:hi], joints[lo:hi]
    mask = np.asarray(collision_mask(p, j), bool) if hi > lo else np.zeros(0, bool)
    idx = np.nonzero(mask)[0]
    stable = np.asarray(stable_mask(p[idx], j[idx]), bool) if len(idx) else np.zeros(0, bool)
    if world > 1:
        g = gather_results({"mask": mask, "stable": stable})
        mask, stable = g["mask"], g["stable"]
    return mask, apply_enough_stable(stable, enough_stable)


def stage_sharded(fn, poses, joints):
    """one per-candidate boolean stage (collision mask or stability) sharded over
    the launch's ranks, gathered in the global order."""
    rank, world = launch_world()
    lo, hi = shard_bounds(len(poses), world, rank)
    out = np.asarray(fn(poses[lo:hi], joints[lo:hi]), bool) if hi > lo else np.zeros(0, bool)
    if world > 1:
        out = gather_results({"m": out})["m"]
    return out
