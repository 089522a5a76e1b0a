"""Candidate sharding across GPUs: one process per GPU, each
evaluates a contiguous slice [r*N/W, (r+1)*N/W) of the candidate batch with the
model replicated; the only exchange is the final gather of the per-candidate
results, after which the order-dependent `enough_stable` prefix rule of the
reference (gravityless_object_grasping.py:151-156) is applied once, globally.
No data-path collective: candidates are independent."""
from __future__ import annotations

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
