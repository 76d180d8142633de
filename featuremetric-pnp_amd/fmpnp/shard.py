"""Multi-GPU sharding of independent refinement problems.

Queries are independent, so a batch is cut into contiguous blocks, one per rank
(one process per GPU, the reference's own scale-out is the same query slicing,
run.py:38-39).  No collective touches the data path; the only exchange is the
optional final gather of the small per-query results (12 doubles + counters).
"""
import time

import torch
import torch.distributed as dist


def shard_range(n_total, rank, world):
    """Contiguous block [lo, hi) of n_total problems for `rank` of `world` (sizes differ by <= 1)."""
    base, extra = divmod(int(n_total), int(world))
    lo = rank * base + min(rank, extra)
    hi = lo + base + (1 if rank < extra else 0)
    return lo, hi


def query_indices(rank, world, per_rank=0, global_batch=0):
    """Global indices of this rank's queries.  Strong scaling (global_batch > 0): a fixed total
    split into contiguous blocks; weak scaling: per_rank queries per rank, i.e. the blocks of
    per_rank * world.  The index is the query's identity everywhere (bench.py seeds its
    synthetic inputs with it), so any rank count refines the same queries."""
    n_total = int(global_batch) if global_batch > 0 else int(per_rank) * int(world)
    return range(*shard_range(n_total, rank, world))


def timed_steps(step, steps, device=None, group=None):
    """Run step(k) for k < steps between two barrier + device-synchronise fences; returns the
    elapsed wall seconds, maximised over ranks (the slowest rank sets the job's time)."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1

    def fence():
        if world > 1:
            dist.barrier(group)
        if device is not None:
            torch.cuda.synchronize(device)

    fence()
    t0 = time.perf_counter()
    for k in range(int(steps)):
        step(k)
    if device is not None:
        torch.cuda.synchronize(device)
    elapsed = time.perf_counter() - t0
    fence()
    return max_over_ranks(elapsed, device=device, group=group)


def refine_sharded(make_problem, n_total, refine_fn, group=None):
    """Refine problems [lo, hi) of this rank and all-gather the per-problem results in
    global order.  make_problem(i) builds problem i; refine_fn(list) returns one result
    dict per problem."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    lo, hi = shard_range(n_total, rank, world)
    local = refine_fn([make_problem(i) for i in range(lo, hi)]) if hi > lo else []
    if world == 1:
        return local
    parts = [None] * world
    dist.all_gather_object(parts, (lo, local), group=group)
    out = []
    for _, res in sorted(parts, key=lambda x: x[0]):
        out.extend(res)
    return out


def device_accounting(device_ids):
    """(n_gpus, ranks_per_device) of a job from the device identity each rank ran on: n_gpus
    counts DISTINCT devices -- two ranks sharing one GPU (a gloo rehearsal on a one-GPU box) are
    one GPU, never two."""
    ids = [tuple(d) if isinstance(d, (list, tuple)) else d for d in device_ids]
    n = len(set(ids))
    return n, (len(ids) / n if n else 0.0)


def gather_device_ids(my_id, group=None):
    """Every rank's device identity (rank order)."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return [my_id]
    parts = [None] * dist.get_world_size(group)
    dist.all_gather_object(parts, my_id, group=group)
    return parts


def max_over_ranks(x, device=None, group=None):
    """Max of a float over ranks (bench timing)."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())
