"""Ego-batch sharding across GPUs.

Every ego scenario is independent and the only shared input is the read-only trajectory table,
so a batch partitions into contiguous per-rank shards with no data-path exchange.  The one
collective is the final gather of per-rank solver telemetry to rank 0 (RCCL over xGMI with the
"nccl" backend on ROCm; gloo in the CPU tests).
"""
import numpy as np

TELEMETRY_FIELDS = ("ok", "max_iter", "infeasible", "numerical", "iters_sum", "iters_max", "n")


def shard_range(total, world, rank):
    """Contiguous [lo, hi) slice of `total` egos owned by `rank` (sizes differ by at most one)."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad world/rank")
    base, extra = divmod(int(total), int(world))
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def telemetry(status, iters):
    """Per-rank summary vector (float64) of one batched solve: status counts, iteration sum/max, size."""
    status = np.asarray(status).ravel()
    iters = np.asarray(iters).ravel()
    counts = [float((status == k).sum()) for k in range(4)]
    return np.array(counts + [float(iters.sum()), float(iters.max(initial=0)), float(status.size)], np.float64)


def gather_telemetry(vec, device=None):
    """All-gather the per-rank telemetry vectors (one collective, after the timed region) and return
    the [world, len(TELEMETRY_FIELDS)] matrix on every rank.  Without an initialised process group,
    returns the local vector as a 1-row matrix."""
    import torch
    import torch.distributed as dist
    v = torch.as_tensor(np.asarray(vec, np.float64), device=device)
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return v.cpu().numpy()[None, :]
    out = [torch.empty_like(v) for _ in range(dist.get_world_size())]
    dist.all_gather(out, v)
    return torch.stack(out).cpu().numpy()


def reduce_telemetry(mat):
    """Whole-job summary from the gathered matrix."""
    mat = np.asarray(mat, np.float64)
    n = mat[:, 6].sum()
    return {"status_counts": {k: int(mat[:, i].sum()) for i, k in enumerate(TELEMETRY_FIELDS[:4])},
            "mean_iters": float(mat[:, 4].sum() / max(n, 1.0)), "max_iters": int(mat[:, 5].max()),
            "egos": int(n), "ranks": int(mat.shape[0])}
