"""Ego-batch sharding across GPUs.

Every ego scenario is independent and the only shared input is the read-only trajectory table,
so a batch partitions into contiguous per-rank shards with no data-path exchange.  The one
collective is the final gather of per-rank solver telemetry to rank 0 (RCCL over xGMI with the
"nccl" backend on ROCm; gloo in the CPU tests).
"""
import numpy as np

TELEMETRY_FIELDS = ("ok", "max_iter", "infeasible", "numerical", "iters_sum", "iters_max", "n", "sqp_unconverged")
SQP_UNCONVERGED, STATUS_MASK = 16, 15     # include/mpcqp.h


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
    counts = [float(((status & STATUS_MASK) == k).sum()) for k in range(4)]
    return np.array(counts + [float(iters.sum()), float(iters.max(initial=0)), float(status.size),
                              float(((status & SQP_UNCONVERGED) != 0).sum())], np.float64)


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
            "egos": int(n), "ranks": int(mat.shape[0]), "sqp_unconverged": int(mat[:, 7].sum())}


# ---------------------------------------------------------------------------------------------
# closed-loop telemetry: each rank runs mpc_closed_loop on its ego shard; one gather
# brings every ego's check quantities, plus the FP32 histories of the first `hist_egos` egos of each
# shard, to rank 0, which applies the restated verdicts (sanity_checks.check_verdicts) to all egos.
# ---------------------------------------------------------------------------------------------
CL_FIELDS = ("ego", "n_steps", "s_final", "max_dev", "u1_min", "u1_max", "u2_min", "u2_max", "max_cpu_ms",
             "min_obs_dist", "red_pass")
HIST_COLS = 7          # s, d, o, k, v of the state after the step, then u1, u2 of the step


def closed_loop_quantities(r, lo, dynamic_obstacle, traffic_light, tl_pos, step_ms=None):
    """[B, len(CL_FIELDS)] float64 check quantities of a closed_loop() result (mpcqp.Solver.closed_loop
    layout) for egos lo .. lo + B - 1.  The solve time each ego saw at a step is that batched step's
    device time (step_ms), the latency of its answer."""
    from sanity_checks import check_quantities
    ns = np.asarray(r["n_steps"])
    B = ns.size
    sm = np.asarray(r["step_ms"] if step_ms is None else step_ms, np.float64)
    out = np.zeros((B, len(CL_FIELDS)))
    for b in range(B):
        n = int(ns[b])
        if n == 0:
            out[b] = [lo + b, 0, r["hist_x"][b, 0, 0], abs(r["hist_x"][b, 0, 1])] + [0.0] * 4 + [0.0, np.nan, 0.0]
            continue
        q = check_quantities(r["hist_x"][b, :n + 1], r["hist_u"][b, :n], sm[:n] / 1e3, r["hist_obs_s"][b, :n],
                             np.asarray(r["hist_tl"][b, :n]) == 0, dynamic_obstacle, traffic_light, tl_pos)
        out[b] = [lo + b, n] + [q[k] for k in CL_FIELDS[2:]]
    return out


def pack_closed_loop(quant, r, rows, hist_egos, max_steps):
    """One rank's gather payload (bytes, the same size on every rank): int32 header (egos, history egos),
    float64 quantities padded to `rows` egos, float32 histories [hist_egos, max_steps, HIST_COLS] (NaN past
    an ego's last step)."""
    B = quant.shape[0]
    h = min(hist_egos, B)
    q = np.full((rows, len(CL_FIELDS)), np.nan)
    q[:B] = quant
    hist = np.full((hist_egos, max_steps, HIST_COLS), np.nan, np.float32)
    if h:
        hist[:h, :, :5] = r["hist_x"][:h, 1:max_steps + 1]
        hist[:h, :, 5:] = r["hist_u"][:h, :max_steps]
    return np.concatenate([np.array([B, h], np.int32).view(np.uint8), q.view(np.uint8).ravel(),
                           hist.view(np.uint8).ravel()])


def unpack_closed_loop(buf, rows, hist_egos, max_steps):
    buf = np.ascontiguousarray(buf, np.uint8)
    B, h = buf[:8].view(np.int32)
    nq = rows * len(CL_FIELDS) * 8
    q = buf[8:8 + nq].view(np.float64).reshape(rows, len(CL_FIELDS))[:B]
    hist = buf[8 + nq:].view(np.float32).reshape(hist_egos, max_steps, HIST_COLS)[:h]
    return q, hist


def gather_closed_loop(payload, device=None):
    """The one collective of the closed loop: gather of every rank's payload to rank 0 (RCCL with the
    "nccl" backend, gloo on CPU).  Returns the list of payloads on rank 0 and None elsewhere; without a
    process group, [payload]."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [payload]
    t = torch.as_tensor(payload, device=device)
    if dist.get_rank() == 0:
        out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
        dist.gather(t, gather_list=out, dst=0)
        return [o.cpu().numpy() for o in out]
    dist.gather(t, dst=0)
    return None


def closed_loop_report(payloads, rows, hist_egos, max_steps, u_min, u_max, s_total):
    """Rank 0: the restated verdicts over every ego of every rank, and the gathered histories."""
    from sanity_checks import check_verdicts
    qs, hists = zip(*(unpack_closed_loop(p, rows, hist_egos, max_steps) for p in payloads))
    q = np.concatenate(qs)
    names = ("destination", "on_road", "steer_ok", "accel_ok", "realtime", "obstacle_ok", "light_ok", "passed")
    counts = dict.fromkeys(names, 0)
    for row in q:
        v = check_verdicts(dict(zip(CL_FIELDS, row)), u_min, u_max, s_total)
        for k in names:
            counts[k] += int(v[k])
    return {"egos": int(q.shape[0]), "ranks": len(payloads), "ego_steps": int(q[:, 1].sum()),
            "checks_passed": counts, "quantities": q, "hist": np.concatenate(hists)}
