"""Ego-batch sharding across GPUs.

Every ego scenario is independent and the only shared input is the read-only trajectory table,
so a batch partitions into contiguous per-rank shards with no data-path exchange.  The one
collective is the final gather to rank 0 of what the reference's run_simulation returns
(trajectory_tracking.py:443): the closed-loop telemetry, plus the per-rank solver summary.

Transports (ShardComm):
  - GPU ranks: RCCL over xGMI through libmpcqp's C ABI (mpc_comm_* / mpc_gather*, include/mpcqp.h).  Rank 0
    makes the RCCL unique id and hands it to the other ranks over a TCP rendezvous on MASTER_ADDR
    (TcpStar; port MPC_COMM_PORT, default MASTER_PORT + 1); the sockets close once the communicator exists.
    No torch on this path.
  - CPU stand-in (tests, bench --device cpu): torch.distributed with gloo, imported only there.
"""
import os
import socket
import struct
import time

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


# ---------------------------------------------------------------------------------------------
# transports
# ---------------------------------------------------------------------------------------------
def _recv_exact(conn, n):
    buf = bytearray()
    while len(buf) < n:
        chunk = conn.recv(n - len(buf))
        if not chunk:
            raise ConnectionError("rendezvous peer closed the connection")
        buf += chunk
    return bytes(buf)


def _send_msg(conn, data):
    conn.sendall(struct.pack("<Q", len(data)) + data)


def _recv_msg(conn):
    return _recv_exact(conn, struct.unpack("<Q", _recv_exact(conn, 8))[0])


class TcpStar:
    """Rendezvous of `world` processes on one TCP star: rank 0 listens on (addr, port), every other rank
    connects once and announces its rank.  Carries small host messages (the RCCL unique id); the data path
    never uses it."""

    def __init__(self, world, rank, addr, port, timeout=300.0):
        self.world, self.rank, self.peers, self.conn = int(world), int(rank), {}, None
        deadline = time.monotonic() + timeout
        if self.rank == 0:
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            try:
                srv.bind((addr, int(port)))
            except OSError as e:
                srv.close()
                raise RuntimeError(f"shard rendezvous: cannot listen on {addr}:{port} ({e}); set MPC_COMM_PORT")
            srv.listen(self.world)
            try:
                while len(self.peers) < self.world - 1:
                    srv.settimeout(max(0.1, deadline - time.monotonic()))
                    conn, _ = srv.accept()
                    conn.settimeout(timeout)
                    r = struct.unpack("<i", _recv_exact(conn, 4))[0]
                    if not (0 < r < self.world) or r in self.peers:
                        conn.close()
                        raise RuntimeError(f"shard rendezvous: unexpected rank {r}")
                    self.peers[r] = conn
            except socket.timeout:
                raise RuntimeError(f"shard rendezvous: {len(self.peers) + 1} of {self.world} ranks arrived")
            finally:
                srv.close()
        else:
            while True:
                try:
                    self.conn = socket.create_connection((addr, int(port)), timeout=5.0)
                    break
                except OSError:
                    if time.monotonic() > deadline:
                        raise RuntimeError(f"shard rendezvous: rank 0 at {addr}:{port} not reachable")
                    time.sleep(0.05)
            self.conn.settimeout(timeout)
            self.conn.sendall(struct.pack("<i", self.rank))

    def bcast(self, data):
        """rank 0's bytes on every rank."""
        if self.rank == 0:
            for r in sorted(self.peers):
                _send_msg(self.peers[r], data)
            return data
        return _recv_msg(self.conn)

    def gather(self, data):
        """Every rank's bytes on rank 0 (rank order), None elsewhere."""
        if self.rank == 0:
            return [data] + [_recv_msg(self.peers[r]) for r in range(1, self.world)]
        _send_msg(self.conn, data)
        return None

    def barrier(self):
        self.gather(b"")
        self.bcast(b"")

    def close(self):
        for c in list(self.peers.values()) + ([self.conn] if self.conn else []):
            try:
                c.close()
            except OSError:
                pass
        self.peers, self.conn = {}, None


class ShardComm:
    """The ranks of one sharded run and their one collective.

    transport 'rccl': libmpcqp's communicator (mpcqp.Comm: ncclGather / ncclAllReduce on the rank's GPU);
              'gloo': torch.distributed on the CPU (the test stand-in);
              'local': world 1, nothing to exchange."""

    def __init__(self, world, rank, transport, native=None):
        self.world, self.rank, self.transport, self.native = int(world), int(rank), transport, native

    @classmethod
    def from_env(cls, device):
        """WORLD_SIZE / RANK / MASTER_ADDR / MASTER_PORT as torch.distributed.run sets them.  device: the rank's
        GPU index (RCCL), or None for the CPU stand-in (gloo)."""
        world = int(os.environ.get("WORLD_SIZE", "1"))
        rank = int(os.environ.get("RANK", "0"))
        # MPC_COMM=rccl runs a world-1 GPU rank through the communicator too (the N > 1 code path on one GPU)
        if world == 1 and not (device is not None and os.environ.get("MPC_COMM") == "rccl"):
            return cls(1, 0, "local")
        if device is None:
            import torch.distributed as dist
            if not dist.is_initialized():
                dist.init_process_group("gloo", init_method="env://", rank=rank, world_size=world)
            return cls(world, rank, "gloo")
        return cls.rccl(world, rank, device)

    @classmethod
    def rccl(cls, world, rank, device, addr=None, port=None):
        """Create the RCCL communicator: rank 0's unique id travels over a TcpStar rendezvous (world > 1)."""
        import mpcqp
        addr = addr or os.environ.get("MASTER_ADDR", "127.0.0.1")
        if port is None:
            port = int(os.environ.get("MPC_COMM_PORT") or int(os.environ.get("MASTER_PORT", "29500")) + 1)
        if world == 1:
            uid = mpcqp.comm_unique_id()
        else:
            star = TcpStar(world, rank, addr, port)
            try:
                uid = star.bcast(mpcqp.comm_unique_id() if rank == 0 else b"")
            finally:
                star.close()
        return cls(world, rank, "rccl", mpcqp.Comm(uid, world, rank, device))

    def gather(self, payload):
        """Gather of one uint8 payload per rank (the same size on every rank) to rank 0: the list of payloads on
        rank 0, None elsewhere."""
        payload = np.ascontiguousarray(payload, np.uint8).ravel()
        if self.transport == "local":
            return [payload]
        if self.transport == "rccl":
            return self.native.gather(payload, root=0)
        import torch
        import torch.distributed as dist
        t = torch.as_tensor(payload)
        if self.rank == 0:
            out = [torch.empty_like(t) for _ in range(self.world)]
            dist.gather(t, gather_list=out, dst=0)
            return [o.numpy() for o in out]
        dist.gather(t, dst=0)
        return None

    def max(self, x):
        """max over ranks of a float (every rank gets it): the measurement's max-over-ranks time."""
        if self.transport == "local":
            return float(x)
        if self.transport == "rccl":
            return self.native.allreduce_max(x)
        import torch
        import torch.distributed as dist
        t = torch.tensor([float(x)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def barrier(self):
        if self.transport == "rccl":
            self.native.barrier()
        elif self.transport == "gloo":
            import torch.distributed as dist
            dist.barrier()

    def close(self):
        if self.transport == "rccl" and self.native is not None:
            self.native.close()
            self.native = None
        elif self.transport == "gloo":
            import torch.distributed as dist
            if dist.is_initialized():
                dist.destroy_process_group()


def telemetry(status, iters):
    """Per-rank summary vector (float64) of one batched solve: status counts, iteration sum/max, size."""
    status = np.asarray(status).ravel()
    iters = np.asarray(iters).ravel()
    counts = [float(((status & STATUS_MASK) == k).sum()) for k in range(4)]
    return np.array(counts + [float(iters.sum()), float(iters.max(initial=0)), float(status.size),
                              float(((status & SQP_UNCONVERGED) != 0).sum())], np.float64)


def gather_telemetry(vec, comm=None):
    """Gather the per-rank telemetry vectors to rank 0 (one collective, after the timed region): the
    [world, len(TELEMETRY_FIELDS)] matrix on rank 0, None on the other ranks; without a communicator (or at
    world 1) the local vector as a 1-row matrix."""
    vec = np.ascontiguousarray(vec, np.float64)
    if comm is None:
        return vec[None, :]
    got = comm.gather(vec.view(np.uint8))
    return None if got is None else np.stack([np.asarray(g, np.uint8).view(np.float64) for g in got])


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


def gather_closed_loop(payload, comm=None):
    """The one collective of the closed loop: gather of every rank's payload to rank 0 (ShardComm: RCCL on
    GPU ranks, gloo in the CPU stand-in).  Returns the list of payloads on rank 0 and None elsewhere; without
    a communicator, [payload]."""
    if comm is None:
        return [np.ascontiguousarray(payload, np.uint8)]
    return comm.gather(payload)


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
