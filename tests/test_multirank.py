"""Multi-rank path on CPU (gloo, world_size 2): contiguous ego shards, no data-path exchange, one
telemetry gather at the end.  The per-rank solver is libmpcqp itself on its host backend
(mpc_create device = -1: the same entries, solver and closed loop as on the GPU); what is under test is the
partition and the collective, run through the product's code path (shard.ShardComm: gloo is the CPU
stand-in for the GPU ranks' RCCL communicator).  The TCP rendezvous that carries the RCCL unique id on GPU
ranks (shard.TcpStar) is tested here too, with 3 processes."""
import os
import socket

import numpy as np
import pytest

from conftest import traj_arrays

WORLD = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, total, outdir):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    sys.path[:0] = [here, root, os.path.join(root, "safe-autonomous-driving-mpc_amd"), os.path.join(root, "oracle")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import mpcqp
    import shard
    import workloads as W
    os.environ.update(WORLD_SIZE=str(world), RANK=str(rank))
    comm = shard.ShardComm.from_env(None)
    assert comm.transport == "gloo"
    lo, hi = shard.shard_range(total, world, rank)
    wb = W.make_batch("C3", B=hi - lo, offset=lo)
    os.environ["MPC_CPU_THREADS"] = "1"
    slv = mpcqp.Solver(*traj_arrays(wb["traj"]), mpcqp.default_params(N=wb["N"], max_obs=wb["max_obs"]), device=-1)
    r = slv.solve_batch(wb["x0"], wb["obs"], wb["n_obs"])
    mat = shard.gather_telemetry(shard.telemetry(r["status"], r["iters"]), comm)
    assert (mat is None) == (rank != 0)
    mx = comm.max(float(rank) + 0.5)
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), U=r["U"], status=r["status"], iters=r["iters"],
             mat=mat if mat is not None else np.zeros(0), lo=lo, hi=hi, mx=mx)
    comm.close()


def test_shard_range_partitions():
    import shard
    for total in (0, 1, 7, 4096, 4097):
        for world in (1, 2, 3, 8):
            parts = [shard.shard_range(total, world, r) for r in range(world)]
            assert parts[0][0] == 0 and parts[-1][1] == total
            assert all(parts[i][1] == parts[i + 1][0] for i in range(world - 1))
            sizes = [b - a for a, b in parts]
            assert max(sizes) - min(sizes) <= 1


def test_make_batch_offset_is_a_slice_of_the_stream():
    import workloads as W
    full = W.make_batch("C3", B=40)
    part = W.make_batch("C3", B=15, offset=20)
    assert np.array_equal(part["x0"], full["x0"][20:35])
    assert np.array_equal(part["obs"], full["obs"][20:35])


@pytest.fixture(scope="module", autouse=True)
def built():
    import __graft_entry__ as g
    g.build()


def test_two_rank_gloo_matches_single_process(tmp_path):
    import torch.multiprocessing as mp
    import mpcqp
    import shard
    import workloads as W
    total = 96
    mp.spawn(_rank_main, args=(WORLD, _free_port(), total, str(tmp_path)), nprocs=WORLD, join=True)
    parts = [np.load(tmp_path / f"rank{r}.npz") for r in range(WORLD)]
    wb = W.make_batch("C3", B=total)
    slv = mpcqp.Solver(*traj_arrays(wb["traj"]), mpcqp.default_params(N=wb["N"], max_obs=wb["max_obs"]), device=-1)
    ref = slv.solve_batch(wb["x0"], wb["obs"], wb["n_obs"])
    U = np.concatenate([p["U"] for p in parts])
    assert np.array_equal(U, ref["U"])                       # shards are independent: bit-identical
    # rank 0 holds the gathered telemetry (one row per rank, its own row first), and it sums to the single-process
    # batch; every rank got the max over ranks
    assert parts[0]["mat"].shape == (WORLD, len(shard.TELEMETRY_FIELDS))
    for rk, p in enumerate(parts):
        assert np.array_equal(parts[0]["mat"][rk], shard.telemetry(p["status"], p["iters"]))
        assert float(p["mx"]) == WORLD - 0.5
    tel = shard.reduce_telemetry(parts[0]["mat"])
    assert tel["egos"] == total and tel["ranks"] == WORLD
    assert tel["status_counts"]["ok"] == int((ref["status"] == 0).sum())
    assert tel["max_iters"] == int(ref["iters"].max())
    assert tel["mean_iters"] == pytest.approx(float(ref["iters"].mean()))


# ---------------------------------------------------------------------------------------------
# closed-loop telemetry: sharded closed loops + one gather of per-ego check quantities and FP32 histories
# ---------------------------------------------------------------------------------------------
CL_TOTAL, CL_STEPS, CL_HIST = 6, 260, 2


def cl_inputs(total):
    """Starts near the traffic light and the car trigger of the trajectory2 preset, so both scenarios run."""
    rng = np.random.default_rng(17)
    s0 = np.where(np.arange(total) % 2 == 0, rng.uniform(440.0, 460.0, total), rng.uniform(690.0, 700.0, total))
    return np.column_stack([s0, rng.normal(0, 0.03, total), np.zeros(total), np.zeros(total),
                            rng.uniform(7.0, 9.0, total)])


def cpu_closed_loop(x_init, max_steps, N=5):
    """mpcqp.Solver.closed_loop on libmpcqp's host backend (device = -1): the closed-loop entry bench.py's
    --closed-loop leg calls, with the trajectory2 FSM and the drop-in SQP default.  Step times are replaced
    by 1 ms so that the check quantities are deterministic."""
    import mpcqp
    import trajectory_tracking as TT
    from trajectory_loader import TrajectoryLoader, builtin_trajectory
    traj = TrajectoryLoader(builtin_trajectory(2))
    os.environ["MPC_CPU_THREADS"] = "1"
    slv = mpcqp.Solver(traj.X_ref, traj.U_ref, mpcqp.default_params(N=N, sqp_iters=TT.SQP_ITERS), device=-1)
    r = slv.closed_loop(x_init, TT.fsm_params(TT.ObstaclesFSM(True, True)), max_steps=max_steps, s_max=traj.s_max)
    slv.close()
    r["step_ms"] = np.ones(max_steps)
    return r, traj


def _cl_rank_main(rank, world, port, outdir):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    sys.path[:0] = [here, root, os.path.join(root, "safe-autonomous-driving-mpc_amd"), os.path.join(root, "oracle")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import shard
    from test_multirank import cl_inputs, cpu_closed_loop, CL_TOTAL, CL_STEPS, CL_HIST
    os.environ.update(WORLD_SIZE=str(world), RANK=str(rank))
    comm = shard.ShardComm.from_env(None)
    lo, hi = shard.shard_range(CL_TOTAL, world, rank)
    r, traj = cpu_closed_loop(cl_inputs(CL_TOTAL)[lo:hi], CL_STEPS)
    q = shard.closed_loop_quantities(r, lo, True, True, 550.0)
    rows = -(-CL_TOTAL // world)
    payloads = shard.gather_closed_loop(shard.pack_closed_loop(q, r, rows, CL_HIST, CL_STEPS), comm)
    if rank == 0:
        rep = shard.closed_loop_report(payloads, rows, CL_HIST, CL_STEPS, (-0.6, -5.0), (0.6, 4.0), traj.s_max)
        np.savez(os.path.join(outdir, "cl_report.npz"), q=rep["quantities"], hist=rep["hist"],
                 passed=rep["checks_passed"]["passed"], ranks=rep["ranks"])
    else:
        assert payloads is None
    comm.close()


def test_two_rank_closed_loop_gather_matches_single_process(tmp_path):
    """Each rank runs the closed loop of its ego shard; rank 0 gathers (one collective) every ego's check
    quantities and the FP32 histories of the first CL_HIST egos of each shard, and applies the verdicts:
    all of it equals the single-process run."""
    import torch.multiprocessing as mp
    import shard
    from sanity_checks import check_verdicts
    mp.spawn(_cl_rank_main, args=(WORLD, _free_port(), str(tmp_path)), nprocs=WORLD, join=True)
    rep = np.load(tmp_path / "cl_report.npz")
    r, traj = cpu_closed_loop(cl_inputs(CL_TOTAL), CL_STEPS)
    q = shard.closed_loop_quantities(r, 0, True, True, 550.0)
    assert int(rep["ranks"]) == WORLD
    assert np.array_equal(rep["q"], q, equal_nan=True)
    # histories: the first CL_HIST egos of each shard, in rank order
    keep = [e for rk in range(WORLD) for e in range(*shard.shard_range(CL_TOTAL, WORLD, rk))[:CL_HIST]]
    exp = np.concatenate([r["hist_x"][keep, 1:CL_STEPS + 1], r["hist_u"][keep, :CL_STEPS]], axis=2).astype(np.float32)
    assert np.array_equal(rep["hist"], exp, equal_nan=True)
    passed = sum(check_verdicts(dict(zip(shard.CL_FIELDS, row)), (-0.6, -5.0), (0.6, 4.0), traj.s_max)["passed"]
                 for row in q)
    assert int(rep["passed"]) == passed
    # the scenarios ran: the light switched for the egos starting before it, the car appeared for the others
    assert (r["hist_tl"][0::2] == 1).any(axis=1).all() and np.isfinite(r["hist_obs_s"][1::2]).any(axis=1).all()


def test_realtime_check_sees_the_slowest_step(capsys):
    """Both restatements of the real-time check (sanity_checks.py:133-139, max(hist_t) per step) must fail an
    ego whose run contains one 151 ms step, and pass an ego that left the loop before that step:
    trajectory_tracking.closed_loop_checks (run_simulation_batch) and shard.closed_loop_quantities +
    check_verdicts (the bench's gathered path)."""
    import shard
    import trajectory_tracking as TT
    from sanity_checks import check_verdicts
    r, traj = cpu_closed_loop(cl_inputs(2), 12)
    r["n_steps"] = np.array([12, 3], np.int32)      # ego 1 left the loop after 3 steps
    r["step_ms"] = np.ones(12)
    r["step_ms"][5] = 151.0                         # a step only ego 0 executed
    fsm = TT.ObstaclesFSM(True, True)
    capsys.readouterr()
    TT.closed_loop_checks(TT.TrajectoryTracker(traj), fsm, traj, r, verbose=True)
    blocks = capsys.readouterr().out.split("=== SANITY CHECKS ===")[1:]
    assert len(blocks) == 2
    assert "Real-time constraint respected : False --> Max CPU time 151.0ms > 150ms" in blocks[0]
    assert "Real-time constraint respected : True" in blocks[1]
    q = shard.closed_loop_quantities(r, 0, True, True, fsm.tl_pos)
    v = [check_verdicts(dict(zip(shard.CL_FIELDS, row)), (-0.6, -5.0), (0.6, 4.0), traj.s_max) for row in q]
    assert not v[0]["realtime"] and v[1]["realtime"]
    assert q[0, shard.CL_FIELDS.index("max_cpu_ms")] == 151.0


# ---------------------------------------------------------------------------------------------
# the GPU ranks' rendezvous: rank 0's RCCL unique id to every rank over TCP (shard.TcpStar)
# ---------------------------------------------------------------------------------------------
def _star_main(rank, world, port, outdir):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.join(os.path.dirname(here), "safe-autonomous-driving-mpc_amd")]
    import shard
    star = shard.TcpStar(world, rank, "127.0.0.1", port, timeout=60.0)
    uid = star.bcast(bytes(range(128)) if rank == 0 else b"")
    got = star.gather(bytes([rank]) * (rank + 1))
    star.barrier()
    star.close()
    np.savez(os.path.join(outdir, f"star{rank}.npz"), uid=np.frombuffer(uid, np.uint8),
             got=np.frombuffer(b"|".join(got), np.uint8) if got is not None else np.zeros(0, np.uint8))


def test_tcp_rendezvous_carries_the_unique_id(tmp_path):
    import torch.multiprocessing as mp
    world = 3
    mp.spawn(_star_main, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        z = np.load(tmp_path / f"star{r}.npz")
        assert bytes(z["uid"]) == bytes(range(128))
    assert bytes(np.load(tmp_path / "star0.npz")["got"]) == b"\x00|\x01\x01|\x02\x02\x02"


def test_gpu_transport_imports_no_torch():
    """The GPU ranks' path (shard.ShardComm.rccl -> mpcqp.Comm) needs no torch: importing shard and mpcqp and
    resolving every mpc_comm_* entry leaves torch unloaded."""
    import subprocess
    import sys
    code = ("import sys; sys.path[:0] = [%r]; import shard, mpcqp; L = mpcqp.lib(); "
            "[getattr(L, n) for n in mpcqp.EXPORTS if n.startswith(('mpc_comm', 'mpc_gather'))]; "
            "assert 'torch' not in sys.modules, 'torch imported'; print('ok')") % os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "safe-autonomous-driving-mpc_amd")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stderr[-2000:]
