"""The offline planner on the GPU (libmpcplan) against the CPU oracle (oracle/plan_oracle.c),
through the C ABI.  Parity with the reference's own chunk solve is unpinned (trajectory_planning.py is not
importable here); the oracle is pinned by tests/test_plan_oracle.py (scipy SLSQP on the restated NLP, the
committed planner outputs, the reference_trajectory_check goldens).

Tolerances: chunks that both sides solve to convergence (status ok / frozen limits) agree to 1e-8 abs on
X, U, S (both converge to the same KKT point to sqp_tol 1e-9; measured <= 8e-13); statuses agree on >= 99% of
the chunks (measured 0.996-1.000), and both sides converge on >= 95% of the chunks whose QP is not infeasible
(the oracle's PLAN_QP_FAILED: e.g. 15 of the 256 traj1 N = 10 chunks start with a curvature outside the
k bounds that 3 s cannot undo, or must stop within the horizon).
"""
import os

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

TOL = 1e-8


@pytest.fixture(scope="module")
def env():
    import __graft_entry__ as g
    g.build()
    import mpcplan
    import plan_oracle as PO
    import workloads as W
    return mpcplan, PO, W


def test_route_eval_matches_oracle(env):
    mpcplan, PO, W = env
    for name in ("traj1", "synth1"):
        r = W.plan_route(name)
        pl = mpcplan.Planner(r)
        orc = PO.PlanOracle(r)
        s = np.concatenate([np.linspace(-2.0, r.s_total + 2.0, 997), r.s])
        k, dk, vm = pl.route_eval(s)
        ko = np.array([orc.kappa(x) for x in s])
        assert np.abs(k - ko[:, 0]).max() <= 1e-12 * (1 + np.abs(ko[:, 0]).max())
        assert np.abs(dk - ko[:, 1]).max() <= 1e-9 * (1 + np.abs(ko[:, 1]).max())
        assert np.array_equal(vm, np.array([orc.vmax(x) for x in s]))
        pl.close()


def compare(label, r, ro):
    both = np.isin(r["status"], (0, 4)) & np.isin(ro["status"], (0, 4))
    agree = float((r["status"] == ro["status"]).mean())
    err = np.array([max(np.abs(r[k][b] - ro[k][b]).max() for k in ("X", "U", "S")) for b in range(len(both))])
    print(f"{label}: B={len(both)} status agree {agree:.3f}, both converged {both.sum()}, max err {err[both].max():.1e}, "
          f"GPU statuses {np.bincount(r['status'], minlength=5).tolist()}, oracle {np.bincount(ro['status'], minlength=5).tolist()}, "
          f"sqp mean {r['sqp'].mean():.1f} max {r['sqp'].max()}")
    assert agree >= 0.99, label
    assert err[both].max() <= TOL, (label, np.flatnonzero(both & (err > TOL)))
    feasible = ro["status"] != 2
    assert both.sum() >= 0.95 * feasible.sum(), (label, int(both.sum()), int(feasible.sum()))
    return both


@pytest.mark.parametrize("N,route", [(10, "traj1"), (20, "traj2"), (20, "synth1"), (40, "synth2")])
def test_chunks_vs_oracle(env, N, route):
    """>= 256 chunks per horizon N in {10, 20, 40}, a quarter of them final chunks (terminal equalities)."""
    mpcplan, PO, W = env
    r = W.plan_route(route)
    wb = W.plan_batch(r, N, 256, seed=N, final_frac=0.25)
    pl = mpcplan.Planner(r, mpcplan.default_params(N=N))
    g = pl.solve_chunks(wb["x0"], wb["s_target"], wb["is_final"])
    o = PO.PlanOracle(r).solve_batch(PO.default_params(N=N), wb["x0"], wb["s_target"], wb["is_final"], num_threads=16)
    compare(f"N={N} {route}", g, o)
    pl.close()


def test_mixed_horizons_one_launch(env):
    """Per-chunk N (the receding-horizon loop's chunks differ in N): one launch over N in {8, 16, 24}; rows past a
    chunk's N are zero, and each chunk equals its own solve at that N."""
    mpcplan, PO, W = env
    r = W.plan_route("synth1")
    parts = [W.plan_batch(r, n, 40, seed=7 + n, final_frac=0.2) for n in (8, 16, 24)]
    x0 = np.concatenate([p["x0"] for p in parts]); st = np.concatenate([p["s_target"] for p in parts])
    fin = np.concatenate([p["is_final"] for p in parts]); N = np.repeat([8, 16, 24], 40).astype(np.int32)
    pl = mpcplan.Planner(r)
    g = pl.solve_chunks(x0, st, fin, N)
    assert g["X"].shape == (120, 25, 5)
    for i, n in enumerate((8, 16, 24)):
        sl = slice(40 * i, 40 * i + 40)
        assert (g["X"][sl, n + 1:] == 0).all() and (g["U"][sl, n:] == 0).all()
        pl.set_params(mpcplan.default_params(N=n))
        one = pl.solve_chunks(x0[sl], st[sl], fin[sl])
        assert np.array_equal(one["X"], g["X"][sl, :n + 1]) and np.array_equal(one["status"], g["status"][sl])
    pl.close()


def test_device_entry_equals_host_entry(env):
    import torch
    mpcplan, PO, W = env
    r = W.plan_route("traj3")
    wb = W.plan_batch(r, 16, 100, seed=11, final_frac=0.3)
    pl = mpcplan.Planner(r, mpcplan.default_params(N=16))
    h = pl.solve_chunks(wb["x0"], wb["s_target"], wb["is_final"])
    dev = torch.device("cuda", 0)
    t = lambda a, dt=torch.float64: torch.as_tensor(a, dtype=dt, device=dev).contiguous()
    x0, st, fin = t(wb["x0"]), t(wb["s_target"]), t(wb["is_final"], torch.int32)
    B = 100
    X = torch.empty((B, 17, 5), dtype=torch.float64, device=dev)
    U = torch.empty((B, 16, 2), dtype=torch.float64, device=dev)
    S = torch.empty((B, 16), dtype=torch.float64, device=dev)
    o = [torch.empty(B, dtype=torch.int32, device=dev) for _ in range(3)]
    stream = torch.cuda.current_stream(dev)
    pl.solve_chunks_device(B, 16, 0, x0.data_ptr(), st.data_ptr(), fin.data_ptr(), X.data_ptr(), U.data_ptr(),
                           S.data_ptr(), *[a.data_ptr() for a in o], stream=stream.cuda_stream)
    torch.cuda.synchronize(dev)
    assert np.array_equal(X.cpu().numpy(), h["X"]) and np.array_equal(U.cpu().numpy(), h["U"])
    assert np.array_equal(o[0].cpu().numpy(), h["status"]) and np.array_equal(o[2].cpu().numpy(), h["sqp"])
    pl.close()


def test_full_trajectory_on_gpu_passes_reference_check(env, capsys):
    """optimize_full_trajectory (trajectory_planning.py:419-559) with every chunk solved on the GPU: the plan
    reaches the destination, stops, and passes the restated reference_trajectory_check (sanity_checks.py:3-75)."""
    mpcplan, PO, W = env
    import sanity_checks as SC
    import trajectory_planning as TP
    for name in ("synth1", "traj1"):
        r = W.plan_route(name)
        X, U, S = TP.optimize_full_trajectory(r)
        out = capsys.readouterr().out
        st = np.array(TP.optimize_full_trajectory.statuses)
        q = SC.plan_check_summary(np.array([-0.6, -5.0]), np.array([0.6, 4.0]), X, U, S, r.s_total)
        print(f"{name}: {len(st)} chunks, N {min(TP.optimize_full_trajectory.horizons)}-"
              f"{max(TP.optimize_full_trajectory.horizons)}, statuses {np.bincount(st, minlength=5).tolist()}, "
              f"{'passed' if q['passed'] else 'FAILED'}")
        assert "===> Checks passed : True" in out, out
        assert q["passed"] and np.isin(st, (0, 4)).mean() >= 0.9


@pytest.mark.parametrize("N", [1, 2, 48, 64])
def test_horizon_extremes_vs_oracle(env, N):
    """The smallest horizons and the largest (PLAN_MAX_N = 64: ~155 KB of LDS per chunk, above the 64 KB
    default, which plan_solve_chunks_device raises with hipFuncSetAttribute): statuses and, on chunks both
    call converged, plans equal to the oracle's within 1e-8."""
    mpcplan, PO, W = env
    r = W.plan_route("synth2")
    wb = W.plan_batch(r, N, 24, seed=100 + N, final_frac=0.25)
    pl = mpcplan.Planner(r, mpcplan.default_params(N=N))
    g = pl.solve_chunks(wb["x0"], wb["s_target"], wb["is_final"])
    pl.close()
    o = PO.PlanOracle(r).solve_batch(PO.default_params(N=N), wb["x0"], wb["s_target"], wb["is_final"], num_threads=16)
    agree = float((g["status"] == o["status"]).mean())
    both = np.isin(g["status"], (0, 4)) & np.isin(o["status"], (0, 4))
    err = max((float(np.abs(g[k][both] - o[k][both]).max()) for k in ("X", "U", "S")), default=0.0) if both.any() else 0.0
    print(f"N={N}: status agree {agree:.3f}, both converged {int(both.sum())}/24, max err {err:.1e}, "
          f"GPU statuses {np.bincount(g['status'], minlength=5).tolist()}")
    assert agree >= 0.99
    if N > 1:         # N = 1 (0.3 s for a 20 m chunk) converges on neither side: statuses agree, plans unchecked
        assert both.sum() >= 0.95 * (o["status"] != 2).sum()
    assert err <= TOL
    assert np.isfinite(g["X"]).all()


def test_device_horizon_out_of_range_is_flagged(env):
    """Per-chunk horizons come from device memory unchecked by the host: a chunk with N[b] = 0 or N[b] > Nmax
    is not solved (zero plan, PLAN_NUMERICAL) and its neighbours are unaffected."""
    import torch
    mpcplan, PO, W = env
    r = W.plan_route("synth1")
    wb = W.plan_batch(r, 12, 6, seed=5)
    pl = mpcplan.Planner(r, mpcplan.default_params(N=12))
    h = pl.solve_chunks(wb["x0"], wb["s_target"], wb["is_final"])
    dev = torch.device("cuda", 0)
    t = lambda a, dt=torch.float64: torch.as_tensor(a, dtype=dt, device=dev).contiguous()
    Nv = t(np.array([12, 0, 12, 13, 12, -3], np.int32), torch.int32)
    x0, st, fin = t(wb["x0"]), t(wb["s_target"]), t(wb["is_final"], torch.int32)
    X = torch.full((6, 13, 5), 7.0, dtype=torch.float64, device=dev)
    o = [torch.full((6,), -1, dtype=torch.int32, device=dev) for _ in range(3)]
    pl.solve_chunks_device(6, 12, Nv.data_ptr(), x0.data_ptr(), st.data_ptr(), fin.data_ptr(), X.data_ptr(), 0, 0,
                           *[a.data_ptr() for a in o], stream=torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize(dev)
    Xh, sth = X.cpu().numpy(), o[0].cpu().numpy()
    for b in (1, 3, 5):
        assert sth[b] == mpcplan.PLAN_NUMERICAL and (Xh[b] == 0).all()
    for b in (0, 2, 4):
        assert sth[b] == h["status"][b] and np.array_equal(Xh[b], h["X"][b])
    pl.close()


def test_batched_receding_loop_on_gpu(env, capsys):
    """optimize_full_trajectory_batch on the GPU: 48 plans on trajectory1's route from starts spread along it
    (the first at the reference's start) advance together, one launch per round; the first plan equals the
    single-route loop's, and the plans reach the destination and pass the restated checks."""
    mpcplan, PO, W = env
    import trajectory_planning as TP
    r = W.plan_route("traj1")
    X1, U1, S1 = TP.optimize_full_trajectory(r, check=False)
    rng = np.random.default_rng(4)
    starts = np.zeros((48, 5))
    for b in range(1, 48):
        s0 = rng.uniform(1.0, r.s_total - 30.0)
        starts[b] = (s0, rng.normal(0, 0.05), rng.normal(0, 0.01), r.k_ref_fun(s0), rng.uniform(0.2, 0.9) * r.v_max_fun(s0))
    plans, summary = TP.optimize_full_trajectory_batch(r, starts)
    assert np.array_equal(plans[0][0], X1) and np.array_equal(plans[0][1], U1)
    passed = np.array([q["passed"] for q in summary])
    print(f"batched GPU plans: {passed.sum()}/48 pass the checks, chunks per plan "
          f"{min(len(q['statuses']) for q in summary)}-{max(len(q['statuses']) for q in summary)}")
    assert passed.mean() >= 0.9
    assert all(abs(p[0][-1, 0] - r.s_total) < 1e-3 for p in plans)


@pytest.mark.gpu
def test_device_loop_equals_round_loop(env, capsys):
    """plan_optimize_device (each plan's chunk loop on its own wavefront) gives the round-by-round host loop's
    plans bit for bit: the same chunk solver on the same chunk inputs (start, target, final flag, N).  Also with
    the loop cut into launches of 2 chunks (plans continue from their last start), and max_chunks honoured."""
    mpcplan, PO, W = env
    import trajectory_planning as TP
    r = W.plan_route("traj1")
    rng = np.random.default_rng(11)
    starts = np.zeros((40, 5))
    for b in range(1, 40):
        s0 = rng.uniform(1.0, r.s_total - 30.0)
        starts[b] = (s0, rng.normal(0, 0.05), rng.normal(0, 0.01), r.k_ref_fun(s0), rng.uniform(0.2, 0.9) * r.v_max_fun(s0))
    starts[1, 0] = -12.0                 # before the route: vmax[int(s / 5):] counts from the end, as in Python
    starts[2, 0] = -5.0 * len(r.vmax) - 10.0    # int(s / 5) before -len: the whole array, avg[0]
    starts[3, 0] = r.s_total - 0.05      # already there: no chunk
    pd, sd = TP.optimize_full_trajectory_batch(r, starts, device_loop=True)
    assert sd[3]["statuses"] == []
    ph, sh = TP.optimize_full_trajectory_batch(r, starts, device_loop=False)
    for b in range(40):
        assert sd[b]["statuses"] == sh[b]["statuses"] and sd[b]["horizons"] == sh[b]["horizons"]
        for i in range(3):
            assert np.array_equal(pd[b][i], ph[b][i]), (b, i)
    # launches of 2 chunks each
    opt = TP.TrajectoryOptimizer()
    pieces, st, hz = [[] for _ in range(40)], [[] for _ in range(40)], [[] for _ in range(40)]
    TP._device_loop(r, starts, 20, 10000, 0, pieces, st, hz, opt, seg=2)
    for b in range(40):
        assert st[b] == sd[b]["statuses"] and hz[b] == sd[b]["horizons"]
        if pieces[b]:
            assert np.array_equal(np.concatenate([p[0] for p in pieces[b]]), pd[b][0])
    # max_chunks caps every plan, as in the host loop
    pc, sc = TP.optimize_full_trajectory_batch(r, starts, max_chunks=3)
    pc2, sc2 = TP.optimize_full_trajectory_batch(r, starts, max_chunks=3, device_loop=False)
    assert all(len(q["statuses"]) <= 3 for q in sc)
    for b in range(40):
        assert np.array_equal(pc[b][0], pc2[b][0])
    with capsys.disabled():
        print(f"\ndevice loop = round loop on 40 plans, chunks per plan "
              f"{min(len(q['statuses']) for q in sd)}-{max(len(q['statuses']) for q in sd)}")


def test_longest_first_order_changes_nothing(env, monkeypatch):
    """plan_solve_chunks_device dispatches the chunks by a route-curvature score, highest first (plan_order_*_
    kernel, a scheduling hint): every chunk's plan, status and counts equal the index-order launch's bit for bit
    (PLAN_ORDER=0 at plan_create), including batches on two streams of one context at once."""
    import torch
    mpcplan, PO, W = env
    r = W.plan_route("traj3")
    wb = W.plan_batch(r, 14, 2048, seed=21, final_frac=0.1)
    dev = torch.device("cuda", 0)
    t = lambda a, dt=torch.float64: torch.as_tensor(a, dtype=dt, device=dev).contiguous()
    x0, st, fin = t(wb["x0"]), t(wb["s_target"]), t(wb["is_final"], torch.int32)
    B = 2048

    def run(pl, stream):
        X = torch.empty((B, 15, 5), dtype=torch.float64, device=dev)
        o = [torch.empty(B, dtype=torch.int32, device=dev) for _ in range(3)]
        pl.solve_chunks_device(B, 14, 0, x0.data_ptr(), st.data_ptr(), fin.data_ptr(), X.data_ptr(), 0, 0,
                               *[a.data_ptr() for a in o], stream=stream.cuda_stream)
        return X, o
    monkeypatch.setenv("PLAN_ORDER", "0")
    plain = mpcplan.Planner(r, mpcplan.default_params(N=14))
    monkeypatch.setenv("PLAN_ORDER", "1")
    ordered = mpcplan.Planner(r, mpcplan.default_params(N=14))
    s0, s1 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    s0.wait_stream(torch.cuda.current_stream(dev))
    s1.wait_stream(torch.cuda.current_stream(dev))
    Xa, oa = run(plain, s0)
    Xb, ob = run(ordered, s0)
    Xc, oc = run(ordered, s1)          # the same context on a second stream at the same time
    torch.cuda.synchronize(dev)
    for Xo, oo in ((Xb, ob), (Xc, oc)):
        assert torch.equal(Xo, Xa)
        for a, b in zip(oo, oa):
            assert torch.equal(a, b)
    print(f"\nordered dispatch == index order on {B} traj3 chunks; statuses "
          f"{np.bincount(oa[0].cpu().numpy(), minlength=5).tolist()}")
    plain.close()
    ordered.close()


def test_graph_capture_after_eager_warmup(env):
    """an eager call on a stream (which takes a longest-first order buffer), then the same call
    captured into a HIP graph on that stream and replayed, interleaved with eager calls on the same context:
    the captured call must not use the pool (index order), so replays and eager calls never rewrite each
    other's order[]; every replay and every eager call equals the index-order result bit for bit."""
    import torch
    mpcplan, PO, W = env
    r = W.plan_route("traj3")
    B = 1024
    wb = W.plan_batch(r, 14, B, seed=41, final_frac=0.1)
    dev = torch.device("cuda", 0)
    t = lambda a, dt=torch.float64: torch.as_tensor(a, dtype=dt, device=dev).contiguous()
    x0, st, fin = t(wb["x0"]), t(wb["s_target"]), t(wb["is_final"], torch.int32)
    ref = mpcplan.Planner(r, mpcplan.default_params(N=14)).solve_chunks(wb["x0"], wb["s_target"], wb["is_final"])
    pl = mpcplan.Planner(r, mpcplan.default_params(N=14))
    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))

    def outputs():
        return torch.empty((B, 15, 5), dtype=torch.float64, device=dev), [torch.empty(B, dtype=torch.int32, device=dev)
                                                                          for _ in range(3)]

    def call(X, o, stream):
        pl.solve_chunks_device(B, 14, 0, x0.data_ptr(), st.data_ptr(), fin.data_ptr(), X.data_ptr(), 0, 0,
                               *[a.data_ptr() for a in o], stream=stream)

    def check(X, o, what):
        assert np.array_equal(X.cpu().numpy(), ref["X"]), what
        assert np.array_equal(o[0].cpu().numpy(), ref["status"]) and np.array_equal(o[2].cpu().numpy(), ref["sqp"]), what

    Xe, oe = outputs()
    with torch.cuda.stream(side):
        call(Xe, oe, side.cuda_stream)                    # eager warm-up: the side stream gets a pool buffer
    torch.cuda.synchronize(dev)
    check(Xe, oe, "eager")
    Xg, og = outputs()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        call(Xg, og, torch.cuda.current_stream(dev).cuda_stream)
    for k in range(3):
        Xg.zero_()
        g.replay()
        Xe2, oe2 = outputs()
        call(Xe2, oe2, side.cuda_stream)                  # an eager call right behind the replay
        torch.cuda.synchronize(dev)
        check(Xg, og, f"replay {k}")
        check(Xe2, oe2, f"eager after replay {k}")
    pl.close()


def test_order_pool_reuse_across_many_streams(env):
    """More concurrent streams than the pool holds (8): buffers are reused least recently used, each only after
    the kernel that last read it has finished; every launch equals the index-order result."""
    import torch
    mpcplan, PO, W = env
    r = W.plan_route("traj3")
    B = 512
    wb = W.plan_batch(r, 12, B, seed=43, final_frac=0.1)
    dev = torch.device("cuda", 0)
    t = lambda a, dt=torch.float64: torch.as_tensor(a, dtype=dt, device=dev).contiguous()
    x0, st, fin = t(wb["x0"]), t(wb["s_target"]), t(wb["is_final"], torch.int32)
    ref = mpcplan.Planner(r, mpcplan.default_params(N=12)).solve_chunks(wb["x0"], wb["s_target"], wb["is_final"])
    pl = mpcplan.Planner(r, mpcplan.default_params(N=12))
    streams = [torch.cuda.Stream(dev) for _ in range(12)]
    outs = []
    for rep in range(2):
        for s in streams:
            s.wait_stream(torch.cuda.current_stream(dev))
            X = torch.empty((B, 13, 5), dtype=torch.float64, device=dev)
            o = [torch.empty(B, dtype=torch.int32, device=dev) for _ in range(3)]
            pl.solve_chunks_device(B, 12, 0, x0.data_ptr(), st.data_ptr(), fin.data_ptr(), X.data_ptr(), 0, 0,
                                   *[a.data_ptr() for a in o], stream=s.cuda_stream)
            outs.append((X, o))
    torch.cuda.synchronize(dev)
    for X, o in outs:
        assert np.array_equal(X.cpu().numpy(), ref["X"]) and np.array_equal(o[0].cpu().numpy(), ref["status"])
    pl.close()


def test_residency_groups(env):
    """plan_chunks_per_cu is non-increasing in Nmax and at least 1 up to PLAN_MAX_N; Planner.horizon_groups
    puts each horizon in one launch whose residency equals its own launch's; the grouped launches (per-chunk N,
    LDS sized for the group's largest horizon) give each chunk's plan bit for bit as one launch per horizon."""
    mpcplan, PO, W = env
    r = W.plan_route("traj3")
    pl = mpcplan.Planner(r, mpcplan.default_params(N=16))
    occ = [pl.chunks_per_cu(n) for n in range(1, mpcplan.PLAN_MAX_N + 1)]
    assert min(occ) >= 1 and all(a >= b for a, b in zip(occ, occ[1:])), occ
    hs = [13, 14, 16, 17, 25, 28, 32]
    groups = pl.horizon_groups(hs)
    assert sorted(n for n in hs if any(lo <= n <= hi for lo, hi in groups)) == hs
    for lo, hi in groups:
        for n in hs:
            if lo <= n <= hi:
                assert pl.chunks_per_cu(n) == pl.chunks_per_cu(hi)
    parts = {n: W.plan_batch(r, n, 24, seed=30 + n, final_frac=0.2) for n in hs}
    for lo, hi in groups:
        mem = [n for n in hs if lo <= n <= hi]
        x0 = np.concatenate([parts[n]["x0"] for n in mem]); st = np.concatenate([parts[n]["s_target"] for n in mem])
        fin = np.concatenate([parts[n]["is_final"] for n in mem]); N = np.repeat(mem, 24).astype(np.int32)
        g = pl.solve_chunks(x0, st, fin, N)
        for i, n in enumerate(mem):
            pl.set_params(mpcplan.default_params(N=n))
            one = pl.solve_chunks(parts[n]["x0"], parts[n]["s_target"], parts[n]["is_final"])
            sl = slice(24 * i, 24 * i + 24)
            assert np.array_equal(one["X"], g["X"][sl, :n + 1]) and np.array_equal(one["status"], g["status"][sl])
    print(f"\nchunks per CU by Nmax: {dict(zip(range(1, 65), occ))}; groups of {hs}: {groups}")
    pl.close()


def test_device_loop_needs_no_torch(env):
    """The device chunk loop (plan_optimize, host buffers) runs in a fresh process that never imports torch:
    the planner's HIP runtime is the only one initialised there, and the plans equal the round loop's."""
    import subprocess
    import sys
    code = (
        "import sys, numpy as np\n"
        f"sys.path[:0] = [{os.path.join(ROOT, 'safe-autonomous-driving-mpc_amd')!r}, {ROOT!r}]\n"
        "import workloads as W, trajectory_planning as TP\n"
        "r = W.plan_route('traj1')\n"
        "starts = np.zeros((4, 5)); starts[1:, 0] = [40.0, 120.0, 200.0]; starts[1:, 4] = 5.0\n"
        "pd, sd = TP.optimize_full_trajectory_batch(r, starts)\n"
        "ph, sh = TP.optimize_full_trajectory_batch(r, starts, device_loop=False)\n"
        "assert all(np.array_equal(a[0], b[0]) for a, b in zip(pd, ph))\n"
        "assert 'torch' not in sys.modules, 'torch was imported'\n"
        "print('ok', [len(q['statuses']) for q in sd])\n")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.startswith("ok")
