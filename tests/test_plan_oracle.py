"""The offline planner's CPU oracle (oracle/plan_oracle.c, test infrastructure) against what pins it
(the reference module trajectory_planning.py is not importable, so the chunk solve is
"parity unpinned" against the reference's own outputs):
  - the route functions k_ref_fun / v_max_fun (trajectory_planning.py:437-477) against the reference's own
    scipy construction (routes.Route, scipy CubicSpline / interp1d);
  - the NLP functions against the numpy restatement (oracle/plan_ref.py) of :50-89, :128-170, :181-210;
  - the defect rule against the committed planner outputs (trajectories/*.json: v_{k+1} - v_k = +dt u2);
  - the chunk optimum against scipy SLSQP (the reference's solver) on the same restated NLP, tight;
  - the receding-horizon loop (package trajectory_planning.optimize_full_trajectory, :419-559) driven by the
    oracle on a route: the planned trajectory passes the restated reference_trajectory_check.
"""
import numpy as np
import pytest

from conftest import load_golden  # noqa: F401


@pytest.fixture(scope="module")
def env():
    import __graft_entry__ as g
    g.build()
    import plan_oracle as PO
    import plan_ref as PR
    import workloads as W
    return PO, PR, W


def test_route_functions_match_scipy(env):
    PO, PR, W = env
    for name in ("traj1", "synth1"):
        r = W.plan_route(name)
        orc = PO.PlanOracle(r)
        rng = np.random.default_rng(0)
        ss = np.concatenate([rng.uniform(0.0, r.s_total, 300), r.s[1:-1:7], [r.s_total, r.s_total + 3.0]])
        for s in ss:
            k, dk = orc.kappa(s)
            assert abs(k - r.k_ref_fun(s)) <= 1e-10 * (1 + abs(k)), (name, s)
            assert abs(dk - PR.dkappa(r, s)) <= 1e-7 * (1 + abs(dk)), (name, s)
            assert orc.vmax(s) == r.v_max_fun(s), (name, s)
        # below the first knot: the reference's interp1d('previous') gives NaN, the restatement the first limit
        assert np.isnan(r.v_max_fun(-1.0)) and orc.vmax(-1.0) == r.vmax[0]


def test_nlp_functions_match_numpy_restatement(env):
    PO, PR, W = env
    r = W.plan_route("traj2")
    orc = PO.PlanOracle(r)
    p = PO.default_params(N=10)
    rng = np.random.default_rng(1)
    for _ in range(50):
        xa = np.array([rng.uniform(5, r.s_total - 20), rng.normal(0, 0.3), rng.normal(0, 0.1), rng.normal(0, 0.2),
                       rng.uniform(0, 14)])
        xb = xa + np.array([rng.uniform(0, 4), *rng.normal(0, 0.05, 4)])
        u = rng.normal(0, 0.5, 2)
        ch = PR.Chunk(r, 1, 0.3, xa, xa[0] + 20, False)
        X = np.stack([xa, xb])
        assert np.abs(orc.defect(p, xa, xb, u) - ch.defect(X, u[None], 0)).max() <= 1e-12
        z = np.concatenate([X.ravel(), u, [0.05]])
        assert abs(orc.cost(p, 1, xa, X, u, np.array([0.05])) - ch.cost(z)) <= 1e-12 * (1 + abs(ch.cost(z)))


def test_defect_rule_of_the_committed_planner_outputs(env):
    """The k and v rows of the Hermite-Simpson defect are linear (k_dot = u1, v_dot = u2) and independent of
    the route: the committed planner outputs satisfy the forward rule x_{k+1} = x_k + dt/6 (...) to 1e-7
    (defect_sign = +1), and violate the committed source's literal sign (-1) by 2 dt |u|."""
    PO, PR, W = env
    r = W.plan_route("traj1")
    orc = PO.PlanOracle(r)
    for i in (1, 2, 3):
        X, U = W.loader(i).X_ref, W.loader(i).U_ref
        fwd = np.array([orc.defect(PO.default_params(), X[k], X[k + 1], U[k])[3:] for k in range(len(U))])
        bwd = np.array([orc.defect(PO.default_params(defect_sign=-1.0), X[k], X[k + 1], U[k])[3:] for k in range(len(U))])
        assert np.abs(fwd).max() <= 1e-7, i
        assert np.abs(bwd - 2 * 0.3 * U).max() <= 1e-7 and np.abs(bwd).max() > 1.0, i


@pytest.mark.parametrize("N,final", [(10, 0), (12, 1)])
def test_oracle_optimum_matches_slsqp(env, N, final):
    """Chunks the oracle solves (status ok) against scipy SLSQP on the restated NLP (analytic Jacobians,
    ftol 1e-14): the same point to 1e-6 when SLSQP converges from the reference's initial guess, and SLSQP
    started at the oracle's answer stays there (a KKT point of the reference's NLP)."""
    PO, PR, W = env
    r = W.plan_route("traj1")
    orc = PO.PlanOracle(r)
    wb = W.plan_batch(r, N, 6, seed=3, final_frac=float(final))
    o = orc.solve_batch(PO.default_params(N=N), wb["x0"], wb["s_target"], wb["is_final"])
    checked = 0
    for b in range(6):
        if o["status"][b] != 0:
            continue
        ch = PR.Chunk(r, N, 0.3, wb["x0"][b], wb["s_target"][b], bool(wb["is_final"][b]))
        z = np.concatenate([o["X"][b].ravel(), o["U"][b].ravel(), o["S"][b]])
        assert np.abs(ch.eq(z)).max() <= 1e-9 and ch.ineq(z).min() >= -1e-9
        rt, _ = ch.slsqp(ftol=1e-14, maxiter=400, jac=True, z0=z)
        assert np.abs(rt.x - z).max() <= 1e-6, (b, np.abs(rt.x - z).max())
        assert rt.fun >= ch.cost(z) - 1e-8
        checked += 1
        if checked == 3:
            break
    assert checked >= 2


def _slsqp_from(job):
    """Worker of test_oracle_optimum_matches_slsqp_bench_mix: SLSQP (analytic Jacobians, ftol 1e-14) on the
    restated chunk NLP started at the oracle's answer z; returns (max |x - z|, SLSQP cost, cost at z, max |eq|,
    min ineq)."""
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "safe-autonomous-driving-mpc_amd"), os.path.join(root, "oracle")]
    import plan_ref as PR
    import workloads as W
    route, n, x0, st, fin, z = job
    ch = PR.Chunk(W.plan_route(route), n, 0.3, x0, st, fin)
    rt, _ = ch.slsqp(ftol=1e-14, maxiter=400, jac=True, z0=z)
    return float(np.abs(rt.x - z).max()), float(rt.fun), float(ch.cost(z)), float(np.abs(ch.eq(z)).max()), \
        float(ch.ineq(z).min())


def test_oracle_optimum_matches_slsqp_bench_mix(env, capsys):
    """The same check over the chunks bench.py's planner leg solves (workloads.plan_batch_ref on traj3: 20 m
    chunks with the reference's horizon rule, N = 13..17, final chunks N = 25..32): for every horizon, four
    chunks the oracle solves to convergence are KKT points of the restated NLP that scipy SLSQP (analytic
    Jacobians, ftol 1e-14) started there does not leave (1e-6), at no lower cost.  (8 worker processes: the
    N = 32 problems take ~10 s each.)"""
    import multiprocessing as mp
    from concurrent.futures import ProcessPoolExecutor
    PO, PR, W = env
    r = W.plan_route("traj3")
    orc = PO.PlanOracle(r)
    wb = W.plan_batch_ref(r, 2048, seed=7)
    o = orc.solve_batch(PO.default_params(N=int(wb["N"].max())), wb["x0"], wb["s_target"], wb["is_final"], N=wb["N"],
                        num_threads=8)
    per_n, jobs = {}, []
    for b in range(len(wb["N"])):
        n = int(wb["N"][b])
        if o["status"][b] != 0 or per_n.get(n, 0) >= 4:
            continue
        z = np.concatenate([o["X"][b][:n + 1].ravel(), o["U"][b][:n].ravel(), o["S"][b][:n]])
        jobs.append(("traj3", n, wb["x0"][b], float(wb["s_target"][b]), bool(wb["is_final"][b]), z))
        per_n[n] = per_n.get(n, 0) + 1
    with ProcessPoolExecutor(8, mp_context=mp.get_context("spawn")) as ex:
        res = list(ex.map(_slsqp_from, jobs))
    worst = 0.0
    for job, (d, fun, cost, eq, ineq) in zip(jobs, res):
        assert eq <= 1e-9 and ineq >= -1e-9, job[:2]
        assert d <= 1e-6, (job[:2], d)
        assert fun >= cost - 1e-8, job[:2]
        worst = max(worst, d)
    finals = sorted({int(n) for n, f in zip(wb["N"], wb["is_final"]) if f})
    with capsys.disabled():
        print(f"\nbench mix: horizons {sorted(per_n)} (final-chunk horizons {finals}), chunks checked {len(jobs)}, "
              f"largest SLSQP move {worst:.1e}")
    assert all(per_n.get(n, 0) >= 4 for n in set(int(x) for x in wb["N"])), per_n
    assert set(range(13, 18)) <= set(per_n) and set(range(25, 33)) <= set(per_n)


def test_receding_horizon_loop_with_oracle_passes_check(env, capsys):
    """optimize_full_trajectory (:419-559) with the oracle as the chunk solver on a synthetic route: the planned
    trajectory reaches the destination, stops, and passes the restated reference_trajectory_check."""
    PO, PR, W = env
    import sanity_checks as SC
    import trajectory_planning as TP
    r = W.plan_route("synth1")
    orc = PO.PlanOracle(r)

    def solve_chunk(x0, st, fin, N):
        o = orc.solve_batch(PO.default_params(N=N), np.asarray(x0)[None], st, int(fin))
        return o["X"][0], o["U"][0], o["S"][0], o["status"][0]

    X, U, S = TP.optimize_full_trajectory(r, solve_chunk=solve_chunk)
    out = capsys.readouterr().out
    q = SC.plan_check_summary(np.array([-0.6, -5.0]), np.array([0.6, 4.0]), X, U, S, r.s_total)
    st = np.array(TP.optimize_full_trajectory.statuses)
    print(f"{len(st)} chunks, statuses {np.bincount(st, minlength=5).tolist()}, final s {X[-1, 0]:.3f} / "
          f"{r.s_total:.3f}, v_end {X[-1, 4]:.2e}")
    assert "===> Checks passed : True" in out, out
    assert q["passed"] and abs(X[-1, 0] - r.s_total) < 1e-6 and abs(X[-1, 4]) < 1e-9
    assert np.isin(st, (0, 4)).mean() >= 0.9


def test_batched_receding_loop_equals_the_single_loop(env, capsys):
    """optimize_full_trajectory_batch: B plans on one route advance together, one batched chunk solve per
    round with per-chunk horizons.  With the oracle as the batch solver, a plan from the reference's start
    equals optimize_full_trajectory's plan exactly, and plans from other starts on the route reach the
    destination and pass the restated checks."""
    PO, PR, W = env
    import trajectory_planning as TP
    r = W.plan_route("synth1")
    orc = PO.PlanOracle(r)

    def solve_chunk(x0, st, fin, N):
        o = orc.solve_batch(PO.default_params(N=N), np.asarray(x0)[None], st, int(fin))
        return o["X"][0], o["U"][0], o["S"][0], o["status"][0]

    def solve_chunks(x0, st, fin, N):
        return orc.solve_batch(PO.default_params(N=int(N.max())), x0, st, fin, N=N, num_threads=8)

    X1, U1, S1 = TP.optimize_full_trajectory(r, solve_chunk=solve_chunk, check=False)
    starts = np.zeros((3, 5))
    for b, s0 in ((1, 400.0), (2, 1100.0)):
        starts[b] = (s0, 0.02, 0.0, r.k_ref_fun(s0), 0.6 * r.v_max_fun(s0))
    plans, summary = TP.optimize_full_trajectory_batch(r, starts, solve_chunks=solve_chunks)
    X, U, S = plans[0]
    assert np.array_equal(X, X1) and np.array_equal(U, U1) and np.array_equal(S, S1)
    assert summary[0]["statuses"] == TP.optimize_full_trajectory.statuses
    for b in range(3):
        assert summary[b]["passed"], (b, summary[b])
        assert abs(plans[b][0][-1, 0] - r.s_total) < 1e-6
    print("batched plans: chunks", [len(q["statuses"]) for q in summary])
