"""The SQP path pinned to the reference's nonlinear problem, on the CPU oracle.

tests/golden/nlp_golden.npz (make_goldens.gen_nlp) holds, for 60 instances of the C1-C5 shapes and the
reference default N=5, the optimum of the reference's own cost/constraints (trajectory_tracking.py:116-211)
from the reference warm start: SLSQP at ftol 1e-12 / maxiter 1000, continued with
central-FD derivatives of the same functions and a golden-side FD-SQP, and certified by a KKT check of
the reference functions (`certified`: feasible and within ~1e-6 of the local optimum).

The build's Gauss-Newton SQP (sqp_iters QPs, each re-linearised about the previous solution, stopping at
sqp_tol) is a different algorithm with the same fixed points: on every certified case it must land on the
golden optimum within the BASELINE 1e-5 gate (measured: <= 1e-7).  The closed-loop test replays the
reference's trajectory2 FSM run (closedloop_golden) with the oracle's SQP in the shim's run_simulation.
"""
import json

import numpy as np
import pytest

from conftest import golden_cases, traj_arrays

TOL_NLP = 1e-5        # BASELINE.json gate, now against the reference NLP optimum
TOL_NLP_MEAS = 2e-7   # what the SQP reaches (golden certificate floor ~1e-8..6e-8 on the obstacle cases)


def nlp_cases():
    cases, _ = golden_cases("nlp_golden")
    return cases


def sqp_errors(oracles, c, Ks):
    import oracle as O
    orc = oracles[int(c["traj"])]
    ob = c["obs"]
    out = []
    for K in Ks:
        p = O.default_params(N=int(c["N"]), max_obs=len(ob), sqp_iters=K)
        r = orc.solve(p, c["x0"], ob if len(ob) else None)
        out.append((float(np.abs(r["U"] - c["U_nlp"]).max()), r))
    return out


def test_nlp_golden_coverage():
    cases = nlp_cases()
    assert len(cases) >= 60
    shapes = {(int(c["traj"]), int(c["N"])) for c in cases}
    assert {(1, 10), (1, 20), (2, 20), (3, 30), (3, 40), (2, 5)} <= shapes
    cert = [c for c in cases if bool(c["certified"])]
    assert len(cert) >= 45
    # every shape has certified cases, obstacle shapes included
    assert {(int(c["traj"]), int(c["N"])) for c in cert} == shapes
    for c in cert:
        k = json.loads(str(c["kkt"]))
        assert k["prim"] <= 1e-9 and k["err_est"] <= 1e-6


MAX_OTHER_OPTIMA = 1   # certified cases where the SQP may converge to a different local optimum (case 34)


def classify(U, U_cap_more, c, feasible_fn):
    """'nlp' when U is the golden optimum (TOL_NLP_MEAS); 'other' when U is a different converged local
    optimum of the same problem: the SQP stopped moving (more iterations change nothing) and U satisfies the
    reference constraints; else 'bad'."""
    e = float(np.abs(U.ravel() - c["U_nlp"]).max())
    if e <= TOL_NLP_MEAS:
        return "nlp", e
    if np.array_equal(U, U_cap_more) and feasible_fn(U) >= -1e-9:
        return "other", e
    return "bad", e


def test_oracle_sqp_reaches_reference_nlp_optimum(oracles):
    """Default drop-in SQP (trajectory_tracking.SQP_ITERS QPs at most, sqp_tol 1e-10) vs the certified
    golden optimum; also reports the error after K = 1..4 QPs (K = 1 is the single tracking QP).  The
    reference problem is not convex: from the same warm start a local solver may settle in a different
    local optimum than SLSQP's path did; that is allowed for at most MAX_OTHER_OPTIMA cases, each a
    converged, feasible KKT point (the SQP's fixed points are the problem's KKT points)."""
    import oracle as O
    import trajectory_tracking as TT
    worst, rows, other = 0.0, [], []
    for j, c in enumerate(nlp_cases()):
        if not bool(c["certified"]):
            continue
        errs = sqp_errors(oracles, c, (1, 2, 3, 4, TT.SQP_ITERS, TT.SQP_ITERS + 20))
        orc, ob = oracles[int(c["traj"])], c["obs"]
        p = O.default_params(N=int(c["N"]), max_obs=len(ob))
        kind, e = classify(errs[-2][1]["U"], errs[-1][1]["U"], c,
                           lambda U: orc.constraints(p, c["x0"], ob if len(ob) else None, U.ravel()).min())
        rows.append((j, int(c["traj"]), int(c["N"]), len(ob), kind, [f"{x[0]:.1e}" for x in errs[:-1]]))
        assert kind != "bad", (j, e)
        assert e <= TOL_NLP or kind == "other", (j, e)
        if kind == "nlp":
            worst = max(worst, e)
            assert errs[-2][1]["status"] == 0
        else:
            other.append(j)
    for r in rows:
        print("case %d traj%d N=%d obs=%d %s  |U-U_nlp| after K=1,2,3,4,cap: %s" % r)
    print(f"worst |U_sqp - U_nlp| over {len(rows) - len(other)} certified cases: {worst:.2e}; "
          f"other local optima: {other}")
    assert len(other) <= MAX_OTHER_OPTIMA


def test_certified_optimum_is_no_worse_than_appendix_c_slsqp(oracles):
    """SURVEY App. C's stage-1 point (SLSQP, ftol 1e-12, 2-point FD derivatives) is not a precise pin: its
    distance to the certified optimum spans 2e-7 .. O(1) (FD-limited, or stopped by the max() kink / line
    search).  The certified point is feasible and its reference cost is never above the stage-1 cost of a
    feasible stage-1 point (restated cost/constraints, oracle)."""
    import oracle as O
    d = []
    for c in nlp_cases():
        if not bool(c["certified"]):
            continue
        orc, ob = oracles[int(c["traj"])], c["obs"]
        p = O.default_params(N=int(c["N"]), max_obs=len(ob))
        o = ob if len(ob) else None
        f_cert, f_1 = orc.cost(p, c["x0"], c["U_nlp"]), orc.cost(p, c["x0"], c["U_slsqp"])
        assert orc.constraints(p, c["x0"], o, c["U_nlp"]).min() >= -1e-9
        if orc.constraints(p, c["x0"], o, c["U_slsqp"]).min() >= -1e-9:
            assert f_cert <= f_1 + 1e-9 * (1 + abs(f_1)), (f_cert, f_1)
        d.append(float(np.abs(c["U_slsqp"] - c["U_nlp"]).max()))
    print(f"|U_appC - U_certified|: min {min(d):.1e}, median {np.median(d):.1e}, max {max(d):.1e}")


class OracleTracker:
    """TrajectoryTracker surface over the CPU oracle (test-only stand-in for the GPU solver), so the shim's
    run_simulation can replay the reference closed loop on the CPU."""

    def __init__(self, traj, N, sqp_iters):
        import oracle as O
        import trajectory_tracking as TT
        base = TT.TrajectoryTracker(traj)
        for k, v in vars(base).items():
            setattr(self, k, v)
        self.N = N
        self.sqp_iters = sqp_iters
        self.orc = O.Oracle(traj.X_ref, traj.U_ref)
        self.O = O

    def dynamics(self, x, u, k_ref):
        s, d, o, k, v = x
        return np.array([v, v * o, v * (k - k_ref), u[0], u[1]])

    def solve(self, x0, obstacles):
        ob = np.array([[o["s"], o["v"]] for o in obstacles]).reshape(-1, 2)
        p = self.O.default_params(N=self.N, max_obs=len(ob), sqp_iters=self.sqp_iters)
        r = self.orc.solve(p, x0, ob if len(ob) else None)
        self.last_status = r["status"]
        return r["u0"].copy(), r["Xpred"], 0.0


@pytest.mark.parametrize("tag,ti,N,preset", [("traj2_N5_fsm", 2, 5, "trajectory2"),
                                             ("traj3_N5_fsm", 3, 5, "trajectory3")])
def test_oracle_closed_loop_vs_reference_run(tag, ti, N, preset):
    """run_simulation with the FSM (trajectory_tracking.py:377-443) driven by the oracle's SQP: the same
    number of steps as the reference's own run (+-2), the checks pass, and the lateral offset and speed
    stay close to the reference's (its SLSQP stops at ftol 1e-3, so its run is itself inexact)."""
    import contextlib
    import io
    import trajectory_tracking as TT
    from conftest import load_golden
    from trajectory_loader import TrajectoryLoader, builtin_trajectory
    import oracle as O
    O.build()
    traj = TrajectoryLoader(builtin_trajectory(ti))
    mpc = OracleTracker(traj, N, TT.SQP_ITERS)
    fsm = TT.ObstaclesFSM(dynamic_obstacle=True, traffic_light=True, preset=preset)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        hx, hu, ht, hp, hobs, htl, _ = TT.run_simulation(mpc, fsm, traj, max_steps=4000)
    g = load_golden("closedloop_golden")
    gx = g[f"{tag}_hist_x"]
    print(f"{tag}: oracle SQP closed loop {len(hu)} steps, reference {len(gx) - 1}")
    assert abs(len(hu) - (len(gx) - 1)) <= 2, (len(hu), len(gx) - 1)
    assert "===> Checks passed : True" in buf.getvalue(), buf.getvalue()[-600:]
    m = min(len(hx), len(gx))
    dd, dv = np.abs(hx[:m, 1] - gx[:m, 1]).max(), np.abs(hx[:m, 4] - gx[:m, 4]).max()
    print(f"  max |d - d_ref_run| = {dd:.3f} m, max |v - v_ref_run| = {dv:.3f} m/s, median |dv| = "
          f"{np.median(np.abs(hx[:m, 4] - gx[:m, 4])):.2e}")
    assert dd < 0.1 and dv < 2.0


@pytest.mark.parametrize("N", [10, 20])
def test_oracle_closed_loop_traj2_long_horizon(N):
    """The reference scenario (trajectory2, FSM car + light, start [0,0,0,0,0.5]) at N = 10 and 20 with the
    drop-in SQP default: the ego reaches the destination and every restated check passes (a single QP at the
    braking warm start stops for good behind the FSM car at these horizons)."""
    import contextlib
    import io
    import trajectory_tracking as TT
    from trajectory_loader import TrajectoryLoader, builtin_trajectory
    traj = TrajectoryLoader(builtin_trajectory(2))
    mpc = OracleTracker(traj, N, TT.SQP_ITERS)
    fsm = TT.ObstaclesFSM(dynamic_obstacle=True, traffic_light=True)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        hx, hu, *_ = TT.run_simulation(mpc, fsm, traj, max_steps=3000)
    print(f"traj2 N={N} FSM: {len(hu)} steps")
    assert len(hu) < 3000
    assert "===> Checks passed : True" in buf.getvalue(), buf.getvalue()[-600:]


def test_second_start_on_the_other_optima(oracles):
    """the certified cases where the drop-in SQP lands on another local optimum (case 34:
    trajectory3, N=30, two obstacles) re-solved from a second start, the unbraked reference controls (the
    warm start of :224-246 without the obstacle braking), keeping the lower reference cost.  Measured: from
    that start the SQP converges (status 0, stops moving) at cost 112.2747, against 120.8911 from the braked
    start and 112.2721 at the golden optimum SLSQP's path reached, yet 5e-2 away from it in U: a third local
    optimum of the non-convex problem, 0.002% above the golden cost.  So the two-start rule recovers the
    cost but not the point; MAX_OTHER_OPTIMA stays at the one such case, and the product keeps one start
    (a second SQP would double every solve for 1 of 52 certified cases)."""
    import oracle as O
    import trajectory_tracking as TT
    seen = 0
    for j, c in enumerate(nlp_cases()):
        if not bool(c["certified"]):
            continue
        orc, ob = oracles[int(c["traj"])], c["obs"]
        o = ob if len(ob) else None
        p = O.default_params(N=int(c["N"]), max_obs=len(ob), sqp_iters=TT.SQP_ITERS)
        r1 = orc.solve(p, c["x0"], o)
        if float(np.abs(r1["U"] - c["U_nlp"].ravel()).max()) <= TOL_NLP_MEAS:
            continue
        seen += 1
        r2 = orc.solve(p, c["x0"], o, ubar=orc.warm_start(p, c["x0"], None).reshape(-1, 2))
        f1, f2, fg = (orc.cost(p, c["x0"], U) for U in (r1["U"], r2["U"], c["U_nlp"]))
        best = r2 if f2 < f1 else r1
        fb = min(f1, f2)
        e = float(np.abs(best["U"] - c["U_nlp"].ravel()).max())
        print(f"case {j}: braked start cost {f1:.4f}, unbraked start cost {f2:.4f}, golden {fg:.4f}; "
              f"best |U - U_nlp| = {e:.2e}")
        assert best["status"] == 0
        assert orc.constraints(p, c["x0"], o, best["U"]).min() >= -1e-9
        assert fb <= fg * (1 + 1e-4), (j, fb, fg)
    assert seen <= MAX_OTHER_OPTIMA
