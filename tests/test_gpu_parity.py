"""GPU parity of the HIP path (libmpcqp.so through its C ABI) against the reference goldens
and the CPU oracle.  Tolerances:
  lookups, warm start, nominal rollout / predict: bit-exact (FP64 integer-free arithmetic
      identical to numpy; the kernel is compiled with -ffp-contract=off);
  QP(ubar) solution U*: <= 5e-8 abs vs the KKT-certified golden (the BASELINE gate is 1e-5)
      and <= 1e-9 vs the oracle (same warm start, QP and solver) on the FULL per-GPU batch of every
      configuration (measured round 2: 4.8e-13 on C2, 5.6e-11 on C5); statuses identical, except flips
      between infeasible/numerical on badly infeasible elastic problems, and elastic instances where the
      two sides certified different points of the same elastic optimum: both checked by objective value
      (check_vs_oracle) and counted in the printed summary.
"""
import json

import numpy as np
import pytest

from conftest import golden_cases, load_golden, traj_arrays

pytestmark = pytest.mark.gpu

TOL_U = 1e-9          # GPU vs oracle (same warm start, QP, PDIP and polish), N <= 30
TOL_U_N40 = 5e-9      # N = 40: cond(H) ~ 1.5e9; measured 1.4e-9 on one of the 8192 C5 instances


def tol_u(N):
    return TOL_U if N <= 30 else TOL_U_N40
TOL_GATE = 1e-5       # BASELINE.json parity gate vs the certified golden
TOL_CERT = 5e-8       # what the solver actually reaches vs the certified golden (oracle: 9.8e-9)


@pytest.fixture(scope="module")
def lib():
    import __graft_entry__ as g
    g.build()
    import mpcqp
    return mpcqp


@pytest.fixture(scope="module")
def solvers(lib):
    return {i: lib.Solver(*traj_arrays(i), lib.default_params(), device=0) for i in (1, 2, 3)}


def set_p(lib, slv, N, max_obs=0, **kw):
    p = lib.default_params(N=int(N), max_obs=int(max_obs), **kw)
    slv.set_params(p)
    return p


def pack_obs(obs_list, B=None):
    if B is None:
        B = len(obs_list)
    mo = max([len(o) for o in obs_list] + [0])
    if mo == 0:
        return None, None, 0
    a = np.zeros((B, mo, 2))
    n = np.zeros(B, np.int32)
    for b, o in enumerate(obs_list):
        o = np.asarray(o).reshape(-1, 2)
        a[b, :len(o)] = o
        n[b] = len(o)
    return a, n, mo


@pytest.mark.parametrize("ti", [1, 2, 3])
def test_lookup_bit_exact(solvers, ti):
    """mpc_lookup == TrajectoryLoader.get_state/get_control (trajectory_loader.py:86-102)."""
    g = load_golden("interp_golden")
    st, ct = solvers[ti].lookup(g[f"t{ti}_s"])
    assert np.array_equal(st, g[f"t{ti}_state"])
    assert np.array_equal(ct, g[f"t{ti}_control"])


@pytest.mark.parametrize("ti", [1, 2, 3])
def test_lookup_knots_vs_oracle(solvers, ti):
    """The device interval search (bucket index + stepping) finds the binary search's interval at every
    knot, one ulp either side of it, between knots, before s[0] and past s_max (oracle: bisection)."""
    import oracle as O
    X, U = traj_arrays(ti)
    orc = O.Oracle(X, U)
    knots = X[:, 0]
    s = np.concatenate([knots, np.nextafter(knots, -np.inf), np.nextafter(knots, np.inf),
                        0.5 * (knots[1:] + knots[:-1]), [-5.0, -1e-300, orc.s_max * 0.999999, orc.s_max + 3.0],
                        np.random.default_rng(ti).uniform(-1.0, orc.s_max + 1.0, 2000)])
    st, ct = solvers[ti].lookup(s)
    for i, v in enumerate(s):
        assert np.array_equal(st[i], orc.get_state(v)), (i, v)
        assert np.array_equal(ct[i], orc.get_control(v)), (i, v)


def test_warm_start_and_predict_bit_exact(lib, solvers):
    """sqp_iters=0 returns the warm start (:224-246) and predict(x0, ubar) (:87-114) unchanged."""
    cases, _ = golden_cases("warmstart_golden")
    import oracle as O
    for c in cases:
        slv = solvers[int(c["traj"])]
        obs, n, mo = pack_obs([c["obs"]])
        set_p(lib, slv, c["N"], mo, sqp_iters=0)
        r = slv.solve_batch(c["x0"][None], obs, n)
        assert np.array_equal(r["U"][0].ravel(), c["ubar"]), c["x0"]
        orc = O.Oracle(*traj_arrays(int(c["traj"])))
        Xo = orc.predict(O.default_params(N=int(c["N"])), c["x0"], c["ubar"])
        assert np.array_equal(r["Xpred"][0], Xo)
        assert r["status"][0] == 0 and r["iters"][0] == 0


def test_predict_matches_reference_model_golden(lib, solvers):
    """Xpred with a given U and sqp_iters=0 is the reference predict() bit for bit."""
    cases, _ = golden_cases("model_golden")
    for c in cases:
        slv = solvers[int(c["traj"])]
        set_p(lib, slv, c["N"], 0, sqp_iters=0)
        r = slv.solve_batch(c["x0"][None], ubar=c["U"].reshape(1, -1, 2))
        assert np.array_equal(r["Xpred"][0], c["X"])


def test_qp_solution_vs_certified_golden(lib, solvers):
    """The 1e-5 gate of BASELINE.json, at identical linearisation points."""
    cases, g = golden_cases("qp_golden")
    rho = float(g["rho"])
    worst = 0.0
    for c in cases:
        if not bool(c["ok_elastic"]):
            continue
        slv = solvers[int(c["traj"])]
        obs, n, mo = pack_obs([c["obs"]])
        set_p(lib, slv, c["N"], mo, elastic_rho=rho)
        r = slv.solve_batch(c["x0"][None], obs, n, ubar=c["ubar"].reshape(1, -1, 2))
        err = float(np.abs(r["U"][0].ravel() - c["U_elastic"]).max())
        worst = max(worst, err)
        assert err <= TOL_GATE, (err, int(r["status"][0]), int(r["iters"][0]), json.loads(str(c["fdcheck"])))
        assert err <= TOL_CERT, err
        if bool(c["feasible"]):
            assert int(r["status"][0]) == 0
        else:
            from test_oracle_golden import golden_violation, params
            import oracle as O
            viol = golden_violation(O.Oracle(*traj_arrays(int(c["traj"]))), params(c["N"], c["obs"].shape[0]), c)
            assert int(r["status"][0]) == 2 or (viol <= 1e-5 and int(r["status"][0]) == 0)
    print(f"worst |U_gpu - U*_golden| = {worst:.3e}")


def elastic_objective(orc, p, x0, obs, U):
    """Objective of the elastic QP(ubar) at U: the quadratic model plus
    rho * (soft-row violation); ubar is the reference warm start.  Box rows are hard."""
    ubar = orc.warm_start(p, x0, obs)
    q = orc.build_qp(p, x0, obs, ubar)
    du = np.asarray(U, np.float64).ravel() - ubar
    ax = q["A"] @ du
    viol = np.maximum(q["lo"] - ax, 0.0) + np.maximum(ax - q["hi"], 0.0)
    return 0.5 * du @ q["H"] @ du + q["f"] @ du + q["c0"] + p.elastic_rho * viol.sum()


def check_vs_oracle(r, ro, ctx=None, label="", tol=TOL_U, xtol=1e-8):
    """Status and U/Xpred parity, returns the summary dict (printed by the callers).
    Statuses must agree, except flips between infeasible (2) and numerical (3): both mean "no certified
    solution of the hard QP"; they happen on badly infeasible elastic problems (rho = 1e5), where the last
    interior-point iterates of the two implementations differ by rounding, and the side that certified
    its elastic optimum (status 2, KKT-checked by the polish) must have an objective no worse than the
    other's.  U must agree to TOL_U wherever both sides certified a solution, except on elastic instances
    (status 2 on both) whose two answers have the same elastic objective to 1e-9 relative: the polish can
    certify two points of one flat elastic optimum ("Elastic-problem tolerance").
    The SQP-unconverged flag (16) is compared separately: it must agree wherever U agrees."""
    flag_g, flag_o = (r["status"] & 16) != 0, (ro["status"] & 16) != 0
    r = dict(r, status=r["status"] & 15)
    ro = dict(ro, status=ro["status"] & 15)
    agree = r["status"] == ro["status"]
    mism = ~agree
    assert np.isin(r["status"][mism], (2, 3)).all() and np.isin(ro["status"][mism], (2, 3)).all(), \
        (label, r["status"][mism], ro["status"][mism])
    orc = p = x0 = obs = n_obs = None
    if ctx is not None:
        orc, p, x0, obs, n_obs = ctx
    obj = lambda i, U: elastic_objective(orc, p, x0[i], None if obs is None else obs[i, :n_obs[i]], U)
    for i in np.flatnonzero(mism):
        assert ctx is not None, (label, "status flip without context", i)
        fg, fo = obj(i, r["U"][i]), obj(i, ro["U"][i])
        cert, other = (fg, fo) if r["status"][i] == 2 else (fo, fg)
        assert cert <= other + 1e-6 * (1.0 + abs(other)), (label, i, fg, fo, r["status"][i], ro["status"][i])
    cert = np.isin(r["status"], (0, 2)) & np.isin(ro["status"], (0, 2))
    err = np.abs(r["U"] - ro["U"]).reshape(len(cert), -1).max(axis=1)
    alt = 0
    for i in np.flatnonzero(cert & (err > tol)):
        both_elastic = bool(r["status"][i] == 2 and ro["status"][i] == 2)
        assert ctx is not None and both_elastic, (label, int(i), float(err[i]), int(r["status"][i]), int(ro["status"][i]))
        fg, fo = obj(i, r["U"][i]), obj(i, ro["U"][i])
        assert abs(fg - fo) <= 1e-9 * (1.0 + abs(fo)), (label, i, err[i], fg, fo)
        alt += 1
    ok = cert & (err <= tol)
    xe = np.abs(r["Xpred"] - ro["Xpred"]).reshape(len(cert), -1).max(axis=1)
    assert xe[ok].max(initial=0.0) <= xtol, (label, xe[ok].max())
    assert np.array_equal(flag_g[ok], flag_o[ok]), (label, np.flatnonzero(ok & (flag_g != flag_o)))
    s = dict(label=label, B=len(cert), status_agree=float(agree.mean()), flips_2_3=int(mism.sum()),
             sqp_unconverged=int(flag_g.sum()),
             elastic_alt_optima=alt, max_err_U=float(err[ok].max(initial=0.0)),
             max_err_Xpred=float(xe[ok].max(initial=0.0)))
    print(json.dumps(s))
    return s


@pytest.mark.parametrize("cfg", ["C1", "C2", "C3", "C4", "C5"])
def test_vs_oracle_full_batch(lib, solvers, cfg):
    """The full per-GPU batch of every BASELINE configuration (bench.py's inputs: C2 4096, C3 8192,
    C4 4096, C5 8192; C1 64 egos): GPU == oracle (warm start + QP + predict) to TOL_U."""
    import oracle as O
    import workloads as W
    B = 64 if cfg == "C1" else W.CONFIGS[cfg]["B"] // W.CONFIGS[cfg]["gpus"]
    wb = W.make_batch(cfg, B=B)
    slv = solvers[wb["traj"]]
    set_p(lib, slv, wb["N"], wb["max_obs"])
    r = slv.solve_batch(wb["x0"], wb["obs"], wb["n_obs"])
    orc = O.Oracle(*traj_arrays(wb["traj"]))
    po = O.default_params(N=wb["N"], max_obs=wb["max_obs"])
    ro = orc.solve_batch(po, wb["x0"], wb["obs"], wb["n_obs"])
    check_vs_oracle(r, ro, ctx=(orc, po, wb["x0"], wb["obs"], wb["n_obs"]), label=f"{cfg} B={B}", tol=tol_u(wb["N"]))
    assert np.array_equal(r["u0"], r["U"][:, 0, :])


@pytest.mark.parametrize("cfg,B,nsqp", [("C2", 4096, 3), ("C3", 2048, 10), ("C4", 1024, 10)])
def test_sqp_relinearisation_vs_oracle(lib, solvers, cfg, B, nsqp):
    """SQP outer iterations on device: QP(U*) re-linearised about the previous
    solution, `sqp_iters` times; same fixed-point path as the oracle's orc_solve loop."""
    import oracle as O
    import workloads as W
    wb = W.make_batch(cfg, B=B, seed=99)
    slv = solvers[wb["traj"]]
    set_p(lib, slv, wb["N"], wb["max_obs"], sqp_iters=nsqp)
    r = slv.solve_batch(wb["x0"], wb["obs"], wb["n_obs"])
    orc = O.Oracle(*traj_arrays(wb["traj"]))
    po = O.default_params(N=wb["N"], max_obs=wb["max_obs"], sqp_iters=nsqp)
    ro = orc.solve_batch(po, wb["x0"], wb["obs"], wb["n_obs"])
    # up to 10 re-linearisations carry the last-bit differences of each QP into the next linearisation
    # point: measured 3.5e-9 (C3) and 2.0e-9 (C4) on elastic instances, <= 9e-11 on the hard (status 0)
    # ones; the N = 30 rollout of the C4 one's U moves Xpred by 2.9e-8
    check_vs_oracle(r, ro, label=f"SQP {cfg} K={nsqp}", tol=1e-8, xtol=1e-7)
    assert (r["iters"] >= 0).all()


def test_full_size_C2_properties(lib, solvers):
    """BASELINE metric config (traj1, N=20, B=4096): size-independent properties + oracle subset."""
    import oracle as O
    import workloads as W
    wb = W.make_batch("C2")
    slv = solvers[1]
    p = set_p(lib, slv, 20, 0)
    r = slv.solve_batch(wb["x0"])
    assert r["U"].shape == (4096, 20, 2)
    assert set(np.unique(r["status"])) <= {0, 2}
    U = r["U"]
    assert (U[..., 0] >= p.u_min[0] - 1e-9).all() and (U[..., 0] <= p.u_max[0] + 1e-9).all()
    assert (U[..., 1] >= p.u_min[1] - 1e-9).all() and (U[..., 1] <= p.u_max[1] + 1e-9).all()
    # deterministic: same inputs -> bit-identical outputs
    r2 = slv.solve_batch(wb["x0"])
    assert np.array_equal(r["U"], r2["U"]) and np.array_equal(r["iters"], r2["iters"])
    orc = O.Oracle(*traj_arrays(1))
    ro = orc.solve_batch(O.default_params(N=20), wb["x0"])
    assert np.abs(r["U"] - ro["U"]).max() <= TOL_U


def test_edge_cases(lib, solvers):
    import oracle as O
    X, Uref = traj_arrays(1)
    orc = O.Oracle(X, Uref)
    slv = solvers[1]
    smax = orc.s_max
    x0s = np.array([
        [smax - 0.3, 0.0, 0.0, 0.0, 3.0],       # horizon runs past s_max (get_state returns the last row)
        [smax + 5.0, 0.1, 0.0, 0.0, 1.0],       # already past the end
        [10.0, 0.0, 0.0, 0.0, 0.0],             # standing still
        [50.0, 0.9, 0.05, 0.0, 8.0],            # far outside the lane margin -> elastic
        [-3.0, 0.0, 0.0, 0.0, 0.5],             # s < 0: left extrapolation
        [100.0, 0.0, 0.0, 0.0, 12.0],
    ])
    obs_lists = [[], [], [(12.0, 0.0)], [(53.0, 0.0)], [], [(104.0, 1.0), (400.0, 3.0)]]
    obs, n, mo = pack_obs(obs_lists)
    for N in (1, 2, 20, 63):
        set_p(lib, slv, N, mo)
        r = slv.solve_batch(x0s, obs, n)
        po = O.default_params(N=N, max_obs=mo)
        ro = orc.solve_batch(po, x0s, obs, n)
        # instance 5 (obstacle 4 m ahead at 12 m/s) is the badly infeasible elastic case of check_vs_oracle
        check_vs_oracle(r, ro, ctx=(orc, po, x0s, obs, n), label=f"edge N={N}", tol=tol_u(N))
        assert np.isfinite(r["Xpred"]).all()
    # obstacle inside 5 m: infeasible, still returns a control (the reference always returns one)
    assert r["status"][2] == 2 and r["status"][3] == 2
    # an empty batch is a no-op
    set_p(lib, slv, 20, 0)
    r = slv.solve_batch(np.zeros((0, 5)))
    assert r["U"].shape == (0, 20, 2)


def test_shim_solve_matches_oracle(lib):
    """TrajectoryTracker.solve (trajectory_tracking.py:213-263 surface) on the GPU."""
    import oracle as O
    import trajectory_tracking as TT
    from trajectory_loader import TrajectoryLoader, builtin_trajectory
    traj = TrajectoryLoader(builtin_trajectory(2))
    mpc = TT.TrajectoryTracker(traj)
    mpc.N = 20
    x0 = np.array([700.0, 0.05, 0.0, traj.get_state(700.0)[3], 8.0])
    obs = [{"s": 730.0, "v": 4.0, "type": "car"}, {"s": 760.0, "v": 0.0, "type": "light"}]
    u0, pred_X, t = mpc.solve(x0, obs)
    orc = O.Oracle(traj.X_ref, traj.U_ref)
    ro = orc.solve(O.default_params(N=20, max_obs=2, sqp_iters=TT.SQP_ITERS), x0, [(730.0, 4.0), (760.0, 0.0)])
    assert pred_X.shape == (21, 5) and u0.shape == (2,)
    assert np.abs(u0 - ro["u0"]).max() <= TOL_U
    assert np.abs(pred_X - ro["Xpred"]).max() <= 1e-8
    assert t >= 0.0 and mpc.last_status == ro["status"]


def test_closed_loop_config1(lib):
    """Config 1 (traj1, N=10, single ego, closed loop): the restated sanity checks pass and the
    trajectory stays close to the reference's own closed loop (closedloop_golden)."""
    import io
    import contextlib
    import trajectory_tracking as TT
    from trajectory_loader import TrajectoryLoader, builtin_trajectory
    traj = TrajectoryLoader(builtin_trajectory(1))
    mpc = TT.TrajectoryTracker(traj)
    mpc.N = 10
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        hx, hu, ht, hp, hobs, htl, _ = TT.run_simulation(mpc, TT.ObstaclesFSM(), traj, max_steps=2000)
    assert "===> Checks passed : True" in buf.getvalue(), buf.getvalue()[-800:]
    g = load_golden("closedloop_golden")
    ref_x = g["c1_traj1_N10_hist_x"]
    # the reference's SLSQP stops at ftol=1e-3 (trajectory_tracking.py:255) and the exact NLP optimum brakes a
    # step apart from it: steps within +-2, lateral offsets within 0.1 m over the whole run (the bar of the FSM
    # runs and of the host backend's config-1 loop, tests/test_cpu_backend.py)
    assert abs(len(hx) - len(ref_x)) <= 2
    m = min(len(hx), len(ref_x))
    assert np.abs(hx[:m, 1] - ref_x[:m, 1]).max() < 0.1


def test_global_pose_device_vs_golden(lib, solvers):
    """mpc_global_pose == TrajectoryLoader.get_global_pose (trajectory_loader.py:104-116); device sin/cos
    may differ from libm by an ulp, so 1e-9 m / rad."""
    g = load_golden("pose_golden")
    for i in (1, 2, 3):
        P = solvers[i].global_pose(g[f"t{i}_s"], g[f"t{i}_d"])
        assert np.abs(P - g[f"t{i}_pose"]).max() <= 1e-9, i


def test_create_from_json_matches(lib, tmp_path):
    """mpc_create_from_json on the reference's JSON format == mpc_create on the same arrays."""
    import ctypes
    X, U = traj_arrays(3)
    path = tmp_path / "trajectory3.json"
    path.write_text(json.dumps({"X": X.tolist(), "U": U.tolist()}))
    p = lib.default_params(N=10)
    h = ctypes.c_void_p()
    rc = lib.lib().mpc_create_from_json(str(path).encode(), ctypes.byref(p), 0, ctypes.byref(h))
    assert rc == 0, lib.last_error()
    s = np.linspace(-5.0, 2000.0, 777)
    st = np.empty((s.size, 5)); ct = np.empty((s.size, 2))
    assert lib.lib().mpc_lookup(h, s.size, lib._p(s), lib._p(st), lib._p(ct)) == 0
    lib.lib().mpc_destroy(h)
    st2, ct2 = lib.Solver(X, U, p).lookup(s)
    assert np.array_equal(st, st2) and np.array_equal(ct, ct2)
