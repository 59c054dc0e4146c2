"""Pin the CPU oracle to the reference (golden vectors captured by tests/golden/make_goldens.py).

Each test names the reference function it pins.  CPU only.
"""
import json

import numpy as np
import pytest

from conftest import golden_cases, load_golden

import oracle as O


def params(N, nobs=0, **kw):
    return O.default_params(N=int(N), max_obs=int(nobs), **kw)


@pytest.mark.parametrize("ti", [1, 2, 3])
def test_interp_bit_exact(oracles, ti):
    """TrajectoryLoader.get_state / get_control, trajectory_loader.py:86-102 (scipy interp1d linear)."""
    g = load_golden("interp_golden")
    orc = oracles[ti]
    S = g[f"t{ti}_s"]
    st = np.array([orc.get_state(s) for s in S])
    ct = np.array([orc.get_control(s) for s in S])
    assert np.array_equal(st, g[f"t{ti}_state"])
    assert np.array_equal(ct, g[f"t{ti}_control"])


def test_model_predict_cost_constraints(oracles):
    """TrajectoryTracker.predict (:87-114) bit-exact; cost (:116-152), constraints (:155-211) to 1e-12."""
    cases, _ = golden_cases("model_golden")
    assert len(cases) >= 50
    for c in cases:
        orc = oracles[int(c["traj"])]
        p = params(c["N"])
        X = orc.predict(p, c["x0"], c["U"])
        assert np.array_equal(X, c["X"])
        cost = orc.cost(p, c["x0"], c["U"])
        assert abs(cost - float(c["cost"])) <= 1e-12 * (1 + abs(float(c["cost"])))
        g = orc.constraints(p, c["x0"], c["obs"], c["U"])
        assert g.shape == c["cons"].shape
        assert np.abs(g - c["cons"]).max() <= 1e-12


def test_warm_start_bit_exact(oracles):
    """u_init of TrajectoryTracker.solve (:224-246, sticky brake rule), bit-exact."""
    cases, _ = golden_cases("warmstart_golden")
    for c in cases:
        orc = oracles[int(c["traj"])]
        p = params(c["N"])
        ub = orc.warm_start(p, c["x0"], c["obs"])
        assert np.array_equal(ub, c["ubar"]), (c["x0"], c["obs"])


def test_qp_matrices(oracles):
    """QP(ubar) of SURVEY Appendix B: the oracle's dense build vs the golden build
    (which the generator validated against central-FD of the reference predict/cost/constraints)."""
    cases, _ = golden_cases("qpdata_golden")
    for c in cases:
        orc = oracles[int(c["traj"])]
        p = params(c["N"])
        q = orc.build_qp(p, c["x0"], c["obs"], c["ubar"])
        for k in ("H", "f", "A", "blo", "bhi"):
            ref = c[k]
            assert q[k].shape == ref.shape, k
            assert np.abs(q[k] - ref).max() <= 1e-10 * (1 + np.abs(ref).max()), k
        assert abs(q["c0"] - float(c["c0"])) <= 1e-12 * (1 + abs(float(c["c0"])))
        for k in ("lo", "hi"):
            ref = c[k]
            fin = np.isfinite(ref)
            assert np.array_equal(fin, np.isfinite(q[k])), k
            assert np.abs(q[k][fin] - ref[fin]).max() <= 1e-12, k


def golden_violation(orc, p, c):
    """max elastic slack of the certified solution (0 when the hard QP(ubar) is feasible)."""
    q = orc.build_qp(p, c["x0"], c["obs"], c["ubar"])
    ax = q["A"] @ (c["U_elastic"] - c["ubar"])
    return float(max(0.0, np.max(q["lo"] - ax), np.max(ax - q["hi"])))


TOL_QP = 5e-8      # measured worst 9.8e-9 over the 114 cases


def test_qp_solution_vs_certified_golden(oracles):
    """Oracle PDIP vs the KKT-certified solution of QP(ubar) (hard QP when feasible == elastic)."""
    cases, g = golden_cases("qp_golden")
    rho = float(g["rho"])
    worst = 0.0
    nfeas = 0
    for c in cases:
        if not bool(c["ok_elastic"]):
            continue
        orc = oracles[int(c["traj"])]
        p = params(c["N"], elastic_rho=rho)
        r = orc.solve(p, c["x0"], c["obs"], ubar=c["ubar"])
        err = np.abs(r["U"] - c["U_elastic"]).max()
        worst = max(worst, err)
        # BASELINE gate is 1e-5; the oracle agrees with the certified optimum to ~1e-8
        assert err <= TOL_QP, (err, r["status"], r["iters"], json.loads(str(c["kkt_elastic"])))
        viol = golden_violation(orc, p, c)
        if bool(c["feasible"]):
            nfeas += 1
            assert r["status"] == 0, r
            assert np.abs(r["U"] - c["U_hard"]).max() <= TOL_QP
        elif viol > 1e-5:
            assert r["status"] == 2, (r, viol)
        else:
            assert r["status"] in (0, 2), (r, viol)
    assert nfeas >= 40
    print("worst |U - U*| =", worst)


def test_global_pose_bit_exact(oracles):
    """orc_global_pose == TrajectoryLoader.get_global_pose (trajectory_loader.py:32-62,104-116)."""
    g = load_golden("pose_golden")
    for i in (1, 2, 3):
        P = np.array([oracles[i].global_pose(s, d) for s, d in zip(g[f"t{i}_s"], g[f"t{i}_d"])])
        assert np.array_equal(P, g[f"t{i}_pose"])
