"""Pin oracle/slsqp_port.py — the reference's own CPU solve path (warm start + scipy SLSQP) restated —
to the reference's outputs.  CPU only.

model_golden / warmstart_golden / solve_golden were captured from the reference itself by
tests/golden/make_goldens.py; solve_golden holds what TrajectoryTracker.solve
(trajectory_tracking.py:213-263) returned on seeded instances (U, nit, status, fun).
"""
import json

import numpy as np
import pytest
import scipy

from conftest import golden_cases, load_golden

import slsqp_port as SP
from trajectory_loader import TrajectoryLoader, builtin_trajectory

_LD = {}


def tracker(ti, N):
    ti = int(ti)
    if ti not in _LD:
        _LD[ti] = TrajectoryLoader(builtin_trajectory(ti))
    return SP.SlsqpTracker(_LD[ti], int(N))


def obs_list(a):
    return [{"s": float(s), "v": float(v)} for s, v in np.asarray(a, dtype=np.float64).reshape(-1, 2)]


def test_model_bit_exact_vs_reference():
    """predict (:87-114), cost (:116-152), constraints (:155-211): same accumulation order -> bit-exact."""
    cases, _ = golden_cases("model_golden")
    for c in cases:
        tr = tracker(c["traj"], c["N"])
        assert np.array_equal(tr.predict(c["x0"], c["U"]), c["X"])
        assert tr.cost(c["U"], c["x0"]) == float(c["cost"])
        g = tr.constraints(c["x0"], obs_list(c["obs"]))["fun"](c["U"])
        assert np.array_equal(g, c["cons"])


def test_warm_start_bit_exact_vs_reference():
    """u_init handed to minimize (:224-246)."""
    cases, _ = golden_cases("warmstart_golden")
    for c in cases:
        tr = tracker(c["traj"], c["N"])
        assert np.array_equal(tr.warm_start(c["x0"], obs_list(c["obs"])), c["ubar"])


def test_pool_timing_leg_runs():
    """bench.py's cpu_reference leg: the bounded process-pool timing over a config's egos."""
    import workloads as W
    wb = W.make_batch("C1", B=4)
    done, dt = SP.time_batch(wb["traj"], wb["N"], wb["x0"], budget_s=0.5, procs=2)
    assert done >= 2 and dt > 0.0


def test_solve_matches_reference_solve():
    """The whole SLSQP solve (:254-263) against the reference's own solve() outputs."""
    g = load_golden("solve_golden")
    meta = json.loads(str(g["meta_json"]))
    if meta.get("scipy") != scipy.__version__:
        pytest.skip(f"solve_golden was captured with scipy {meta.get('scipy')}, this is {scipy.__version__}")
    cases, _ = golden_cases("solve_golden")
    assert len(cases) >= 10
    for c in cases:
        tr = tracker(c["traj"], c["N"])
        u0, pX, _, r = tr.solve(c["x0"], obs_list(c["obs"]))
        assert int(r.nit) == int(c["nit"]) and int(r.status) == int(c["status"])
        assert np.array_equal(r.x, c["U"])
        assert np.array_equal(u0, c["u0"])
        assert np.array_equal(pX, c["predX"])
        assert float(r.fun) == float(c["fun"])
