"""libmpcplan's host backend (plan_create(..., device = -1, ...), csrc/plan_host.h): the offline planner's chunk
solve on the CPU behind the same C ABI (VERDICT r05 "missing" 4: the reference's planner is CPU code,
trajectory_planning.py:381-387).  Checked here, without a GPU:
  - bit for bit against the planner oracle (oracle/plan_oracle.c, same algorithm and IEEE operation sequence)
    on a mixed batch of intermediate and final chunks (every output: X, U, S, status, iterations, QPs);
  - the route functions (k_ref_fun, its derivative, v_max_fun) against the oracle's;
  - plan_optimize's receding-horizon loop against the package loop driven by the oracle (identical plans);
  - the drop-in's full trajectory on the host backend passes the restated reference_trajectory_check;
  - device entries on a host context fail with PLAN_E_DEVICE.
"""
import numpy as np
import pytest


@pytest.fixture(scope="module")
def env():
    import __graft_entry__ as g
    g.build()
    import mpcplan
    import plan_oracle as PO
    import workloads as W
    return mpcplan, PO, W


def _batch(W, r, n=48, seed=11):
    """intermediate and final chunks of several horizons along the route"""
    rng = np.random.default_rng(seed)
    x0 = np.zeros((n, 5))
    s0 = rng.uniform(0.0, r.s_total - 45.0, n)
    x0[:, 0] = s0
    x0[:, 1] = rng.uniform(-0.05, 0.05, n)
    x0[:, 3] = [r.k_ref_fun(s) for s in s0]
    x0[:, 4] = [rng.uniform(0.3, 0.9) * r.v_max_fun(s) for s in s0]
    fin = (np.arange(n) % 4 == 3).astype(np.int32)
    st = np.where(fin == 1, np.minimum(s0 + 35.0, r.s_total), s0 + 20.0)
    N = np.array([(13, 16, 20, 26)[i % 4] for i in range(n)], np.int32)
    return x0, st, fin, N


def test_host_backend_equals_oracle_bit_for_bit(env):
    mpcplan, PO, W = env
    r = W.plan_route("synth1")
    x0, st, fin, N = _batch(W, r)
    pl = mpcplan.Planner(r, mpcplan.default_params(N=int(N.max())), device=-1)
    got = pl.solve_chunks(x0, st, fin, N)
    orc = PO.PlanOracle(r)
    ref = orc.solve_batch(PO.default_params(N=int(N.max())), x0, st, fin, N=N, num_threads=4)
    for k in ("X", "U", "S", "status", "iters", "sqp"):
        assert np.array_equal(got[k], ref[k]), k
    print("statuses", np.bincount(got["status"], minlength=5).tolist(), "QPs", int(got["sqp"].sum()))
    assert np.isin(got["status"], (0, 4)).mean() >= 0.9


def test_host_route_functions_equal_oracle(env):
    mpcplan, PO, W = env
    r = W.plan_route("traj1")
    pl = mpcplan.Planner(r, device=-1)
    orc = PO.PlanOracle(r)
    s = np.concatenate([np.linspace(-3.0, r.s_total + 3.0, 401), np.asarray(r.s[:50], np.float64)])
    k, dk, vm = pl.route_eval(s)
    for i, si in enumerate(s):
        ko, dko = orc.kappa(si)
        assert k[i] == ko and dk[i] == dko and vm[i] == orc.vmax(si), (i, si)


def test_host_optimize_loop_equals_oracle_loop(env):
    """plan_optimize on the host backend (the receding-horizon loop of plan_loop_kernel, trajectory_planning.py
    :478-559) gives the plans the package loop gives with the oracle as its batched chunk solver."""
    mpcplan, PO, W = env
    import trajectory_planning as TP
    r = W.plan_route("synth1")
    orc = PO.PlanOracle(r)

    def solve_chunks(x0, st, fin, N):
        return orc.solve_batch(PO.default_params(N=int(N.max())), x0, st, fin, N=N, num_threads=4)

    starts = np.zeros((3, 5))
    for b, s0 in ((1, 400.0), (2, 1100.0)):
        starts[b] = (s0, 0.02, 0.0, r.k_ref_fun(s0), 0.6 * r.v_max_fun(s0))
    ref, qref = TP.optimize_full_trajectory_batch(r, starts, solve_chunks=solve_chunks)
    got, qgot = TP.optimize_full_trajectory_batch(r, starts, device=-1)
    for b in range(3):
        for a, c in zip(got[b], ref[b]):
            assert np.array_equal(a, c), b
        assert qgot[b]["statuses"] == qref[b]["statuses"] and qgot[b]["passed"], (b, qgot[b])
    print("host-backend plans: chunks", [len(q["statuses"]) for q in qgot])


def test_dropin_full_trajectory_on_host_backend(env, capsys):
    """The package optimize_full_trajectory (the reference's per-chunk loop, :419-559) on the host backend:
    the plan reaches the destination and passes the restated reference_trajectory_check (:557)."""
    mpcplan, PO, W = env
    import trajectory_planning as TP
    r = W.plan_route("traj1")
    X, U, S = TP.optimize_full_trajectory(r, device=-1)
    out = capsys.readouterr().out
    assert "===> Checks passed : True" in out, out
    assert abs(X[-1, 0] - r.s_total) < 1e-6 and abs(X[-1, 4]) < 1e-9
    TP.release_planners()


def test_device_entries_refuse_a_host_context(env):
    mpcplan, PO, W = env
    import ctypes as C
    r = W.plan_route("synth1")
    pl = mpcplan.Planner(r, device=-1)
    L = mpcplan.lib()
    n = C.c_int(0)
    assert L.plan_chunks_per_cu(pl.h, 16, C.byref(n)) == -2
    assert b"host context" in L.plan_last_error()
    rc = L.plan_solve_chunks_device(pl.h, 1, 16, None, None, None, None, None, None, None, None, None, None, None)
    assert rc == -2
    with pytest.raises(mpcplan.PlanError):
        mpcplan.Planner(r, device=-2)
