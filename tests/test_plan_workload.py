"""The planner benchmark's chunk generator (workloads.plan_batch_ref): chunks posed as
optimize_full_trajectory (trajectory_planning.py:491-515) poses them, and rank shards that together are the
single-process batch (bench.py's plan leg shards by offset)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "safe-autonomous-driving-mpc_amd")]


def test_chunks_follow_the_reference_sizing_rule():
    import workloads as W
    r = W.plan_route("traj3")
    wb = W.plan_batch_ref(r, 2000, seed=3)
    s0, st, fin, N = wb["x0"][:, 0], wb["s_target"], wb["is_final"], wb["N"]
    assert np.all(np.diff(N) >= 0)                                   # sorted by horizon
    D = st - s0
    assert np.allclose(D[fin == 0], 20.0)
    assert np.all(st[fin == 1] == r.s_total) and np.all((D[fin == 1] >= 30.0 - 1e-9) & (D[fin == 1] <= 40.0 + 1e-9))
    for i in range(0, 2000, 97):
        assert N[i] == int(np.ceil(D[i] / r.avg_speed_from(s0[i]) * 2.0 / 0.3))
        assert wb["x0"][i, 3] == r.k_ref_fun(s0[i])
        assert 0.0 <= wb["x0"][i, 4] <= 0.9 * r.v_max_fun(s0[i]) + 1e-12
    assert 0.05 <= fin.mean() <= 0.15


def test_rank_shards_make_up_the_batch():
    import workloads as W
    r = W.plan_route("traj2")
    full = W.plan_batch_ref(r, 600, seed=9)
    parts = [W.plan_batch_ref(r, 200, seed=9, offset=o) for o in (0, 200, 400)]
    key = lambda w: sorted(map(tuple, np.column_stack([w["x0"], w["s_target"], w["is_final"], w["N"]]).tolist()))
    merged = {k: np.concatenate([p[k] for p in parts]) for k in ("x0", "s_target", "is_final", "N")}
    assert key(merged) == key(full)


def test_graphhopper_route_dict_is_accepted():
    """optimize_full_trajectory takes the reference's own route object (path_planning.get_route's dict:
    (lon, lat) points and max_speed details): routes.from_graphhopper projects it to local metres as
    global2local does (WGS84 ENU, first point at the origin) and builds the same route as from_waypoints."""
    import routes
    pts = [(-73.5673, 45.5017), (-73.5660, 45.5025), (-73.5640, 45.5030), (-73.5631, 45.5049)]
    loc = routes.global2local(pts)
    assert loc[0] == (0.0, 0.0)
    # local tangent plane vs the small-distance approximation (east = R_N cos(lat) dlon, north = R_M dlat)
    a, f = 6378137.0, 1 / 298.257223563
    e2 = f * (2 - f)
    lat0 = np.radians(45.5017)
    rn = a / np.sqrt(1 - e2 * np.sin(lat0) ** 2)
    rm = a * (1 - e2) / (1 - e2 * np.sin(lat0) ** 2) ** 1.5
    for (lon, lat), (e, n) in zip(pts, loc):
        assert abs(e - rn * np.cos(lat0) * np.radians(lon + 73.5673)) < 0.05
        assert abs(n - rm * np.radians(lat - 45.5017)) < 0.05
    ms = [[0, 2, 50], [2, 3, None]]
    r1 = routes.from_graphhopper({"points": pts, "max_speed": ms})
    r2 = routes.from_waypoints(loc, [tuple(m) for m in ms])
    assert np.array_equal(r1.s, r2.s) and np.array_equal(r1.vmax, r2.vmax)
    assert np.isclose(r1.vmax[0], 50 / 3.6) and np.isclose(r1.vmax[-1], 30 / 3.6)
