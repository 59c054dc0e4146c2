"""The planner drop-in takes the reference's own route functions.

optimize_full_trajectory (/root/reference/trajectory_planning.py:437-477) builds k_ref_fun and v_max_fun as
closures over s_to_t (interp1d), the reference path's CubicSpline pair and v_max_interpolator (interp1d
'previous'), and hands them to a new TrajectoryOptimizer per chunk (:517-520).  `reference_closures` below
restates those lines (no import of the reference); the package must recover the route from them bit for bit
and share one device context for the whole route.
"""
import numpy as np
import pytest
from scipy.interpolate import interp1d


def reference_closures(detailed_points, reference_path_spline, speed_limits):
    """trajectory_planning.py:435-477, restated: the route functions exactly as the reference builds them.
    speed_limits: [((_, _), (idx_start, idx_end), value)] as get_path_and_speed_limits returns them."""
    points = np.array(detailed_points)
    distances = np.sqrt(np.diff(points[:, 0]) ** 2 + np.diff(points[:, 1]) ** 2)        # :412
    s_values = np.concatenate([[0], np.cumsum(distances)])                              # :413
    s_total = s_values[-1]
    t_max = len(detailed_points) - 1                                                     # :440
    t_values = np.linspace(0.0, t_max, len(detailed_points))
    s_to_t = interp1d(s_values, t_values, kind='linear', fill_value='extrapolate')

    def k_ref_fun(s):                                                                    # :445-459
        t = float(s_to_t(s))
        x_spline, y_spline = reference_path_spline
        x_dt = x_spline(t, 1)
        y_dt = y_spline(t, 1)
        x_ddt = x_spline(t, 2)
        y_ddt = y_spline(t, 2)
        denom = (x_dt ** 2 + y_dt ** 2) ** 1.5 + 1e-9
        if denom < 1e-8:
            denom = 1e-8
        k = (x_dt * y_ddt - y_dt * x_ddt) / denom
        return float(k)

    v_max_array = np.ones(len(detailed_points))                                          # :464-467
    for limit in speed_limits:
        (_, _), (idx_start, idx_end), value = limit
        v_max_array[idx_start: idx_end + 1] = value
    v_max_interpolator = interp1d(s_values, v_max_array, kind='previous', fill_value="extrapolate")

    def v_max_fun(s):                                                                    # :472-473
        return float(v_max_interpolator(s))

    def v_min_fun(s):                                                                    # :476-477
        return 0
    return k_ref_fun, v_min_fun, v_max_fun, v_max_array, s_total


def reference_inputs(route):
    """The reference's (detailed_points, spline, speed_limits) for a routes.Route: its way-points, a spline made
    the way path_planning.create_spline makes it (:146-162), and the speed-limit intervals of its array."""
    from scipy.interpolate import CubicSpline
    pts = [tuple(p) for p in route.points]
    t = np.arange(len(pts))
    spline = (CubicSpline(t, route.points[:, 0]), CubicSpline(t, route.points[:, 1]))
    v, lim, i = route.vmax, [], 0
    while i < len(v):
        j = i
        while j + 1 < len(v) and v[j + 1] == v[i]:
            j += 1
        lim.append(((None, None), (i, j), float(v[i])))
        i = j + 1
    return pts, spline, lim


@pytest.fixture(scope="module")
def mods():
    import routes
    import trajectory_planning as TP
    import workloads as W
    return routes, TP, W


@pytest.mark.parametrize("name", ["traj1", "traj3", "synth1"])
def test_route_recovered_from_reference_closures_bit_for_bit(mods, name):
    routes, TP, W = mods
    r = W.plan_route(name)
    pts, spline, lim = reference_inputs(r)
    k_ref_fun, v_min_fun, v_max_fun, v_max_array, s_total = reference_closures(pts, spline, lim)
    got = TP.route_from_functions(k_ref_fun, v_max_fun)
    for a in ("s", "cx", "cy", "vmax"):
        assert np.array_equal(getattr(got, a), getattr(r, a)), a
    assert got.s_total == r.s_total == s_total
    assert got.content_key() == r.content_key()
    assert np.array_equal(v_max_array, r.vmax)
    # the recovered route's own functions are the closures' (same objects underneath)
    for s in np.linspace(-3.0, s_total + 3.0, 211):
        assert got.k_ref_fun(s) == k_ref_fun(s) == r.k_ref_fun(s)
        vm, vr = got.v_max_fun(s), v_max_fun(s)
        assert (vm == vr) or (np.isnan(vm) and np.isnan(vr))
    # the same closures map to the same cached route object; bound methods map to their route
    assert TP.route_from_functions(k_ref_fun, v_max_fun) is got
    assert TP.route_from_functions(r.k_ref_fun, r.v_max_fun) is r


def test_route_recovery_rejects_other_callables(mods):
    routes, TP, W = mods
    r = W.plan_route("synth1")
    pts, spline, lim = reference_inputs(r)
    k_ref_fun, _, v_max_fun, _, _ = reference_closures(pts, spline, lim)
    with pytest.raises(TypeError):
        TP.route_from_functions(lambda s: 0.0, v_max_fun)
    with pytest.raises(TypeError):
        TP.route_from_functions(k_ref_fun, lambda s: 10.0)
    with pytest.raises(TypeError):
        TP.route_from_functions(r.k_ref_fun, W.plan_route("synth2").v_max_fun)


def test_closures_computing_something_else_are_refused(mods):
    """closures over the very objects route_from_functions recovers the route from, but returning
    something else (a scaled curvature, a modified limit), would be replaced by the device's curvature / limit
    and solve a different NLP: they are evaluated against the recovered route and raise TypeError."""
    routes, TP, W = mods
    r = W.plan_route("traj1")
    pts, spline, lim = reference_inputs(r)
    k_ref_fun, _, v_max_fun, _, _ = reference_closures(pts, spline, lim)
    cells = TP._closure(k_ref_fun)
    s_to_t, sp = cells["s_to_t"], cells["reference_path_spline"]
    vint = TP._closure(v_max_fun)["v_max_interpolator"]

    def k_scaled(s):
        t = float(s_to_t(s))
        x_spline, y_spline = sp
        return 2.0 * float((x_spline(t, 1) * y_spline(t, 2) - y_spline(t, 1) * x_spline(t, 2)) /
                           ((x_spline(t, 1) ** 2 + y_spline(t, 1) ** 2) ** 1.5 + 1e-9))

    def v_capped(s):
        return min(float(vint(s)), 5.0)
    with pytest.raises(TypeError, match="k_ref_fun"):
        TP.route_from_functions(k_scaled, v_max_fun)
    with pytest.raises(TypeError, match="v_max_fun"):
        TP.route_from_functions(k_ref_fun, v_capped)
    assert TP.route_from_functions(k_ref_fun, v_max_fun).content_key() == r.content_key()


def test_nonconstant_v_min_is_refused(mods):
    """The device rows take one v_min per chunk; the reference calls v_min_fun(s_k) per stage (:259), so a
    v_min_fun that varies over the chunk raises instead of solving a different NLP (checked before any device
    call)."""
    routes, TP, W = mods
    r = W.plan_route("synth1")
    opt = TP.TrajectoryOptimizer(horizon=6.0, N=20, dt=0.3)
    with pytest.raises(TypeError, match="v_min_fun"):
        opt.optimize(np.zeros(5), 20.0, r.s_total, r.k_ref_fun, lambda s: 0.1 * s, r.v_max_fun, False)


@pytest.mark.gpu
def test_reference_loop_with_closures_equals_optimize_full_trajectory(mods):
    """The reference's chunk loop (:481-554) restated with the reference's closures and a new
    TrajectoryOptimizer(horizon, N, dt) per chunk (:517), through the package's optimize: the plan equals
    optimize_full_trajectory(route) bit for bit, and the whole route creates one device context."""
    import __graft_entry__ as g
    g.build()
    import mpcplan
    routes, TP, W = mods
    r = W.plan_route("traj1")
    X1, U1, S1 = TP.optimize_full_trajectory(r, check=False)
    pts, spline, lim = reference_inputs(r)
    k_ref_fun, v_min_fun, v_max_fun, v_max_array, s_total = reference_closures(pts, spline, lim)
    TP.release_planners()
    TP._ROUTES.clear()
    made = mpcplan.Planner.created
    X_full, U_full, S_full = [], [], []
    current_x0 = np.array([0.0, 0.0, 0.0, 0.0, 0.0])
    remaining_dist, max_chunk_size = s_total, 20
    while remaining_dist > 0.1:
        if remaining_dist < max_chunk_size * 2:
            chunk_size, is_final_chunk = remaining_dist, True
        else:
            chunk_size, is_final_chunk = max_chunk_size, False
        current_s = current_x0[0]
        s_target = current_s + chunk_size
        avg_speed = np.mean(v_max_array[int(current_s / 5):])
        horizon = chunk_size / avg_speed * 2.0
        dt = 0.3
        N = int(np.ceil(horizon / dt))
        optimizer = TP.TrajectoryOptimizer(horizon=horizon, N=N, dt=dt)
        X, U, S = optimizer.optimize(current_x0, s_target, s_total, k_ref_fun, v_min_fun, v_max_fun, is_final_chunk)
        if not is_final_chunk:
            c = int(N / 2)
            X_full.append(X[:c + 1] if not X_full else X[1:c + 1])
            U_full.append(U[:c])
            S_full.append(S[:c])
        else:
            X_full.append(X[1:])
            U_full.append(U)
            S_full.append(S)
        current_x0 = X_full[-1][-1]
        remaining_dist = s_total - current_x0[0]
    assert mpcplan.Planner.created - made == 1
    assert np.array_equal(np.concatenate(X_full), X1)
    assert np.array_equal(np.concatenate(U_full), U1)
    assert np.array_equal(np.concatenate(S_full), S1)
    print(f"\nreference loop with the reference's closures: {len(X_full)} chunks, one context, plan == "
          f"optimize_full_trajectory's")
