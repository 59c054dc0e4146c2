"""Routes for the offline planner: the reference path that optimize_full_trajectory builds
(trajectory_planning.py:393-477) as the plain arrays libmpcplan takes (include/mpcplan.h, plan_create).

The reference gets its route from the GraphHopper HTTP API and projects it with pymap3d
(path_planning.py:19-107); both are network/third-party steps outside this build's scope.  Everything after
the projection is restated here from the source:
  - densification of the way-points to <= 5 m (add_extra_points, get_reference_path: path_planning.py:123-143,
    :182-195);
  - the parametric CubicSpline x(t), y(t) over t = 0..M-1 (create_spline, :146-162; scipy's CubicSpline, the
    same library and default not-a-knot end conditions, so the coefficients are the reference's);
  - s_values, the cumulative chord length (unpack_reference_path, trajectory_planning.py:411-414);
  - the speed-limit array over the detailed points (get_speed_limits, path_planning.py:203-243, 30 km/h for
    missing values; trajectory_planning.py:464-467).
Inputs without the network: `from_waypoints` (local x, y way-points + GraphHopper-style max_speed intervals),
`from_trajectory` (the global line of a committed trajectory, the way trajectory_loader.py:32-62 rebuilds it)
and `synthetic` (a documented generator: curvature profile + speed-limit bands).
"""
import math

import numpy as np
from scipy.interpolate import CubicSpline, PPoly, interp1d


def _is_interp1d(f, kind):
    return isinstance(f, interp1d) and getattr(f, "_kind", None) == kind


def add_extra_points(p1, p2, threshold=5.0):
    """path_planning.add_extra_points (:123-143): recursive midpoints while the gap exceeds 5 m."""
    if threshold < math.dist(p1, p2):
        mid = ((p1[0] + p2[0]) / 2, (p1[1] + p2[1]) / 2)
        return add_extra_points(p1, mid, threshold) + [mid] + add_extra_points(mid, p2, threshold)
    return []


def densify(points):
    """get_reference_path (path_planning.py:182-195): original points with the extra points between them."""
    out = []
    for i in range(len(points) - 1):
        out.append(tuple(points[i]))
        out += add_extra_points(tuple(points[i]), tuple(points[i + 1]))
    out.append(tuple(points[-1]))
    return out


class Route:
    """A planner route: detailed way-points (M, 2) in local metres and the speed limit at each (m/s)."""

    def __init__(self, detailed_points, v_max_points, name="route"):
        pts = np.asarray(detailed_points, np.float64)
        if pts.ndim != 2 or pts.shape[1] != 2 or pts.shape[0] < 3:
            raise ValueError("need at least 3 detailed way-points (M, 2)")
        t = np.arange(len(pts))
        spline = (CubicSpline(t, pts[:, 0]), CubicSpline(t, pts[:, 1]))              # create_spline
        dist = np.sqrt(np.diff(pts[:, 0]) ** 2 + np.diff(pts[:, 1]) ** 2)              # :412
        s = np.concatenate([[0], np.cumsum(dist)])                                     # :413
        self._set(name, pts, spline, s, v_max_points)

    def _set(self, name, pts, spline, s, v_max_points, s_to_t=None, vint=None):
        self.name = name
        self.points = pts
        self.spline = spline
        self.s = np.ascontiguousarray(s, np.float64)
        if self.s.ndim != 1 or self.s.size < 3 or not (np.diff(self.s) > 0).all():
            raise ValueError("consecutive way-points must be distinct (s strictly increasing, at least 3 points)")
        self.s_total = float(self.s[-1])                                               # :414
        self.cx = np.ascontiguousarray(spline[0].c.T, np.float64)                     # [M-1][4], cubic first
        self.cy = np.ascontiguousarray(spline[1].c.T, np.float64)
        if self.cx.shape != (self.s.size - 1, 4) or self.cy.shape != self.cx.shape:
            raise ValueError("the spline must have one cubic piece per way-point interval")
        self.vmax = np.ascontiguousarray(v_max_points, np.float64)
        if self.vmax.shape != self.s.shape:
            raise ValueError("one speed limit per detailed way-point")
        # the reference's own route functions (trajectory_planning.py:440-473), for checks and the drop-in
        M = self.s.size
        self._s_to_t = s_to_t if s_to_t is not None else interp1d(self.s, np.linspace(0.0, M - 1, M), kind="linear",
                                                                   fill_value="extrapolate")
        self._vint = vint if vint is not None else interp1d(self.s, self.vmax, kind="previous",
                                                            fill_value="extrapolate")

    @classmethod
    def from_reference_functions(cls, s_to_t, spline, v_max_interpolator, name="route"):
        """The route behind the closures optimize_full_trajectory builds (trajectory_planning.py:440-473): s_to_t
        (interp1d linear, s_values -> t_values), the CubicSpline pair of the reference path, and
        v_max_interpolator (interp1d 'previous' over the speed-limit array).  The arrays are taken from those
        objects as they are (no refit), so the device route is the reference's own spline and limits."""
        if not (_is_interp1d(s_to_t, "linear") and _is_interp1d(v_max_interpolator, "previous")):
            raise TypeError("s_to_t must be interp1d(kind='linear') and v_max_interpolator interp1d(kind='previous')")
        s = np.asarray(s_to_t.x, np.float64)
        M = s.size
        if not np.array_equal(np.asarray(s_to_t.y, np.float64), np.linspace(0.0, M - 1, M)):
            raise ValueError("s_to_t must map s_values to t = 0 .. M-1 (trajectory_planning.py:440-442)")
        if not np.array_equal(np.asarray(v_max_interpolator.x, np.float64), s):
            raise ValueError("v_max_interpolator and s_to_t are over different s_values")
        if len(spline) != 2 or not all(isinstance(p, PPoly) for p in spline):
            raise TypeError("the reference path spline must be a pair of scipy CubicSpline objects")
        for p in spline:
            if p.c.shape != (4, M - 1) or not np.array_equal(np.asarray(p.x, np.float64), np.arange(M, dtype=np.float64)):
                raise ValueError("the spline pair must be cubic over t = 0 .. M-1 (path_planning.create_spline)")
        pts = np.column_stack([np.append(spline[0].c[3], spline[0](M - 1.0)), np.append(spline[1].c[3], spline[1](M - 1.0))])
        r = cls.__new__(cls)
        r._set(name, pts, tuple(spline), s, np.asarray(v_max_interpolator.y, np.float64), s_to_t, v_max_interpolator)
        return r

    def content_key(self):
        """sha256 over the arrays the device holds (s, cx, cy, vmax): equal keys = the same device route."""
        k = getattr(self, "_key", None)
        if k is None:
            import hashlib
            h = hashlib.sha256()
            for a in (self.s, self.cx, self.cy, self.vmax):
                h.update(np.ascontiguousarray(a, np.float64).tobytes())
            k = self._key = h.hexdigest()
        return k

    @property
    def M(self):
        return len(self.s)

    def k_ref_fun(self, s):
        """trajectory_planning.py:445-459 (scipy evaluation, as the reference)."""
        t = float(self._s_to_t(s))
        xs, ys = self.spline
        x_dt, y_dt, x_ddt, y_ddt = xs(t, 1), ys(t, 1), xs(t, 2), ys(t, 2)
        denom = (x_dt ** 2 + y_dt ** 2) ** 1.5 + 1e-9
        if denom < 1e-8:
            denom = 1e-8
        return float((x_dt * y_ddt - y_dt * x_ddt) / denom)

    def v_max_fun(self, s):
        """trajectory_planning.py:470-473 (NaN below the first knot, as interp1d 'previous' gives)."""
        return float(self._vint(s))

    def avg_speed_from(self, current_s):
        """np.mean(v_max_array[int(current_s / 5):]) of optimize_full_trajectory (:507)."""
        return float(np.mean(self.vmax[int(current_s / 5):]))


def speed_limit_array(original_points, detailed_points, max_speed):
    """get_speed_limits (path_planning.py:203-243) + trajectory_planning.py:464-467: the limit (m/s) at every
    detailed point; max_speed = [(start_idx, end_idx, km/h or None)] over the ORIGINAL points."""
    det = [tuple(p) for p in detailed_points]
    v = np.ones(len(det))
    for start, end, kmh in max_speed:
        kmh = 30.0 if kmh is None else kmh
        i0 = det.index(tuple(original_points[start]))
        i1 = det.index(tuple(original_points[end]))
        v[i0:i1 + 1] = kmh / 3.6
    return v


def from_waypoints(points, max_speed, name="route"):
    """A route from local way-points (the output of path_planning.global2local) and GraphHopper-style
    max_speed intervals over them."""
    pts = [tuple(map(float, p)) for p in points]
    det = densify(pts)
    return Route(det, speed_limit_array(pts, det, max_speed), name)


# WGS84 (pymap3d's default ellipsoid, which path_planning.global2local uses through geodetic2enu)
_WGS84_A = 6378137.0
_WGS84_F = 1.0 / 298.257223563


def _geodetic2ecef(lat, lon, h):
    e2 = _WGS84_F * (2.0 - _WGS84_F)
    la, lo = np.radians(lat), np.radians(lon)
    n = _WGS84_A / np.sqrt(1.0 - e2 * np.sin(la) ** 2)
    return ((n + h) * np.cos(la) * np.cos(lo), (n + h) * np.cos(la) * np.sin(lo), (n * (1.0 - e2) + h) * np.sin(la))


def global2local(points):
    """path_planning.global2local (:91-108): (lon, lat) way-points to local east/north metres with the first
    point as origin (geodetic -> ECEF -> ENU on WGS84, altitude 0; pymap3d is not installed here, so the
    projection is restated)."""
    lon0, lat0 = points[0]
    x0, y0, z0 = _geodetic2ecef(lat0, lon0, 0.0)
    la0, lo0 = np.radians(lat0), np.radians(lon0)
    out = []
    for lon, lat in points:
        x, y, z = _geodetic2ecef(lat, lon, 0.0)
        dx, dy, dz = x - x0, y - y0, z - z0
        east = -np.sin(lo0) * dx + np.cos(lo0) * dy
        north = -np.sin(la0) * np.cos(lo0) * dx - np.sin(la0) * np.sin(lo0) * dy + np.cos(la0) * dz
        out.append((float(east), float(north)))
    return out


def from_graphhopper(route, name="route"):
    """The route dict path_planning.get_route returns (:50-88: 'points' as (lon, lat), 'max_speed' details
    [[start, end, km/h or None]] over them), projected and densified as get_path_and_speed_limits does
    (:170-262).  Fetching it (GraphHopper over HTTP) stays out of scope."""
    pts = global2local([(float(lon), float(lat)) for lon, lat in route["points"]])
    return from_waypoints(pts, [tuple(iv) for iv in route.get("max_speed", [])], name)


def global_line(X):
    """The global (x, y) line of a committed trajectory, integrated like trajectory_loader.py:32-62."""
    s = X[:, 0].copy()
    for i in range(1, len(s)):                          # monotone fix, trajectory_loader.py:26-30
        if s[i] <= s[i - 1]:
            s[i] = s[i - 1] + 1e-5
    x, y, psi = [0.0], [0.0], [0.0]
    for i in range(1, len(s)):
        ds = s[i] - s[i - 1]
        pn = psi[-1] + X[i - 1, 3] * ds
        pa = (psi[-1] + pn) / 2.0
        x.append(x[-1] + np.cos(pa) * ds)
        y.append(y[-1] + np.sin(pa) * ds)
        psi.append(pn)
    return np.column_stack([x, y])


def from_trajectory(X, bands=((0.0, 50.0),), min_gap=1.0, name="route"):
    """Synthetic input of realistic geometry: the global line of a committed planner output as way-points
    (points closer than min_gap dropped), densified to <= 5 m, with speed-limit bands: (fraction of the
    way-points where the band starts, km/h)."""
    g = global_line(np.asarray(X, np.float64))
    keep = [0]
    for i in range(1, len(g)):
        if np.hypot(*(g[i] - g[keep[-1]])) >= min_gap:
            keep.append(i)
    pts = [tuple(map(float, g[i])) for i in keep]
    n = len(pts)
    iv = []
    for b, (frac, kmh) in enumerate(bands):
        start = int(frac * (n - 1))
        end = int(bands[b + 1][0] * (n - 1)) if b + 1 < len(bands) else n - 1
        iv.append((start, end, kmh))
    return from_waypoints(pts, iv, name)


def synthetic(length=1500.0, seed=0, spacing=12.0, name=None):
    """Documented synthetic route: way-points every `spacing` m along a heading that follows a random
    piecewise-constant curvature profile (straights, and arcs of radius 15-200 m, turns up to 90 degrees),
    with speed-limit bands of 30 / 40 / 50 km/h changing every 150-500 m (numpy default_rng(seed))."""
    rng = np.random.default_rng(seed)
    pts, psi, s = [(0.0, 0.0)], 0.0, 0.0
    seg_k, seg_left = 0.0, 0.0
    while s < length:
        if seg_left <= 0.0:
            if rng.uniform() < 0.45:
                seg_k, seg_left = 0.0, rng.uniform(40.0, 200.0)
            else:
                radius = rng.uniform(15.0, 200.0)
                turn = rng.uniform(0.2, np.pi / 2)
                seg_k, seg_left = rng.choice([-1.0, 1.0]) / radius, turn * radius
        step = min(spacing, seg_left) if seg_left > 1.0 else spacing
        psi_new = psi + seg_k * step
        pa = 0.5 * (psi + psi_new)
        x, y = pts[-1]
        pts.append((x + np.cos(pa) * step, y + np.sin(pa) * step))
        psi, s, seg_left = psi_new, s + step, seg_left - step
    n = len(pts)
    iv, i = [], 0
    while i < n - 1:
        j = min(n - 1, i + int(rng.uniform(150.0, 500.0) / spacing))
        iv.append((i, j, float(rng.choice([30.0, 40.0, 50.0]))))
        i = j
    return from_waypoints(pts, iv, name or f"synthetic{seed}")
