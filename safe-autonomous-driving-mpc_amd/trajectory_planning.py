"""Drop-in surface of the reference's offline planner (trajectory_planning.py) on libmpcplan (MI355X).

`TrajectoryOptimizer` keeps the reference's constructor, attributes, `dynamics`, `unpack` / `pack`, `cost`
and `optimize(x0, s_target, s_total, k_ref_fun, v_min_fun, v_max_fun, is_final_chunk)` signature
(trajectory_planning.py:8-391).  The NLP is solved on the GPU (include/mpcplan.h), so the route functions
must be ones whose route can be put on the device: the closures optimize_full_trajectory itself builds
(:442-473; the route is read from their s_to_t, CubicSpline pair and v_max_interpolator) or a routes.Route's
bound k_ref_fun / v_max_fun.  An arbitrary Python callable raises TypeError.  One device context per distinct
route is shared by all optimizers (planner_for), so the reference's optimizer-per-chunk loop uploads the
route once.  `optimize_full_trajectory(route, max_chunk_size=20)` restates the chunked receding-horizon
loop (:419-559) and ends with reference_trajectory_check (:557).  Route acquisition (path_planning.py,
GraphHopper over HTTP) is out of scope: routes.py builds the route from local way-points.
"""
import math
import threading
import time

import numpy as np

import mpcplan
from sanity_checks import reference_trajectory_check

SQP_ITERS = 100


class TrajectoryOptimizer:
    """trajectory_planning.py:8-391; the solve runs on the GPU (mpcplan.Planner)."""

    def __init__(self, horizon=None, N=None, dt=None, w_y=10.0, w_s=10.0, w_u=0.1, w_slack=100.0, device=0):
        self.T = horizon
        self.N = N
        self.dt = dt
        self.w_y = float(w_y)
        self.w_s = float(w_s)
        self.w_u = float(w_u)
        self.w_slack = float(w_slack)
        self.u_min = np.array([-0.6, -5.0])
        self.u_max = np.array([0.6, 4.0])
        self.k_min = -0.8
        self.k_max = 0.8
        self.a_max = 6.0
        self.device = device
        self.last_status = None

    @staticmethod
    def dynamics(x, u, k_ref):
        """:50-89"""
        s, d, o, k, v = x
        u1, u2 = u
        denom = 1 - d * k_ref
        if abs(denom) < 1e-4:
            denom = 1e-4 * np.sign(denom) if denom != 0 else 1e-4
        s_dot = (v * np.cos(o)) / denom
        return np.array([s_dot, v * np.sin(o), v * k - s_dot * k_ref, u1, u2])

    def unpack(self, z):
        """:91-113"""
        N = self.N
        X = z[0:(N + 1) * 5].reshape(N + 1, 5)
        U = z[(N + 1) * 5:(N + 1) * 5 + N * 2].reshape(N, 2)
        return X, U, z[(N + 1) * 5 + N * 2:]

    @staticmethod
    def pack(X, U, S):
        """:115-126"""
        return np.concatenate([X.ravel(), U.ravel(), S.ravel()])

    def cost(self, z, x0, s_total):
        """:128-170"""
        X, U, S = self.unpack(z)
        denom = max(1, s_total - x0[0])
        c = 0.0
        for k in range(self.N):
            s_k, d_k, o_k, _, _ = X[k]
            c += (self.w_y * (d_k ** 2 + o_k ** 2) + self.w_s * ((s_total - s_k) / denom) ** 2
                  + self.w_u * (U[k] @ U[k]) + self.w_slack * S[k] ** 2)
        return c

    def params(self, route_vmin=0.0):
        p = mpcplan.default_params(N=int(self.N), dt=float(self.dt), w_y=self.w_y, w_s=self.w_s, w_u=self.w_u,
                                   w_slack=self.w_slack, u_min=self.u_min, u_max=self.u_max, k_min=self.k_min,
                                   k_max=self.k_max, a_max=self.a_max, v_min=float(route_vmin), sqp_iters=SQP_ITERS)
        return p

    def planner(self, route, v_min=0.0):
        """A context of its own for `route` with this optimizer's parameters (the caller closes it).  optimize()
        itself uses the route's shared context (planner_for) under the module lock instead."""
        return mpcplan.Planner(route, self.params(v_min), device=self.device)

    def optimize(self, x0, s_target, s_total, k_ref_fun, v_min_fun, v_max_fun, is_final_chunk):
        """:351-390 — returns (X [N+1,5], U [N,2], S [N]); the chunk's status is left in self.last_status.

        k_ref_fun / v_max_fun are either a routes.Route's bound methods or the closures optimize_full_trajectory
        builds (:445-473); the route is recovered from them (route_from_functions) and its device context is
        shared by every optimizer on this device (the reference makes a new optimizer per chunk, :517).
        v_min_fun must be constant over the chunk (the reference's is 0, :476-477): the device rows take one
        v_min."""
        route = route_from_functions(k_ref_fun, v_max_fun)
        if abs(float(s_total) - route.s_total) > 1e-9 * max(1.0, route.s_total):
            raise ValueError("s_total must be the route's total length")
        s0 = float(x0[0])
        vs = [float(v_min_fun(s)) for s in (s0, 0.5 * (s0 + float(s_target)), float(s_target))]
        if not (vs[0] == vs[1] == vs[2]):
            raise TypeError("v_min_fun must be constant over the chunk (the device rows take one v_min; the "
                            f"reference's is 0): got {vs} at s = x0, midpoint, s_target")
        with _LOCK:
            pl = planner_for(route, self.device)
            pl.set_params(self.params(vs[0]))
            r = pl.solve_chunks(np.asarray(x0, np.float64)[None], float(s_target), int(bool(is_final_chunk)),
                                int(self.N))
        self.last_status = int(r["status"][0])
        return r["X"][0], r["U"][0], r["S"][0]


# ---- route recovery and the per-route context cache --------------------------------------------------------

_ROUTES = {}          # ids of (s_to_t, spline pair, v_max_interpolator) -> routes.Route holding those objects
_PLANNERS = {}        # (route content key, device) -> mpcplan.Planner
MAX_CACHED_ROUTES = 8


def _closure(f):
    code, cells = getattr(f, "__code__", None), getattr(f, "__closure__", None)
    if code is None or not cells:
        return {}
    out = {}
    for name, c in zip(code.co_freevars, cells):
        try:
            out[name] = c.cell_contents
        except ValueError:          # an empty cell
            pass
    return out


def route_from_functions(k_ref_fun, v_max_fun):
    """The routes.Route that k_ref_fun / v_max_fun evaluate.

    - bound methods of one routes.Route: that route;
    - the closures of optimize_full_trajectory (trajectory_planning.py:442-473): k_ref_fun closes over s_to_t
      (interp1d linear, s_values -> t) and the reference path's CubicSpline pair, v_max_fun over
      v_max_interpolator (interp1d 'previous' over v_max_array).  The arrays are read from those objects
      (s_to_t.x, the splines' .c, v_max_interpolator.y), not refitted.
    Anything else raises TypeError: an arbitrary callable cannot be evaluated on the device."""
    import routes
    from scipy.interpolate import PPoly, interp1d
    r = getattr(k_ref_fun, "__self__", None)
    if isinstance(r, routes.Route):
        if getattr(v_max_fun, "__self__", None) is not r:
            raise TypeError("k_ref_fun and v_max_fun must be bound to the same routes.Route")
        return r
    ck, cv = _closure(k_ref_fun), _closure(v_max_fun)
    s_to_t = [v for v in ck.values() if isinstance(v, interp1d) and getattr(v, "_kind", None) == "linear"]
    spl = [v for v in ck.values() if isinstance(v, (tuple, list)) and len(v) == 2
           and all(isinstance(p, PPoly) for p in v)]
    vint = [v for v in cv.values() if isinstance(v, interp1d) and getattr(v, "_kind", None) == "previous"]
    if len(s_to_t) != 1 or len(spl) != 1 or len(vint) != 1:
        raise TypeError("the GPU planner evaluates the route on the device: pass k_ref_fun / v_max_fun of a "
                        "routes.Route, or the closures of trajectory_planning.optimize_full_trajectory (k_ref_fun "
                        "over s_to_t and the CubicSpline pair, v_max_fun over v_max_interpolator)")
    key = (id(s_to_t[0]), id(spl[0]), id(vint[0]))
    hit = _ROUTES.get(key)
    # the objects are the key while they live; a hit must still hold the very same objects
    if hit is not None and hit._s_to_t is s_to_t[0] and hit._vint is vint[0] and hit.spline[0] is spl[0][0]:
        r = hit
        _ROUTES[key] = _ROUTES.pop(key)                 # most recently used last
    else:
        r = routes.Route.from_reference_functions(s_to_t[0], spl[0], vint[0], name="reference-closures")
        while len(_ROUTES) >= MAX_CACHED_ROUTES:
            _ROUTES.pop(next(iter(_ROUTES)))
        _ROUTES[key] = r
    _verify_closures(k_ref_fun, v_max_fun, r)
    return r


_VERIFIED = {}        # (id(k_ref_fun), id(v_max_fun)) -> (k_ref_fun, v_max_fun, route) checked against the route


def _verify_closures(k_ref_fun, v_max_fun, route, samples=96):
    """The recovered route replaces the caller's closures on the device, so they must compute what the route
    computes: k_ref_fun / v_max_fun are evaluated at up to `samples` knots and interval midpoints spread over
    the route and compared bit for bit with the route's own k_ref_fun / v_max_fun (a closure over the same
    objects that returns something else -- heading, a scaled curvature, a modified limit -- raises
    TypeError).  Checked once per pair of function objects."""
    key = (id(k_ref_fun), id(v_max_fun))
    got = _VERIFIED.get(key)
    if got is not None and got[0] is k_ref_fun and got[1] is v_max_fun and got[2] is route:
        return
    s = np.asarray(route.s, np.float64)
    idx = np.unique(np.linspace(0, s.size - 2, min(samples // 2, s.size - 1)).astype(int))
    pts = np.concatenate([s[idx], 0.5 * (s[idx] + s[idx + 1]), s[-1:]])
    same = lambda a, b: (a == b) or (np.isnan(a) and np.isnan(b))
    for x in pts:
        x = float(x)
        if not same(float(k_ref_fun(x)), route.k_ref_fun(x)):
            raise TypeError(f"k_ref_fun({x}) = {float(k_ref_fun(x))!r} differs from the curvature of the route it "
                            f"closes over ({route.k_ref_fun(x)!r}): the device evaluates the reference's curvature "
                            "(trajectory_planning.py:445-459) only")
        if not same(float(v_max_fun(x)), route.v_max_fun(x)):
            raise TypeError(f"v_max_fun({x}) = {float(v_max_fun(x))!r} differs from the route's speed limit "
                            f"({route.v_max_fun(x)!r}): the device evaluates the reference's limit "
                            "(trajectory_planning.py:470-473) only")
    while len(_VERIFIED) >= MAX_CACHED_ROUTES:
        _VERIFIED.pop(next(iter(_VERIFIED)))
    _VERIFIED[key] = (k_ref_fun, v_max_fun, route)


_LOCK = threading.RLock()     # planner_for + set_params + solve of the shared contexts (not re-entrant in C)


def planner_for(route, device=0):
    """One libmpcplan context per distinct route (content hash of its device arrays) and device, shared by every
    TrajectoryOptimizer: the reference's per-chunk optimizers (:517) reuse it, so a route is uploaded once.
    At most MAX_CACHED_ROUTES contexts are kept, least recently used closed first; release_planners() closes
    all.  The contexts are shared and a C context is not re-entrant: callers hold _LOCK from here through
    their solve (TrajectoryOptimizer.optimize does)."""
    key = (route.content_key(), int(device))
    with _LOCK:
        pl = _PLANNERS.pop(key, None)
        if pl is None:
            while len(_PLANNERS) >= MAX_CACHED_ROUTES:
                _PLANNERS.pop(next(iter(_PLANNERS))).close()
            pl = mpcplan.Planner(route, device=device)
        _PLANNERS[key] = pl                              # most recently used last
        return pl


def release_planners():
    """Close every cached planner context."""
    with _LOCK:
        while _PLANNERS:
            _PLANNERS.popitem()[1].close()


def optimize_full_trajectory(route, max_chunk_size=20, max_chunks=10000, device=0, verbose=False, check=True,
                             solve_chunk=None):
    """The chunked receding-horizon planner of trajectory_planning.py:419-559 on a routes.Route (or the
    reference's GraphHopper route dict, converted by routes.from_graphhopper): returns
    (X, U, S) and runs the restated reference_trajectory_check on the result (:557).  max_chunks caps the
    loop (the reference has no cap); per-chunk statuses and horizons are left in
    `optimize_full_trajectory.statuses` / `.horizons`.  solve_chunk(x0, s_target, is_final, N) -> (X, U, S,
    status) replaces the GPU chunk solve (tests drive this loop with the CPU oracle)."""
    if isinstance(route, dict):                               # the reference's GraphHopper route object
        import routes
        route = routes.from_graphhopper(route)
    v_min_fun = lambda s: 0                                   # :476-477
    X_full, U_full, S_full, statuses, horizons = [], [], [], [], []
    current_x0 = np.array([0.0, 0.0, 0.0, 0.0, 0.0])          # :486
    s_total = route.s_total
    if verbose:
        print(f"Total Distance : {s_total:.2f} m")
    remaining = s_total
    opt = TrajectoryOptimizer(device=device)
    n = 0
    while remaining > 0.1 and n < max_chunks:                  # :491
        if remaining < max_chunk_size * 2:
            chunk_size, is_final = remaining, True
        else:
            chunk_size, is_final = max_chunk_size, False
        current_s = current_x0[0]
        s_target = current_s + chunk_size
        if verbose:
            print(f"==> Distance traveled --> {current_s:.2f} m ({current_s / s_total * 100:.2f}%)")
        avg_speed = route.avg_speed_from(current_s)            # :507
        est_time = chunk_size / avg_speed
        horizon = est_time * 2.0
        dt = 0.3
        N = int(np.ceil(horizon / dt))
        if N > mpcplan.PLAN_MAX_N:
            raise ValueError(f"chunk horizon N={N} exceeds PLAN_MAX_N={mpcplan.PLAN_MAX_N}")
        opt.T, opt.N, opt.dt = horizon, N, dt
        if solve_chunk is None:
            X, U, S = opt.optimize(current_x0, s_target, s_total, route.k_ref_fun, v_min_fun, route.v_max_fun,
                                   is_final)
            statuses.append(opt.last_status)
        else:
            X, U, S, st = solve_chunk(current_x0, s_target, is_final, N)
            statuses.append(int(st))
        horizons.append(N)
        if not is_final:                                       # :523-541
            commit = int(N / 2)
            Xs, Us, Ss = X[:commit + 1], U[:commit], S[:commit]
            X_full.append(Xs if not X_full else Xs[1:])
            U_full.append(Us)
            S_full.append(Ss)
        else:
            X_full.append(X[1:])
            U_full.append(U)
            S_full.append(S)
        current_x0 = X_full[-1][-1]                            # :548
        remaining = s_total - current_x0[0]
        n += 1
    X_final = np.concatenate(X_full, axis=0)
    U_final = np.concatenate(U_full, axis=0)
    S_final = np.concatenate(S_full, axis=0)
    optimize_full_trajectory.statuses = statuses
    optimize_full_trajectory.horizons = horizons
    if check:
        reference_trajectory_check(TrajectoryOptimizer(device=device), X_final, U_final, S_final, s_total)
    return X_final, U_final, S_final


def _commit(pieces, X, U, S, n, fin):
    """:523-541: the first int(N/2) intervals of a non-final chunk, the whole final chunk; returns the next start."""
    if not fin:
        c = int(n / 2)
        pieces.append((X[:c + 1] if not pieces else X[1:c + 1], U[:c], S[:c]))
    else:
        pieces.append((X[1:], U, S))
    return pieces[-1][0][-1]


def _device_loop(route, starts, max_chunk_size, max_chunks, device, pieces, statuses, horizons, opt, seg=64,
                 timing=None):
    """optimize_full_trajectory_batch's chunk loop as plan_optimize_device launches: every plan advances on its
    own wavefront, up to `seg` chunks per launch (plans still running continue from their last start).

    One launch size (the longest final chunk's horizon) for every plan: the fleet lasts as long as its slowest
    plan, whose chunks run back to back on one wavefront, so sizing the intermediate chunks' launches for their
    own (shorter) horizon to raise the residency, then solving the longer final chunks in launches of their
    own, measured slower (0.58-0.63 s against 0.49-0.53 s for 1024 trajectory1 plans): the
    slowest final chunk then starts only after every plan's intermediate chunks."""
    s_total = route.s_total
    vm = np.asarray(route.vmax, np.float64)
    avg = np.array([float(np.mean(vm[i:])) for i in range(vm.size)])     # route.avg_speed_from(5 i), :507
    nb = int(np.max(np.ceil(2.0 * max_chunk_size / avg * 2.0 / 0.3)))
    Nmax = min(max(nb, 1), mpcplan.PLAN_MAX_N)
    opt.N, opt.dt = Nmax, 0.3
    pl = mpcplan.Planner(route, opt.params(0.0), device=device)
    cur = np.asarray(starts, np.float64).copy()
    used = np.zeros(cur.shape[0], int)

    def commit(b, X, U, S, n, fin, status):
        statuses[b].append(int(status))
        horizons[b].append(int(n))
        cur[b] = _commit(pieces[b], X[:n + 1], U[:n], S[:n], n, fin)
        used[b] += 1

    def loop(act, Nm):
        """loop launches sized for Nm over the plans act"""
        while act.size:
            # slots per plan: enough for the longest remaining distance at about half a chunk committed per
            # intermediate chunk (plans that use them all continue in the next launch)
            est = int(np.ceil(float(np.max(s_total - cur[act, 0])) / (0.5 * max_chunk_size))) + 4
            C_ = int(min(seg, est, max_chunks - used[act].min()))
            if C_ <= 0:
                break
            # longest remaining distance first: a launch lasts as long as its slowest wavefront's chain, and
            # with more plans than resident slots the plans dispatched last start late (results are per plan)
            act = act[np.argsort(-(s_total - cur[act, 0]), kind="stable")]
            t0 = time.perf_counter()
            r = pl.optimize_device(cur[act], max_chunk_size, C_, avg, Nm, device=device)
            if timing is not None:
                timing.setdefault("launches", []).append({"kind": "loop", "Nmax": int(Nm), "plans": int(act.size),
                                                          "slots": C_, "seconds": time.perf_counter() - t0})
            nxt = []
            for i, b in enumerate(act):
                nc = int(r["nchunks"][i])
                for j in range(min(abs(nc) - (1 if nc < 0 else 0), max_chunks - used[b])):
                    commit(b, r["X"][i, j], r["U"][i, j], r["S"][i, j], int(r["N"][i, j]), int(r["is_final"][i, j]),
                           r["status"][i, j])
                if used[b] >= max_chunks or s_total - cur[b, 0] <= 0.1:
                    continue
                if nc < 0:
                    raise ValueError(f"chunk horizon of plan {b} exceeds PLAN_MAX_N={mpcplan.PLAN_MAX_N} (or its "
                                     f"start lies past the end of the route)")
                if nc == C_:
                    nxt.append(b)
            act = np.array(nxt, dtype=int)

    try:
        loop(np.arange(cur.shape[0]), Nmax)
    finally:
        pl.close()


def optimize_full_trajectory_batch(route, starts, max_chunk_size=20, max_chunks=10000, device=0, solve_chunks=None,
                                   device_loop=True):
    """The chunk loop of optimize_full_trajectory (trajectory_planning.py:491-548) for B plans on one route at
    once, from B start states (e.g. a fleet re-planning from where each vehicle is): every round solves the
    current chunk of each unfinished plan in one batched call, each chunk with its own horizon (the
    reference's N rule) and its own final-chunk flag.  Plan b follows exactly the chunk sequence
    optimize_full_trajectory would run from starts[b] (start (0, 0, 0, 0, 0) = the reference's).

    Returns (plans, summary): plans[b] = (X, U, S); summary[b] = sanity_checks.plan_check_summary of the plan
    plus 'statuses' and 'horizons' of its chunks.  solve_chunks(x0 [n,5], s_target [n], is_final [n], N [n])
    -> dict(X, U, S, status) replaces the GPU batch (tests drive this loop with the CPU oracle).
    device_loop (GPU, the default): the whole loop runs on the device (plan_optimize_device), each plan on its
    own wavefront with no barrier across plans; False: one batched chunk launch per round, the host loop
    below.  Both give the same plans bit for bit (the same chunk solver on the same chunk inputs)."""
    from sanity_checks import plan_check_summary
    if isinstance(route, dict):
        import routes
        route = routes.from_graphhopper(route)
    t_start = time.perf_counter()
    timing = {}
    starts = np.atleast_2d(np.asarray(starts, np.float64))
    B = starts.shape[0]
    s_total = route.s_total
    cur = starts.copy()
    pieces = [[] for _ in range(B)]
    statuses = [[] for _ in range(B)]
    horizons = [[] for _ in range(B)]
    done = np.zeros(B, bool)
    opt = TrajectoryOptimizer(device=device)
    pl = None
    if solve_chunks is None and device_loop:
        _device_loop(route, starts, max_chunk_size, max_chunks, device, pieces, statuses, horizons, opt,
                     timing=timing)
        max_chunks = 0                                                 # the host loop below does not run
    for _ in range(max_chunks):
        act = np.flatnonzero(~done & (s_total - cur[:, 0] > 0.1))
        done[~done & (s_total - cur[:, 0] <= 0.1)] = True
        if act.size == 0:
            break
        rem = s_total - cur[act, 0]
        fin = (rem < max_chunk_size * 2).astype(np.int32)
        size = np.where(fin == 1, rem, max_chunk_size)
        st = cur[act, 0] + size
        N = np.array([int(np.ceil(size[i] / route.avg_speed_from(cur[b, 0]) * 2.0 / 0.3))
                      for i, b in enumerate(act)], np.int32)
        if N.max() > mpcplan.PLAN_MAX_N:
            raise ValueError(f"chunk horizon N={N.max()} exceeds PLAN_MAX_N={mpcplan.PLAN_MAX_N}")
        if solve_chunks is None:
            if pl is None:
                opt.N, opt.dt = int(N.max()), 0.3
                pl = mpcplan.Planner(route, opt.params(0.0), device=device)
            r = pl.solve_chunks(cur[act], st, fin, N)
        else:
            r = solve_chunks(cur[act], st, fin, N)
        for i, b in enumerate(act):
            n = int(N[i])
            X, U, S = r["X"][i, :n + 1], r["U"][i, :n], r["S"][i, :n]
            statuses[b].append(int(r["status"][i]))
            horizons[b].append(n)
            cur[b] = _commit(pieces[b], X, U, S, n, fin[i])
    if pl is not None:
        pl.close()
    timing["loop_seconds"] = time.perf_counter() - t_start
    plans, summary = [], []
    for b in range(B):
        if not pieces[b]:
            plans.append((starts[b][None], np.zeros((0, 2)), np.zeros(0)))
            summary.append({"passed": False, "statuses": [], "horizons": []})
            continue
        X = np.concatenate([p[0] for p in pieces[b]])
        U = np.concatenate([p[1] for p in pieces[b]])
        S = np.concatenate([p[2] for p in pieces[b]])
        plans.append((X, U, S))
        q = plan_check_summary(opt.u_min, opt.u_max, X, U, S, s_total)
        q["statuses"], q["horizons"] = statuses[b], horizons[b]
        summary.append(q)
    timing["seconds"] = time.perf_counter() - t_start
    optimize_full_trajectory_batch.timing = timing
    return plans, summary
