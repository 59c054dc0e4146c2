"""Golden-vector capture for the tracking-QP hot path.

RUN ONLY IN THE BUILD CONTAINER (needs /root/reference, read-only).  Never shipped
to / executed on the GPU box: the fixtures it writes (tests/golden/*.npz) are the
only thing the tests read.

What it pins:
  interp      TrajectoryLoader.get_state / get_control     trajectory_loader.py:86-102
  model       TrajectoryTracker.predict / cost / constraints  trajectory_tracking.py:87-211
  warmstart   the u_init that solve() hands to minimize      trajectory_tracking.py:224-246,254
  qp          QP(ubar) = Gauss-Newton linearisation of predict/cost/constraints about
              the warm start, validated here against the reference's
              own functions (bit-identical nominal rollout, cost/constraint values at ubar,
              central-FD Jacobians), solved tightly by scipy SLSQP + an exact active-set
              polish (independent of the build's PDIP), hard and elastic (L1) variants.
  solve       reference solve() outputs (behavioural check)  trajectory_tracking.py:213-263
  closedloop  run_simulation histories                       trajectory_tracking.py:377-443

The trajectories are also converted (data only) to ../../safe-autonomous-driving-mpc_amd/data.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_goldens.py [--only NAME]
"""
import argparse
import io
import json
import os
import platform
import sys
import time
import contextlib

sys.dont_write_bytecode = True
REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
PKG_DATA = os.path.join(REPO, "safe-autonomous-driving-mpc_amd", "data")

import numpy as np
import scipy
from scipy.optimize import minimize as sp_minimize

sys.path.insert(0, REF)
import trajectory_loader as RL   # noqa: E402  (reference, read-only)
import trajectory_tracking as RT  # noqa: E402
import sanity_checks as RS        # noqa: E402

VERSIONS = dict(python=platform.python_version(), numpy=np.__version__, scipy=scipy.__version__)
RHO_DEFAULT = 1.0e5   # elastic L1 penalty, must equal mpc_params.elastic_rho default

TRAJ = {i: os.path.join(REF, "trajectories", f"trajectory{i}.json") for i in (1, 2, 3)}
_LOADERS = {}


def loader(i):
    if i not in _LOADERS:
        _LOADERS[i] = RL.TrajectoryLoader(TRAJ[i])
    return _LOADERS[i]


def tracker(i, N):
    t = RT.TrajectoryTracker(loader(i))
    t.N = N
    return t


def save(name, **arrs):
    path = os.path.join(HERE, name + ".npz")
    meta = dict(VERSIONS)
    meta["generator"] = "tests/golden/make_goldens.py"
    arrs["meta_json"] = np.array(json.dumps(meta))
    np.savez_compressed(path, **arrs)
    print(f"wrote {path}  ({os.path.getsize(path)/1024:.1f} KiB)")


# ----------------------------------------------------------------------------------------
# data conversion (trajectory JSON -> npz, verbatim float64 arrays)
# ----------------------------------------------------------------------------------------
def convert_trajectories():
    os.makedirs(PKG_DATA, exist_ok=True)
    for i, p in TRAJ.items():
        with open(p) as f:
            d = json.load(f)
        out = os.path.join(PKG_DATA, f"trajectory{i}.npz")
        np.savez_compressed(out, X=np.asarray(d["X"], np.float64), U=np.asarray(d["U"], np.float64),
                            S=np.asarray(d["S"], np.float64))
        print("wrote", out)


# ----------------------------------------------------------------------------------------
# 1. interpolation
# ----------------------------------------------------------------------------------------
def gen_interp():
    out = {}
    rng = np.random.default_rng(11)
    for i in (1, 2, 3):
        ld = loader(i)
        s_kn = ld.interp_d.x
        smax = ld.s_max
        knots = s_kn if len(s_kn) < 200 else s_kn[rng.choice(len(s_kn), 200, replace=False)]
        su = ld.interp_u1.x
        mids = 0.5 * (s_kn[:-1] + s_kn[1:])
        mids = mids if len(mids) < 150 else mids[rng.choice(len(mids), 150, replace=False)]
        extra = np.array([-5.0, -1e-3, 0.0, 1e-12, smax, smax - 1e-9, smax + 1e-9, smax + 3.0,
                          su[-1], su[-1] + 0.5 * (smax - su[-1]), np.nextafter(smax, 0)])
        rnd = rng.uniform(-2.0, smax + 2.0, 300)
        S = np.concatenate([knots, mids, extra, rnd])
        st = np.array([ld.get_state(float(s)) for s in S])
        ct = np.array([ld.get_control(float(s)) for s in S])
        out[f"t{i}_s"] = S
        out[f"t{i}_state"] = st
        out[f"t{i}_control"] = ct
    save("interp_golden", **out)


def gen_pose():
    """TrajectoryLoader global geometry (trajectory_loader.py:32-62) and get_global_pose
    (:104-116) on the reference's own trajectories: knots, mid-segments, s < 0, s >= s_max."""
    out = {}
    rng = np.random.default_rng(12)
    for i in (1, 2, 3):
        ld = loader(i)
        smax = ld.s_max
        S = np.concatenate([rng.uniform(-3.0, smax + 3.0, 250), ld.interp_d.x[:40], [smax, smax + 1.0, -1.0, 0.0]])
        D = rng.uniform(-1.5, 1.5, S.size)
        P = np.array([ld.get_global_pose(float(s), float(d)) for s, d in zip(S, D)])
        out[f"t{i}_s"] = S
        out[f"t{i}_d"] = D
        out[f"t{i}_pose"] = P
        out[f"t{i}_gx"] = np.asarray(ld.global_x)
        out[f"t{i}_gy"] = np.asarray(ld.global_y)
        out[f"t{i}_gpsi"] = np.asarray(ld.global_psi)
    save("pose_golden", **out)


# ----------------------------------------------------------------------------------------
# instance generators
# ----------------------------------------------------------------------------------------
def draw_x0(ld, rng, s_lo=0.0, s_hi_frac=0.8):
    s0 = rng.uniform(s_lo, s_hi_frac * ld.s_max)
    ref = ld.get_state(s0)
    return np.array([s0, ref[1] + rng.normal(0, 0.05), ref[2] + rng.normal(0, 0.01), ref[3],
                     max(0.5, ref[4] + rng.normal(0, 0.5))])


def draw_obstacles(kind, x0, rng):
    s0 = x0[0]
    if kind == 0:
        return []
    if kind == "fsm":   # car and/or red light snapshot, like ObstaclesFSM (trajectory_tracking.py:330-374)
        obs = []
        if rng.uniform() < 0.7:
            obs.append({"s": s0 + rng.uniform(8.0, 70.0), "v": 4.0, "type": "car"})
        if rng.uniform() < 0.5:
            obs.append({"s": s0 + rng.uniform(6.0, 99.0), "v": 0.0, "type": "light"})
        return obs
    n = int(kind)
    return [{"s": s0 + 25.0 + 50.0 * i + rng.uniform(0, 10), "v": rng.uniform(2, 10), "type": "car"}
            for i in range(n)]


# ----------------------------------------------------------------------------------------
# 2. model golden: predict / cost / constraints
# ----------------------------------------------------------------------------------------
def gen_model():
    rng = np.random.default_rng(22)
    cases = []
    for (ti, N, ok) in [(1, 5, 0), (1, 10, 0), (1, 20, 1), (2, 20, "fsm"), (2, 10, 2), (3, 30, 1),
                        (3, 40, 8), (1, 40, 0), (3, 20, 2), (2, 30, 8)]:
        for rep in range(6):
            ld = loader(ti)
            tr = tracker(ti, N)
            x0 = draw_x0(ld, rng, s_hi_frac=1.02 if rep == 5 else 0.8)
            if rep == 4:
                x0[0] = ld.s_max - rng.uniform(0, 3)      # horizon runs past s_max
            obs = draw_obstacles(ok, x0, rng)
            U = np.column_stack([rng.uniform(-0.6, 0.6, N), rng.uniform(-5, 4, N)]).ravel()
            X = tr.predict(x0, U)
            c = tr.cost(U, x0)
            g = tr.constraints(x0, obs)["fun"](U)
            cases.append(dict(traj=ti, N=N, x0=x0, obs=np.array([[o["s"], o["v"]] for o in obs]).reshape(-1, 2),
                              U=U, X=X, cost=c, cons=g))
    out = {"n": np.array(len(cases))}
    for j, c in enumerate(cases):
        for k, v in c.items():
            out[f"c{j}_{k}"] = np.asarray(v)
    save("model_golden", **out)


# ----------------------------------------------------------------------------------------
# 3. warm start golden (captures the exact u_init solve() passes to minimize)
# ----------------------------------------------------------------------------------------
class _Captured(Exception):
    pass


def capture_warmstart(tr, x0, obs):
    box = {}

    def stub(fun, x0_, args=(), method=None, bounds=None, constraints=None, options=None):
        box["u"] = np.array(x0_, dtype=np.float64).copy()
        raise _Captured()
    orig = RT.minimize
    RT.minimize = stub
    try:
        tr.solve(x0, obs)
    except _Captured:
        pass
    finally:
        RT.minimize = orig
    return box["u"]


def gen_warmstart():
    rng = np.random.default_rng(33)
    cases = []
    for (ti, N, ok) in [(1, 5, 0), (1, 20, 0), (2, 20, "fsm"), (2, 10, 1), (3, 30, 2), (3, 40, 8),
                        (1, 10, 1), (2, 40, "fsm")]:
        for rep in range(8):
            ld = loader(ti)
            tr = tracker(ti, N)
            x0 = draw_x0(ld, rng)
            if rep == 6:
                x0[0] = ld.s_max - rng.uniform(0, 4)
            if rep == 7:
                x0[4] = rng.uniform(0.0, 0.2)
            obs = draw_obstacles(ok, x0, rng)
            if rep == 5 and ok != 0:     # obstacle just at the 40 m brake threshold
                obs = [{"s": x0[0] + 40.0 + x0[4] * 0.2 * 2 + 1e-9, "v": 1.0, "type": "car"}]
            u = capture_warmstart(tr, x0, obs)
            cases.append(dict(traj=ti, N=N, x0=x0, obs=np.array([[o["s"], o["v"]] for o in obs]).reshape(-1, 2),
                              ubar=u))
    out = {"n": np.array(len(cases))}
    for j, c in enumerate(cases):
        for k, v in c.items():
            out[f"c{j}_{k}"] = np.asarray(v)
    save("warmstart_golden", **out)


# ----------------------------------------------------------------------------------------
# 4. QP(ubar) golden
# ----------------------------------------------------------------------------------------
def seg_slope(interp, s):
    """Slope of scipy interp1d 'linear' at s (searchsorted-left, clip [1, T-1]),
    scipy/interpolate/_interpolate.py:457-483."""
    x, y = interp.x, interp.y
    i = int(np.searchsorted(x, s))
    i = min(max(i, 1), len(x) - 1)
    return (y[i] - y[i - 1]) / (x[i] - x[i - 1])


def build_qp(tr, ld, x0, obs, ubar, gn=True):
    """Appendix B of SURVEY.md, in deviation coordinates dU = U - ubar.

    Returns dict with H, f, c0 (objective 0.5 dU'H dU + f'dU + c0), rows A (m x n),
    lo/hi (+-inf where absent), soft flags, box lo/hi, plus intermediate data."""
    N, dt = tr.N, tr.dt
    n = 2 * N
    Xbar = tr.predict(x0, ubar)                       # nominal rollout == reference predict
    smax = ld.s_max
    kap = np.zeros(N)
    dkap = np.zeros(N)
    G = np.zeros((N + 1, 5, n))
    for k in range(N):
        s, d, o, kk, v = Xbar[k]
        kap[k] = ld.get_state(s)[3]
        dkap[k] = 0.0 if (s >= smax or not gn) else seg_slope(ld.interp_k, s)
        J = np.zeros((5, 5))
        J[0, 4] = 1.0
        J[1, 2] = v
        J[1, 4] = o
        J[2, 3] = v
        J[2, 4] = kk - kap[k]
        J[2, 0] = -v * dkap[k]
        A = np.eye(5) + dt * J
        G[k + 1] = A @ G[k]
        G[k + 1, 3, 2 * k] += dt
        G[k + 1, 4, 2 * k + 1] += dt
    w = np.array([tr.w_d, tr.w_o, tr.w_v])
    H = np.zeros((n, n))
    f = np.zeros(n)
    c0 = 0.0
    refs = np.zeros((N + 1, 3))
    drefs = np.zeros((N + 1, 3))
    for k in range(1, N + 1):
        s = Xbar[k, 0]
        xr = ld.get_state(s)
        refs[k] = [xr[1], xr[2], xr[4]]
        if s < smax and gn:
            drefs[k] = [seg_slope(ld.interp_d, s), seg_slope(ld.interp_o, s), seg_slope(ld.interp_v, s)]
        for j, (idx, wj) in enumerate(zip((1, 2, 4), w)):
            m = np.zeros(5)
            m[idx] = 1.0
            m[0] = -drefs[k, j]
            r0 = Xbar[k, idx] - refs[k, j]
            Mrow = m @ G[k]
            H += 2 * wj * np.outer(Mrow, Mrow)
            f += 2 * wj * r0 * Mrow
            c0 += wj * r0 * r0
    wu = np.tile([tr.w_u1, tr.w_u2], N)
    H += 2 * np.diag(wu)
    f += 2 * wu * ubar
    c0 += float(np.sum(wu * ubar * ubar))
    sl = tr.lane_width / 2.0 - tr.vehicle_radius - tr.safe_lane_margin
    L = tr.wheelbase
    rows, lo, hi = [], [], []
    for k in range(1, N + 1):
        s, d, o, kk, v = Xbar[k]
        Gk = G[k]
        for c in (0.0, L / 2.0, L):
            p = np.zeros(5)
            p[1] = 1.0
            p[2] = c
            pv = d + c * o
            rows.append(p @ Gk)
            lo.append(-sl - pv)
            hi.append(sl - pv)
        if len(obs):
            shat = min(ob["s"] + ob["v"] * (k * dt) for ob in obs)
            rows.append(Gk[0])
            lo.append(-np.inf)
            hi.append(shat - tr.obstacle_safety_distance - s)
            rows.append(Gk[0] + tr.max_time_2_obs * Gk[4])
            lo.append(-np.inf)
            hi.append(shat - s - tr.max_time_2_obs * v)
        rows.append(Gk[4])
        lo.append(-v)
        hi.append(np.inf)
    A = np.array(rows)
    lo = np.array(lo)
    hi = np.array(hi)
    umin = np.tile(tr.u_min, N)
    umax = np.tile(tr.u_max, N)
    return dict(H=H, f=f, c0=c0, A=A, lo=lo, hi=hi, blo=umin - ubar, bhi=umax - ubar,
                Xbar=Xbar, kap=kap, dkap=dkap, refs=refs, drefs=drefs, G=G)


def qp_rows_ge(qp):
    """All constraints as a_i' x >= b_i; returns (A, b, soft mask)."""
    A, lo, hi = qp["A"], qp["lo"], qp["hi"]
    n = A.shape[1]
    Ar, br, soft = [], [], []
    for i in range(A.shape[0]):
        if np.isfinite(lo[i]):
            Ar.append(A[i]); br.append(lo[i]); soft.append(True)
        if np.isfinite(hi[i]):
            Ar.append(-A[i]); br.append(-hi[i]); soft.append(True)
    I = np.eye(n)
    for j in range(n):
        Ar.append(I[j]); br.append(qp["blo"][j]); soft.append(False)
        Ar.append(-I[j]); br.append(-qp["bhi"][j]); soft.append(False)
    return np.array(Ar), np.array(br), np.array(soft)


def _kkt_solve(K, rhs):
    sol = np.linalg.lstsq(K, rhs, rcond=None)[0]
    for _ in range(3):                       # iterative refinement (ill-conditioned at N=40)
        sol = sol + np.linalg.lstsq(K, rhs - K @ sol, rcond=None)[0]
    return sol


def active_set_polish(H, f, A, b, soft, rho, x_init, hard, max_rounds=400):
    """Exact solve of min 0.5x'Hx + f'x [+ rho*sum(xi)] s.t. A x (+xi) >= b by a
    primal-dual active-set iteration started from a near-solution.

    Row states: W (active, multiplier in [0, cap]), V (violated, multiplier == rho; soft only).
    Returns (x, lam, ok, kkt); ok means the exact KKT certificate below holds
    (relative stationarity / primal / multiplier-sign residuals <= 1e-9)."""
    m, n = A.shape
    anorm = np.abs(A).max(axis=1)
    cap = np.where(soft & (not hard), rho, np.inf)
    r = A @ x_init - b
    sc = 1.0 + np.abs(b) + anorm * np.abs(x_init).max()
    W = set(np.where(np.abs(r) <= 1e-6 * sc)[0])
    V = set() if hard else set(np.where((r < -1e-6 * sc) & soft)[0])
    W -= V
    seen = set()
    for rnd in range(max_rounds):
        Wl = sorted(W)
        g = f.copy()
        for i in V:
            g -= rho * A[i]
        nw = len(Wl)
        K = np.zeros((n + nw, n + nw))
        K[:n, :n] = H
        if nw:
            Aw = A[Wl]
            K[:n, n:] = -Aw.T
            K[n:, :n] = Aw
        rhs = np.concatenate([-g, b[Wl] if nw else np.zeros(0)])
        sol = _kkt_solve(K, rhs)
        x = sol[:n]
        lw = sol[n:]
        r = A @ x - b
        sc = 1.0 + np.abs(b) + anorm * np.abs(x).max()
        lam = np.zeros(m)
        for i in V:
            lam[i] = rho
        for j, i in enumerate(Wl):
            lam[i] = lw[j]
        lsc = 1.0 + (np.abs(lw).max() if nw else 0.0)
        cand = []
        for j, i in enumerate(Wl):
            if lw[j] < -1e-9 * lsc:
                cand.append((lw[j] / lsc, "dropW", i))
            elif lw[j] > cap[i] * (1 + 1e-9):
                cand.append((-(lw[j] - cap[i]) / lsc, "toV", i))
        if not cand:
            for i in range(m):
                if i in W:
                    continue
                if i in V:
                    if r[i] > 1e-9 * sc[i]:
                        cand.append((-r[i] / sc[i], "fromV", i))
                elif r[i] < -1e-9 * sc[i]:
                    cand.append((r[i] / sc[i], "addW", i))
        if not cand:
            stat = H @ x + f - A.T @ lam
            ssc = 1.0 + np.abs(f).max() + np.abs(H @ x).max() + np.abs(A.T @ lam).max()
            nonV = [i for i in range(m) if i not in V]
            prim = float(max(0.0, float(-(r[nonV] / sc[nonV]).min()))) if nonV else 0.0
            kkt = dict(stat=float(np.abs(stat).max() / ssc), prim=prim,
                       comp=float(max([abs(r[i]) / sc[i] for i in W] + [0.0])), nW=len(W), nV=len(V),
                       rounds=rnd)
            ok = kkt["stat"] < 1e-9 and prim < 1e-9 and kkt["comp"] < 1e-9
            return x, lam, ok, kkt
        cand.sort()
        _, act, i = cand[0]
        key = (frozenset(W), frozenset(V))
        if key in seen:            # cycling guard: take the second-worst move
            _, act, i = cand[min(1, len(cand) - 1)]
        seen.add(key)
        if act == "dropW":
            W.discard(i)
        elif act == "toV":
            W.discard(i); V.add(i)
        elif act == "fromV":
            V.discard(i); W.add(i)
        elif act == "addW":
            W.add(i)
    return x, lam, False, {"rounds": max_rounds}


def ipm_dense(H, f, A, b, soft, rho, tol=1e-11, max_iter=120):
    """Dense Mehrotra primal-dual IPM for  min 0.5x'Hx + f'x + rho*sum(xi)
    s.t. A x + xi >= b (soft rows, xi >= 0), A x >= b (hard rows).  Golden-side only:
    its answer is used solely to seed active_set_polish, whose exact KKT certificate is
    what pins the fixture."""
    m, n = A.shape
    sf = soft.astype(float)
    x = np.zeros(n)
    r0 = A @ x - b
    xi = np.where(soft, np.maximum(-r0, 0.0) + 1e-2, 0.0)
    s = np.where(soft, r0 + xi, np.maximum(r0, 1.0))
    lam = np.ones(m)
    nu = np.where(soft, rho - 1.0, 0.0)     # dual-feasible for xi from the start
    M = m + int(soft.sum())
    for it in range(max_iter):
        rd = H @ x + f - A.T @ lam
        rp = A @ x + xi - s - b
        rx = np.where(soft, rho - lam - nu, 0.0)
        mu = (s @ lam + xi @ nu) / M
        if (np.abs(rd).max() < tol * (1 + np.abs(f).max()) and np.abs(rp).max() < tol * (1 + np.abs(b).max())
                and np.abs(rx).max() < tol * rho and mu < tol):
            break
        d = s / lam + np.where(soft, xi / np.where(soft, nu, 1.0), 0.0)
        K = H + A.T @ (A / d[:, None])
        reg = 0.0
        while True:
            try:
                Lc = np.linalg.cholesky(K + reg * np.eye(n))
                break
            except np.linalg.LinAlgError:
                reg = max(1e-14 * np.abs(np.diag(K)).max(), 10 * reg)

        def solve(r4, r5):
            rhs = -rp - r4 / lam + np.where(soft, (r5 + xi * rx) / np.where(soft, nu, 1.0), 0.0)
            dx = np.linalg.solve(Lc.T, np.linalg.solve(Lc, -rd + A.T @ (rhs / d)))
            dl = (rhs - A @ dx) / d
            ds = -(r4 + s * dl) / lam
            dn = np.where(soft, rx - dl, 0.0)
            dxi = np.where(soft, -(r5 + xi * dn) / np.where(soft, nu, 1.0), 0.0)
            return dx, dl, ds, dn, dxi

        def maxstep(v, dv):
            neg = dv < 0
            return min(1.0, float(np.min(-v[neg] / dv[neg]))) if neg.any() else 1.0
        dx, dl, ds, dn, dxi = solve(s * lam, xi * nu)
        ap = min(maxstep(s, ds), maxstep(np.where(soft, xi, 1.0), np.where(soft, dxi, 0.0)))
        ad = min(maxstep(lam, dl), maxstep(np.where(soft, nu, 1.0), np.where(soft, dn, 0.0)))
        a = min(ap, ad)
        mua = ((s + a * ds) @ (lam + a * dl) + (xi + a * dxi) @ (nu + a * dn)) / M
        sig = (mua / mu) ** 3
        dx, dl, ds, dn, dxi = solve(s * lam + ds * dl - sig * mu, xi * nu + dxi * dn - sig * mu * sf)
        ap = min(maxstep(s, ds), maxstep(np.where(soft, xi, 1.0), np.where(soft, dxi, 0.0)))
        ad = min(maxstep(lam, dl), maxstep(np.where(soft, nu, 1.0), np.where(soft, dn, 0.0)))
        a = min(1.0, 0.995 * min(ap, ad))
        x += a * dx; s += a * ds; lam += a * dl; xi += a * dxi; nu += a * dn
    return x, lam, it


def solve_qp_tight(qp, rho, hard):
    """Hard QP: scipy SLSQP (ftol 1e-15) seeds the polish.  Elastic QP: ipm_dense seeds it.
    Either way the returned x carries an exact active-set KKT certificate (ok flag)."""
    H, f = qp["H"], qp["f"]
    A, b, soft = qp_rows_ge(qp)
    n = H.shape[0]
    if hard:
        res = sp_minimize(lambda x: 0.5 * x @ H @ x + f @ x, np.zeros(n), jac=lambda x: H @ x + f,
                          method="SLSQP", constraints=[{"type": "ineq", "fun": lambda x: A @ x - b,
                                                        "jac": lambda x: A}],
                          options={"ftol": 1e-15, "maxiter": 3000})
        xs = res.x
        info = dict(seed="slsqp", status=int(res.status), nit=int(res.nit))
    else:
        xs, _, it = ipm_dense(H, f, A, b, soft, rho)
        info = dict(seed="ipm", nit=int(it))
    x, lam, ok, kkt = active_set_polish(H, f, A, b, soft, rho, xs, hard)
    kkt.update(info)
    kkt["seed_dist"] = float(np.abs(x - xs).max())
    return x, lam, ok, kkt, None


def fd_checks(tr, x0, obs, ubar, qp):
    """Validate the QP against the reference's own functions."""
    N = tr.N
    n = 2 * N
    h = 1e-6
    G = qp["G"]
    # jacobian of reference predict wrt U (central FD)
    Gfd = np.zeros_like(G)
    for j in range(n):
        e = np.zeros(n); e[j] = h
        Gfd[:, :, j] = (tr.predict(x0, ubar + e) - tr.predict(x0, ubar - e)) / (2 * h)
    errG = np.abs(Gfd - G).max()
    # cost value and gradient
    cref = tr.cost(ubar, x0)
    gfd = np.array([(tr.cost(ubar + h * e, x0) - tr.cost(ubar - h * e, x0)) / (2 * h) for e in np.eye(n)])
    errc = abs(cref - qp["c0"]) / (1 + abs(cref))
    errg = np.abs(gfd - qp["f"]).max() / (1 + np.abs(gfd).max())
    # constraints at ubar: reference rows vs our rows (mapping with the max split / min over obstacles)
    gref = tr.constraints(x0, obs)["fun"](ubar)
    per = 7 + len(obs)
    errcon = 0.0
    ri = 0
    for k in range(N):
        blk = gref[k * per:(k + 1) * per]
        # lane: [sl-d, d+sl, sl-vf, vf+sl, sl-vfull, vfull+sl]
        for c in range(3):
            errcon = max(errcon, abs(blk[2 * c] - qp["hi"][ri]), abs(blk[2 * c + 1] - (-qp["lo"][ri])))
            ri += 1
        if len(obs):
            mref = min(blk[6:6 + len(obs)])
            mine = min(qp["hi"][ri], qp["hi"][ri + 1])
            errcon = max(errcon, abs(mref - mine))
            ri += 2
        errcon = max(errcon, abs(blk[-1] - (-qp["lo"][ri])))
        ri += 1
    return dict(errG=float(errG), errc=float(errc), errg=float(errg), errcon=float(errcon))


def gen_qp(quick=False):
    rng = np.random.default_rng(44)
    plan = [  # (traj, N, obstacles kind, count)
        (1, 10, 0, 12), (1, 20, 0, 30), (2, 20, "fsm", 24), (3, 30, 2, 14), (3, 40, 8, 10),
        (1, 5, 0, 6), (2, 10, 1, 8), (1, 40, 0, 4), (2, 30, "fsm", 6),
    ]
    if quick:
        plan = [(1, 10, 0, 3), (1, 20, 0, 3)]
    cases = []
    t0 = time.time()
    for (ti, N, ok, cnt) in plan:
        ld = loader(ti)
        tr = tracker(ti, N)
        for rep in range(cnt):
            x0 = draw_x0(ld, rng)
            if rep == cnt - 1 and cnt > 3:
                x0[0] = ld.s_max - rng.uniform(0.5, 5.0)     # horizon beyond the end
            if rep == cnt - 2 and cnt > 3:
                x0[1] += 0.3                                 # pushed towards / over the lane margin
            obs = draw_obstacles(ok, x0, rng)
            ubar = capture_warmstart(tr, x0, obs)
            qp = build_qp(tr, ld, x0, obs, ubar)
            chk = fd_checks(tr, x0, obs, ubar, qp)
            # nominal rollout bit-identical to reference predict by construction; re-assert
            assert np.array_equal(qp["Xbar"], tr.predict(x0, ubar))
            xe, le, oke, kkte, _ = solve_qp_tight(qp, RHO_DEFAULT, hard=False)
            if oke and kkte.get("nV", 1) == 0:
                # elastic slack inactive: the hard QP is feasible; solve it independently (SLSQP seed)
                xh, lh, okh, kkth, _ = solve_qp_tight(qp, RHO_DEFAULT, hard=True)
            else:
                xh, lh, okh, kkth = xe, le, False, {"skipped": "elastic slack active -> hard QP infeasible"}
            feasible = bool(okh)
            if feasible:
                # exact-penalty consistency: elastic == hard when rho > max multiplier
                assert np.abs(xh - xe).max() < 1e-7 or lh.max() >= RHO_DEFAULT, (np.abs(xh - xe).max(), lh.max())
            c = dict(traj=ti, N=N, x0=x0, obs=np.array([[o["s"], o["v"]] for o in obs]).reshape(-1, 2), ubar=ubar,
                     U_hard=ubar + xh, U_elastic=ubar + xe, feasible=feasible, ok_elastic=oke,
                     lam_max=float(lh.max()) if feasible else float(le.max()),
                     kkt_hard=json.dumps(kkth), kkt_elastic=json.dumps(kkte), fdcheck=json.dumps(chk),
                     obj_elastic=float(0.5 * xe @ qp["H"] @ xe + qp["f"] @ xe + qp["c0"]))
            cases.append(c)
            print(f"  qp case {len(cases)} traj{ti} N={N} obs={len(obs)} feasible={feasible} "
                  f"okE={oke} lam={c['lam_max']:.3g} chk={chk} ({time.time()-t0:.0f}s)", flush=True)
    out = {"n": np.array(len(cases)), "rho": np.array(RHO_DEFAULT)}
    for j, c in enumerate(cases):
        for k, v in c.items():
            out[f"c{j}_{k}"] = np.asarray(v)
    save("qp_golden" if not quick else "qp_golden_quick", **out)


def gen_qpdata():
    """Full QP matrices for a few small cases: pins the oracle's QP builder element-wise."""
    rng = np.random.default_rng(55)
    out = {}
    j = 0
    for (ti, N, ok) in [(1, 5, 0), (1, 10, 0), (2, 10, "fsm"), (3, 10, 8), (1, 20, 0), (2, 8, 1)]:
        ld = loader(ti)
        tr = tracker(ti, N)
        x0 = draw_x0(ld, rng)
        obs = draw_obstacles(ok, x0, rng)
        if ok == 1:
            x0[0] = ld.s_max - 2.0
            obs = [{"s": x0[0] + 30.0, "v": 2.0, "type": "car"}]
        ubar = capture_warmstart(tr, x0, obs)
        qp = build_qp(tr, ld, x0, obs, ubar)
        d = dict(traj=ti, N=N, x0=x0, obs=np.array([[o["s"], o["v"]] for o in obs]).reshape(-1, 2), ubar=ubar,
                 H=qp["H"], f=qp["f"], c0=qp["c0"], A=qp["A"], lo=qp["lo"], hi=qp["hi"], blo=qp["blo"],
                 bhi=qp["bhi"], Xbar=qp["Xbar"], kap=qp["kap"], dkap=qp["dkap"], refs=qp["refs"],
                 drefs=qp["drefs"])
        for k, v in d.items():
            out[f"c{j}_{k}"] = np.asarray(v)
        j += 1
    out["n"] = np.array(j)
    save("qpdata_golden", **out)


# ----------------------------------------------------------------------------------------
# 5. reference solve() outputs (behavioural)
# ----------------------------------------------------------------------------------------
def gen_solve():
    rng = np.random.default_rng(66)
    cases = []
    for (ti, N, ok, cnt) in [(1, 5, 0, 6), (1, 10, 0, 4), (2, 5, "fsm", 6), (1, 20, 0, 2), (2, 10, 1, 3)]:
        ld = loader(ti)
        tr = tracker(ti, N)
        for rep in range(cnt):
            x0 = draw_x0(ld, rng)
            obs = draw_obstacles(ok, x0, rng)
            rec = {}
            orig = RT.minimize

            def wrap(*a, **kw):
                r = orig(*a, **kw)
                rec["r"] = r
                return r
            RT.minimize = wrap
            try:
                u0, pX, tsol = tr.solve(x0, obs)
            finally:
                RT.minimize = orig
            r = rec["r"]
            cases.append(dict(traj=ti, N=N, x0=x0, obs=np.array([[o["s"], o["v"]] for o in obs]).reshape(-1, 2),
                              u0=u0, U=r.x, predX=pX, nit=r.nit, status=r.status, fun=r.fun,
                              solve_time=tsol))
            print(f"  solve case traj{ti} N={N} status={r.status} nit={r.nit} t={tsol:.3f}", flush=True)
    out = {"n": np.array(len(cases))}
    for j, c in enumerate(cases):
        for k, v in c.items():
            out[f"c{j}_{k}"] = np.asarray(v)
    save("solve_golden", **out)


# ----------------------------------------------------------------------------------------
# 5b. tight NLP optimum of the reference's own problem ("Tight NLP optimum")
# ----------------------------------------------------------------------------------------
def _central_jac(fun, x, h=1e-4):
    """Fourth-order central finite differences of a vector (or scalar) function of the reference:
    (-f(x+2h) + 8 f(x+h) - 8 f(x-h) + f(x-2h)) / 12h.  Its rounding noise (~eps |f| / h) is what limits
    the certificates below on the high-cost obstacle cases (|f| ~ 1e3); the h^4 truncation is negligible."""
    f0 = np.atleast_1d(fun(x))
    J = np.zeros((f0.size, x.size))
    for j in range(x.size):
        e = np.zeros(x.size)
        e[j] = h
        f = lambda t: np.atleast_1d(fun(x + t * e))
        J[:, j] = (-f(2) + 8 * f(1) - 8 * f(-1) + f(-2)) / (12 * h)
    return J


def split_constraints(tr, x0, obs):
    """The reference's constraint function (trajectory_tracking.py:155-211) with each obstacle row
    s_o + v_o k dt - s - max(5, 1.5 v) >= 0 (:194-204) written as its two smooth rows (- 5 and - 1.5 v):
    the same feasible set without the kink of max() that stops SLSQP's line search (status 8) whenever an
    obstacle row is active at v = 5 / 1.5.  Rows are taken from the reference's own output."""
    base = tr.constraints(x0, obs)["fun"]
    if not obs:
        return base
    per = 7 + len(obs)
    osd, tg = tr.obstacle_safety_distance, tr.max_time_2_obs

    def g(U):
        c = base(U)
        X = tr.predict(x0, U)
        out = []
        for k in range(tr.N):
            blk = c[k * per:(k + 1) * per]
            v = X[k + 1, 4]
            m = max(osd, v * tg)
            out.extend(blk[:6])
            for i in range(len(obs)):
                out.append(blk[6 + i] + m - osd)
                out.append(blk[6 + i] + m - v * tg)
            out.append(blk[-1])
        return np.array(out)
    return g


def nlp_kkt(tr, ld, x0, obs, U, act_tol=1e-7):
    """KKT check of the reference NLP (cost :116-152, constraints :155-211 in the split form, bounds :249)
    at U with central-FD derivatives of the reference functions: multipliers of the active rows by
    non-negative least squares (stationarity `stat`, relative to 1 + |grad|), and `err_est`, the
    length of the equality-constrained Newton step on the active set with the Gauss-Newton Hessian of
    build_qp at U -- an estimate of the distance of U to the local optimum, in U units."""
    from scipy.optimize import nnls
    N = tr.N
    g = _central_jac(lambda u: tr.cost(u, x0), U)[0]
    cf = split_constraints(tr, x0, obs)
    c = cf(U)
    A = _central_jac(cf, U)
    lo = np.tile(tr.u_min, N)
    hi = np.tile(tr.u_max, N)
    rows, rhs = [], []
    for i in np.flatnonzero(c <= act_tol):
        rows.append(A[i]); rhs.append(c[i])
    for j in np.flatnonzero(U - lo <= act_tol):
        rows.append(np.eye(2 * N)[j]); rhs.append(U[j] - lo[j])
    for j in np.flatnonzero(hi - U <= act_tol):
        rows.append(-np.eye(2 * N)[j]); rhs.append(hi[j] - U[j])
    n = 2 * N
    H = build_qp(tr, ld, x0, obs, U)["H"]
    if rows:
        Aa = np.array(rows)
        lam, _ = nnls(Aa.T, g, maxiter=5000)
        res = g - Aa.T @ lam
        na = len(rows)
        K = np.zeros((n + na, n + na))
        K[:n, :n] = H
        K[:n, n:] = -Aa.T
        K[n:, :n] = Aa
        sol = np.linalg.lstsq(K, np.concatenate([-g, -np.array(rhs)]), rcond=None)[0]
        du = sol[:n]
    else:
        lam = np.zeros(0)
        res = g
        du = np.linalg.solve(H, -g)
    return dict(stat=float(np.abs(res).max() / (1.0 + np.abs(g).max())), prim=float(max(0.0, -c.min(initial=0.0))),
                n_active=len(rows), lam_max=float(lam.max(initial=0.0)), err_est=float(np.abs(du).max()))


def solve_nlp_case(args):
    """One reference NLP, solved twice:
      stage 1 = SURVEY App. C exactly: minimize(cost, ubar, SLSQP, bounds, constraints), ftol 1e-12,
                maxiter 1000, scipy's 2-point finite-difference derivatives (the reference's solve(),
                trajectory_tracking.py:254-256, only tighter);
      stage 2 = continuation from stage 1 on the same reference functions with the obstacle rows split
                (split_constraints) and central-FD derivatives (2-point FD limits stage 1 to ~1e-5 in U,
                and the max() kink stops its line search).
    `certified` = stage 2 converged (SLSQP status 0) to a feasible point whose KKT check (nlp_kkt) puts it
    within 1e-7 of the local optimum."""
    ti, N, ok, seed = args
    rng = np.random.default_rng(seed)
    ld = loader(ti)
    tr = tracker(ti, N)
    x0 = draw_x0(ld, rng)
    obs = draw_obstacles(ok, x0, rng)
    ubar = capture_warmstart(tr, x0, obs)
    cons = tr.constraints(x0, obs)
    bounds = [(tr.u_min[0], tr.u_max[0]), (tr.u_min[1], tr.u_max[1])] * N
    t0 = time.time()
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        r1 = sp_minimize(tr.cost, ubar, args=(x0,), method="SLSQP", bounds=bounds, constraints=cons,
                         options={"ftol": 1e-12, "maxiter": 1000})
        t1 = time.time() - t0
        sg = split_constraints(tr, x0, obs)
        cons2 = {"type": "ineq", "fun": sg, "jac": lambda u: _central_jac(sg, u)}
        r2 = sp_minimize(tr.cost, r1.x, args=(x0,), jac=lambda u, x: _central_jac(lambda v: tr.cost(v, x), u)[0],
                         method="SLSQP", bounds=bounds, constraints=cons2, options={"ftol": 1e-15, "maxiter": 150})
    k1 = nlp_kkt(tr, ld, x0, obs, r1.x)
    U, kk, stage, n3 = r2.x, nlp_kkt(tr, ld, x0, obs, r2.x), 2, 0
    if not (kk["prim"] <= 1e-9 and kk["err_est"] <= 1e-8):
        U3, n3 = fd_sqp(tr, ld, x0, obs, r2.x)
        k3 = nlp_kkt(tr, ld, x0, obs, U3)
        if k3["prim"] <= max(kk["prim"], 1e-9) and k3["err_est"] < kk["err_est"]:
            U, kk, stage = U3, k3, 3
    feasible = bool(kk["prim"] <= 1e-9)
    certified = bool(feasible and kk["err_est"] <= 1e-6 and kk["stat"] <= 1e-6)
    return dict(traj=ti, N=N, x0=x0, obs=np.array([[o["s"], o["v"]] for o in obs]).reshape(-1, 2), ubar=ubar,
                U_nlp=U, U_slsqp=r1.x, nit1=r1.nit, status1=r1.status, nit2=r2.nit, status2=r2.status, stage=stage,
                nit3=n3, fun=float(tr.cost(U, x0)), fun_slsqp=float(r1.fun), feasible=feasible, certified=certified,
                kkt=json.dumps(kk), kkt_slsqp=json.dumps(k1), seconds=time.time() - t0, seconds1=t1)


def fd_sqp(tr, ld, x0, obs, U, iters=25):
    """Stage 3, used when SLSQP stops short (status 8 on degenerate or kinked problems): Newton-type SQP
    on the reference's own functions, golden-side -- gradient and constraint Jacobian by central FD of
    cost() and the split constraints, the Gauss-Newton Hessian of build_qp, each QP solved exactly by
    active_set_polish.  Stops when the step is below 1e-12."""
    N = tr.N
    n = 2 * N
    cf = split_constraints(tr, x0, obs)
    lo = np.tile(tr.u_min, N)
    hi = np.tile(tr.u_max, N)
    U = np.clip(np.array(U, np.float64), lo, hi)
    best, best_step = U.copy(), np.inf
    for it in range(iters):
        g = _central_jac(lambda u: tr.cost(u, x0), U)[0]
        c = cf(U)
        A = _central_jac(cf, U)
        H = build_qp(tr, ld, x0, obs, U)["H"]
        Aall = np.vstack([A, np.eye(n), -np.eye(n)])
        b = np.concatenate([-c, lo - U, U - hi])
        d, _, ok, _ = active_set_polish(H, g, Aall, b, np.zeros(len(b), bool), RHO_DEFAULT, np.zeros(n), True)
        step = float(np.abs(d).max())
        if step < best_step:            # past the FD noise floor the steps jitter: keep the calmest point
            best, best_step = U.copy(), step
        U = np.clip(U + d, lo, hi)
        if step < 1e-12:
            return U, it + 1
    return best, iters


NLP_PLAN = [  # (traj, N, obstacle kind, count): the C1-C5 shapes plus the reference default N=5
    (1, 10, 0, 10), (1, 20, 0, 12), (2, 20, "fsm", 12), (3, 30, 2, 10), (3, 40, 8, 8), (2, 5, "fsm", 8),
]


def gen_nlp(procs=8):
    import multiprocessing as mp
    jobs = []
    seed = 7700
    for (ti, N, ok, cnt) in NLP_PLAN:
        for _ in range(cnt):
            jobs.append((ti, N, ok, seed))
            seed += 1
    t0 = time.time()
    with mp.get_context("fork").Pool(procs) as pool:
        cases = []
        for c in pool.imap(solve_nlp_case, jobs):
            cases.append(c)
            k = json.loads(c["kkt"])
            print(f"  nlp case {len(cases)} traj{c['traj']} N={c['N']} obs={len(c['obs'])} feasible={c['feasible']} "
                  f"certified={c['certified']} nit={c['nit1']}+{c['nit2']} st={c['status1']},{c['status2']} "
                  f"err_est={k['err_est']:.1e} stat={k['stat']:.1e} prim={k['prim']:.1e} "
                  f"|U_slsqp-U|={np.abs(c['U_slsqp'] - c['U_nlp']).max():.1e} ({time.time()-t0:.0f}s)", flush=True)
    out = {"n": np.array(len(cases))}
    for j, c in enumerate(cases):
        for k, v in c.items():
            out[f"c{j}_{k}"] = np.asarray(v)
    save("nlp_golden", **out)


# ----------------------------------------------------------------------------------------
# 6. closed loop (run_simulation) histories
# ----------------------------------------------------------------------------------------
def gen_closedloop():
    out = {}
    runs = [("c1_traj1_N10", 1, 10, False, False), ("traj2_N5_fsm", 2, 5, True, True),
            ("traj3_N5_fsm", 3, 5, True, True)]
    if os.environ.get("CL_ONLY"):
        runs = [r for r in runs if r[0] in os.environ["CL_ONLY"].split(",")]
        old = os.path.join(HERE, "closedloop_golden.npz")
        if os.path.exists(old):
            with np.load(old, allow_pickle=False) as z:
                out.update({k: z[k] for k in z.files if k != "meta_json"})
    for (tag, ti, N, dyn, tl) in runs:
        ld = loader(ti)
        tr = tracker(ti, N)
        fsm = RT.ObstaclesFSM(dynamic_obstacle=dyn, traffic_light=tl)
        if ti == 3:
            # the trajectory3 preset, commented out in the reference (trajectory_tracking.py:311-327);
            # overwrite the attributes of the active (trajectory2) preset
            fsm.obs_trigger_s = 5.0
            fsm.obs_start_s = fsm.obs_s = 150.0
            fsm.obs_v = 4.0
            fsm.obs_end_s = 850.0
            fsm.tl_pos = 2000.0
            fsm.tl_trigger_s = 100.0
            fsm.tl_stop_duration = 20.0
        t0 = time.time()
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            hx, hu, ht, hp, hobs, htl, _ = RT.run_simulation(tr, fsm, ld)
        log = buf.getvalue()
        passed = "===> Checks passed : True" in log
        print(f"  closed loop {tag}: {len(hu)} steps in {time.time()-t0:.1f}s; checks passed={passed}")
        out[f"{tag}_hist_x"] = hx
        out[f"{tag}_hist_u"] = hu
        out[f"{tag}_hist_obs_s"] = np.array(hobs, dtype=np.float64)
        out[f"{tag}_hist_tl_red"] = np.array([s == "RED" for s in htl])
        out[f"{tag}_hist_t"] = ht
        out[f"{tag}_log"] = np.array(log)
    save("closedloop_golden", **out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="")
    ap.add_argument("--quick", action="store_true")
    a = ap.parse_args()
    todo = a.only.split(",") if a.only else ["convert", "interp", "pose", "model", "warmstart", "qpdata", "qp",
                                              "solve", "closedloop"]
    fns = dict(convert=convert_trajectories, interp=gen_interp, pose=gen_pose, model=gen_model, warmstart=gen_warmstart,
               qpdata=gen_qpdata, qp=lambda: gen_qp(a.quick), solve=gen_solve, closedloop=gen_closedloop,
               nlp=gen_nlp)
    for t in todo:
        print(f"== {t}")
        fns[t]()


if __name__ == "__main__":
    main()
