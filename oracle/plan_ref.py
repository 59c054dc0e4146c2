"""numpy restatement of the offline planner's chunk NLP (TrajectoryOptimizer, trajectory_planning.py:8-391)
for scipy SLSQP, the reference's own solver.  TEST INFRASTRUCTURE ONLY (tests/test_plan_oracle.py): it
checks that the oracle's SQP lands on the optimum SLSQP finds for the same functions.  The reference module
is not importable, so the functions are restated from its source:
  dynamics :50-89, unpack :91-113, cost :128-170, the Hermite-Simpson defects :181-210 (forward rule, see
  include/mpcplan.h), the initial-state, terminal and inequality rows :212-349, the initial guess :357-376,
  SLSQP with maxiter 500 / ftol 1e-4 :381-387.
The route functions are routes.Route.k_ref_fun / v_max_fun (the reference's :445-473); d kappa / ds for
the analytic Jacobians comes from the same scipy splines."""
import time

import numpy as np
from scipy.optimize import minimize

W_Y, W_S, W_U, W_SL = 10.0, 10.0, 0.1, 100.0
U_MIN, U_MAX = np.array([-0.6, -5.0]), np.array([0.6, 4.0])
K_MIN, K_MAX, A_MAX = -0.8, 0.8, 6.0


def dkappa(route, s):
    """d k_ref_fun / ds from the scipy splines (same pieces as k_ref_fun)."""
    t = float(route._s_to_t(s))
    i = int(np.clip(np.searchsorted(route.s, s, side="left"), 1, len(route.s) - 1))
    slope = 1.0 / (route.s[i] - route.s[i - 1])
    xs, ys = route.spline
    x1, y1, x2, y2, x3, y3 = xs(t, 1), ys(t, 1), xs(t, 2), ys(t, 2), xs(t, 3), ys(t, 3)
    q = x1 * x1 + y1 * y1
    den = q ** 1.5 + 1e-9
    k = (x1 * y2 - y1 * x2) / den
    return float(((x1 * y3 - y1 * x3) - k * 3.0 * np.sqrt(q) * (x1 * x2 + y1 * y2)) / den * slope)


def dyn(x, u, kr):
    s, d, o, k, v = x
    den = 1 - d * kr
    if abs(den) < 1e-4:
        den = 1e-4 * np.sign(den) if den != 0 else 1e-4
    sd = v * np.cos(o) / den
    return np.array([sd, v * np.sin(o), v * k - sd * kr, u[0], u[1]])


def dyn_jac(x, u, kr, dkr):
    """F = df/dx (kappa = kappa(s)) and df/du."""
    s, d, o, k, v = x
    den = 1 - d * kr
    guard = abs(den) < 1e-4
    if guard:
        den = 1e-4 * np.sign(den) if den != 0 else 1e-4
    c, sn = np.cos(o), np.sin(o)
    sd = v * c / den
    F = np.zeros((5, 5))
    # s_dot
    dsd = np.zeros(5)
    dsd[4] = c / den
    dsd[2] = -v * sn / den
    if not guard:
        dsd[1] = v * c * kr / den ** 2
        dsd[0] = v * c * d * dkr / den ** 2
    F[0] = dsd
    F[1, 2] = v * c
    F[1, 4] = sn
    F[2] = -kr * dsd
    F[2, 0] += -dkr * sd
    F[2, 3] += v
    F[2, 4] += k
    G = np.zeros((5, 2))
    G[3, 0] = G[4, 1] = 1.0
    return F, G


class Chunk:
    def __init__(self, route, N, dt, x0, s_target, final):
        self.r, self.N, self.dt, self.x0, self.st, self.final = route, N, dt, np.asarray(x0, float), s_target, final
        self.nz = 5 * (N + 1) + 3 * N

    def unpack(self, z):
        N = self.N
        return z[:5 * (N + 1)].reshape(N + 1, 5), z[5 * (N + 1):5 * (N + 1) + 2 * N].reshape(N, 2), z[5 * (N + 1) + 2 * N:]

    def cost(self, z):
        X, U, S = self.unpack(z)
        den = max(1, self.r.s_total - self.x0[0])
        c = 0.0
        for k in range(self.N):
            c += W_Y * (X[k, 1] ** 2 + X[k, 2] ** 2) + W_S * ((self.r.s_total - X[k, 0]) / den) ** 2 + \
                W_U * (U[k] @ U[k]) + W_SL * S[k] ** 2
        return c

    def defect(self, X, U, k):
        h, x0, x1, u = self.dt, X[k], X[k + 1], U[k]
        f0, f1 = dyn(x0, u, self.r.k_ref_fun(x0[0])), dyn(x1, u, self.r.k_ref_fun(x1[0]))
        xm = 0.5 * (x0 + x1) + h / 8 * (f0 - f1)
        fm = dyn(xm, u, self.r.k_ref_fun(xm[0]))
        return x1 - (x0 + h / 6 * (f0 + 4 * fm + f1))     # forward HS (the committed trajectories' rule)

    def defect_jac(self, X, U, k):
        h, x0, x1, u = self.dt, X[k], X[k + 1], U[k]
        kap = self.r.k_ref_fun
        f0, f1 = dyn(x0, u, kap(x0[0])), dyn(x1, u, kap(x1[0]))
        F0, G = dyn_jac(x0, u, kap(x0[0]), dkappa(self.r, x0[0]))
        F1, _ = dyn_jac(x1, u, kap(x1[0]), dkappa(self.r, x1[0]))
        xm = 0.5 * (x0 + x1) + h / 8 * (f0 - f1)
        Fm, _ = dyn_jac(xm, u, kap(xm[0]), dkappa(self.r, xm[0]))
        I = np.eye(5)
        D0 = -I - h / 6 * (F0 + 4 * Fm @ (0.5 * I + h / 8 * F0))
        D1 = I - h / 6 * (4 * Fm @ (0.5 * I - h / 8 * F1) + F1)
        Du = -h * G
        return D0, D1, Du

    # constraint functions in the reference's sense (>= 0 / == 0), forward defect
    def eq(self, z):
        X, U, S = self.unpack(z)
        out = [self.defect(X, U, k) for k in range(self.N)] + [X[0] - self.x0]
        if self.final:
            out.append([X[-1, 0] - self.st, X[-1, 4]])
        return np.concatenate(out)

    def ineq(self, z):
        X, U, S = self.unpack(z)
        N, out = self.N, []
        if not self.final:
            out.append(X[N, 0] - self.st / 2)
        for k in range(N + 1):
            sl = S[k] if k < N else 0.0
            out += [X[k, 4] + sl - 0.0, self.r.v_max_fun(X[k, 0]) - (X[k, 4] + sl),
                    A_MAX - X[k, 3] * X[k, 4] ** 2, A_MAX + X[k, 3] * X[k, 4] ** 2]
        for k in range(N + 1):
            out += [X[k, 3] - K_MIN, K_MAX - X[k, 3]]
        for k in range(N):
            out += [U[k, 0] - U_MIN[0], U_MAX[0] - U[k, 0], U[k, 1] - U_MIN[1], U_MAX[1] - U[k, 1], S[k]]
        return np.array(out)

    def ineq_jac(self, z):
        X, U, S = self.unpack(z)
        N, nz = self.N, self.nz
        rows = []
        def row(pairs):
            r = np.zeros(nz)
            for j, v in pairs:
                r[j] += v
            rows.append(r)
        iS = lambda k: 5 * (N + 1) + 2 * N + k
        iU = lambda k, c: 5 * (N + 1) + 2 * k + c
        if not self.final:
            row([(5 * N, 1.0)])
        for k in range(N + 1):
            sl = [(iS(k), 1.0)] if k < N else []
            row([(5 * k + 4, 1.0)] + sl)
            row([(5 * k + 4, -1.0)] + [(j, -v) for j, v in sl])
            kk, v = X[k, 3], X[k, 4]
            row([(5 * k + 3, -v * v), (5 * k + 4, -2 * kk * v)])
            row([(5 * k + 3, v * v), (5 * k + 4, 2 * kk * v)])
        for k in range(N + 1):
            row([(5 * k + 3, 1.0)])
            row([(5 * k + 3, -1.0)])
        for k in range(N):
            row([(iU(k, 0), 1.0)]); row([(iU(k, 0), -1.0)]); row([(iU(k, 1), 1.0)]); row([(iU(k, 1), -1.0)])
            row([(iS(k), 1.0)])
        return np.array(rows)

    def eq_jac(self, z):
        return self.lin(z)[2]

    def cost_grad(self, z):
        return self.lin_cost(z)[1]

    def lin_cost(self, z):
        N, nz = self.N, self.nz
        X, U, S = self.unpack(z)
        den = max(1, self.r.s_total - self.x0[0])
        H = np.zeros(nz)
        g = np.zeros(nz)
        for k in range(N):
            H[5 * k + 0] = 2 * W_S / den ** 2
            g[5 * k + 0] = -2 * W_S * (self.r.s_total - X[k, 0]) / den ** 2
            H[5 * k + 1] = H[5 * k + 2] = 2 * W_Y
            g[5 * k + 1], g[5 * k + 2] = 2 * W_Y * X[k, 1], 2 * W_Y * X[k, 2]
            iu = 5 * (N + 1) + 2 * k
            H[iu] = H[iu + 1] = 2 * W_U
            g[iu], g[iu + 1] = 2 * W_U * U[k, 0], 2 * W_U * U[k, 1]
            isl = 5 * (N + 1) + 2 * N + k
            H[isl] = 2 * W_SL
            g[isl] = 2 * W_SL * S[k]
        return H, g

    def z_init(self):
        N = self.N
        X = np.zeros((N + 1, 5))
        X[:, 0] = np.linspace(self.x0[0], self.st, N + 1)
        X[:, 4] = np.linspace(self.x0[4], 0.0, N + 1) if self.final else self.x0[4]
        return np.concatenate([X.ravel(), np.zeros(2 * N), np.zeros(N)])

    def slsqp(self, ftol=1e-4, maxiter=500, z0=None, jac=False):
        cons = [{"type": "eq", "fun": self.eq}, {"type": "ineq", "fun": self.ineq}]
        if jac:
            cons[0]["jac"], cons[1]["jac"] = self.eq_jac, self.ineq_jac
            t = time.perf_counter()
            r = minimize(self.cost, self.z_init() if z0 is None else z0, jac=self.cost_grad, method="SLSQP",
                         constraints=cons, options={"maxiter": maxiter, "ftol": ftol})
            return r, time.perf_counter() - t
        t = time.perf_counter()
        r = minimize(self.cost, self.z_init() if z0 is None else z0, method="SLSQP", constraints=cons,
                     options={"maxiter": maxiter, "ftol": ftol})
        return r, time.perf_counter() - t

    # ---------------- Gauss-Newton SQP with a dense interior point per QP ----------------
    def lin(self, z):
        """Dense linearisation: cost H, g; equalities A dz = b; inequalities C dz >= d (rows of ineq())."""
        N, nz = self.N, self.nz
        X, U, S = self.unpack(z)
        den = max(1, self.r.s_total - self.x0[0])
        H = np.zeros(nz)
        g = np.zeros(nz)
        for k in range(N):
            H[5 * k + 0] = 2 * W_S / den ** 2
            g[5 * k + 0] = -2 * W_S * (self.r.s_total - X[k, 0]) / den ** 2
            H[5 * k + 1] = H[5 * k + 2] = 2 * W_Y
            g[5 * k + 1], g[5 * k + 2] = 2 * W_Y * X[k, 1], 2 * W_Y * X[k, 2]
            iu = 5 * (N + 1) + 2 * k
            H[iu] = H[iu + 1] = 2 * W_U
            g[iu], g[iu + 1] = 2 * W_U * U[k, 0], 2 * W_U * U[k, 1]
            isl = 5 * (N + 1) + 2 * N + k
            H[isl] = 2 * W_SL
            g[isl] = 2 * W_SL * S[k]
        A, b = [], []
        for k in range(N):
            D0, D1, Du = self.defect_jac(X, U, k)
            row = np.zeros((5, nz))
            row[:, 5 * k:5 * k + 5] = D0
            row[:, 5 * (k + 1):5 * (k + 1) + 5] = D1
            iu = 5 * (N + 1) + 2 * k
            row[:, iu:iu + 2] = Du
            A.append(row)
            b.append(-self.defect(X, U, k))
        row = np.zeros((5, nz))
        row[:, :5] = np.eye(5)
        A.append(row)
        b.append(self.x0 - X[0])
        if self.final:
            row = np.zeros((2, nz))
            row[0, 5 * N] = 1
            row[1, 5 * N + 4] = 1
            A.append(row)
            b.append(np.array([self.st - X[N, 0], -X[N, 4]]))
        A, b = np.vstack(A), np.concatenate(b)
        C, c0 = self.ineq_jac(z), self.ineq(z)
        return np.diag(H), g, A, b, C, -c0




def slsqp_job(job):
    """One chunk through the reference's solve (for bench.py's cpu_reference leg, a process-pool worker):
    job = (route name of workloads.plan_route, x0, s_target, is_final, N)."""
    import workloads as W
    name, x0, st, fin, N = job
    Chunk(W.plan_route(name), N, 0.3, x0, st, fin).slsqp()
    return 1
