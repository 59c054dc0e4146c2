"""ctypes wrapper of liborcmpc.so — the CPU restatement (oracle) of the reference hot path.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, always as the checker / the timed CPU baseline, never as the product.
See mpc_oracle.h for what each function restates (reference file:line).
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liborcmpc.so")

_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int)


class MpcParams(C.Structure):
    """Layout of `mpc_params` in include/mpcqp.h (shared with the product ABI)."""
    _fields_ = [
        ("N", C.c_int), ("max_obs", C.c_int), ("dt", C.c_double),
        ("u_min", C.c_double * 2), ("u_max", C.c_double * 2),
        ("vehicle_radius", C.c_double),
        ("w_d", C.c_double), ("w_o", C.c_double), ("w_v", C.c_double), ("w_u1", C.c_double), ("w_u2", C.c_double),
        ("obstacle_safety_distance", C.c_double), ("max_time_2_obs", C.c_double), ("wheelbase", C.c_double),
        ("lane_width", C.c_double), ("safe_lane_margin", C.c_double),
        ("brake_distance", C.c_double), ("brake_accel", C.c_double),
        ("linearization", C.c_int), ("sqp_iters", C.c_int), ("max_iter", C.c_int), ("polish", C.c_int),
        ("tol", C.c_double), ("tol_mu", C.c_double), ("elastic_rho", C.c_double), ("sqp_tol", C.c_double),
    ]


def build(quiet=True):
    subprocess.run(["make", "-C", HERE], check=True, capture_output=quiet)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.orc_default_params.argtypes = [C.POINTER(MpcParams)]
        L.orc_table_create.restype = C.c_void_p
        L.orc_table_create.argtypes = [_dp, C.c_int, _dp, C.c_int]
        L.orc_table_destroy.argtypes = [C.c_void_p]
        L.orc_s_max.restype = C.c_double
        L.orc_s_max.argtypes = [C.c_void_p]
        L.orc_get_state.argtypes = [C.c_void_p, C.c_double, _dp]
        L.orc_get_control.argtypes = [C.c_void_p, C.c_double, _dp]
        L.orc_state_slopes.argtypes = [C.c_void_p, C.c_double, _dp]
        L.orc_global_pose.argtypes = [C.c_void_p, C.c_double, C.c_double, _dp]
        L.orc_warm_start.argtypes = [C.c_void_p, C.POINTER(MpcParams), _dp, _dp, C.c_int, _dp]
        L.orc_predict.argtypes = [C.c_void_p, C.POINTER(MpcParams), _dp, _dp, _dp]
        L.orc_cost.restype = C.c_double
        L.orc_cost.argtypes = [C.c_void_p, C.POINTER(MpcParams), _dp, _dp]
        L.orc_constraints.restype = C.c_int
        L.orc_constraints.argtypes = [C.c_void_p, C.POINTER(MpcParams), _dp, _dp, C.c_int, _dp, _dp]
        L.orc_build_qp.restype = C.c_int
        L.orc_build_qp.argtypes = [C.c_void_p, C.POINTER(MpcParams), _dp, _dp, C.c_int, _dp, _dp, _dp, _dp,
                                   _dp, _dp, _dp, _dp, _dp]
        L.orc_solve.restype = C.c_int
        L.orc_solve.argtypes = [C.c_void_p, C.POINTER(MpcParams), _dp, _dp, C.c_int, _dp, _dp, _dp, _dp, _ip]
        L.orc_solve_batch.restype = C.c_int
        L.orc_solve_batch.argtypes = [C.c_void_p, C.POINTER(MpcParams), C.c_int, _dp, _dp, _ip, _dp, _dp, _dp,
                                      _dp, _ip, _ip, C.c_int]
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(_dp)


def _pi(a):
    return None if a is None else a.ctypes.data_as(_ip)


def default_params(**kw):
    p = MpcParams()
    lib().orc_default_params(C.byref(p))
    for k, v in kw.items():
        if k in ("u_min", "u_max"):
            getattr(p, k)[0], getattr(p, k)[1] = v
        else:
            setattr(p, k, v)
    return p


def _obs_arr(obs):
    if obs is None or len(obs) == 0:
        return np.zeros((0, 2)), 0
    a = np.ascontiguousarray(np.asarray(obs, np.float64).reshape(-1, 2))
    return a, a.shape[0]


class Oracle:
    """CPU oracle bound to one reference trajectory (X [T,5], U [T-1,2])."""

    def __init__(self, X, U):
        self.X = np.ascontiguousarray(X, np.float64)
        self.U = np.ascontiguousarray(U, np.float64)
        self.h = lib().orc_table_create(_p(self.X), self.X.shape[0], _p(self.U), self.U.shape[0])
        if not self.h:
            raise ValueError("bad trajectory table")
        self.s_max = lib().orc_s_max(self.h)

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.orc_table_destroy(self.h)
            self.h = None

    def get_state(self, s):
        out = np.zeros(5)
        lib().orc_get_state(self.h, float(s), _p(out))
        return out

    def get_control(self, s):
        out = np.zeros(2)
        lib().orc_get_control(self.h, float(s), _p(out))
        return out

    def global_pose(self, s, d):
        out = np.zeros(3)
        lib().orc_global_pose(self.h, float(s), float(d), _p(out))
        return out

    def state_slopes(self, s):
        out = np.zeros(4)
        lib().orc_state_slopes(self.h, float(s), _p(out))
        return out

    def warm_start(self, p, x0, obs=None):
        o, n = _obs_arr(obs)
        ub = np.zeros(2 * p.N)
        x0 = np.ascontiguousarray(x0, np.float64)
        lib().orc_warm_start(self.h, C.byref(p), _p(x0), _p(o), n, _p(ub))
        return ub

    def predict(self, p, x0, U):
        X = np.zeros((p.N + 1, 5))
        lib().orc_predict(self.h, C.byref(p), _p(np.ascontiguousarray(x0, np.float64)),
                          _p(np.ascontiguousarray(U, np.float64)), _p(X))
        return X

    def cost(self, p, x0, U):
        return lib().orc_cost(self.h, C.byref(p), _p(np.ascontiguousarray(x0, np.float64)),
                              _p(np.ascontiguousarray(U, np.float64)))

    def constraints(self, p, x0, obs, U):
        o, n = _obs_arr(obs)
        out = np.zeros(p.N * (7 + n))
        m = lib().orc_constraints(self.h, C.byref(p), _p(np.ascontiguousarray(x0, np.float64)), _p(o), n,
                                  _p(np.ascontiguousarray(U, np.float64)), _p(out))
        return out[:m]

    def build_qp(self, p, x0, obs, ubar):
        o, n_o = _obs_arr(obs)
        n = 2 * p.N
        mmax = 6 * p.N
        H = np.zeros((n, n)); f = np.zeros(n); c0 = np.zeros(1); A = np.zeros((mmax, n))
        lo = np.zeros(mmax); hi = np.zeros(mmax); blo = np.zeros(n); bhi = np.zeros(n)
        m = lib().orc_build_qp(self.h, C.byref(p), _p(np.ascontiguousarray(x0, np.float64)), _p(o), n_o,
                               _p(np.ascontiguousarray(ubar, np.float64)), _p(H), _p(f), _p(c0), _p(A), _p(lo),
                               _p(hi), _p(blo), _p(bhi))
        return dict(H=H, f=f, c0=float(c0[0]), A=A[:m], lo=lo[:m], hi=hi[:m], blo=blo, bhi=bhi)

    def solve(self, p, x0, obs=None, ubar=None):
        o, n = _obs_arr(obs)
        u0 = np.zeros(2); U = np.zeros(2 * p.N); X = np.zeros((p.N + 1, 5)); it = C.c_int(0)
        ub = None if ubar is None else np.ascontiguousarray(ubar, np.float64)
        st = lib().orc_solve(self.h, C.byref(p), _p(np.ascontiguousarray(x0, np.float64)), _p(o), n, _p(ub),
                             _p(u0), _p(U), _p(X), C.byref(it))
        return dict(u0=u0, U=U, Xpred=X, status=st, iters=it.value)

    def solve_batch(self, p, x0, obs=None, n_obs=None, ubar=None, num_threads=0):
        """x0 [B,5]; obs [B,max_obs,2]; n_obs [B]; ubar [B,N,2] or None."""
        x0 = np.ascontiguousarray(x0, np.float64)
        B = x0.shape[0]
        N = p.N
        obs = None if obs is None else np.ascontiguousarray(obs, np.float64)
        n_obs = None if n_obs is None else np.ascontiguousarray(n_obs, np.int32)
        ub = None if ubar is None else np.ascontiguousarray(ubar, np.float64)
        u0 = np.zeros((B, 2)); U = np.zeros((B, N, 2)); X = np.zeros((B, N + 1, 5))
        st = np.zeros(B, np.int32); it = np.zeros(B, np.int32)
        rc = lib().orc_solve_batch(self.h, C.byref(p), B, _p(x0), _p(obs), _pi(n_obs), _p(ub), _p(u0), _p(U),
                                   _p(X), _pi(st), _pi(it), int(num_threads))
        if rc != 0:
            raise RuntimeError(f"orc_solve_batch rc={rc}")
        return dict(u0=u0, U=U, Xpred=X, status=st, iters=it)
