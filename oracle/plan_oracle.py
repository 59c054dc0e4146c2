"""ctypes binding of the planner oracle (oracle/liborcplan.so, plan_oracle.c). TEST INFRASTRUCTURE ONLY:
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it as the checker of libmpcplan."""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int)


class PlanParams(C.Structure):
    """plan_params of include/mpcplan.h."""
    _fields_ = [("N", C.c_int), ("dt", C.c_double), ("w_y", C.c_double), ("w_s", C.c_double), ("w_u", C.c_double),
                ("w_slack", C.c_double), ("u_min", C.c_double * 2), ("u_max", C.c_double * 2), ("k_min", C.c_double),
                ("k_max", C.c_double), ("a_max", C.c_double), ("v_min", C.c_double), ("defect_sign", C.c_double),
                ("sqp_iters", C.c_int), ("sqp_tol", C.c_double), ("max_iter", C.c_int), ("tol", C.c_double)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        L = C.CDLL(os.path.join(HERE, "liborcplan.so"))
        L.orc_plan_default_params.argtypes = [C.POINTER(PlanParams)]
        L.orc_route_create.argtypes = [_dp, C.c_int, _dp, _dp, _dp, C.POINTER(C.c_void_p)]
        L.orc_route_destroy.argtypes = [C.c_void_p]
        L.orc_route_kappa.restype = C.c_double
        L.orc_route_kappa.argtypes = [C.c_void_p, C.c_double, _dp]
        L.orc_route_vmax.restype = C.c_double
        L.orc_route_vmax.argtypes = [C.c_void_p, C.c_double]
        L.orc_plan_dynamics.argtypes = [_dp, C.c_double, C.c_double, C.c_double, _dp]
        L.orc_plan_defect.argtypes = [C.c_void_p, C.POINTER(PlanParams), _dp, _dp, C.c_double, C.c_double, _dp]
        L.orc_plan_cost.restype = C.c_double
        L.orc_plan_cost.argtypes = [C.c_void_p, C.POINTER(PlanParams), C.c_int, _dp, _dp, _dp, _dp]
        L.orc_plan_batch.argtypes = [C.c_void_p, C.POINTER(PlanParams), C.c_int, _ip, _dp, _dp, _ip, _dp, _dp, _dp,
                                     _ip, _ip, _ip, C.c_int]
        _lib = L
    return _lib


def default_params(**kw):
    p = PlanParams()
    lib().orc_plan_default_params(C.byref(p))
    for k, v in kw.items():
        if k in ("u_min", "u_max"):
            getattr(p, k)[0], getattr(p, k)[1] = v
        else:
            setattr(p, k, v)
    return p


def _p(a):
    return None if a is None else a.ctypes.data_as(_dp)


def _pi(a):
    return None if a is None else a.ctypes.data_as(_ip)


class PlanOracle:
    """The oracle on one route (routes.Route)."""

    def __init__(self, route):
        self.route = route
        self._arr = [np.ascontiguousarray(a, np.float64) for a in (route.s, route.cx, route.cy, route.vmax)]
        h = C.c_void_p()
        rc = lib().orc_route_create(_p(self._arr[0]), len(route.s), _p(self._arr[1]), _p(self._arr[2]),
                                    _p(self._arr[3]), C.byref(h))
        if rc != 0:
            raise ValueError(f"orc_route_create failed ({rc})")
        self.h = h

    def __del__(self):
        if getattr(self, "h", None) and self.h.value:
            lib().orc_route_destroy(self.h)

    def kappa(self, s):
        dk = C.c_double()
        k = lib().orc_route_kappa(self.h, float(s), C.byref(dk))
        return k, dk.value

    def vmax(self, s):
        return lib().orc_route_vmax(self.h, float(s))

    def defect(self, p, xa, xb, u):
        out = np.empty(5)
        lib().orc_plan_defect(self.h, C.byref(p), _p(np.ascontiguousarray(xa, np.float64)),
                              _p(np.ascontiguousarray(xb, np.float64)), float(u[0]), float(u[1]), _p(out))
        return out

    def cost(self, p, N, x0, X, U, S):
        a = [np.ascontiguousarray(v, np.float64) for v in (x0, X, U, S)]
        return lib().orc_plan_cost(self.h, C.byref(p), int(N), *[_p(v) for v in a])

    def solve_batch(self, p, x0, s_target, is_final=None, N=None, num_threads=0):
        x0 = np.ascontiguousarray(x0, np.float64).reshape(-1, 5)
        B = x0.shape[0]
        st = np.ascontiguousarray(np.broadcast_to(np.asarray(s_target, np.float64), (B,)))
        fin = None if is_final is None else np.ascontiguousarray(np.broadcast_to(np.asarray(is_final, np.int32), (B,)))
        Nv = None if N is None else np.ascontiguousarray(np.broadcast_to(np.asarray(N, np.int32), (B,)))
        Nmax = int(p.N if Nv is None else Nv.max())
        X = np.empty((B, Nmax + 1, 5)); U = np.empty((B, Nmax, 2)); S = np.empty((B, Nmax))
        status = np.empty(B, np.int32); iters = np.empty(B, np.int32); sqp = np.empty(B, np.int32)
        rc = lib().orc_plan_batch(self.h, C.byref(p), B, _pi(Nv), _p(x0), _p(st), _pi(fin), _p(X), _p(U), _p(S),
                                  _pi(status), _pi(iters), _pi(sqp), int(num_threads))
        if rc != 0:
            raise ValueError(f"orc_plan_batch failed ({rc})")
        return dict(X=X, U=U, S=S, status=status, iters=iters, sqp=sqp)
