"""ctypes binding of libmpcplan.so (include/mpcplan.h): the MI355X batched offline planner.

The product's host boundary for SURVEY 8(f)4.  It loads the in-tree HIP library and fails loudly when it
is missing or when no GPU is present: there is no host fallback (oracle/plan_oracle.c is the tests'
checker and is never used here).
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libmpcplan.so")

PLAN_OK, PLAN_NOT_CONVERGED, PLAN_QP_FAILED, PLAN_NUMERICAL, PLAN_FROZEN_LIMITS = 0, 1, 2, 3, 4
STATUS_NAMES = {0: "ok", 1: "not_converged", 2: "qp_failed", 3: "numerical", 4: "frozen_limits"}
PLAN_MAX_N = 64

_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int)


class PlanParams(C.Structure):
    """plan_params of include/mpcplan.h (TrajectoryOptimizer.__init__, trajectory_planning.py:14-47)."""
    _fields_ = [("N", C.c_int), ("dt", C.c_double), ("w_y", C.c_double), ("w_s", C.c_double), ("w_u", C.c_double),
                ("w_slack", C.c_double), ("u_min", C.c_double * 2), ("u_max", C.c_double * 2), ("k_min", C.c_double),
                ("k_max", C.c_double), ("a_max", C.c_double), ("v_min", C.c_double), ("defect_sign", C.c_double),
                ("sqp_iters", C.c_int), ("sqp_tol", C.c_double), ("max_iter", C.c_int), ("tol", C.c_double)]


class PlanError(RuntimeError):
    pass


EXPORTS = ["plan_default_params", "plan_create", "plan_solve_chunks", "plan_solve_chunks_device", "plan_optimize_device",
           "plan_optimize", "plan_route_eval", "plan_chunks_per_cu", "plan_set_params", "plan_last_error", "plan_version", "plan_destroy"]

_lib = None


def lib():
    """Load libmpcplan.so (raises if it has not been built: run __graft_entry__.build())."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise PlanError(f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    L = C.CDLL(LIB_PATH)
    L.plan_default_params.argtypes = [C.POINTER(PlanParams)]
    L.plan_create.restype = C.c_int
    L.plan_create.argtypes = [_dp, C.c_int, _dp, _dp, _dp, C.POINTER(PlanParams), C.c_int, C.POINTER(C.c_void_p)]
    L.plan_solve_chunks.restype = C.c_int
    L.plan_solve_chunks.argtypes = [C.c_void_p, C.c_int, _ip, _dp, _dp, _ip, _dp, _dp, _dp, _ip, _ip, _ip]
    L.plan_solve_chunks_device.restype = C.c_int
    L.plan_solve_chunks_device.argtypes = [C.c_void_p, C.c_int, C.c_int] + [C.c_void_p] * 11
    L.plan_optimize_device.restype = C.c_int
    L.plan_optimize_device.argtypes = ([C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_double, C.c_int, C.c_void_p,
                                        C.c_int] + [C.c_void_p] * 10)
    L.plan_optimize.restype = C.c_int
    L.plan_optimize.argtypes = ([C.c_void_p, C.c_int, C.c_int, _dp, C.c_double, C.c_int, _dp, C.c_int] + [_dp] * 3 +
                                [_ip] * 6)
    L.plan_route_eval.restype = C.c_int
    L.plan_route_eval.argtypes = [C.c_void_p, C.c_int, _dp, _dp, _dp, _dp]
    L.plan_chunks_per_cu.restype = C.c_int
    L.plan_chunks_per_cu.argtypes = [C.c_void_p, C.c_int, _ip]
    L.plan_set_params.restype = C.c_int
    L.plan_set_params.argtypes = [C.c_void_p, C.POINTER(PlanParams)]
    L.plan_last_error.restype = C.c_char_p
    L.plan_version.restype = C.c_int
    L.plan_destroy.argtypes = [C.c_void_p]
    _lib = L
    return L


def last_error():
    return lib().plan_last_error().decode()


def default_params(**kw):
    p = PlanParams()
    lib().plan_default_params(C.byref(p))
    for k, v in kw.items():
        if k in ("u_min", "u_max"):
            getattr(p, k)[0], getattr(p, k)[1] = float(v[0]), float(v[1])
        else:
            setattr(p, k, v)
    return p


def _check(rc, what):
    if rc != 0:
        raise PlanError(f"{what} failed (rc={rc}): {last_error()}")


def _p(a):
    return None if a is None else a.ctypes.data_as(_dp)


def _pi(a):
    return None if a is None else a.ctypes.data_as(_ip)


class Planner:
    """One libmpcplan context: a device-resident route (routes.Route) and the planner parameters."""

    created = 0          # contexts created in this process (plan_create calls that succeeded)

    def __init__(self, route, params=None, device=0):
        self.route = route
        self.device = int(device)
        self.params = params if params is not None else default_params()
        arr = [np.ascontiguousarray(a, np.float64) for a in (route.s, route.cx, route.cy, route.vmax)]
        h = C.c_void_p()
        _check(lib().plan_create(_p(arr[0]), len(arr[0]), _p(arr[1]), _p(arr[2]), _p(arr[3]), C.byref(self.params),
                                 int(device), C.byref(h)), "plan_create")
        self.h = h
        Planner.created += 1

    def close(self):
        if getattr(self, "h", None) and self.h.value:
            lib().plan_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_params(self, params):
        _check(lib().plan_set_params(self.h, C.byref(params)), "plan_set_params")
        self.params = params

    def solve_chunks(self, x0, s_target, is_final=None, N=None):
        """B chunks: x0 [B,5], s_target [B], is_final [B] (or scalar), N [B] (or scalar; default params.N).
        Returns dict(X [B,Nmax+1,5], U [B,Nmax,2], S [B,Nmax], status, iters, sqp)."""
        x0 = np.ascontiguousarray(x0, np.float64).reshape(-1, 5)
        B = x0.shape[0]
        st = np.ascontiguousarray(np.broadcast_to(np.asarray(s_target, np.float64), (B,)))
        fin = None if is_final is None else np.ascontiguousarray(np.broadcast_to(np.asarray(is_final, np.int32), (B,)))
        Nv = None if N is None else np.ascontiguousarray(np.broadcast_to(np.asarray(N, np.int32), (B,)))
        Nmax = int(self.params.N if Nv is None else Nv.max(initial=1))
        X = np.empty((B, Nmax + 1, 5)); U = np.empty((B, Nmax, 2)); S = np.empty((B, Nmax))
        status = np.empty(B, np.int32); iters = np.empty(B, np.int32); sqp = np.empty(B, np.int32)
        _check(lib().plan_solve_chunks(self.h, B, _pi(Nv), _p(x0), _p(st), _pi(fin), _p(X), _p(U), _p(S), _pi(status),
                                       _pi(iters), _pi(sqp)), "plan_solve_chunks")
        return dict(X=X, U=U, S=S, status=status, iters=iters, sqp=sqp)

    def solve_chunks_device(self, B, Nmax, N_ptr, x0_ptr, st_ptr, fin_ptr, X_ptr, U_ptr, S_ptr, status_ptr, iters_ptr,
                            sqp_ptr, stream=0):
        """Device-pointer variant (ints are raw device addresses, e.g. torch tensor.data_ptr(); 0 = NULL)."""
        _check(lib().plan_solve_chunks_device(self.h, int(B), int(Nmax), N_ptr or None, x0_ptr, st_ptr, fin_ptr or None,
                                              X_ptr or None, U_ptr or None, S_ptr or None, status_ptr or None,
                                              iters_ptr or None, sqp_ptr or None, C.c_void_p(stream)),
               "plan_solve_chunks_device")

    def chunks_per_cu(self, Nmax):
        """plan_chunks_per_cu: chunks resident per compute unit for a launch sized for Nmax."""
        n = C.c_int(0)
        _check(lib().plan_chunks_per_cu(self.h, int(Nmax), C.byref(n)), "plan_chunks_per_cu")
        return n.value

    def horizon_groups(self, horizons):
        """Launch groups for a batch of mixed horizons: runs of consecutive distinct horizons (ascending) whose
        launch sized for the run's largest horizon keeps the residency each would reach alone
        (include/mpcplan.h, plan_chunks_per_cu).  Returns [(N_lo, N_hi), ...]."""
        hs = sorted({int(n) for n in np.asarray(horizons).ravel()})
        groups = []
        for n in hs:
            if groups and self.chunks_per_cu(n) == self.chunks_per_cu(groups[-1][0]):
                groups[-1] = (groups[-1][0], n)
            else:
                groups.append((n, n))
        return groups

    def optimize_device(self, starts, max_chunk_size, max_chunks, avg, Nmax, device=None):
        """The chunk loop of optimize_full_trajectory for B plans on the device (plan_optimize: host buffers,
        the kernel is plan_optimize_device's), up to max_chunks chunks each.  starts [B,5]; avg [nav] =
        mean(vmax[i:]).  Returns dict of numpy arrays: X [B,C,Nmax+1,5], U [B,C,Nmax,2], S [B,C,Nmax], N,
        is_final, status, iters, sqp [B,C] (C = max_chunks slots; slots past nchunks[b] are not written) and
        nchunks [B].  Needs no torch (device: the context's; the argument is kept for callers)."""
        starts = np.ascontiguousarray(starts, np.float64).reshape(-1, 5)
        avg = np.ascontiguousarray(avg, np.float64)
        B, Cn, Nm = starts.shape[0], int(max_chunks), int(Nmax)
        out = dict(X=np.empty((B, Cn, Nm + 1, 5)), U=np.empty((B, Cn, Nm, 2)), S=np.empty((B, Cn, Nm)))
        for k in ("N", "is_final", "status", "iters", "sqp"):
            out[k] = np.empty((B, Cn), np.int32)
        out["nchunks"] = np.empty(B, np.int32)
        _check(lib().plan_optimize(self.h, B, Nm, _p(starts), float(max_chunk_size), Cn, _p(avg), int(avg.size),
                                   *[_p(out[k]) for k in ("X", "U", "S")],
                                   *[_pi(out[k]) for k in ("N", "is_final", "status", "iters", "sqp", "nchunks")]),
               "plan_optimize")
        return out

    def route_eval(self, s):
        """kappa(s), d kappa / ds and v_max(s) on the device (k_ref_fun / v_max_fun)."""
        s = np.ascontiguousarray(s, np.float64).ravel()
        k, dk, vm = np.empty_like(s), np.empty_like(s), np.empty_like(s)
        _check(lib().plan_route_eval(self.h, s.size, _p(s), _p(k), _p(dk), _p(vm)), "plan_route_eval")
        return k, dk, vm
