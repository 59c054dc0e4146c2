"""ctypes binding of libmpcqp.so (include/mpcqp.h) — the MI355X batched tracking-MPC solver.

This is the product's host boundary.  It loads the in-tree HIP library and fails loudly when
it is missing or when a GPU context is asked for without a GPU: nothing falls back silently.  device=-1
selects the library's host backend explicitly (csrc/cpu_backend.h; BASELINE config 1's CPU path).  The
CPU restatement in oracle/ is test infrastructure and is never used here.
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libmpcqp.so")

MPC_OK, MPC_MAX_ITER, MPC_INFEASIBLE, MPC_NUMERICAL = 0, 1, 2, 3
# flag OR-ed onto the last QP's status when the SQP (sqp_iters > 1, sqp_tol > 0) stopped unconverged
MPC_SQP_UNCONVERGED, MPC_STATUS_MASK = 16, 15
STATUS_NAMES = {0: "ok", 1: "max_iter", 2: "infeasible", 3: "numerical"}
MAX_N = 63
MAX_OBS = 64

_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int)


class MpcParams(C.Structure):
    """`mpc_params` of include/mpcqp.h (mirrors TrajectoryTracker.__init__, trajectory_tracking.py:17-47)."""
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


class MpcFsm(C.Structure):
    """`mpc_fsm` of include/mpcqp.h (ObstaclesFSM parameters, trajectory_tracking.py:286-304)."""
    _fields_ = [("dynamic_obstacle", C.c_int), ("traffic_light", C.c_int),
                ("obs_trigger_s", C.c_double), ("obs_start_s", C.c_double), ("obs_v", C.c_double),
                ("obs_end_s", C.c_double), ("tl_pos", C.c_double), ("tl_trigger_s", C.c_double),
                ("tl_stop_duration", C.c_double)]


class MpcError(RuntimeError):
    pass


EXPORTS = ["mpc_default_params", "mpc_create", "mpc_solve_batch", "mpc_solve_batch_device", "mpc_lookup",
           "mpc_set_params", "mpc_get_params", "mpc_last_error", "mpc_version", "mpc_destroy", "mpc_default_fsm",
           "mpc_closed_loop", "mpc_global_pose", "mpc_read_trajectory_json", "mpc_create_from_json",
           "mpc_comm_unique_id", "mpc_comm_create", "mpc_comm_info", "mpc_gather", "mpc_gather_host",
           "mpc_comm_allreduce_max", "mpc_comm_barrier", "mpc_comm_destroy"]
COMM_UID_BYTES = 128

_lib = None


def lib():
    """Load libmpcqp.so (raises if it has not been built: run __graft_entry__.build())."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise MpcError(f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    L = C.CDLL(LIB_PATH)
    L.mpc_default_params.argtypes = [C.POINTER(MpcParams)]
    L.mpc_create.restype = C.c_int
    L.mpc_create.argtypes = [_dp, C.c_int, _dp, C.c_int, C.POINTER(MpcParams), C.c_int, C.POINTER(C.c_void_p)]
    L.mpc_solve_batch.restype = C.c_int
    L.mpc_solve_batch.argtypes = [C.c_void_p, C.c_int, _dp, _dp, _ip, _dp, _dp, _dp, _dp, _ip, _ip]
    L.mpc_solve_batch_device.restype = C.c_int
    L.mpc_solve_batch_device.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                         C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    L.mpc_lookup.restype = C.c_int
    L.mpc_lookup.argtypes = [C.c_void_p, C.c_int, _dp, _dp, _dp]
    L.mpc_set_params.restype = C.c_int
    L.mpc_set_params.argtypes = [C.c_void_p, C.POINTER(MpcParams)]
    L.mpc_get_params.restype = C.c_int
    L.mpc_get_params.argtypes = [C.c_void_p, C.POINTER(MpcParams)]
    L.mpc_last_error.restype = C.c_char_p
    L.mpc_version.restype = C.c_int
    L.mpc_destroy.argtypes = [C.c_void_p]
    L.mpc_default_fsm.argtypes = [C.POINTER(MpcFsm)]
    L.mpc_global_pose.restype = C.c_int
    L.mpc_global_pose.argtypes = [C.c_void_p, C.c_int, _dp, _dp, _dp]
    L.mpc_read_trajectory_json.restype = C.c_int
    L.mpc_read_trajectory_json.argtypes = [C.c_char_p, _dp, C.c_int, _dp, C.c_int, _ip, _ip]
    L.mpc_create_from_json.restype = C.c_int
    L.mpc_create_from_json.argtypes = [C.c_char_p, C.POINTER(MpcParams), C.c_int, C.POINTER(C.c_void_p)]
    L.mpc_closed_loop.restype = C.c_int
    L.mpc_closed_loop.argtypes = [C.c_void_p, C.c_int, _dp, C.POINTER(MpcFsm), C.c_int, C.c_double, _dp, _dp, _dp,
                                  _ip, _ip, _ip, _dp]
    L.mpc_comm_unique_id.restype = C.c_int
    L.mpc_comm_unique_id.argtypes = [C.c_char_p]
    L.mpc_comm_create.restype = C.c_int
    L.mpc_comm_create.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_void_p)]
    L.mpc_comm_info.restype = C.c_int
    L.mpc_comm_info.argtypes = [C.c_void_p, _ip, _ip, _ip]
    L.mpc_gather.restype = C.c_int
    L.mpc_gather.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_int, C.c_void_p]
    L.mpc_gather_host.restype = C.c_int
    L.mpc_gather_host.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_int]
    L.mpc_comm_allreduce_max.restype = C.c_int
    L.mpc_comm_allreduce_max.argtypes = [C.c_void_p, _dp]
    L.mpc_comm_barrier.restype = C.c_int
    L.mpc_comm_barrier.argtypes = [C.c_void_p]
    L.mpc_comm_destroy.argtypes = [C.c_void_p]
    _lib = L
    return L


def last_error():
    return lib().mpc_last_error().decode()


def default_params(**kw):
    p = MpcParams()
    lib().mpc_default_params(C.byref(p))
    for k, v in kw.items():
        if k in ("u_min", "u_max"):
            arr = getattr(p, k)
            arr[0], arr[1] = float(v[0]), float(v[1])
        else:
            setattr(p, k, v)
    return p


def default_fsm(**kw):
    f = MpcFsm()
    lib().mpc_default_fsm(C.byref(f))
    for k, v in kw.items():
        setattr(f, k, v)
    return f


def read_trajectory_json(path):
    """Native reader of the reference trajectory JSON (mpc_read_trajectory_json): returns (X [T,5], U [Tu,2])."""
    T, Tu = C.c_int(), C.c_int()
    b = os.fsencode(path)
    _check(lib().mpc_read_trajectory_json(b, None, 0, None, 0, C.byref(T), C.byref(Tu)), "mpc_read_trajectory_json")
    X = np.empty((T.value, 5))
    U = np.empty((Tu.value, 2))
    _check(lib().mpc_read_trajectory_json(b, X.ctypes.data_as(_dp), T.value, U.ctypes.data_as(_dp), Tu.value,
                                          C.byref(T), C.byref(Tu)), "mpc_read_trajectory_json")
    return X, U


def _p(a):
    return None if a is None else a.ctypes.data_as(_dp)


def _pi(a):
    return None if a is None else a.ctypes.data_as(_ip)


def _check(rc, what):
    if rc != 0:
        raise MpcError(f"{what} failed (rc={rc}): {last_error()}")


class Solver:
    """One libmpcqp context: device-resident reference table + parameters (one HIP device)."""

    def __init__(self, X, U, params=None, device=0):
        self.X = np.ascontiguousarray(X, np.float64)
        self.U = np.ascontiguousarray(U, np.float64)
        if self.X.ndim != 2 or self.X.shape[1] != 5 or self.U.ndim != 2 or self.U.shape[1] != 2:
            raise ValueError("X must be [T,5] and U [Tu,2]")
        self.params = params if params is not None else default_params()
        h = C.c_void_p()
        _check(lib().mpc_create(_p(self.X), self.X.shape[0], _p(self.U), self.U.shape[0], C.byref(self.params),
                                int(device), C.byref(h)), "mpc_create")
        self.h = h

    def close(self):
        if getattr(self, "h", None) and self.h.value:
            lib().mpc_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_params(self, params):
        _check(lib().mpc_set_params(self.h, C.byref(params)), "mpc_set_params")
        self.params = params

    def solve_batch(self, x0, obs=None, n_obs=None, ubar=None):
        """x0 [B,5]; obs [B,max_obs,2] (s, v); n_obs [B]; ubar [B,N,2] or None (reference warm start).
        Returns dict(u0 [B,2], U [B,N,2], Xpred [B,N+1,5], status [B], iters [B])."""
        p = self.params
        N, mo = p.N, p.max_obs
        x0 = np.ascontiguousarray(x0, np.float64).reshape(-1, 5)
        B = x0.shape[0]
        if obs is not None and np.asarray(obs).size > 0 and mo == 0:
            # the library refuses this too (MPC_E_ARG): an obstacle slab must never be dropped silently
            raise ValueError("obstacles given but params.max_obs == 0: set max_obs to the slab width")
        if obs is not None and mo > 0:
            obs = np.ascontiguousarray(obs, np.float64).reshape(B, mo, 2)
            n_obs = (np.full(B, mo, np.int32) if n_obs is None
                     else np.ascontiguousarray(n_obs, np.int32).reshape(B))
        else:
            obs, n_obs = None, None
        ub = None if ubar is None else np.ascontiguousarray(ubar, np.float64).reshape(B, N, 2)
        u0 = np.empty((B, 2)); U = np.empty((B, N, 2)); X = np.empty((B, N + 1, 5))
        st = np.empty(B, np.int32); it = np.empty(B, np.int32)
        _check(lib().mpc_solve_batch(self.h, B, _p(x0), _p(obs), _pi(n_obs), _p(ub), _p(u0), _p(U), _p(X), _pi(st),
                                     _pi(it)), "mpc_solve_batch")
        return dict(u0=u0, U=U, Xpred=X, status=st, iters=it)

    def solve_batch_device(self, B, x0_ptr, obs_ptr, nobs_ptr, ubar_ptr, u0_ptr, U_ptr, X_ptr, st_ptr, it_ptr,
                           stream=0):
        """Device-pointer variant (ints are raw device addresses, e.g. torch tensor.data_ptr())."""
        _check(lib().mpc_solve_batch_device(self.h, int(B), x0_ptr, obs_ptr, nobs_ptr, ubar_ptr, u0_ptr, U_ptr,
                                            X_ptr, st_ptr, it_ptr, C.c_void_p(stream)), "mpc_solve_batch_device")

    def closed_loop(self, x_init, fsm=None, max_steps=1000, s_stop=None, s_max=None):
        """Batched run_simulation (trajectory_tracking.py:377-443) on the device.
        x_init [B,5]; fsm: MpcFsm or None; the loop runs while s <= s_stop (default s_max - 1, :395).
        Returns dict(hist_x [B,max_steps+1,5], hist_u [B,max_steps,2], hist_obs_s [B,max_steps],
        hist_tl [B,max_steps], hist_status [B,max_steps], n_steps [B], step_ms [max_steps])."""
        x_init = np.ascontiguousarray(x_init, np.float64).reshape(-1, 5)
        B = x_init.shape[0]
        if s_stop is None:
            if s_max is None:
                raise ValueError("give s_stop or s_max")
            s_stop = s_max - 1.0
        hx = np.empty((B, max_steps + 1, 5)); hu = np.empty((B, max_steps, 2)); ho = np.empty((B, max_steps))
        ht = np.empty((B, max_steps), np.int32); hs = np.empty((B, max_steps), np.int32)
        ns = np.empty(B, np.int32); sm = np.empty(max_steps)
        _check(lib().mpc_closed_loop(self.h, B, _p(x_init), None if fsm is None else C.byref(fsm), int(max_steps),
                                     float(s_stop), _p(hx), _p(hu), _p(ho), _pi(ht), _pi(hs), _pi(ns), _p(sm)),
               "mpc_closed_loop")
        return dict(hist_x=hx, hist_u=hu, hist_obs_s=ho, hist_tl=ht, hist_status=hs, n_steps=ns, step_ms=sm)

    def global_pose(self, s, d):
        """TrajectoryLoader.get_global_pose on the device table, batched: s, d [n] -> [n, 3] (x, y, psi)."""
        s = np.ascontiguousarray(s, np.float64).ravel()
        d = np.ascontiguousarray(d, np.float64).ravel()
        if s.shape != d.shape:
            raise ValueError("s and d must have the same length")
        out = np.empty((s.size, 3))
        _check(lib().mpc_global_pose(self.h, s.size, _p(s), _p(d), _p(out)), "mpc_global_pose")
        return out

    def lookup(self, s):
        s = np.ascontiguousarray(s, np.float64).ravel()
        st = np.empty((s.size, 5)); ct = np.empty((s.size, 2))
        _check(lib().mpc_lookup(self.h, s.size, _p(s), _p(st), _p(ct)), "mpc_lookup")
        return st, ct


def comm_unique_id():
    """mpc_comm_unique_id: the RCCL unique id (COMM_UID_BYTES bytes) that rank 0 hands to every rank."""
    buf = C.create_string_buffer(COMM_UID_BYTES)
    _check(lib().mpc_comm_unique_id(buf), "mpc_comm_unique_id")
    return buf.raw


class Comm:
    """One libmpcqp ego-shard communicator (mpc_comm_*: RCCL over xGMI behind the C ABI, include/mpcqp.h).
    Collective construction: every rank of `nranks` calls it with rank 0's unique id."""

    def __init__(self, uid, nranks, rank, device):
        if len(uid) != COMM_UID_BYTES:
            raise ValueError(f"uid must be {COMM_UID_BYTES} bytes")
        h = C.c_void_p()
        _check(lib().mpc_comm_create(uid, int(nranks), int(rank), int(device), C.byref(h)), "mpc_comm_create")
        self.h, self.nranks, self.rank, self.device = h, int(nranks), int(rank), int(device)

    def gather(self, payload, root=0):
        """mpc_gather_host of a uint8 payload (the same size on every rank): the list of every rank's payload on
        the root, None elsewhere."""
        buf = np.ascontiguousarray(payload, np.uint8).ravel()
        out = np.empty(buf.size * self.nranks, np.uint8) if self.rank == root else None
        _check(lib().mpc_gather_host(self.h, buf.ctypes.data, buf.size, None if out is None else out.ctypes.data,
                                     int(root)), "mpc_gather_host")
        return None if out is None else [out[i * buf.size:(i + 1) * buf.size] for i in range(self.nranks)]

    def gather_device(self, send_ptr, nbytes, recv_ptr, root=0, stream=0):
        """mpc_gather on device buffers (raw addresses), asynchronous on `stream`."""
        _check(lib().mpc_gather(self.h, send_ptr, int(nbytes), recv_ptr, int(root), C.c_void_p(stream)),
               "mpc_gather")

    def allreduce_max(self, x):
        v = C.c_double(float(x))
        _check(lib().mpc_comm_allreduce_max(self.h, C.byref(v)), "mpc_comm_allreduce_max")
        return v.value

    def barrier(self):
        _check(lib().mpc_comm_barrier(self.h), "mpc_comm_barrier")

    def close(self):
        if getattr(self, "h", None) and self.h.value:
            lib().mpc_comm_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
