"""CPU-side checks of the drop-in boundary: libmpcqp.so builds, loads, exports exactly the
entry points include/mpcqp.h declares, and fails loudly (no CPU fallback) without a GPU."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import PKG, ROOT, traj_arrays

HEADER = os.path.join(ROOT, "include", "mpcqp.h")
LIB = os.path.join(PKG, "libmpcqp.so")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[A-Za-z_][A-Za-z0-9_]*\s*\*?\s*(mpc_[a-z_]+)\s*\(", src, flags=re.M)
    return sorted(set(names))


@pytest.fixture(scope="module")
def built():
    import __graft_entry__ as g
    g.build()
    return LIB


def test_header_declares_the_boundary():
    names = declared_functions()
    for n in ("mpc_create", "mpc_solve_batch", "mpc_solve_batch_device", "mpc_last_error", "mpc_destroy",
              "mpc_default_params", "mpc_lookup", "mpc_set_params", "mpc_get_params", "mpc_version",
              "mpc_default_fsm", "mpc_closed_loop"):
        assert n in names


def test_library_exports_every_declared_symbol(built):
    out = subprocess.run(["nm", "-D", "--defined-only", built], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\sT\s+(mpc_[a-z_]+)$", out, flags=re.M))
    missing = [n for n in declared_functions() if n not in exported]
    assert not missing, missing
    L = ctypes.CDLL(built)
    for n in declared_functions():
        assert hasattr(L, n)


def test_python_binding_matches_exports(built):
    import mpcqp
    assert sorted(mpcqp.EXPORTS) == declared_functions()


def test_params_struct_layout_and_defaults(built):
    """mpc_params mirrors TrajectoryTracker.__init__ (trajectory_tracking.py:17-47)."""
    import mpcqp
    import oracle as O
    p = mpcqp.default_params()
    assert ctypes.sizeof(mpcqp.MpcParams) == ctypes.sizeof(O.MpcParams)
    q = O.default_params()
    for f, _ in mpcqp.MpcParams._fields_:
        a, b = getattr(p, f), getattr(q, f)
        if f in ("u_min", "u_max"):
            assert list(a) == list(b)
        else:
            assert a == b, f
    assert (p.dt, p.N, list(p.u_min), list(p.u_max)) == (0.2, 5, [-0.6, -5.0], [0.6, 4.0])
    assert (p.w_d, p.w_o, p.w_v, p.w_u1, p.w_u2) == (10.0, 10.0, 5.0, 0.5, 0.5)
    assert (p.obstacle_safety_distance, p.max_time_2_obs, p.wheelbase, p.lane_width, p.safe_lane_margin) == \
        (5.0, 1.5, 2.8, 3.0, 0.1)


def test_no_gpu_fails_loudly(built):
    """Without a HIP device mpc_create must fail (MPC_E_DEVICE), never fall back to the CPU."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    import mpcqp
    X, U = traj_arrays(1)
    with pytest.raises(mpcqp.MpcError, match="no HIP device"):
        mpcqp.Solver(X, U)


def test_argument_errors(built):
    import mpcqp
    X, U = traj_arrays(1)
    p = mpcqp.default_params(N=0)
    h = ctypes.c_void_p()
    Xc = np.ascontiguousarray(X)
    Uc = np.ascontiguousarray(U)
    rc = mpcqp.lib().mpc_create(mpcqp._p(Xc), X.shape[0], mpcqp._p(Uc), U.shape[0], ctypes.byref(p), 0,
                                ctypes.byref(h))
    assert rc == -1 and "N out of range" in mpcqp.last_error()
    rc = mpcqp.lib().mpc_solve_batch(None, 1, None, None, None, None, None, None, None, None, None)
    assert rc == -1


def test_shim_surface_matches_reference():
    """TrajectoryTracker / ObstaclesFSM / run_simulation keep the reference's public surface."""
    import trajectory_tracking as TT
    t = TT.TrajectoryTracker()        # no-argument constructor (sanity_checks.py:114-115 usage)
    for a in ("dt", "N", "u_min", "u_max", "vehicle_radius", "w_d", "w_o", "w_v", "w_u1", "w_u2",
              "obstacle_safety_distance", "max_time_2_obs", "wheelbase", "lane_width", "safe_lane_margin"):
        assert hasattr(t, a)
    for m in ("dynamics", "unpack", "pack", "predict", "cost", "constraints", "solve"):
        assert callable(getattr(t, m))
    f = TT.ObstaclesFSM(dynamic_obstacle=True, traffic_light=True)
    obs, st = f.update(0.2, 0.0, 1.0)
    assert obs == [] and st == "RED"


def test_fsm_struct_defaults(built):
    """mpc_fsm mirrors ObstaclesFSM.__init__ (trajectory_tracking.py:286-304, trajectory2 preset)."""
    import mpcqp
    import trajectory_tracking as TT
    f = mpcqp.default_fsm()
    assert f.dynamic_obstacle == 0 and f.traffic_light == 0
    for k, v in TT.FSM_PRESETS["trajectory2"].items():
        assert getattr(f, k) == v, k
    g = TT.fsm_params(TT.ObstaclesFSM(dynamic_obstacle=True, traffic_light=False, preset="trajectory3"))
    assert g.dynamic_obstacle == 1 and g.traffic_light == 0 and g.obs_trigger_s == 5.0 and g.tl_pos == 2000.0
    assert TT.fsm_params(TT.ObstaclesFSM()) is None
    rc = mpcqp.lib().mpc_closed_loop(None, 1, None, None, 10, 0.0, None, None, None, None, None, None, None)
    assert rc == -1 and "ctx" in mpcqp.last_error()


def test_native_json_reader(built, tmp_path):
    """mpc_read_trajectory_json reads the reference's trajectory format (trajectory_loader.py:13-24)
    exactly: written here from the bundled arrays (X, U, S, plus an unknown key), read back bit-exact."""
    import json
    import mpcqp
    from conftest import traj_arrays
    X, U = traj_arrays(2)
    path = tmp_path / "trajectory2.json"
    path.write_text(json.dumps({"meta": {"a": [1, 2, {"b": None}], "ok": True}, "X": X.tolist(), "U": U.tolist(),
                                "S": list(range(len(U)))}, indent=4))
    Xr, Ur = mpcqp.read_trajectory_json(str(path))
    assert np.array_equal(Xr, X) and np.array_equal(Ur, U)
    with pytest.raises(mpcqp.MpcError, match="File not found"):
        mpcqp.read_trajectory_json(str(tmp_path / "missing.json"))
    bad = tmp_path / "bad.json"
    bad.write_text('{"X": [[0, 1, 2, 3]], "U": []}')
    with pytest.raises(mpcqp.MpcError, match="wrong width"):
        mpcqp.read_trajectory_json(str(bad))


def test_host_global_pose_matches_reference_golden():
    """The shim's TrajectoryLoader.get_global_pose == reference (trajectory_loader.py:104-116), bit-exact."""
    from conftest import load_golden
    from trajectory_loader import TrajectoryLoader, builtin_trajectory
    g = load_golden("pose_golden")
    for i in (1, 2, 3):
        ld = TrajectoryLoader(builtin_trajectory(i))
        assert np.array_equal(ld.global_x, g[f"t{i}_gx"]) and np.array_equal(ld.global_psi, g[f"t{i}_gpsi"])
        P = np.array([ld.get_global_pose(s, d) for s, d in zip(g[f"t{i}_s"], g[f"t{i}_d"])])
        assert np.array_equal(P, g[f"t{i}_pose"])
