"""CPU-side checks of the planner's drop-in boundary: libmpcplan.so builds, loads, exports exactly the entry
points include/mpcplan.h declares, its params struct mirrors TrajectoryOptimizer.__init__
(trajectory_planning.py:14-47) and the oracle's, and it fails loudly without a GPU (no host fallback)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import PKG, ROOT

HEADER = os.path.join(ROOT, "include", "mpcplan.h")
LIB = os.path.join(PKG, "libmpcplan.so")


def declared_functions():
    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[A-Za-z_][A-Za-z0-9_]*\s*\*?\s*(plan_[a-z_]+)\s*\(", src, flags=re.M)))


@pytest.fixture(scope="module")
def built():
    import __graft_entry__ as g
    g.build()
    return LIB


def test_library_exports_every_declared_symbol(built):
    out = subprocess.run(["nm", "-D", "--defined-only", built], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\sT\s+(plan_[a-z_]+)$", out, flags=re.M))
    names = declared_functions()
    assert len(names) == 12 and not [n for n in names if n not in exported]
    import mpcplan
    assert sorted(mpcplan.EXPORTS) == names


def test_params_mirror_the_reference_and_the_oracle(built):
    import mpcplan
    import plan_oracle as PO
    p, q = mpcplan.default_params(), PO.default_params()
    assert ctypes.sizeof(mpcplan.PlanParams) == ctypes.sizeof(PO.PlanParams)
    for f, _ in mpcplan.PlanParams._fields_:
        a, b = getattr(p, f), getattr(q, f)
        assert (list(a) == list(b)) if f in ("u_min", "u_max") else a == b, f
    assert (p.dt, p.w_y, p.w_s, p.w_u, p.w_slack) == (0.3, 10.0, 10.0, 0.1, 100.0)
    assert (list(p.u_min), list(p.u_max), p.k_min, p.k_max, p.a_max, p.v_min) == ([-0.6, -5.0], [0.6, 4.0], -0.8, 0.8,
                                                                                   6.0, 0.0)


def test_no_gpu_fails_loudly(built):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    import mpcplan
    import workloads as W
    with pytest.raises(mpcplan.PlanError, match="no HIP device"):
        mpcplan.Planner(W.plan_route("traj1"))


def test_argument_errors(built):
    import mpcplan
    import workloads as W
    r = W.plan_route("traj1")
    h = ctypes.c_void_p()
    a = [np.ascontiguousarray(x, np.float64) for x in (r.s, r.cx, r.cy, r.vmax)]
    bad = a[0].copy()
    bad[3] = bad[2]
    p = mpcplan.default_params()
    rc = mpcplan.lib().plan_create(mpcplan._p(bad), len(bad), mpcplan._p(a[1]), mpcplan._p(a[2]), mpcplan._p(a[3]),
                                   ctypes.byref(p), 0, ctypes.byref(h))
    assert rc == -1 and "strictly increasing" in mpcplan.last_error()
    p = mpcplan.default_params(N=65)
    rc = mpcplan.lib().plan_create(*[mpcplan._p(x) for x in a[:1]], len(a[0]), *[mpcplan._p(x) for x in a[1:]],
                                   ctypes.byref(p), 0, ctypes.byref(h))
    assert rc == -1 and "N out of range" in mpcplan.last_error()
    rc = mpcplan.lib().plan_solve_chunks(None, 1, None, None, None, None, None, None, None, None, None, None)
    assert rc == -1


def test_drop_in_surface():
    """TrajectoryOptimizer keeps the reference's constructor, attributes and methods (:8-391); its dynamics
    and cost agree with the numpy restatement the oracle tests use."""
    import plan_ref as PR
    import trajectory_planning as TP
    import workloads as W
    t = TP.TrajectoryOptimizer(horizon=3.0, N=10, dt=0.3)
    for a in ("T", "N", "dt", "w_y", "w_s", "w_u", "w_slack", "u_min", "u_max", "k_min", "k_max", "a_max"):
        assert hasattr(t, a)
    for m in ("dynamics", "unpack", "pack", "cost", "optimize"):
        assert callable(getattr(t, m))
    r = W.plan_route("traj1")
    x = np.array([10.0, 0.1, 0.02, 0.05, 6.0])
    assert np.array_equal(t.dynamics(x, [0.1, -0.5], 0.03), PR.dyn(x, np.array([0.1, -0.5]), 0.03))
    rng = np.random.default_rng(2)
    z = rng.normal(0, 1, 5 * 11 + 3 * 10)
    ch = PR.Chunk(r, 10, 0.3, x, 30.0, False)
    assert abs(t.cost(z, x, r.s_total) - ch.cost(z)) <= 1e-12 * abs(ch.cost(z))
    with pytest.raises(TypeError, match="routes.Route"):
        t.optimize(x, 30.0, r.s_total, lambda s: 0.0, lambda s: 0, lambda s: 13.0, False)


def test_horizon_groups_follow_the_residency(built):
    """Planner.horizon_groups (host logic; residency stubbed, plan_chunks_per_cu needs a GPU): consecutive
    horizons share a launch while the launch sized for the largest keeps each one's residency."""
    import mpcplan
    pl = object.__new__(mpcplan.Planner)
    occ = lambda n: 4 if n <= 17 else (3 if n <= 23 else 2)
    pl.chunks_per_cu = occ
    assert pl.horizon_groups([13, 14, 17, 16, 25, 32, 13]) == [(13, 17), (25, 32)]
    assert pl.horizon_groups(np.array([20, 18, 24, 30])) == [(18, 20), (24, 30)]
    assert pl.horizon_groups([5]) == [(5, 5)]
    assert pl.horizon_groups([]) == []
    pl.h = None
