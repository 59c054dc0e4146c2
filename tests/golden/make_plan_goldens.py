"""Golden capture for the offline planner's acceptance check.

RUN ONLY IN THE BUILD CONTAINER (needs /root/reference, read-only).  Never shipped to / executed on
the GPU box (.gpurunignore): only the fixture it writes, tests/golden/plancheck_golden.npz, is read by
the tests.

trajectory_planning.py itself is not importable here (it imports path_planning, which needs pymap3d,
dotenv and an API key), so the planner's NLP solve is "parity unpinned".  What the reference
does hold for the planner path:
  - its committed outputs, trajectories/trajectory{1,2,3}.json (X, U, S of optimize_full_trajectory);
  - reference_trajectory_check (sanity_checks.py:3-75), which is importable.
This script runs reference_trajectory_check on the three committed trajectories and on perturbations
that drive every branch (destination, full stop, reverse driving, the curvature-rate and acceleration
checks with the AND at :48 and :54, lateral deviation, slack), and records the printed text.  The
optimizer argument only supplies u_min / u_max (TrajectoryOptimizer.__init__, trajectory_planning.py:35-36).

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_plan_goldens.py
"""
import contextlib
import io
import json
import os
import platform
import sys

sys.dont_write_bytecode = True
REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))

import numpy as np

sys.path.insert(0, REF)
import sanity_checks as RS  # noqa: E402  (reference, read-only)


class _Opt:
    """Stands in for TrajectoryOptimizer() in reference_trajectory_check: u_min / u_max only (:35-36)."""
    u_min = np.array([-0.6, -5.0])
    u_max = np.array([0.6, 4.0])


def traj(i):
    d = json.load(open(os.path.join(REF, "trajectories", f"trajectory{i}.json")))
    return np.array(d["X"]), np.array(d["U"]), np.array(d["S"])


def cases():
    out = []
    for i in (1, 2, 3):
        X, U, S = traj(i)
        out.append((f"traj{i}", X, U, S, float(X[-1, 0])))
    X, U, S = traj(1)
    st = float(X[-1, 0])
    out.append(("dest_short", X, U, S, st + 0.6))
    out.append(("dest_edge", X, U, S, st + 0.5))
    X2 = X.copy(); X2[-1, 4] = 0.2
    out.append(("no_stop", X2, U, S, st))
    X2 = X.copy(); X2[40, 4] = -0.15
    out.append(("reverse", X2, U, S, st))
    U2 = U.copy(); U2[10, 0] = -0.75
    out.append(("u1_low_only", X, U2, S, st))            # the AND at :48: passes
    U2 = U.copy(); U2[10, 0] = -0.75; U2[20, 0] = 0.75
    out.append(("u1_both", X, U2, S, st))
    U2 = U.copy(); U2[30, 1] = 4.2
    out.append(("u2_high_only", X, U2, S, st))           # the AND at :54: passes
    U2 = U.copy(); U2[30, 1] = 4.2; U2[31, 1] = -5.2
    out.append(("u2_both", X, U2, S, st))
    X2 = X.copy(); X2[50, 1] = -1.6
    out.append(("lateral", X2, U, S, st))
    S2 = S.copy(); S2[5] = -0.2
    out.append(("slack", X, U, S2, st))
    X2 = X.copy(); X2[-1, 4] = 0.2; X2[50, 1] = 1.7
    U2 = U.copy(); U2[10, 0] = -0.75; U2[20, 0] = 0.75
    out.append(("many", X2, U2, S, st + 3.0))            # several failures; passed stays False
    return out


def main():
    res = {}
    names = []
    for name, X, U, S, st in cases():
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            RS.reference_trajectory_check(_Opt(), X, U, S, st)
        names.append(name)
        res[f"{name}_X"], res[f"{name}_U"], res[f"{name}_S"] = X, U, S
        res[f"{name}_s_total"] = np.array(st)
        res[f"{name}_text"] = np.array(buf.getvalue())
    res["names"] = np.array(names)
    res["versions"] = np.array(json.dumps(dict(python=platform.python_version(), numpy=np.__version__)))
    np.savez_compressed(os.path.join(HERE, "plancheck_golden.npz"), **res)
    print(f"wrote {len(names)} cases")


if __name__ == "__main__":
    main()
