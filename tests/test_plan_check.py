"""The offline planner's acceptance check, restated (package sanity_checks.reference_trajectory_check,
reference sanity_checks.py:3-75), against the reference's own printed verdicts captured by
tests/golden/make_plan_goldens.py: the three committed planner outputs (trajectories/*.json) and
perturbations that drive every branch, including the AND at :48 / :54."""
import contextlib
import io

import numpy as np

from conftest import load_golden


class _Opt:
    u_min = np.array([-0.6, -5.0])
    u_max = np.array([0.6, 4.0])


def test_reference_trajectory_check_matches_golden_text():
    import sanity_checks as SC
    g = load_golden("plancheck_golden")
    names = [str(n) for n in g["names"]]
    assert len(names) == 14
    for n in names:
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            SC.reference_trajectory_check(_Opt(), g[f"{n}_X"], g[f"{n}_U"], g[f"{n}_S"], float(g[f"{n}_s_total"]))
        assert buf.getvalue() == str(g[f"{n}_text"]), n
        q = SC.plan_check_summary(_Opt.u_min, _Opt.u_max, g[f"{n}_X"], g[f"{n}_U"], g[f"{n}_S"],
                                  float(g[f"{n}_s_total"]))
        assert q["passed"] == ("===> Checks passed : True" in str(g[f"{n}_text"])), n
