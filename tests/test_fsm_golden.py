"""ObstaclesFSM, the closed-loop prints and the acceptance checks, pinned to the reference's own
closed-loop runs (tests/golden/closedloop_golden.npz, captured by make_goldens.gen_closedloop from
run_simulation, trajectory_tracking.py:377-443).  CPU only: the golden histories are replayed through
the shim's host-side restatements.

  - ObstaclesFSM.update (trajectory_tracking.py:330-374): fed the golden (s, v) of every step, it must
    reproduce the golden car positions and light states bit for bit, for the trajectory2 preset
    (:292-308, active in the reference) and the trajectory3 preset (:311-327, commented out there);
  - progress_line: the reference's every-50-steps print (:423-435), character for character;
  - trajectory_tracking_check (sanity_checks.py:79-184): the verdict block printed over the golden
    histories equals the block the reference printed.
"""
import contextlib
import io

import numpy as np
import pytest

from conftest import load_golden

RUNS = [("c1_traj1_N10", 1, False, False, "trajectory2"), ("traj2_N5_fsm", 2, True, True, "trajectory2"),
        ("traj3_N5_fsm", 3, True, True, "trajectory3")]


@pytest.fixture(scope="module")
def golden():
    return load_golden("closedloop_golden")


def _replay(g, tag, dyn, tl, preset):
    import trajectory_tracking as TT
    fsm = TT.ObstaclesFSM(dynamic_obstacle=dyn, traffic_light=tl, preset=preset)
    hx = g[f"{tag}_hist_x"]
    obs_s, red, lists = [], [], []
    for j in range(len(hx) - 1):
        obstacles, tl_state = fsm.update(0.2, hx[j, 0], hx[j, 4])
        car = [o["s"] for o in obstacles if o["type"] == "car"]
        obs_s.append(car[0] if car else np.nan)
        red.append(tl_state == "RED")
        lists.append(obstacles)
    return fsm, np.array(obs_s), np.array(red), lists


@pytest.mark.parametrize("tag,ti,dyn,tl,preset", RUNS)
def test_fsm_replay_bit_exact(golden, tag, ti, dyn, tl, preset):
    fsm, obs_s, red, lists = _replay(golden, tag, dyn, tl, preset)
    g_obs = golden[f"{tag}_hist_obs_s"]
    g_red = golden[f"{tag}_hist_tl_red"]
    assert obs_s.shape == g_obs.shape
    # NaN where no car; every position bit-identical (repeated float additions, :345)
    assert np.array_equal(np.isnan(obs_s), np.isnan(g_obs))
    assert np.array_equal(obs_s[~np.isnan(obs_s)], g_obs[~np.isnan(g_obs)])
    assert np.array_equal(red, g_red)
    if dyn:
        # the scenario actually ran: the car appeared, and (trajectory2) the light went GREEN after the wait
        assert np.isfinite(g_obs).sum() > 50
    if tl and ti == 2:
        assert g_red[0] and not g_red[-1]
    # the light is emitted as a v = 0 obstacle at tl_pos while RED and within tl_trigger_s (:357-361)
    for obstacles, x in zip(lists, golden[f"{tag}_hist_x"]):
        lights = [o for o in obstacles if o["type"] == "light"]
        if lights:
            assert lights[0]["v"] == 0.0 and 0 < fsm.tl_pos - x[0] < fsm.tl_trigger_s


@pytest.mark.parametrize("tag,ti,dyn,tl,preset", RUNS)
def test_progress_prints_match_reference(golden, tag, ti, dyn, tl, preset):
    import trajectory_tracking as TT
    log = str(golden[f"{tag}_log"])
    ref_lines = [ln for ln in log.splitlines() if ln.startswith("Step ")]
    fsm = TT.ObstaclesFSM(dynamic_obstacle=dyn, traffic_light=tl, preset=preset)
    hx, hobs, hred = golden[f"{tag}_hist_x"], golden[f"{tag}_hist_obs_s"], golden[f"{tag}_hist_tl_red"]
    mine = [TT.progress_line(j, hx[j + 1], "RED" if hred[j] else "GREEN", hobs[j], fsm)
            for j in range(0, len(hx) - 1, 50)]
    assert mine == ref_lines


@pytest.mark.parametrize("tag,ti,dyn,tl,preset", RUNS)
def test_check_verdicts_match_reference(golden, tag, ti, dyn, tl, preset):
    import trajectory_tracking as TT
    from sanity_checks import check_summary, trajectory_tracking_check
    from trajectory_loader import TrajectoryLoader, builtin_trajectory
    traj = TrajectoryLoader(builtin_trajectory(ti))
    fsm = TT.ObstaclesFSM(dynamic_obstacle=dyn, traffic_light=tl, preset=preset)
    hx, hu, ht = golden[f"{tag}_hist_x"], golden[f"{tag}_hist_u"], golden[f"{tag}_hist_t"]
    hobs, hred = golden[f"{tag}_hist_obs_s"], golden[f"{tag}_hist_tl_red"]
    states = ["RED" if r else "GREEN" for r in hred]
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        passed = trajectory_tracking_check(TT.TrajectoryTracker(), list(hx), list(hu), list(ht), list(hobs), states,
                                           fsm, traj.s_max)
    log = str(golden[f"{tag}_log"])
    ref_block = log[log.index("=== SANITY CHECKS ==="):].strip()
    assert buf.getvalue().strip() == ref_block
    assert passed == ("===> Checks passed : True" in ref_block)
    # the structured form agrees with the printed verdicts
    s = check_summary((-0.6, -5.0), (0.6, 4.0), hx, hu, ht, hobs, hred, dyn, tl, fsm.tl_pos, traj.s_max)
    assert s["passed"] == passed
    # the reference's only failures on these runs are the real-time check (python SLSQP)
    assert s["destination"] and s["on_road"] and s["steer_ok"] and s["accel_ok"] and s["obstacle_ok"] and s["light_ok"]
