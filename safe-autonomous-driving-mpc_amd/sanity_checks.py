"""trajectory_tracking_check — restated acceptance checks over closed-loop telemetry.

Same checks, tolerances and prints as sanity_checks.py:79-184 of the reference
(destination within 1 m, |d| <= 1.5 m, controls within bounds +-0.1, max solve time <= 150 ms,
dynamic-obstacle gap >= 1 m, no RED-light pass).  Returns the bool like the reference.
`check_summary` is the silent, structured form used by the batched closed loop and the bench.

reference_trajectory_check restates the planner's acceptance check (sanity_checks.py:3-75), including its
AND at :48 and :54 (a control check fails only when both of its limits are exceeded); `plan_check_summary`
is its silent form.
"""
import numpy as np

LATERAL_LIMIT = 1.5
CONTROLS_TOL = 0.1
CPU_LIMIT = 150      # ms
SAFETY_DIST = 1.0


def check_quantities(hist_x, hist_u, hist_t, hist_obs_s, hist_tl_red, dynamic_obstacle, traffic_light, tl_pos):
    """What sanity_checks.py:79-184 measures over one closed-loop run (the inputs of the verdicts):
    final s, max |d|, control extremes, max solve time, min gap to the dynamic obstacle (NaN if it never
    existed) and whether the ego crossed tl_pos while the light was RED.  Per ego, on the rank that ran it."""
    hist_x = np.asarray(hist_x, np.float64)
    hist_u = np.asarray(hist_u, np.float64).reshape(-1, 2)
    hist_t = np.asarray(hist_t, np.float64)
    q = {"s_final": float(hist_x[-1, 0]), "max_dev": float(np.max(np.abs(hist_x[:, 1])))}
    q["u1_min"], q["u1_max"] = float(np.min(hist_u[:, 0])), float(np.max(hist_u[:, 0]))
    q["u2_min"], q["u2_max"] = float(np.min(hist_u[:, 1])), float(np.max(hist_u[:, 1]))
    q["max_cpu_ms"] = float(np.max(hist_t) * 1000) if hist_t.size else 0.0
    q["min_obs_dist"] = float("nan")
    if dynamic_obstacle:                                                              # :141-161
        obs_s = np.asarray(hist_obs_s, np.float64)
        valid = ~np.isnan(obs_s)
        if np.any(valid):
            m = min(len(hist_x), len(obs_s))
            q["min_obs_dist"] = float(np.min(obs_s[:m][valid[:m]] - hist_x[:m, 0][valid[:m]]))
    q["red_pass"] = 0.0
    if traffic_light:                                                                 # :163-181
        idx = np.where(hist_x[:, 0] > tl_pos)[0]
        if len(idx) > 0 and idx[0] < len(hist_tl_red) and bool(hist_tl_red[idx[0]]):
            q["red_pass"] = 1.0
    return q


def check_verdicts(q, u_min, u_max, s_total):
    """The verdicts of sanity_checks.py:79-184 from check_quantities' measurements (a dict, or any mapping
    with the same keys: rank 0 applies this to the gathered per-ego summaries of every rank)."""
    v = {"destination": not (q["s_final"] < s_total - 1.0),                            # :97-103
         "on_road": not (q["max_dev"] > LATERAL_LIMIT),                                # :105-111
         "steer_ok": not ((q["u1_min"] < u_min[0] - CONTROLS_TOL) or (q["u1_max"] > u_max[0] + CONTROLS_TOL)),
         "accel_ok": not ((q["u2_min"] < u_min[1] - CONTROLS_TOL) or (q["u2_max"] > u_max[1] + CONTROLS_TOL)),
         "realtime": not (q["max_cpu_ms"] > CPU_LIMIT),                                # :133-139
         "obstacle_ok": bool(np.isnan(q["min_obs_dist"]) or not (q["min_obs_dist"] < SAFETY_DIST)),
         "light_ok": not q["red_pass"]}
    v["passed"] = all(v.values())
    return v


def check_summary(u_min, u_max, hist_x, hist_u, hist_t, hist_obs_s, hist_tl_red, dynamic_obstacle,
                  traffic_light, tl_pos, s_total):
    """All checks of sanity_checks.py:79-184 as a dict of bools (+ the measured quantities)."""
    q = check_quantities(hist_x, hist_u, hist_t, hist_obs_s, hist_tl_red, dynamic_obstacle, traffic_light, tl_pos)
    out = dict(q)
    out.update(check_verdicts(q, u_min, u_max, s_total))
    return out


def trajectory_tracking_check(tracker, hist_x, hist_u, hist_t, hist_obs_s, hist_tl_state, fsm, s_total):
    """Verifies safety, performance and real-time constraints of a tracking run (prints like the reference)."""
    print("\n=== SANITY CHECKS ===")
    red = [s == "RED" for s in hist_tl_state]
    r = check_summary(tracker.u_min, tracker.u_max, hist_x, hist_u, hist_t, hist_obs_s, red,
                      fsm.dynamic_obstacle, fsm.traffic_light, getattr(fsm, "tl_pos", 0.0), s_total)
    if not r["destination"]:
        print(f'Destination reached : False --> Stopped at {r["s_final"]:.1f}/{s_total:.1f} m')
    else:
        print('Destination reached : True')
    if not r["on_road"]:
        print(f'Stayed on road : False --> Max Deviation = {r["max_dev"]:.2f} m')
    else:
        print('Stayed on road : True')
    print(f'Steering controls within limits : {r["steer_ok"]}')
    print(f'Acceleration controls within limits : {r["accel_ok"]}')
    if not r["realtime"]:
        print(f'Real-time constraint respected : False --> Max CPU time {r["max_cpu_ms"]:.1f}ms > {CPU_LIMIT}ms')
    else:
        print('Real-time constraint respected : True')
    if fsm.dynamic_obstacle and not np.isnan(r["min_obs_dist"]):
        if not r["obstacle_ok"]:
            print(f'Dynamic Obstacle Avoided : False --> Min Distance = {r["min_obs_dist"]:.2f} m')
        else:
            print('Dynamic Obstacle Avoided : True')
    if fsm.traffic_light:
        print('Traffic Light Respected : False (Ran a RED light)' if not r["light_ok"]
              else 'Traffic Light Respected : True')
    print(f'===> Checks passed : {r["passed"]}')
    return r["passed"]


# ---------------------------------------------------------------------------------------------
# offline planner acceptance check (sanity_checks.py:3-75)
# ---------------------------------------------------------------------------------------------
PLAN_DISTANCE_TOL = 0.5      # m
PLAN_VELOCITY_TOL = 0.1
PLAN_CONTROLS_TOL = 0.1
PLAN_LATERAL_DEV_TOL = 1.5   # m
PLAN_SLACK_TOL = 0.1


def plan_check_summary(u_min, u_max, X, U, S, s_total):
    """The measurements and verdicts of reference_trajectory_check, without printing."""
    X, U, S = np.asarray(X, np.float64), np.asarray(U, np.float64).reshape(-1, 2), np.asarray(S, np.float64)
    q = {"error_s": abs(X[-1, 0] - s_total), "v_final": X[-1, 4], "min_v": np.min(X[:, 4]),
         "max_lat_dev": np.max(np.abs(X[:, 1])), "max_slack": np.max(np.abs(S))}
    q["destination"] = not (q["error_s"] > PLAN_DISTANCE_TOL)                                 # :19-25
    q["full_stop"] = not (abs(q["v_final"]) > PLAN_VELOCITY_TOL)                             # :27-33
    q["forward"] = not (q["min_v"] < -PLAN_VELOCITY_TOL)                                     # :35-41
    # :48 and :54: a control check fails only if BOTH of its limits are exceeded (the reference's AND)
    q["u1_ok"] = not (np.min(U[:, 0]) < u_min[0] - PLAN_CONTROLS_TOL and np.max(U[:, 0]) > u_max[0] + PLAN_CONTROLS_TOL)
    q["u2_ok"] = not (np.min(U[:, 1]) < u_min[1] - PLAN_CONTROLS_TOL and np.max(U[:, 1]) > u_max[1] + PLAN_CONTROLS_TOL)
    q["lateral_ok"] = not (q["max_lat_dev"] > PLAN_LATERAL_DEV_TOL)                          # :59-65
    q["slack_ok"] = not (q["max_slack"] > PLAN_SLACK_TOL)                                    # :67-73
    passed = q["destination"] and q["full_stop"] and q["forward"]
    if passed:                                                                               # :50-51, :56-57
        passed = q["u1_ok"]
    if passed:
        passed = q["u2_ok"]
    q["passed"] = bool(passed and q["lateral_ok"] and q["slack_ok"])
    return q


def reference_trajectory_check(optimizer, X, U, S, s_total):
    """Verifies the physical feasibility of a planned reference trajectory (prints like the reference,
    sanity_checks.py:3-75; returns None like it, see plan_check_summary for the verdicts)."""
    print("\n=== SANITY CHECKS ===")
    q = plan_check_summary(optimizer.u_min, optimizer.u_max, X, U, S, s_total)
    print(f'Final destination reached : False --> Error = {q["error_s"]} m' if not q["destination"]
          else 'Final destination reached : True')
    print(f'Full stop at the end : False --> Final velocity = {q["v_final"] * 3.6} km/h' if not q["full_stop"]
          else 'Full stop at the end : True')
    print(f'Always non-negative velocity : False --> Minimum velocity = {q["min_v"] * 3.6} km/h' if not q["forward"]
          else 'Always non-negative velocity : True')
    print(f'Curvature rate limits respected : {q["u1_ok"]}')
    print(f'Acceleration limits respected : {q["u2_ok"]}')
    print(f'Lateral deviation respected : False --> Maximum lateral deviation : {q["max_lat_dev"]} m'
          if not q["lateral_ok"] else 'Lateral deviation respected : True')
    print(f'Low slack usage : False --> Maximum slack value : {q["max_slack"]}' if not q["slack_ok"]
          else 'Low slack usage : True')
    print(f'===> Checks passed : {q["passed"]}')
