"""Drop-in host surface of the reference tracking MPC, backed by the MI355X library.

Reference: medinammartin3/Safe-Autonomous-Driving-MPC trajectory_tracking.py
  TrajectoryTracker  (:8-263)   same attributes (dt, N, u_min, u_max, weights, safety params),
                                 same methods; solve(x0, obstacles) -> (u0, pred_X, solve_time)
                                 now runs one QP(ubar) instance on the GPU through libmpcqp
                                 (include/mpcqp.h); solve_batch() is the batched form.
  ObstaclesFSM       (:266-374)  same update(dt, s, v) -> (obstacles, 'RED'|'GREEN') contract;
                                 both presets of the reference (trajectory2 active, trajectory3
                                 commented out at :311-327) selectable by name.
  run_simulation     (:377-443)  same loop and returned histories, plus an optional step cap.

What differs by design: the reference's SLSQP on the nonlinear problem
(ftol 1e-3, maxiter 15, finite-difference gradients) is replaced by a Gauss-Newton SQP from the
same warm start: each QP is solved to 1e-9 by a primal-dual interior point on the GPU and re-linearised
about its solution until U moves by at most `sqp_tol` (at most `sqp_iters` QPs; it also stops on a 2-cycle
and after 5 elastic QPs in a row, include/mpcqp.h).  By default solve()
therefore returns the optimum of the reference's own nonlinear problem (pinned to it by
tests/golden/nlp_golden.npz), which its SLSQP only approximates; `sqp_iters = 1` gives the single
tracking QP at the warm start that bench.py times.  Nothing falls back silently: without libmpcqp.so, or
without a GPU for a device index, solve() raises; TrajectoryTracker(X_ref, device=-1) runs the library's host
backend (config 1's CPU path).
"""
import time

import numpy as np

import mpcqp
from sanity_checks import trajectory_tracking_check

# Gauss-Newton SQP cap of the drop-in default: sqp_tol stops it earlier, after 5-8 QPs on 50 of the 52
# certified nlp_golden cases; the slowest (a braking start far inside the obstacle margin) needs 28
SQP_ITERS = 30

# TrajectoryTracker attribute -> mpc_params field
_PARAM_ATTRS = ("dt", "N", "vehicle_radius", "w_d", "w_o", "w_v", "w_u1", "w_u2", "obstacle_safety_distance",
                "max_time_2_obs", "wheelbase", "lane_width", "safe_lane_margin")
_SOLVER_ATTRS = ("linearization", "sqp_iters", "max_iter", "polish", "tol", "tol_mu", "elastic_rho",
                 "brake_distance", "brake_accel", "sqp_tol")


class TrajectoryTracker:
    """Real-time tracking MPC (Frenet kinematic model, x = [s, d, o, k, v], u = [dk/dt, dv/dt])."""

    def __init__(self, X_ref=None, device=0):
        self.X_ref = X_ref
        self.device = device
        # model / horizon (:17-18)
        self.dt = 0.2
        self.N = 5
        # actuator limits (:31-33)
        self.u_min = np.array([-0.6, -5.0])
        self.u_max = np.array([0.6, 4.0])
        self.vehicle_radius = 1.0
        # objective weights (:36-40)
        self.w_d, self.w_o, self.w_v = 10.0, 10.0, 5.0
        self.w_u1, self.w_u2 = 0.5, 0.5
        # safety (:43-47)
        self.obstacle_safety_distance = 5.0
        self.max_time_2_obs = 1.5
        self.wheelbase = 2.8
        self.lane_width = 3.0
        self.safe_lane_margin = 0.1
        # GPU solver knobs.  The SQP defaults make solve() return the optimum of the reference's nonlinear
        # problem (nlp_golden); the other values are those of mpc_default_params
        self.linearization = 1
        self.sqp_iters = SQP_ITERS
        self.sqp_tol = 1e-10
        self.max_iter = 80
        self.polish = 2
        self.tol = 1e-9
        self.tol_mu = 1e-10
        self.elastic_rho = 1e5
        self.brake_distance = 40.0
        self.brake_accel = -2.0
        self.last_status = None
        self.last_iters = None
        self._solver = None
        self._solver_key = None

    # ---- model utilities (host-side numpy, same arithmetic as the reference) --------------
    def dynamics(self, x, u, k_ref):
        """x_dot = [v, v*o, v*(k - k_ref), u1, u2]  (:50-67)."""
        s, d, o, k, v = x
        return np.array([v, v * o, v * (k - k_ref), u[0], u[1]])

    def unpack(self, U_flat):
        return np.asarray(U_flat).reshape(self.N, 2)

    @staticmethod
    def pack(U):
        return np.asarray(U).ravel()

    def predict(self, x0, U_flat):
        """Explicit-Euler rollout over the horizon (:87-114)."""
        U = self.unpack(U_flat)
        X = np.zeros((self.N + 1, 5))
        X[0] = x0
        x = np.array(x0, dtype=np.float64)
        for j in range(self.N):
            x = x + self.dt * self.dynamics(x, U[j], self.X_ref.get_state(x[0])[3])
            X[j + 1] = x
        return X

    def cost(self, U_flat, x0):
        """Tracking + comfort objective (:116-152)."""
        U = self.unpack(U_flat)
        X = self.predict(x0, U_flat)
        c = 0.0
        for row in X[1:]:
            r = self.X_ref.get_state(row[0])
            c += self.w_d * (row[1] - r[1]) ** 2 + self.w_o * (row[2] - r[2]) ** 2 + self.w_v * (row[4] - r[4]) ** 2
        return c + float(np.sum(self.w_u1 * U[:, 0] ** 2 + self.w_u2 * U[:, 1] ** 2))

    def constraints(self, x0, obstacles):
        """{'type': 'ineq', 'fun': g(U) >= 0}, rows in the reference order (:155-211)."""
        sl = self.lane_width / 2.0 - self.vehicle_radius - self.safe_lane_margin

        def g(U_flat):
            X = self.predict(x0, U_flat)
            out = []
            for j in range(1, self.N + 1):
                s, d, o, _, v = X[j]
                for c in (0.0, self.wheelbase / 2.0, self.wheelbase):
                    e = d + c * o
                    out += [sl - e, e + sl]
                for ob in obstacles:
                    out.append(ob["s"] + ob["v"] * (j * self.dt) - s - max(self.obstacle_safety_distance,
                                                                             v * self.max_time_2_obs))
                out.append(v)
            return np.array(out)
        return {"type": "ineq", "fun": g}

    # ---- the GPU path ----------------------------------------------------------------------
    def params(self, max_obs=0):
        p = mpcqp.default_params()
        for a in _PARAM_ATTRS + _SOLVER_ATTRS:
            setattr(p, a, type(getattr(p, a))(getattr(self, a)))
        p.u_min[0], p.u_min[1] = float(self.u_min[0]), float(self.u_min[1])
        p.u_max[0], p.u_max[1] = float(self.u_max[0]), float(self.u_max[1])
        p.max_obs = int(max_obs)
        return p

    def solver(self, max_obs=0):
        """The libmpcqp context for X_ref (created on first use, parameters re-synced every call)."""
        if self.X_ref is None:
            raise ValueError("TrajectoryTracker needs X_ref (a TrajectoryLoader) to solve")
        key = id(self.X_ref)
        p = self.params(max_obs)
        if self._solver is None or self._solver_key != key:
            self._solver = mpcqp.Solver(self.X_ref.X_ref, self.X_ref.U_ref, p, device=self.device)
            self._solver_key = key
        else:
            self._solver.set_params(p)
        return self._solver

    def solve(self, x0, obstacles):
        """u0, pred_X, solve_time for one state (drop-in for :213-263).

        obstacles: list of {'s': position, 'v': speed, ...}; 'type' is ignored like the reference.
        solve_time covers the library call (host->device->host), as the reference timed minimize()."""
        obs = np.array([[float(o["s"]), float(o["v"])] for o in obstacles], dtype=np.float64).reshape(-1, 2)
        slv = self.solver(max_obs=len(obs))
        t0 = time.time()
        r = slv.solve_batch(np.asarray(x0, np.float64).reshape(1, 5),
                            obs.reshape(1, -1, 2) if len(obs) else None,
                            np.array([len(obs)], np.int32) if len(obs) else None)
        solve_time = time.time() - t0
        self.last_status = int(r["status"][0])
        self.last_iters = int(r["iters"][0])
        return r["U"][0][0].copy(), r["Xpred"][0].copy(), solve_time

    def solve_batch(self, x0, obstacles=None, ubar=None):
        """Batched solve: x0 [B,5]; obstacles: list (len B) of obstacle lists, or an array [B,M,2]."""
        x0 = np.asarray(x0, np.float64).reshape(-1, 5)
        B = x0.shape[0]
        obs = n = None
        if obstacles is not None:
            if isinstance(obstacles, np.ndarray):
                obs = obstacles.reshape(B, -1, 2)
                n = np.full(B, obs.shape[1], np.int32)
            else:
                mo = max((len(o) for o in obstacles), default=0)
                if mo:
                    obs = np.zeros((B, mo, 2))
                    n = np.zeros(B, np.int32)
                    for b, lst in enumerate(obstacles):
                        n[b] = len(lst)
                        for i, o in enumerate(lst):
                            obs[b, i] = (o["s"], o["v"])
        slv = self.solver(max_obs=0 if obs is None else obs.shape[1])
        return slv.solve_batch(x0, obs, n, ubar)


# ---------------------------------------------------------------------------------------------
# obstacle scenario state machine (trajectory_tracking.py:266-374)
# ---------------------------------------------------------------------------------------------
FSM_PRESETS = {
    # trajectory_tracking.py:292-308 (active in the reference)
    "trajectory2": dict(obs_trigger_s=710.0, obs_start_s=780.0, obs_v=4.0, obs_end_s=1050.0,
                        tl_pos=550.0, tl_trigger_s=100.0, tl_stop_duration=20.0),
    # trajectory_tracking.py:311-327 (commented out in the reference)
    "trajectory3": dict(obs_trigger_s=5.0, obs_start_s=150.0, obs_v=4.0, obs_end_s=850.0,
                        tl_pos=2000.0, tl_trigger_s=100.0, tl_stop_duration=20.0),
}


class ObstaclesFSM:
    """One dynamic car (WAITING -> ACTIVE -> COMPLETED) and one traffic light
    (RED_APPROACH -> RED_WAITING -> GREEN); update() returns the obstacles the MPC must respect."""

    def __init__(self, dynamic_obstacle=False, traffic_light=False, preset="trajectory2"):
        self.dynamic_obstacle = dynamic_obstacle
        self.traffic_light = traffic_light
        for k, v in FSM_PRESETS[preset].items():
            setattr(self, k, v)
        self.obs_active = False
        self.obs_has_triggered = False
        self.obs_s = self.obs_start_s
        self.tl_state = "RED"
        self.tl_timer = 0.0
        self.tl_waiting = False

    def update(self, dt, s, v):
        active = []
        if self.dynamic_obstacle:
            if s >= self.obs_trigger_s and not self.obs_has_triggered:
                self.obs_has_triggered = self.obs_active = True
            if self.obs_active:
                self.obs_s += self.obs_v * dt
                if self.obs_s > self.obs_end_s:
                    self.obs_active = False
                else:
                    active.append({"s": self.obs_s, "v": self.obs_v, "type": "car"})
        if self.traffic_light and self.tl_state == "RED":
            gap = self.tl_pos - s
            if 0 < gap < self.tl_trigger_s:
                active.append({"s": self.tl_pos, "v": 0.0, "type": "light"})
                if v < 0.1 and gap < 10.0:
                    self.tl_waiting = True
            if self.tl_waiting:
                self.tl_timer += dt
                if self.tl_timer >= self.tl_stop_duration:
                    self.tl_state = "GREEN"
                    self.tl_waiting = False
        return active, self.tl_state


def run_simulation(mpc, fsm, trajectory, max_steps=None, verbose=True):
    """Closed loop of trajectory_tracking.py:377-443 (same histories); max_steps caps the loop
    (the reference has no cap and spins forever if the ego stalls)."""
    x = np.array([0.0, 0.0, 0.0, 0.0, 0.5])
    hist_x, hist_u, hist_t, hist_preds, hist_obs_s, hist_tl_state = [x], [], [], [], [], []
    step = 0
    while x[0] <= trajectory.s_max - 1.0 and (max_steps is None or step < max_steps):
        obstacles, tl_state = fsm.update(mpc.dt, x[0], x[4])
        u, pred_X, cpu = mpc.solve(x, obstacles)
        k_ref = trajectory.get_state(x[0])[3]
        x = x + mpc.dt * mpc.dynamics(x, u, k_ref)       # plant == prediction model (:404-406)
        hist_x.append(x)
        hist_u.append(u)
        hist_t.append(cpu)
        hist_preds.append(pred_X)
        hist_tl_state.append(tl_state)
        car = [o["s"] for o in obstacles if o["type"] == "car"]
        hist_obs_s.append(car[0] if car else np.nan)
        if verbose and step % 50 == 0:
            print(progress_line(step, x, tl_state, hist_obs_s[-1], fsm, mpc.obstacle_safety_distance))
        step += 1
    trajectory_tracking_check(mpc, hist_x, hist_u, hist_t, hist_obs_s, hist_tl_state, fsm, trajectory.s_max)
    return (np.array(hist_x), np.array(hist_u), np.array(hist_t), hist_preds, hist_obs_s, hist_tl_state,
            trajectory)


def progress_line(step, x, tl_state, obstacle_s, fsm, safety_distance=5.0):
    """The reference's progress print of run_simulation (trajectory_tracking.py:423-435), verbatim format."""
    vehicle_info = f"s={x[0]:.1f}m, v={x[4] * 3.6:.1f}km/h"
    if fsm.traffic_light:
        dist_2_tl = fsm.tl_pos - x[0]
        tl_info = (f"color={tl_state}, distance={dist_2_tl:.1f}m" if dist_2_tl > safety_distance
                   else f"color={tl_state}, distance=NaN")
    else:
        tl_info = "NaN"
    obs_info = f"{obstacle_s - x[0]:.1f}m" if not np.isnan(obstacle_s) else "NaN"
    return f"Step {step} | {vehicle_info} | Traffic Light : {tl_info} | Distance to obstacle : {obs_info}"


def fsm_params(fsm):
    """mpc_fsm (include/mpcqp.h) of an ObstaclesFSM, or None when it has no scenario switched on."""
    if fsm is None or not (fsm.dynamic_obstacle or fsm.traffic_light):
        return None
    return mpcqp.default_fsm(dynamic_obstacle=int(bool(fsm.dynamic_obstacle)), traffic_light=int(bool(fsm.traffic_light)),
                             **{k: float(getattr(fsm, k)) for k in FSM_PRESETS["trajectory2"]})


def run_simulation_batch(mpc, fsm, trajectory, x_init=None, B=1, max_steps=2000, checks=False, verbose=False):
    """run_simulation (trajectory_tracking.py:377-443) for B independent egos, entirely on the device
    (mpc_closed_loop): each ego owns a fresh copy of `fsm`'s scenario, the loop runs while
    s <= s_max - 1.  x_init [B,5] defaults to the reference start [0,0,0,0,0.5] (:382).
    Returns the device histories (see mpcqp.Solver.closed_loop); with checks=True also runs the
    restated trajectory_tracking_check on every ego and adds 'checks_passed' [B]."""
    if x_init is None:
        x_init = np.tile(np.array([0.0, 0.0, 0.0, 0.0, 0.5]), (B, 1))
    x_init = np.asarray(x_init, np.float64).reshape(-1, 5)
    r = mpc.solver(max_obs=0).closed_loop(x_init, fsm_params(fsm), max_steps=max_steps, s_max=trajectory.s_max)
    if checks:
        r["checks_passed"] = closed_loop_checks(mpc, fsm, trajectory, r, verbose)
    return r


def closed_loop_checks(mpc, fsm, trajectory, r, verbose=False):
    """The restated trajectory_tracking_check (sanity_checks.py:79-184) on every ego of a closed_loop()
    result (mpcqp.Solver.closed_loop layout); returns the per-ego verdicts [B] (bool)."""
    import contextlib
    import io
    B = np.asarray(r["n_steps"]).size
    ok = np.zeros(B, bool)
    for b in range(B):
        n = int(r["n_steps"][b])
        # the solve time this ego waited for at each of its steps: that batched step's device time
        # (the reference tests max(hist_t) per step, sanity_checks.py:134-135; shard.closed_loop_quantities)
        step_s = np.asarray(r["step_ms"][:n], np.float64) / 1e3
        f = ObstaclesFSM(fsm.dynamic_obstacle, fsm.traffic_light) if fsm is not None else ObstaclesFSM()
        if fsm is not None:
            for k in FSM_PRESETS["trajectory2"]:
                setattr(f, k, getattr(fsm, k))
        buf = io.StringIO()
        tl = ["GREEN" if t == 1 else "RED" for t in r["hist_tl"][b, :n]]
        with contextlib.redirect_stdout(buf):
            ok[b] = bool(trajectory_tracking_check(mpc, list(r["hist_x"][b, :n + 1]), list(r["hist_u"][b, :n]),
                                                   list(step_s), list(r["hist_obs_s"][b, :n]), tl, f,
                                                   trajectory.s_max))
        if verbose:
            print(buf.getvalue())
    return ok


if __name__ == "__main__":
    from trajectory_loader import TrajectoryLoader, builtin_trajectory
    traj = TrajectoryLoader(builtin_trajectory(2))
    run_simulation(TrajectoryTracker(traj), ObstaclesFSM(dynamic_obstacle=True, traffic_light=True), traj)
