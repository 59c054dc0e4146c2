"""Diagnostic: a few egos through the device closed loop with the trajectory2 FSM; prints progress."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "safe-autonomous-driving-mpc_amd")]
import numpy as np
import __graft_entry__ as ge
ge.build()
import trajectory_tracking as TT
from trajectory_loader import TrajectoryLoader, builtin_trajectory

traj = TrajectoryLoader(builtin_trajectory(int(sys.argv[1]) if len(sys.argv) > 1 else 2))
N = int(sys.argv[2]) if len(sys.argv) > 2 else 20
mpc = TT.TrajectoryTracker(traj)
mpc.N = N
mpc.sqp_iters = int(sys.argv[3]) if len(sys.argv) > 3 else 1
x_init = np.array([[0.0, 0, 0, 0, 0.5], [1.0, 0, 0, traj.get_state(1.0)[3], 1.5]])
r = TT.run_simulation_batch(mpc, TT.ObstaclesFSM(True, True), traj, x_init=x_init, max_steps=3000, checks=True,
                            verbose=False)
print("s_max", traj.s_max, "n_steps", r["n_steps"], "checks", r.get("checks_passed"))
for b in range(2):
    n = r["n_steps"][b]
    hx = r["hist_x"][b, :n + 1]
    st = r["hist_status"][b, :n]
    print(f"ego {b}: final s {hx[-1, 0]:.1f} v {hx[-1, 4]:.2f}; status counts {np.bincount(st, minlength=4)}")
    for k in range(0, n, 250):
        print(f"   step {k}: s {hx[k, 0]:.1f} d {hx[k, 1]:.3f} v {hx[k, 4]:.2f} u {r['hist_u'][b, min(k, n - 1)]} "
              f"st {st[min(k, n - 1)]} tl {r['hist_tl'][b, min(k, n - 1)]} car {r['hist_obs_s'][b, min(k, n - 1)]:.1f}")
