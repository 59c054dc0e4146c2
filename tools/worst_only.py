"""Runs the slowest C2 instance alone (B = 2: one wavefront) a few times, for PMC counter passes."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "safe-autonomous-driving-mpc_amd")]
import numpy as np
import mpcqp
import workloads as W

cfg = sys.argv[1] if len(sys.argv) > 1 else "C2"
wb = W.make_batch(cfg)
ld = W.loader(wb["traj"])
slv = mpcqp.Solver(ld.X_ref, ld.U_ref, mpcqp.default_params(N=wb["N"], max_obs=wb["max_obs"]))
r = slv.solve_batch(wb["x0"], wb["obs"], wb["n_obs"])
w = int(np.argmax(r["iters"]))
sel = lambda a: None if a is None else np.repeat(a[w:w + 1], 2, axis=0)
for _ in range(3):
    r2 = slv.solve_batch(sel(wb["x0"]), sel(wb["obs"]), sel(wb["n_obs"]))
print("worst instance", w, "iters", r2["iters"].tolist())
