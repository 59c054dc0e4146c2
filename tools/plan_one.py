"""Smallest planner GPU check: B chunks (default 1) of horizon N on a route, against the oracle.
usage: python tools/plan_one.py [N] [B] [route]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "safe-autonomous-driving-mpc_amd"), ROOT, os.path.join(ROOT, "oracle")]
import numpy as np

import mpcplan
import plan_oracle as PO
import workloads as W

N = int(sys.argv[1]) if len(sys.argv) > 1 else 10
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1
route = sys.argv[3] if len(sys.argv) > 3 else "traj1"
r = W.plan_route(route)
wb = W.plan_batch(r, N, max(B, 4), seed=N, final_frac=0.25)
x0, st, fin = wb["x0"][:B], wb["s_target"][:B], wb["is_final"][:B]
pl = mpcplan.Planner(r, mpcplan.default_params(N=N))
g = pl.solve_chunks(x0, st, fin)
o = PO.PlanOracle(r).solve_batch(PO.default_params(N=N), x0, st, fin)
d = np.abs(g["X"] - o["X"]).reshape(B, -1).max(axis=1)
print(f"N={N} B={B} {route}: status gpu {np.bincount(g['status'], minlength=5).tolist()} oracle "
      f"{np.bincount(o['status'], minlength=5).tolist()} agree {np.mean(g['status'] == o['status']):.3f}; "
      f"max|dX| median {np.median(d):.2e} max {d.max():.2e}", flush=True)
