"""Diagnostic: GPU vs oracle on seeded trajectory1 batches for a list of horizons (no obstacles).
  python tools/debug_n.py [lib.so] N1 N2 ..."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "safe-autonomous-driving-mpc_amd"), os.path.join(ROOT, "oracle")]
import numpy as np
import mpcqp
import oracle as O
import workloads as W

args = sys.argv[1:]
if args and args[0].endswith(".so"):
    mpcqp.LIB_PATH = os.path.join(ROOT, "safe-autonomous-driving-mpc_amd", args.pop(0))
wb = W.make_batch("C2", B=256, seed=5)
ld = W.loader(1)
orc = O.Oracle(ld.X_ref, ld.U_ref)
for N in [int(a) for a in args] or [10, 20, 30]:
    slv = mpcqp.Solver(ld.X_ref, ld.U_ref, mpcqp.default_params(N=N))
    r = slv.solve_batch(wb["x0"])
    ro = orc.solve_batch(O.default_params(N=N), wb["x0"])
    err = np.abs(r["U"] - ro["U"]).reshape(256, -1).max(1)
    print(f"N={N}: max|dU| {err.max():.3e}, status agree {(r['status'] == ro['status']).mean():.3f}, "
          f"iters gpu mean {r['iters'].mean():.2f} max {r['iters'].max()}, oracle mean {ro['iters'].mean():.2f}", flush=True)
    slv.close()
