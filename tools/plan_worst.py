"""The planner's slowest chunks alone (bench.py's plan-leg mix, seed 7), each repeated R times in one launch,
on the product library: wall time per launch.  For PC sampling / single-chunk latency.
usage: python tools/plan_worst.py <route> <B> i1,i2,... [R]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "safe-autonomous-driving-mpc_amd"), ROOT]
import numpy as np  # noqa: E402

import mpcplan  # noqa: E402
import workloads as W  # noqa: E402

if os.environ.get("PLAN_LIB"):      # A/B of library variants
    mpcplan.LIB_PATH = os.path.join(ROOT, "safe-autonomous-driving-mpc_amd", os.environ["PLAN_LIB"])

route, B, idx = sys.argv[1], int(sys.argv[2]), [int(x) for x in sys.argv[3].split(",")]
R = int(sys.argv[4]) if len(sys.argv) > 4 else 1
r = W.plan_route(route)
wb = W.plan_batch_ref(r, B, seed=7)
for i in idx:
    n = int(wb["N"][i])
    pl = mpcplan.Planner(r, mpcplan.default_params(N=n))
    rep = lambda a: np.repeat(a[i:i + 1], R, axis=0)
    for t in range(2):
        t0 = time.perf_counter()
        g = pl.solve_chunks(rep(wb["x0"]), rep(wb["s_target"]), rep(wb["is_final"]))
        dt = time.perf_counter() - t0
    print(f"{route} chunk {i} N={n} x{R}: {dt * 1e3:.1f} ms, sqp {int(g['sqp'][0])}, ipm iters {int(g['iters'][0])}, "
          f"{dt / max(1, int(g['iters'][0])) * 1e6:.1f} us per interior-point iteration", flush=True)
    pl.close()
