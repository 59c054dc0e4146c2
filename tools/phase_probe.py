"""Diagnostic: shader cycles per kernel phase (libmpcqp_prof.so, built with -DMPC_PROF).
Prints the per-instance mean cycles of each phase for one C2 batch."""
import ctypes as C
import json
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "safe-autonomous-driving-mpc_amd")]
import numpy as np
import mpcqp
import workloads as W

import __graft_entry__ as _ge
# the diagnostic twin must be built from the current sources (build() rebuilds it unless its .srchash matches),
# so the phase numbers never describe an older kernel
_ge.build(prof=True)
mpcqp.LIB_PATH = os.path.join(ROOT, "safe-autonomous-driving-mpc_amd", "libmpcqp_prof.so")
mpcqp._lib = None   # build() loaded the product library; load the twin instead
L = mpcqp.lib()
L.mpc_debug_prof.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
cfg = sys.argv[1] if len(sys.argv) > 1 else "C2"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
extra = json.loads(sys.argv[3]) if len(sys.argv) > 3 else {}
worst = os.environ.get("PROBE_WORST")    # >0: B copies of the slowest instance of the config's batch
wb = W.make_batch(cfg, B=B if not worst else None)
ld = W.loader(wb["traj"])
slv = mpcqp.Solver(ld.X_ref, ld.U_ref, mpcqp.default_params(N=wb["N"], max_obs=wb["max_obs"], **extra))
r0 = slv.solve_batch(wb["x0"], wb["obs"], wb["n_obs"])
if worst:
    w = int(np.argmax(r0["iters"]))
    for key in ("x0", "obs", "n_obs"):
        if wb[key] is not None:
            wb[key] = np.repeat(wb[key][w:w + 1], B, axis=0)
    slv.solve_batch(wb["x0"], wb["obs"], wb["n_obs"])
buf = (C.c_ulonglong * 16)()
L.mpc_debug_prof(None, 1)
r = slv.solve_batch(wb["x0"], wb["obs"], wb["n_obs"])
L.mpc_debug_prof(buf, 0)
names = ["setup+crossover", "iter top", "residuals", "dual_norms", "weights", "riccati_factor", "pass rows",
         "riccati_solve", "update", "polish", "outputs", "pass step"]
it = r["iters"].astype(float)
tot = sum(buf[i] for i in range(12))
print(f"{cfg} B={B} mean iters {it.mean():.2f} max {it.max():.0f}; mean cycles/instance {tot / B:.0f}")
for i, n in enumerate(names):
    c = buf[i] / B
    print(f"  {n:16s} {c:12.0f} cyc/inst  {100 * buf[i] / tot:5.1f}%  {c / max(it.mean(), 1):9.0f} cyc/iter")
