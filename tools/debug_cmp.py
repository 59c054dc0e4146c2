"""Diagnostic: GPU vs oracle on a seeded batch; prints the instances whose status or U differ."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "safe-autonomous-driving-mpc_amd"), os.path.join(ROOT, "oracle")]
import numpy as np
import __graft_entry__ as ge
ge.build()
import mpcqp
import oracle as O
import workloads as W

cfg = sys.argv[1] if len(sys.argv) > 1 else "C5"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 128
seed = int(sys.argv[3]) if len(sys.argv) > 3 else 1234
seed = None if seed < 0 else seed        # < 0: the config's own seed (the bench batch)
wb = W.make_batch(cfg, B=B, seed=seed)
ld = W.loader(wb["traj"])
slv = mpcqp.Solver(ld.X_ref, ld.U_ref, mpcqp.default_params(N=wb["N"], max_obs=wb["max_obs"]))
r = slv.solve_batch(wb["x0"], wb["obs"], wb["n_obs"])
orc = O.Oracle(ld.X_ref, ld.U_ref)
ro = orc.solve_batch(O.default_params(N=wb["N"], max_obs=wb["max_obs"]), wb["x0"], wb["obs"], wb["n_obs"])
err = np.abs(r["U"] - ro["U"]).reshape(B, -1).max(axis=1)
bad = np.flatnonzero((r["status"] != ro["status"]) | (err > 1e-6))
print(f"{cfg} B={B}: status agree {np.mean(r['status'] == ro['status']):.4f}, max err {err.max():.3e}")
print("gpu status counts", np.bincount(r["status"], minlength=4), "oracle", np.bincount(ro["status"], minlength=4))
for i in bad[:20]:
    print(f"  #{i}: gpu st {r['status'][i]} it {r['iters'][i]}  oracle st {ro['status'][i]} it {ro['iters'][i]}  "
          f"|dU| {err[i]:.3e}  x0 {np.array2string(wb['x0'][i], precision=4)}")
d = r["iters"].astype(int) - ro["iters"].astype(int)
print("iteration difference gpu - oracle: max", d.max(), "min", d.min(), "n(|d|>2)", int((np.abs(d) > 2).sum()),
      "gpu max", r["iters"].max(), "oracle max", ro["iters"].max())
for i in np.argsort(-np.abs(d))[:5]:
    print(f"  #{i}: gpu st {r['status'][i]} it {r['iters'][i]}  oracle st {ro['status'][i]} it {ro['iters'][i]}  |dU| {err[i]:.3e}")
