"""Tail-latency probe: is the batch time set by throughput or by the slowest instance?
Times one launch of (a) the full C2 batch, (b) B copies of its slowest instance, (c) that instance
alone, (d) B copies of a crossover-certified instance."""
import os
import sys
import json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "safe-autonomous-driving-mpc_amd")]
import numpy as np
import torch
import mpcqp
import workloads as W

cfg = sys.argv[1] if len(sys.argv) > 1 else "C2"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
wb = W.make_batch(cfg, B=B)
N, mo = wb["N"], wb["max_obs"]
ld = W.loader(wb["traj"])
slv = mpcqp.Solver(ld.X_ref, ld.U_ref, mpcqp.default_params(N=N, max_obs=mo))
dev = torch.device("cuda", 0)
stream = torch.cuda.current_stream(dev)
ptr = lambda x: 0 if x is None else x.data_ptr()


def run(x0n, obsn, nobn, reps=5):
    b = x0n.shape[0]
    t = lambda a, dt=torch.float64: torch.as_tensor(a, dtype=dt, device=dev).contiguous()
    x0 = t(x0n)
    obs = t(obsn) if obsn is not None else None
    nob = t(nobn, torch.int32) if nobn is not None else None
    u0 = torch.empty((b, 2), dtype=torch.float64, device=dev)
    Uo = torch.empty((b, N, 2), dtype=torch.float64, device=dev)
    Xo = torch.empty((b, N + 1, 5), dtype=torch.float64, device=dev)
    st = torch.empty(b, dtype=torch.int32, device=dev)
    it = torch.empty(b, dtype=torch.int32, device=dev)
    args = lambda: (b, ptr(x0), ptr(obs), ptr(nob), 0, ptr(u0), ptr(Uo), ptr(Xo), ptr(st), ptr(it), stream.cuda_stream)
    for _ in range(2):
        slv.solve_batch_device(*args())
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        slv.solve_batch_device(*args())
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps, it.cpu().numpy()


ms, its = run(wb["x0"], wb["obs"], wb["n_obs"])
w = int(np.argmax(its))
easy = int(np.argmin(its))
sel = lambda a, i, n: None if a is None else np.repeat(a[i:i + 1], n, axis=0)
res = {"full": ms, "max_iters": int(its.max()), "worst": w}
res["worst_xB"], _ = run(sel(wb["x0"], w, B), sel(wb["obs"], w, B), sel(wb["n_obs"], w, B))
res["worst_x1"], _ = run(sel(wb["x0"], w, 1), sel(wb["obs"], w, 1), sel(wb["n_obs"], w, 1))
res["worst_x2"], _ = run(sel(wb["x0"], w, 2), sel(wb["obs"], w, 2), sel(wb["n_obs"], w, 2))
res["worst_x1024"], _ = run(sel(wb["x0"], w, 1024), sel(wb["obs"], w, 1024), sel(wb["n_obs"], w, 1024))
res["worst_x2048"], _ = run(sel(wb["x0"], w, 2048), sel(wb["obs"], w, 2048), sel(wb["n_obs"], w, 2048))
res["easy_xB"], _ = run(sel(wb["x0"], easy, B), sel(wb["obs"], easy, B), sel(wb["n_obs"], easy, B))
print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in res.items()}), flush=True)
