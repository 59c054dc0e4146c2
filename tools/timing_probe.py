"""Cost breakdown of the solver kernel on the GPU: times one C2 batch under truncated settings."""
import os
import sys
import json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "safe-autonomous-driving-mpc_amd")]
import numpy as np
import torch
import __graft_entry__ as ge
ge.build()
import mpcqp
if os.environ.get("PROBE_LIB"):          # time an alternative in-tree build of the same ABI
    mpcqp.LIB_PATH = os.path.join(ROOT, "safe-autonomous-driving-mpc_amd", os.environ["PROBE_LIB"])
import workloads as W

cfg = sys.argv[1] if len(sys.argv) > 1 else "C2"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
wb = W.make_batch(cfg, B=B)
N, mo = wb["N"], wb["max_obs"]
ld = W.loader(wb["traj"])
slv = mpcqp.Solver(ld.X_ref, ld.U_ref, mpcqp.default_params(N=N, max_obs=mo))
dev = torch.device("cuda", 0)
t = lambda a, dt=torch.float64: torch.as_tensor(a, dtype=dt, device=dev).contiguous()
x0 = t(wb["x0"]); obs = t(wb["obs"]) if wb["obs"] is not None else None
nob = t(wb["n_obs"], torch.int32) if wb["n_obs"] is not None else None
u0 = torch.empty((B, 2), dtype=torch.float64, device=dev); Uo = torch.empty((B, N, 2), dtype=torch.float64, device=dev)
Xo = torch.empty((B, N + 1, 5), dtype=torch.float64, device=dev)
st = torch.empty(B, dtype=torch.int32, device=dev); it = torch.empty(B, dtype=torch.int32, device=dev)
ptr = lambda x: 0 if x is None else x.data_ptr()
stream = torch.cuda.current_stream(dev)
res = {}
for name, kw in [("warm+predict only (sqp_iters=0)", dict(sqp_iters=0)),
                 ("max_iter=1 nopolish", dict(max_iter=1, polish=0)),
                 ("max_iter=5 nopolish", dict(max_iter=5, polish=0)),
                 ("max_iter=10 nopolish", dict(max_iter=10, polish=0)),
                 ("full nopolish", dict(polish=0)),
                 ("full", dict())]:
    slv.set_params(mpcqp.default_params(N=N, max_obs=mo, **kw))
    for _ in range(2):
        slv.solve_batch_device(B, ptr(x0), ptr(obs), ptr(nob), 0, ptr(u0), ptr(Uo), ptr(Xo), ptr(st), ptr(it), stream.cuda_stream)
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(5):
        slv.solve_batch_device(B, ptr(x0), ptr(obs), ptr(nob), 0, ptr(u0), ptr(Uo), ptr(Xo), ptr(st), ptr(it), stream.cuda_stream)
    e1.record(stream); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 5
    res[name] = dict(ms=round(ms, 4), mean_iters=float(it.float().mean().item()))
    print(f"{name:40s} {ms:8.3f} ms   mean iters {res[name]['mean_iters']:.2f}", flush=True)
json.dump(res, open(os.path.join(ROOT, "gpurun_out", f"probe_{cfg}.json"), "w"), indent=1)
