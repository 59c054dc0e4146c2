"""Diagnostic: does the order of instances in a batch change the batch time?  Times the config's batch
in its natural order, sorted by the previous solve's iteration count (longest first / shortest first),
and randomly shuffled.  A large gap means the makespan suffers from the last round of long waves."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "safe-autonomous-driving-mpc_amd")]
import numpy as np
import torch
import mpcqp
import workloads as W

cfg = sys.argv[1] if len(sys.argv) > 1 else "C5"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
wb = W.make_batch(cfg, B=B)
N, mo = wb["N"], wb["max_obs"]
ld = W.loader(wb["traj"])
slv = mpcqp.Solver(ld.X_ref, ld.U_ref, mpcqp.default_params(N=N, max_obs=mo))
dev = torch.device("cuda", 0)
stream = torch.cuda.current_stream(dev)
ptr = lambda x: 0 if x is None else x.data_ptr()


def timed(perm, reps=10):
    t = lambda a, dt=torch.float64: torch.as_tensor(np.ascontiguousarray(a[perm]), dtype=dt, device=dev)
    x0 = t(wb["x0"])
    obs = t(wb["obs"]) if wb["obs"] is not None else None
    nob = t(wb["n_obs"], torch.int32) if wb["n_obs"] is not None else None
    o = [torch.empty((B, 2), dtype=torch.float64, device=dev), torch.empty((B, N, 2), dtype=torch.float64, device=dev),
         torch.empty((B, N + 1, 5), dtype=torch.float64, device=dev), torch.empty(B, dtype=torch.int32, device=dev),
         torch.empty(B, dtype=torch.int32, device=dev)]
    args = (B, ptr(x0), ptr(obs), ptr(nob), 0) + tuple(ptr(a) for a in o) + (stream.cuda_stream,)
    slv.solve_batch_device(*args)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
    ev[0].record(stream)
    for i in range(reps):
        slv.solve_batch_device(*args)
        ev[i + 1].record(stream)
    torch.cuda.synchronize()
    ms = np.median([ev[i].elapsed_time(ev[i + 1]) for i in range(reps)])
    return ms, o[4].cpu().numpy()


ident = np.arange(B)
ms0, it = timed(ident)
inv = np.empty(B, dtype=np.int64)
rng = np.random.default_rng(0)
print(f"{cfg} B={B}: natural order {ms0:.3f} ms (iters mean {it.mean():.2f} max {it.max()})", flush=True)
for name, perm in (("longest first", np.argsort(-it, kind="stable")), ("shortest first", np.argsort(it, kind="stable")),
                   ("shuffled", rng.permutation(B))):
    ms, _ = timed(perm)
    print(f"{cfg} B={B}: {name:15s} {ms:.3f} ms", flush=True)
