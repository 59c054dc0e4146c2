"""Planner concurrency probe: one typical chunk (the median-work chunk of a small traj3 batch) replicated B
times, B = 256 .. 4096, HIP events on the launch stream.  256 copies put one chunk on each CU, 1024 four
(the LDS limit at N = 16): the time per launch against B shows whether the chunks on one CU slow each other
down (LDS bandwidth, instruction cache) or run side by side.  Usage: python tools/plan_conc.py [N]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "safe-autonomous-driving-mpc_amd"), ROOT]
import numpy as np
import torch

import mpcplan
import workloads as W

if os.environ.get("PLAN_LIB"):      # A/B of library variants
    mpcplan.LIB_PATH = os.path.join(ROOT, "safe-autonomous-driving-mpc_amd", os.environ["PLAN_LIB"])

N = int(sys.argv[1]) if len(sys.argv) > 1 else 16
dev = torch.device("cuda", 0)
r = W.plan_route("traj3")
pl = mpcplan.Planner(r, mpcplan.default_params(N=N))
t = lambda a, dt=torch.float64: torch.as_tensor(np.ascontiguousarray(a), dtype=dt, device=dev).contiguous()
stream = torch.cuda.current_stream(dev)


def run(x0, st, fin, reps=3):
    B = x0.shape[0]
    X = torch.empty((B, N + 1, 5), dtype=torch.float64, device=dev)
    U = torch.empty((B, N, 2), dtype=torch.float64, device=dev)
    S = torch.empty((B, N), dtype=torch.float64, device=dev)
    o = [torch.empty(B, dtype=torch.int32, device=dev) for _ in range(3)]
    a = [t(x0), t(st), t(fin, torch.int32)]
    call = lambda: pl.solve_chunks_device(B, N, 0, a[0].data_ptr(), a[1].data_ptr(), a[2].data_ptr(), X.data_ptr(),
                                          U.data_ptr(), S.data_ptr(), *[v.data_ptr() for v in o],
                                          stream=stream.cuda_stream)
    call()
    torch.cuda.synchronize(dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
    ev[0].record(stream)
    for i in range(reps):
        call()
        ev[i + 1].record(stream)
    torch.cuda.synchronize(dev)
    ms = float(np.median([ev[i].elapsed_time(ev[i + 1]) for i in range(reps)]))
    return ms, o[2].cpu().numpy(), o[1].cpu().numpy()


wb = W.plan_batch(r, N, 256, seed=N, final_frac=0.0)
_, sq, it = run(wb["x0"], wb["s_target"], wb["is_final"])
work = sq * 4 + it
order = np.argsort(work)
for name, i in (("median", order[len(order) // 2]), ("light", order[len(order) // 10])):
    print(f"{name} chunk {i}: sqp {sq[i]} ipm {it[i]}", flush=True)
    for B in (1, 64, 256, 512, 768, 1024, 2048, 4096):
        rep = lambda v: np.repeat(np.asarray(v)[i:i + 1], B, axis=0)
        ms, _, _ = run(rep(wb["x0"]), rep(wb["s_target"]), rep(wb["is_final"]))
        print(f"  B={B:5d}: {ms:8.3f} ms/launch  {B / ms * 1e3:10.0f} chunks/s", flush=True)
pl.close()
