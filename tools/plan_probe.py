"""Planner throughput probe: plan_solve_chunks_device on B chunks of horizon N (workloads.plan_batch), HIP
events on the launch stream.  Usage: python tools/plan_probe.py N B [route] [final_frac]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "safe-autonomous-driving-mpc_amd"), ROOT]
import numpy as np
import torch

import mpcplan
import workloads as W

if os.environ.get("PLAN_LIB"):      # A/B of library variants (gpu_plan_lib_ab.sh (removed in round 6))
    mpcplan.LIB_PATH = os.path.join(ROOT, "safe-autonomous-driving-mpc_amd", os.environ["PLAN_LIB"])

N = int(sys.argv[1]) if len(sys.argv) > 1 else 20
route = sys.argv[3] if len(sys.argv) > 3 else "traj1"
ff = float(sys.argv[4]) if len(sys.argv) > 4 else 0.25
dev = torch.device("cuda", 0)
r = W.plan_route(route)
for B in [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "4096,16384,65536").split(",")]:
    t0 = time.perf_counter()
    wb = W.plan_batch(r, N, B, seed=N, final_frac=ff)
    tg = time.perf_counter() - t0
    pl = mpcplan.Planner(r, mpcplan.default_params(N=N))
    t = lambda a, dt=torch.float64: torch.as_tensor(a, dtype=dt, device=dev).contiguous()
    x0, st, fin = t(wb["x0"]), t(wb["s_target"]), t(wb["is_final"], torch.int32)
    X = torch.empty((B, N + 1, 5), dtype=torch.float64, device=dev)
    U = torch.empty((B, N, 2), dtype=torch.float64, device=dev)
    S = torch.empty((B, N), dtype=torch.float64, device=dev)
    o = [torch.empty(B, dtype=torch.int32, device=dev) for _ in range(3)]
    stream = torch.cuda.current_stream(dev)
    call = lambda: pl.solve_chunks_device(B, N, 0, x0.data_ptr(), st.data_ptr(), fin.data_ptr(), X.data_ptr(),
                                          U.data_ptr(), S.data_ptr(), *[a.data_ptr() for a in o],
                                          stream=stream.cuda_stream)
    call()
    torch.cuda.synchronize(dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    ev[0].record(stream)
    for i in range(3):
        call()
        ev[i + 1].record(stream)
    torch.cuda.synchronize(dev)
    ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(3)]
    sq, it, stt = o[2].cpu().numpy(), o[1].cpu().numpy(), o[0].cpu().numpy()
    print(f"N={N} B={B} route={route}: {np.mean(ms):.2f} ms/launch = {B / np.mean(ms) * 1e3:.0f} chunks/s; "
          f"sqp mean {sq.mean():.2f} max {sq.max()}, ipm mean {it.mean():.1f} max {it.max()}, "
          f"status {np.bincount(stt, minlength=5).tolist()} (gen {tg:.1f}s)", flush=True)
    if os.environ.get("PLAN_DUMP"):     # results for a bit-for-bit A/B of library variants
        np.savez(os.path.join(ROOT, "gpurun_out", f"plan_dump_{os.environ.get('PLAN_LIB', 'libmpcplan.so')}_{N}_{B}.npz"),
                 X=X.cpu().numpy(), U=U.cpu().numpy(), S=S.cpu().numpy(), status=stt, iters=it, sqp=sq)
    pl.close()
