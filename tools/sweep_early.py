"""Diagnostic sweep of the early-polish policy (env MPC_EARLY_MU / MPC_EARLY_ROUNDS read by the
experimental build): C2 batch time and mean iterations per setting, each in a fresh process."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = r'''
import os, sys, json
sys.path[:0] = [%r, %r]
import numpy as np, torch, mpcqp, workloads as W
wb = W.make_batch("C2", B=4096); N = wb["N"]
ld = W.loader(wb["traj"]); slv = mpcqp.Solver(ld.X_ref, ld.U_ref, mpcqp.default_params(N=N))
dev = torch.device("cuda", 0)
x0 = torch.as_tensor(wb["x0"], device=dev)
o = {k: torch.empty(s, dtype=torch.float64, device=dev) for k, s in (("u0", (4096, 2)), ("U", (4096, N, 2)), ("X", (4096, N + 1, 5)))}
st = torch.empty(4096, dtype=torch.int32, device=dev); it = torch.empty(4096, dtype=torch.int32, device=dev)
s = torch.cuda.current_stream(dev)
f = lambda: slv.solve_batch_device(4096, x0.data_ptr(), 0, 0, 0, o["u0"].data_ptr(), o["U"].data_ptr(), o["X"].data_ptr(), st.data_ptr(), it.data_ptr(), s.cuda_stream)
for _ in range(3): f()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(s)
for _ in range(10): f()
e1.record(s); torch.cuda.synchronize()
print(json.dumps(dict(ms=e0.elapsed_time(e1) / 10, iters=float(it.float().mean()), status=np.bincount(st.cpu().numpy(), minlength=4).tolist())))
''' % (ROOT, os.path.join(ROOT, "safe-autonomous-driving-mpc_amd"))
for mu in ("0", "1e-1", "1e-2", "1e-3", "1e-5"):
    for rounds in ("1", "2"):
        if mu == "0" and rounds == "2":
            continue
        env = dict(os.environ, MPC_EARLY_MU=mu, MPC_EARLY_ROUNDS=rounds)
        r = subprocess.run([sys.executable, "-c", CODE], env=env, capture_output=True, text=True, timeout=240)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")]
        print(f"early_mu={mu:6s} rounds={rounds}: {line[-1] if line else r.stderr[-300:]}", flush=True)
