"""Diagnostic: the C2 step with and without the Xpred output (2.4 MB fewer bytes left dirty by the crossover
kernel), 300 launches each, HIP events; run it under rocprofv3 --kernel-trace --stats to split the step into
kernel time and kernel-boundary time.   usage: python tools/boundary_probe.py [with|without]"""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "safe-autonomous-driving-mpc_amd")]
import torch  # noqa: E402  (before libmpcqp, as bench.py)
import mpcqp  # noqa: E402
import workloads as W  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "with"
wb = W.make_batch("C2")
ld = W.loader(wb["traj"])
B, N = wb["x0"].shape[0], wb["N"]
slv = mpcqp.Solver(ld.X_ref, ld.U_ref, mpcqp.default_params(N=N, max_obs=0))
dev = torch.device("cuda", 0)
x0 = torch.as_tensor(wb["x0"], dtype=torch.float64, device=dev).contiguous()
u0 = torch.empty((B, 2), dtype=torch.float64, device=dev)
U = torch.empty((B, N, 2), dtype=torch.float64, device=dev)
X = torch.empty((B, N + 1, 5), dtype=torch.float64, device=dev)
st = torch.empty(B, dtype=torch.int32, device=dev)
it = torch.empty(B, dtype=torch.int32, device=dev)
s = torch.cuda.current_stream(dev)
xp = X.data_ptr() if mode == "with" else 0


def step():
    slv.solve_batch_device(B, x0.data_ptr(), 0, 0, 0, u0.data_ptr(), U.data_ptr(), xp, st.data_ptr(), it.data_ptr(),
                           stream=s.cuda_stream)


for _ in range(5):
    step()
torch.cuda.synchronize(dev)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
reps = 300
e0.record(s)
for _ in range(reps):
    step()
e1.record(s)
torch.cuda.synchronize(dev)
print(f"{mode} Xpred: {e0.elapsed_time(e1) / reps * 1e3:.1f} us per step")
