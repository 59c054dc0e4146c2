"""Oracle A/B of the planner SQP's switch to the exact Lagrangian Hessian after a fixed number of Gauss-Newton
iterations (PLAN_EXACT_AFTER, oracle/plan_oracle.c) on the bench's chunk mix and the parity batches: statuses,
SQP / interior-point iteration counts (mean, p99, max) and 8-thread oracle time.  Each setting runs in a child
process (the oracle reads the variable once).

  python tools/plan_exact_ab.py [B] [after ...]       (after -1 = off, the round-4 rule)
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = r"""
import sys, time, numpy as np
sys.path[:0] = [ROOT + '/safe-autonomous-driving-mpc_amd', ROOT + '/oracle']
import plan_oracle as PO, workloads as W
B = int(sys.argv[1])
def stats(label, o, dt):
    st, sq, it = o['status'], o['sqp'], o['iters']
    print(f"  {label:14s} status {np.bincount(st, minlength=5).tolist()} sqp mean {sq.mean():.2f} p99 {np.percentile(sq, 99):.0f} "
          f"max {sq.max()} | ipm mean {it.mean():.1f} p99 {np.percentile(it, 99):.0f} max {it.max()} | {dt:.1f} s", flush=True)
r = W.plan_route('traj3')
wb = W.plan_batch_ref(r, B, seed=7)
po = PO.PlanOracle(r)
t0 = time.time()
o = po.solve_batch(PO.default_params(N=int(wb['N'].max())), wb['x0'], wb['s_target'], wb['is_final'], N=wb['N'], num_threads=8)
stats('bench traj3', o, time.time() - t0)
for N, route, seed in ((10, 'traj1', 10), (20, 'traj2', 20), (20, 'synth1', 20), (40, 'synth2', 40)):
    rr = W.plan_route(route)
    b = W.plan_batch(rr, N, 256, seed=seed, final_frac=0.25)
    t0 = time.time()
    o = PO.PlanOracle(rr).solve_batch(PO.default_params(N=N), b['x0'], b['s_target'], b['is_final'], num_threads=8)
    stats(f'{route} N={N}', o, time.time() - t0)
"""


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    for a in (sys.argv[2:] or ["-1", "10", "20"]):
        print(f"PLAN_EXACT_AFTER={a}", flush=True)
        env = dict(os.environ)
        if a != "-1":
            env["PLAN_EXACT_AFTER"] = a
        subprocess.run([sys.executable, "-c", "ROOT = %r\n" % ROOT + CODE, str(B)], env=env, check=True)


if __name__ == "__main__":
    main()
