import sys; sys.path[:0]=['safe-autonomous-driving-mpc_amd']
import mpcplan, workloads as W
pl = mpcplan.Planner(W.plan_route('traj3'), mpcplan.default_params(N=17), device=0)
print('chunks_per_cu', {n: pl.chunks_per_cu(n) for n in (13, 16, 17, 18, 24, 25, 33)})
