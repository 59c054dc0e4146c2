# planner A/B timing by repetition (PLAN_DBG bits, csrc/plan.hip) in the throughput regime: N = 16,
# 65536 chunks of traj3 in one launch (the average chunk, not the tail chunk, sets the time there)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for d in 0 1 2 4 8 16 32 64 0; do
  PLAN_DBG=$d timeout -k 10 120 python -u tools/plan_probe.py 16 65536 traj3 0.1 > gpurun_out/plan_ab2_$d.log 2>&1 || exit 1
  echo "PLAN_DBG=$d"; grep "N=16" gpurun_out/plan_ab2_$d.log
done
