# planner launch-time scan: fixed horizon, growing batch (throughput vs tail), then the kernel stats of one run
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/plan_probe.py 16 1024,4096,16384 traj3 0.1 > gpurun_out/plan_scan.log 2>&1 || exit 1
cat gpurun_out/plan_scan.log
