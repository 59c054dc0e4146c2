# round-4 profiles in one call: tracker kernel stats of the C2 bench and its phase cycles (MPC_PROF build),
# then the planner's kernel stats (N = 16, 16384 chunks on traj3) and its bench leg
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/stats_C2 $R/gpurun_out/stats_plan
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/stats_C2 -o run --output-format csv -- python3 $R/bench.py --config C2 --steps 20 --warmup 3 --no-cpu --inflight 0 --nlp-steps 0 --closed-loop 0 --plan-chunks 0 > $R/gpurun_out/stats_C2.log 2>&1 || { echo "stats C2 failed"; tail $R/gpurun_out/stats_C2.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/stats_plan -o run --output-format csv -- python3 $R/tools/plan_probe.py 16 16384 traj3 0.1 > $R/gpurun_out/stats_plan.log 2>&1 || { echo "stats plan failed"; tail $R/gpurun_out/stats_plan.log; exit 1; }
cd $R
bash tools/gpu_phase.sh > /dev/null || { echo "phase failed"; exit 1; }
find gpurun_out/stats_C2 gpurun_out/stats_plan -name "*kernel_stats.csv" | while read f; do echo "== $f"; cut -c1-160 "$f"; done
tail -3 gpurun_out/stats_C2.log | cut -c1-300
grep "N=16" gpurun_out/stats_plan.log
