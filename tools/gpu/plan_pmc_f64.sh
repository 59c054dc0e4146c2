# Planner kernel: kernel stats and the executed-FP64 counter pass (7 SQ counters, its own run) over
# tools/plan_probe.py (N = 16, 16384 chunks on traj3), summarised by tools/pmc_f64.py plan.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/stats_plan $R/gpurun_out/pmc_f64_plan
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/stats_plan -o run --output-format csv -- python3 $R/tools/plan_probe.py 16 16384 traj3 0.1 > $R/gpurun_out/stats_plan.log 2>&1 || { echo "stats plan failed"; tail $R/gpurun_out/stats_plan.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $R/gpurun_out/pmc_f64_plan -o run --output-format csv -- python3 $R/tools/plan_probe.py 16 16384 traj3 0.1 > $R/gpurun_out/pmc_f64_plan.log 2>&1 || { echo "pmc plan failed"; tail $R/gpurun_out/pmc_f64_plan.log; exit 1; }
cd $R && python3 tools/pmc_f64.py plan $(find gpurun_out/stats_plan -name "*kernel_stats.csv" | head -1)
