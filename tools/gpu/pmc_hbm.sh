# C2 HBM bytes per step from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; each its own run) plus the
# kernel-trace stats, each time-limited; summarise afterwards with tools/pmc_summary.py C2 <round> <commit>
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_stats $R/gpurun_out/pmc_fetch $R/gpurun_out/pmc_write
B="python3 $R/bench.py --no-cpu --inflight 0 --nlp-steps 0 --closed-loop 0 --plan-chunks 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_stats -o run --output-format csv -- $B --steps 20 --warmup 3 > $R/gpurun_out/prof_stats.log 2>&1 || { echo "stats failed"; tail $R/gpurun_out/prof_stats.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch -o run --output-format csv -- $B --steps 3 --warmup 1 > $R/gpurun_out/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; tail $R/gpurun_out/pmc_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write -o run --output-format csv -- $B --steps 3 --warmup 1 > $R/gpurun_out/pmc_write.log 2>&1 || { echo "pmc write failed"; tail $R/gpurun_out/pmc_write.log; exit 1; }
cd $R && bash tools/gpu/configs.sh
