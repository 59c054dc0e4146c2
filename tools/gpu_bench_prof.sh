# one GPU call: bench, kernel-trace stats, two PMC passes (HBM bytes), each time-limited
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --cpu-seconds 15 > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_stats $R/gpurun_out/pmc_fetch $R/gpurun_out/pmc_write
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_stats -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu --inflight 0 > $R/gpurun_out/prof_stats.log 2>&1 || { echo "stats failed"; tail $R/gpurun_out/prof_stats.log; exit 1; }
tail -1 $R/gpurun_out/prof_stats.log
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --inflight 0 > $R/gpurun_out/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; tail $R/gpurun_out/pmc_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --inflight 0 > $R/gpurun_out/pmc_write.log 2>&1 || { echo "pmc write failed"; tail $R/gpurun_out/pmc_write.log; exit 1; }
cd $R && python tools/pmc_summary.py C2
find gpurun_out/prof_stats -name "*kernel_stats*"
