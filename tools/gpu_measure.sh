# One GPU call: every config at the current commit (tools/gpu_configs.sh), then per config in $PMC_CFGS
# (default C2) a kernel-stats run and the executed-FP64 counter pass (tools/gpu_f64_pmc.sh), summarised with
# the stats by tools/pmc_f64.py.  Each GPU step is time-limited; the first failure ends the script.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
bash tools/gpu_configs.sh || exit 1
for c in ${PMC_CFGS:-C2}; do
  cd /tmp && export TMPDIR=/tmp
  rm -rf $R/gpurun_out/stats_$c
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/stats_$c -o run --output-format csv -- python3 $R/bench.py --config $c --steps 20 --warmup 3 --no-cpu --inflight 0 --nlp-steps 0 --closed-loop 0 --plan-chunks 0 > $R/gpurun_out/stats_$c.log 2>&1 || { echo "stats $c failed"; tail $R/gpurun_out/stats_$c.log; exit 1; }
  cd $R
  CFG=$c bash tools/gpu_f64_pmc.sh > /dev/null || { echo "f64 pmc $c failed"; exit 1; }
  python3 tools/pmc_f64.py $c $(find gpurun_out/stats_$c -name "*kernel_stats.csv" | head -1)
done
