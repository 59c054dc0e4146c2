# GPU tests, then kernel-trace stats of the C2 bench with and without the crossover kernel's work-list
# atomic (MPC_DBG=1, timing probe only), each step time-limited
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/ -m gpu -q --timeout 300 --timeout-method thread -rA > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed|^E " gpurun_out/gpu_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
  rm -rf $R/gpurun_out/xo_$v
  MPC_DBG=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/xo_$v -o run --output-format csv -- python3 $R/bench.py --config ${CFG:-C2} --steps 20 --warmup 3 --no-cpu --inflight 0 --nlp-steps 0 > $R/gpurun_out/xo_$v.log 2>&1 || { echo "stats $v failed"; tail $R/gpurun_out/xo_$v.log; exit 1; }
  echo "MPC_DBG=$v"; f=$(find $R/gpurun_out/xo_$v -name "*kernel_stats.csv" | head -1); cut -d, -f1-8 "$f" | cut -c1-200
done
