# GPU test pass: the whole -m gpu suite in one process, every test time-limited, then a short bench.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -m gpu -v -s --timeout 300 --timeout-method thread -rA \
    > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed|^E " gpurun_out/gpu_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --cpu-seconds 10 > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
