# GPU round: tests, C5 spot check, configs bench. Every GPU step is time-limited; the first failure ends the script.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -m pytest tests/ -q -m gpu -rA -x > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed|^E " gpurun_out/gpu_tests.log | head -10
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/debug_cmp.py C5 2048 5 > gpurun_out/debug_cmp_C5.log 2>&1 || { echo "debug_cmp failed"; tail -5 gpurun_out/debug_cmp_C5.log; exit 1; }
grep -v amdgpu gpurun_out/debug_cmp_C5.log | head -8
bash tools/gpu_configs.sh
