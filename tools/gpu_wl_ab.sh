# GPU tests, then an A/B of the work-list reset (memset launch vs double-buffered count), time-limited steps
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -q --timeout 300 --timeout-method thread -rA > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed|^E " gpurun_out/gpu_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
ENVVAR=MPC_WL_MEMSET CONFIGS="C2 C3 C4" bash tools/gpu_env_ab.sh
