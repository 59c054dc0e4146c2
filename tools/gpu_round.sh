cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -m pytest tests/ -q -m gpu -rA -x > gpurun_out/gpu_tests.log 2>&1; echo "pytest rc=$?"; grep -E "^(FAILED|ERROR)|passed|failed|^E " gpurun_out/gpu_tests.log | head -10
timeout -k 10 300 python tools/debug_cmp.py C5 2048 5 2>&1 | grep -v amdgpu | head -8
bash tools/gpu_configs.sh
