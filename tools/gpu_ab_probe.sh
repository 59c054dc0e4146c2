# A/B of in-tree library variants (tools/ab_probe.py), then the GPU test suite; each step time-limited
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python tools/ab_probe.py ${AB_LIBS:-libmpcqp_base.so libmpcqp.so} || exit 1
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed|^E " gpurun_out/gpu_tests.log | head -20
exit $rc
