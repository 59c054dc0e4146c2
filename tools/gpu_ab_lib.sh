cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 60 tools/probes/xlane_probe || exit 1
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed|^E " gpurun_out/gpu_tests.log | head -10
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/ab_probe.py libmpcqp_base.so libmpcqp.so --configs C2,C3,C4,C5 --reps 20
