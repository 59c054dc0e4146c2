# GPU A/B of in-tree library variants: parity tests on the product build, then tools/ab_probe.py over
# the libraries named in $LIBS (default: base vs product) on $CONFIGS; every GPU step time-limited
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed|^E " gpurun_out/gpu_tests.log | head -10
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python tools/ab_probe.py ${LIBS:-libmpcqp_base.so libmpcqp.so} --configs=${CONFIGS:-C2,C3,C4,C5} --reps=20
