# GPU A/B of in-tree libmpcqp builds ($LIBS, default: libmpcqp_base.so libmpcqp.so): unless SKIP_TESTS=1 the
# -m gpu suite on the product build first, then tools/ab_probe.py over $CONFIGS in both library orders (a
# box drifts by ~1%, so each variant is timed first once).  Every GPU step time-limited.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed|^E " gpurun_out/gpu_tests.log | head -10
  [ $rc -eq 0 ] || exit $rc
fi
L=${LIBS:-libmpcqp_base.so libmpcqp.so}
R=$(echo $L | awk '{for (i = NF; i > 0; --i) printf "%s ", $i}')
timeout -k 10 600 python tools/ab_probe.py $L --configs=${CONFIGS:-C2,C3,C4,C5} --reps=${REPS:-20} > gpurun_out/ab_fwd.log 2>&1 || { echo "ab fwd failed"; tail gpurun_out/ab_fwd.log; exit 1; }
timeout -k 10 600 python tools/ab_probe.py $R --configs=${CONFIGS:-C2,C3,C4,C5} --reps=${REPS:-20} > gpurun_out/ab_rev.log 2>&1 || { echo "ab rev failed"; tail gpurun_out/ab_rev.log; exit 1; }
grep -v "^WARNING" gpurun_out/ab_fwd.log | tail -20; echo ---; grep -v "^WARNING" gpurun_out/ab_rev.log | tail -20
