# the GPU parity and NLP tests with their measurement prints (-s), each time-limited
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_nlp.py -m gpu -q -s --timeout 300 --timeout-method thread > gpurun_out/parity_report.log 2>&1
rc=$?; echo "pytest rc=$rc"
grep -E "worst|max_dU|\"cfg\"|steps, reference|final s|passed|failed" gpurun_out/parity_report.log | cut -c1-300 | head -40
exit $rc
