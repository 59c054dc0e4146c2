# planner GPU tests (tests/test_gpu_plan.py), time-limited
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_plan.py -v -s --timeout 400 --timeout-method thread -rA > gpurun_out/plan_tests.log 2>&1
rc=$?
grep -E "N=|synth|traj|PASSED|FAILED|ERROR|passed|failed|Error|error" gpurun_out/plan_tests.log | head -60
exit $rc
