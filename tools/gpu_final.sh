# round-end GPU pass: the -m gpu suite, then tools/gpu_bench_prof.sh (bench with the closed-loop leg, kernel
# stats, PMC passes, phase cycles, all configs); the first failure ends the script
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -q --timeout 300 --timeout-method thread -rA > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed|^E " gpurun_out/gpu_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_bench_prof.sh
