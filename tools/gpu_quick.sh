# quick GPU loop: phase profile, timing probe, parity tests (each step time-limited)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python tools/phase_probe.py C2 4096 > gpurun_out/phase.log 2>&1 || { echo "phase probe failed"; tail -20 gpurun_out/phase.log; exit 1; }
grep -v amdgpu.ids gpurun_out/phase.log
timeout -k 10 240 python tools/timing_probe.py C2 4096 > gpurun_out/probe.log 2>&1 || { echo "probe failed"; tail -20 gpurun_out/probe.log; exit 1; }
grep -v amdgpu.ids gpurun_out/probe.log
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -rA -x > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "^(PASSED|FAILED|ERROR)|passed|failed" gpurun_out/gpu_tests.log | tail -20
