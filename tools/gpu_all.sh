# one GPU call: timing probe, parity tests, bench, kernel-trace profile (each step time-limited)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 240 python tools/timing_probe.py C2 4096 > gpurun_out/probe.log 2>&1 || { echo "probe failed"; tail -20 gpurun_out/probe.log; exit 1; }
cat gpurun_out/probe.log | grep -v amdgpu.ids
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -rA > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -8 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 1; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-seconds 5 > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof1 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/prof1.log 2>&1
echo "prof rc=$?"
