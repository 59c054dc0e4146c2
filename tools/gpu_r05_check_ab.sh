# Round 5: the tracker's interior-point checkpoint.  GPU suite on the product build, then
# the A/B against the round-4 build (libmpcqp_base.so) on C2..C5 in both orders, the C2 kernel stats under
# rocprofv3, and the phase cycles of the slowest C2 instance (libmpcqp_prof.so).  Every GPU step time-limited;
# the first failure ends the script.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -m gpu -v -s --timeout 300 --timeout-method thread -rA \
    > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed|^E " gpurun_out/gpu_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/ab_probe.py libmpcqp_base.so libmpcqp.so --configs=C2,C3,C4,C5 --reps=20 \
    > gpurun_out/ab_order1.log 2>&1 || { echo "ab order 1 failed"; tail gpurun_out/ab_order1.log; exit 1; }
cat gpurun_out/ab_order1.log
timeout -k 10 600 python tools/ab_probe.py libmpcqp.so libmpcqp_base.so --configs=C2,C3,C4,C5 --reps=20 \
    > gpurun_out/ab_order2.log 2>&1 || { echo "ab order 2 failed"; tail gpurun_out/ab_order2.log; exit 1; }
cat gpurun_out/ab_order2.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o c2 -- python3 bench.py --steps 20 --warmup 3 \
    --no-cpu --inflight 0 --nlp-steps 0 --closed-loop 0 --plan-chunks 0 > gpurun_out/bench_c2_prof.log 2>&1 \
    || { echo "rocprof failed"; tail gpurun_out/bench_c2_prof.log; exit 1; }
find gpurun_out/prof_c2 -name "*kernel_stats.csv" | head -3
if [ -f safe-autonomous-driving-mpc_amd/libmpcqp_prof.so ]; then
  PROBE_WORST=1 timeout -k 10 200 python tools/phase_probe.py C2 1 > gpurun_out/phase_c2.log 2>&1 \
    || { echo "phase probe failed"; tail -20 gpurun_out/phase_c2.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/phase_c2.log
fi
