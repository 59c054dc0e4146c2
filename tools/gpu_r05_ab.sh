# Round 5 A/B pass: GPU suite on the product builds; the tracker's interior-point checkpoint against the round-4
# build (libmpcqp_base.so) on C2..C5, both orders; the planner's DPP Riccati recursions against the round-4 build
# (libmpcplan_base.so): a latency-bound launch (1024 chunks, its slowest chunk sets the time) and a
# throughput launch (65536 chunks), N = 16 on traj3, both orders; the slowest C2 instance's phase cycles.
# Every GPU step time-limited; the first failure ends the script.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -m gpu -v -s --timeout 300 --timeout-method thread -rA \
    > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed|^E " gpurun_out/gpu_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
for l in libmpcplan_base.so libmpcplan.so libmpcplan.so libmpcplan_base.so; do
  PLAN_LIB=$l timeout -k 10 200 python -u tools/plan_probe.py 16 1024,65536 traj3 0.1 > gpurun_out/plan_ab_$l.log 2>&1 \
    || { echo "$l failed"; tail -3 gpurun_out/plan_ab_$l.log; exit 1; }
  echo "$l:"; grep 'N=' gpurun_out/plan_ab_$l.log
done
timeout -k 10 600 python tools/ab_probe.py libmpcqp_base.so libmpcqp.so --configs=C2,C3,C4,C5 --reps=20 \
    > gpurun_out/ab_order1.log 2>&1 || { echo "ab order 1 failed"; tail gpurun_out/ab_order1.log; exit 1; }
cat gpurun_out/ab_order1.log
timeout -k 10 600 python tools/ab_probe.py libmpcqp.so libmpcqp_base.so --configs=C2,C3,C4,C5 --reps=20 \
    > gpurun_out/ab_order2.log 2>&1 || { echo "ab order 2 failed"; tail gpurun_out/ab_order2.log; exit 1; }
cat gpurun_out/ab_order2.log
PROBE_WORST=1 timeout -k 10 200 python tools/phase_probe.py C2 1 > gpurun_out/phase_c2.log 2>&1 \
    || { echo "phase probe failed"; tail -20 gpurun_out/phase_c2.log; exit 1; }
grep -v amdgpu.ids gpurun_out/phase_c2.log
