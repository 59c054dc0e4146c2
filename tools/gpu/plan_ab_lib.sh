# Round 5: planner library A/B ($A, default the committed-kernel build libmpcplan_head.so, vs $B, default the
# working build libmpcplan.so; both orders): N = 16 traj3 batches of 1024 and 65536, bit-for-bit comparison
# of their results, the two slowest bench-mix chunks alone; then (FULL=1) the planner GPU tests and the fleet
# breakdown.  Each step time-limited.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
A=${A:-libmpcplan_head.so}; B=${B:-libmpcplan.so}
for l in $A $B $A $B; do
  PLAN_DUMP=1 PLAN_LIB=$l timeout -k 10 200 python -u tools/plan_probe.py 16 1024,65536 traj3 0.1 > gpurun_out/ab3_$l.log 2>&1 || { echo "$l failed"; tail -3 gpurun_out/ab3_$l.log; exit 1; }
  echo "$l: $(grep 'N=' gpurun_out/ab3_$l.log | sed 's/route=traj3: //' | cut -c1-120 | tr '\n' ' ')"
  PLAN_LIB=$l timeout -k 10 120 python -u tools/plan_worst.py traj3 65536 18596,6575 1 > gpurun_out/ab3w_$l.log 2>&1 || { echo "$l worst failed"; exit 1; }
  cat gpurun_out/ab3w_$l.log
done
python tools/plan_dump_cmp.py $A $B 16 1024
python tools/plan_dump_cmp.py $A $B 16 65536
rm -f gpurun_out/plan_dump_*.npz
if [ "${FULL:-0}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_plan.py -x -q --timeout 300 --timeout-method thread > gpurun_out/plan_tests.log 2>&1 || { echo "plan tests failed"; tail -30 gpurun_out/plan_tests.log; exit 1; }
  tail -2 gpurun_out/plan_tests.log
  timeout -k 10 300 python -u tools/fleet_probe.py 1024 > gpurun_out/fleet_probe.log 2>&1 || { echo "fleet probe failed"; tail -20 gpurun_out/fleet_probe.log; exit 1; }
  cat gpurun_out/fleet_probe.log
fi
