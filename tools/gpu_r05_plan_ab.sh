# Planner A/B of in-tree builds ($LIBS; both orders): tools/plan_probe.py N = 16, 1024 and 65536 traj3 chunks;
# then the phase cycles of the product build's diagnostic twin (libmpcplan_prof.so).  Each step time-limited.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L="${LIBS:-libmpcplan_base.so libmpcplan_dpp1.so libmpcplan.so}"
R=""; for l in $L; do R="$l $R"; done
for l in $L $R; do
  PLAN_LIB=$l timeout -k 10 200 python -u tools/plan_probe.py 16 1024,65536 traj3 0.1 > gpurun_out/plan_ab_$l.log 2>&1 \
    || { echo "$l failed"; tail -3 gpurun_out/plan_ab_$l.log; exit 1; }
  echo "$l:"; grep 'N=' gpurun_out/plan_ab_$l.log
done
timeout -k 10 300 python tools/plan_phase.py 16 64,1024 traj3 0 > gpurun_out/plan_phase.log 2>&1 || { echo "plan phase failed"; tail -5 gpurun_out/plan_phase.log; exit 1; }
cat gpurun_out/plan_phase.log
