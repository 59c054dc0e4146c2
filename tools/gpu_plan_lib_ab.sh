# planner A/B of in-tree library variants ($LIBS, default: product vs the two scheduler variants), both
# orders, N = 16, 65536 traj3 chunks per launch (tools/plan_probe.py)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L="${LIBS:-libmpcplan.so libmpcplan_maxilp.so libmpcplan_maxocc.so}"
R=""; for l in $L; do R="$l $R"; done
for l in $L $R; do
  PLAN_LIB=$l timeout -k 10 120 python -u tools/plan_probe.py ${PN:-16} ${PB:-65536} traj3 0.1 > gpurun_out/plan_lib_$l.log 2>&1 || { echo "$l failed"; tail -3 gpurun_out/plan_lib_$l.log; exit 1; }
  echo "$l: $(grep 'N=' gpurun_out/plan_lib_$l.log)"
done
