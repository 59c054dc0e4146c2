# Round 5: planner phase cycles (libmpcplan_prof.so, -DPLAN_PROF) of the two slowest bench-mix chunks alone and of
# 1024 N = 16 traj3 chunks (tools/plan_phase.py).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/plan_phase.py bench traj3 65536 18596,6575 > gpurun_out/plan_phase_worst.log 2>&1 || { echo "phase failed"; tail -20 gpurun_out/plan_phase_worst.log; exit 1; }
timeout -k 10 300 python -u tools/plan_phase.py 16 1024 traj3 0 > gpurun_out/plan_phase.log 2>&1 || { echo "phase failed"; tail -20 gpurun_out/plan_phase.log; exit 1; }
grep -v amdgpu.ids gpurun_out/plan_phase_worst.log gpurun_out/plan_phase.log
