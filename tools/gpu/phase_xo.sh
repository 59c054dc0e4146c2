# phase cycles of the crossover kernel alone (MPC_DBG=1: the interior-point launch sees an empty list), C2
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
MPC_DBG=1 timeout -k 10 200 python tools/phase_probe.py ${CFG:-C2} ${PB:-4096} > gpurun_out/xo_phase.log 2>&1 || { echo "phase probe failed"; tail -20 gpurun_out/xo_phase.log; exit 1; }
MPC_DBG=1 timeout -k 10 200 python tools/phase_probe.py ${CFG:-C2} 2 >> gpurun_out/xo_phase.log 2>&1 || { echo "phase probe failed"; tail -20 gpurun_out/xo_phase.log; exit 1; }
grep -v amdgpu.ids gpurun_out/xo_phase.log
