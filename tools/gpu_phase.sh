# phase-cycle probe (diagnostic -DMPC_PROF build): full C2 batch and the slowest instance alone
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python tools/phase_probe.py C2 4096 > gpurun_out/phase.log 2>&1 || { echo "phase probe failed"; tail -20 gpurun_out/phase.log; exit 1; }
PROBE_WORST=1 timeout -k 10 200 python tools/phase_probe.py C2 1 >> gpurun_out/phase.log 2>&1 || { echo "phase probe failed"; tail -20 gpurun_out/phase.log; exit 1; }
timeout -k 10 200 python tools/tail_probe.py C2 4096 >> gpurun_out/phase.log 2>&1 || { echo "tail probe failed"; tail -20 gpurun_out/phase.log; exit 1; }
grep -v amdgpu.ids gpurun_out/phase.log
