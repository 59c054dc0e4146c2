# phase-cycle probe (diagnostic -DMPC_PROF build): full batch and the slowest instance alone, for
# each config in $CONFIGS (default C2)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/phase.log
for c in ${CONFIGS:-C2}; do
  timeout -k 10 200 python tools/phase_probe.py $c ${PB:-4096} >> gpurun_out/phase.log 2>&1 || { echo "phase probe failed"; tail -20 gpurun_out/phase.log; exit 1; }
  PROBE_WORST=1 timeout -k 10 200 python tools/phase_probe.py $c 1 >> gpurun_out/phase.log 2>&1 || { echo "phase probe failed"; tail -20 gpurun_out/phase.log; exit 1; }
done
grep -v amdgpu.ids gpurun_out/phase.log
