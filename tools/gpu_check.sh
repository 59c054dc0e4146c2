cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
nproc > gpurun_out/nproc.txt; rocm-smi --showproductname > gpurun_out/smi.txt 2>&1
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu -rA > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-seconds 5 > gpurun_out/bench.log 2>&1
  echo "bench rc=$?"
fi
tail -5 gpurun_out/gpu_tests.log; tail -3 gpurun_out/bench.log
