# the N = 20 interior-point launch with one deferred instance per wavefront
# (MPC_IPM_GL64=1, GL = 64, B waves) against the shipped two per wavefront (GL = 32).  Parity first (full
# batches vs the oracle with the switch on), then C2/C3 benches in both orders, then the kernel stats.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
if [ "$PROF_ONLY" != 1 ]; then
MPC_IPM_GL64=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "full_batch or full_size or edge or certified" > gpurun_out/gl64_parity.log 2>&1 || { echo "parity with GL64 failed"; tail -20 gpurun_out/gl64_parity.log; exit 1; }
tail -2 gpurun_out/gl64_parity.log
for order in "1 0" "0 1"; do
for c in C2 C3; do
  for v in $order; do
    MPC_IPM_GL64=$v timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --no-cpu --inflight 0 --nlp-steps 0 --closed-loop 0 --plan-chunks 0 > gpurun_out/gl64_${c}_$v.log 2>&1 || { echo "bench $c failed"; tail -5 gpurun_out/gl64_${c}_$v.log; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/gl64_${c}_$v.log').read().strip().splitlines()[-1]); print('$c MPC_IPM_GL64=$v', round(d['ms_per_step'],4), 'ms', d['solver'].get('status_counts', ''))"
  done
done
done
cd /tmp && export TMPDIR=/tmp
fi
for v in 1 0; do
  rm -rf $R/gpurun_out/gl64_prof_$v
  MPC_IPM_GL64=$v timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/gl64_prof_$v -o run --output-format csv -- python3 $R/bench.py --config C2 --steps 20 --warmup 3 --no-cpu --inflight 0 --nlp-steps 0 --closed-loop 0 --plan-chunks 0 > $R/gpurun_out/gl64_prof_$v.log 2>&1 || { echo "prof $v failed"; exit 1; }
  echo "== GL64=$v"; find $R/gpurun_out/gl64_prof_$v -name "*kernel_stats.csv" -exec head -4 {} \; | cut -c1-220
done
