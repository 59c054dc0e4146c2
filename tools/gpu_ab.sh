# A/B of the two-phase launch: GPU parity tests, then C2..C5 benches with the split on and off
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/ -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed|^E " gpurun_out/gpu_tests.log | head -10
[ $rc -eq 0 ] || exit $rc
for c in ${CONFIGS:-C2 C3 C4 C5}; do
  for tp in 1 0; do
    MPC_TWO_PHASE=$tp timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu > gpurun_out/bench_${c}_tp$tp.log 2>&1 || { echo "bench $c failed"; tail -5 gpurun_out/bench_${c}_tp$tp.log; exit 1; }
    python -c "import json,sys; d=json.loads(open('gpurun_out/bench_${c}_tp$tp.log').read().strip().splitlines()[-1]); print('$c two_phase=$tp', round(d['value']), 'solves/s', round(d['ms_per_step'],3), 'ms', d['solver']['mean_iters'], d['solver']['max_iters'], d['solver']['status_counts'])"
  done
done
