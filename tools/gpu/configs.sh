# bench every BASELINE config on one GPU (per-GPU batch), each step time-limited
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for c in C2 C3 C4 C5; do
  timeout -k 10 300 python bench.py --config $c --steps 100 --warmup 5 --no-cpu --nlp-steps 0 --closed-loop 0 --plan-chunks 0 --inflight 0 > gpurun_out/bench_$c.log 2>&1 || { echo "bench $c failed"; tail -5 gpurun_out/bench_$c.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench_$c.log').read().strip().splitlines()[-1]); print('$c', round(d['value']), 'solves/s', round(d['ms_per_step'],3), 'ms', d['solver'])"
done
