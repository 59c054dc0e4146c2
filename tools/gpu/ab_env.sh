# A/B of a runtime switch: bench each config with ENVVAR=0 and =1, twice, interleaved (time-limited steps)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do
for c in ${CONFIGS:-C2 C3 C4}; do
  for v in 1 0; do
    env $ENVVAR=$v timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --no-cpu --inflight 0 --nlp-steps 0 > gpurun_out/envab_${c}_$v.log 2>&1 || { echo "bench $c failed"; tail -5 gpurun_out/envab_${c}_$v.log; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/envab_${c}_$v.log').read().strip().splitlines()[-1]); print('$c $ENVVAR=$v', round(d['ms_per_step'],4), 'ms')"
  done
done
done
