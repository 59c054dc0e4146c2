# GPU tests, A/B of the partitioned work list (MPC_WL_PARTS=1 vs 8), kernel stats of both, and the
# crossover kernel's phase cycles (MPC_DBG=1); every step time-limited, the first failure ends the script
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/ -m gpu -q --timeout 300 --timeout-method thread -rA > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed|^E " gpurun_out/gpu_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for c in C2 C3 C4; do
  for v in 1 8; do
    MPC_WL_PARTS=$v timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --no-cpu --inflight 0 --nlp-steps 0 > gpurun_out/parts_${c}_$v.log 2>&1 || { echo "bench $c failed"; tail -5 gpurun_out/parts_${c}_$v.log; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/parts_${c}_$v.log').read().strip().splitlines()[-1]); print('$c parts=$v', round(d['ms_per_step'],4), 'ms')"
  done
done
done
cd /tmp && export TMPDIR=/tmp
for v in 1 8; do
  rm -rf $R/gpurun_out/parts_prof_$v
  MPC_WL_PARTS=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/parts_prof_$v -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu --inflight 0 --nlp-steps 0 > $R/gpurun_out/parts_prof_$v.log 2>&1 || { echo "stats $v failed"; exit 1; }
done
cd $R
python - <<'PY'
import csv, glob
for v in (1, 8):
    f = glob.glob(f"gpurun_out/parts_prof_{v}/**/*kernel_stats.csv", recursive=True)[0]
    for r in csv.DictReader(open(f)):
        print(v, r["Name"][:42], r["Calls"], "avg us %.2f" % (float(r["AverageNs"]) / 1e3))
PY
bash tools/gpu_xo_phase.sh
