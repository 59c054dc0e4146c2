# Round 5: the GPU test suite (every -m gpu test, product libraries), then the default bench line (all legs).
# Each step time-limited; the first failure ends the script.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -m gpu -v -s --timeout 300 --timeout-method thread -rA \
    > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed|^E " gpurun_out/gpu_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py > gpurun_out/bench_default.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_default.log; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/bench_default.log"):
    if l.startswith("{"):
        d = json.loads(l)
        print({k: d.get(k) for k in ("metric", "value", "ms_per_step")}, "roofline frac", d.get("roofline", {}).get("frac"))
        p = d.get("plan", {})
        print("plan", {k: p.get(k) for k in ("value", "ms_per_step", "launch_groups", "status_counts_rank0")})
        print("plan roofline", {k: p.get("roofline", {}).get(k) for k in ("executed_frac", "source")})
        print("pipelined", p.get("pipelined", {}).get("value"), "cpu", p.get("cpu_baseline", {}).get("value"), "parity", p.get("parity_sample"))
        f = p.get("fleet", {})
        print("fleet", {k: f.get(k) for k in ("seconds", "plans_per_s", "chunks", "checks_passed")}, f.get("breakdown", {}).get("launches"))
PY
