# Round 5: residency-class launches (bench plan leg) and the two-tier device chunk loop (fleet): the planner's
# GPU tests, then bench.py's plan leg and fleet alone (tracker legs minimal), each step time-limited.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_plan.py -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/plan_tests.log 2>&1 || { echo "plan tests failed"; tail -30 gpurun_out/plan_tests.log; exit 1; }
grep -E "passed|failed|chunks per CU" gpurun_out/plan_tests.log | tail -5
timeout -k 10 600 python -u bench.py --no-cpu --inflight 0 --nlp-steps 0 --closed-loop 0 --steps 3 --warmup 1 \
    > gpurun_out/bench_groups.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_groups.log; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/bench_groups.log"):
    if l.startswith("{"):
        p = json.loads(l).get("plan", {})
        print({k: p.get(k) for k in ("value", "ms_per_step", "launch_groups", "status_counts_rank0")})
        print("pipelined", p.get("pipelined", {}).get("value"))
        f = p.get("fleet", {})
        print("fleet", {k: f.get(k) for k in ("seconds", "plans_per_s", "chunks", "checks_passed")}, f.get("round_loop"))
PY
