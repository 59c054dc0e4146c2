# Round 5 planner measurements: the default bench (every leg), the planner leg with the index-order dispatch
# (PLAN_ORDER=0) for the longest-first A/B, the planner phase cycles (libmpcplan_prof.so) and the planner's
# kernel stats and executed-FP64 counter pass (tools/gpu_plan_pmc.sh).  Every GPU step time-limited.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log | cut -c1-400
PLAN_ORDER=0 timeout -k 10 400 python bench.py --no-cpu --inflight 0 --nlp-steps 0 --closed-loop 0 --plan-fleet 0 \
    > gpurun_out/bench_noorder.log 2>&1 || { echo "bench noorder failed"; tail -5 gpurun_out/bench_noorder.log; exit 1; }
python -c "import json,sys; d=json.loads(open('gpurun_out/bench_noorder.log').read().strip().splitlines()[-1]); p=d['plan']; print('index order: plan', p['value'], p['ms_per_step'], 'pipelined', p['pipelined']['value'])"
timeout -k 10 300 python tools/plan_phase.py 16 64,1024 traj3 0 > gpurun_out/plan_phase.log 2>&1 || { echo "plan phase failed"; tail -5 gpurun_out/plan_phase.log; exit 1; }
cat gpurun_out/plan_phase.log
bash tools/gpu_plan_pmc.sh
