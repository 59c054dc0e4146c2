# the multi-rank code path of bench.py on one GPU: MPC_COMM=rccl makes a world-1 rank use libmpcqp's RCCL
# communicator (barrier, max-over-ranks time, telemetry and closed-loop gathers), first as a plain process,
# then under torch.distributed.run as the driver launches N ranks (each step time-limited)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
A="--steps 20 --warmup 3 --no-cpu --nlp-steps 0 --inflight 0 --plan-chunks 4096 --plan-fleet 0 --closed-loop 256"
MPC_COMM=rccl timeout -k 10 300 python bench.py $A > gpurun_out/comm_plain.log 2>&1 || { echo "plain failed"; tail -20 gpurun_out/comm_plain.log; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/comm_plain.log').read().strip().splitlines()[-1]); print('plain', d['comm']['transport'], round(d['value']), d['n_gpus'], d['closed_loop'].get('checks_passed', {}).get('passed'), d['plan'].get('value'))"
MPC_COMM=rccl timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 $A > gpurun_out/comm_torchrun.log 2>&1 || { echo "torchrun failed"; tail -20 gpurun_out/comm_torchrun.log; exit 1; }
python -c "import json; d=json.loads([l for l in open('gpurun_out/comm_torchrun.log').read().strip().splitlines() if l.startswith('{')][-1]); print('torchrun', d['comm']['transport'], round(d['value']), d['n_gpus'], d['closed_loop'].get('checks_passed', {}).get('passed'), d['plan'].get('value'))"
