# SQ counter passes over the planner kernel (N = 16, 16384 chunks on traj3): stall classes, instruction
# fetch, LDS activity and bank conflicts; each pass a run of its own, the profiled program after --.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/plan_sq1 $R/gpurun_out/plan_sq2
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS -d $R/gpurun_out/plan_sq1 -o run --output-format csv -- python3 $R/tools/plan_probe.py 16 16384 traj3 0.1 > $R/gpurun_out/plan_sq1.log 2>&1 || { echo "plan sq1 failed"; tail $R/gpurun_out/plan_sq1.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_WAVES -d $R/gpurun_out/plan_sq2 -o run --output-format csv -- python3 $R/tools/plan_probe.py 16 16384 traj3 0.1 > $R/gpurun_out/plan_sq2.log 2>&1 || { echo "plan sq2 failed"; tail $R/gpurun_out/plan_sq2.log; exit 1; }
cd $R && python3 - <<'PY' | tee gpurun_out/plan_sq.log
import csv, glob, collections
for d in ('plan_sq1', 'plan_sq2'):
    f = glob.glob(f'gpurun_out/{d}/**/*counter_collection.csv', recursive=True)
    if not f:
        print('no csv', d); continue
    agg = collections.Counter()
    for row in csv.DictReader(open(f[0])):
        if 'plan_chunk_kernel' in row.get('Kernel_Name', ''):
            agg[row['Counter_Name']] += float(row['Counter_Value'])
    print(d, ' '.join(f'{a}={v:.4g}' for a, v in sorted(agg.items())))
PY
