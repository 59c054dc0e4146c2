# Round 5: SQ counters of the slowest bench-mix chunk alone (tools/plan_worst.py, one wave): instruction mix
# (VALU / SALU / LDS / VMEM, FP64 FMA / MUL / ADD) and wait classes, two passes of 8 SQ counters each.
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/plan_sqw1 $R/gpurun_out/plan_sqw2
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS -d $R/gpurun_out/plan_sqw1 -o run --output-format csv -- python3 $R/tools/plan_worst.py traj3 65536 18596 1 > $R/gpurun_out/plan_sqw1.log 2>&1 || { echo "sq1 failed"; tail $R/gpurun_out/plan_sqw1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VMEM SQ_ACTIVE_INST_SCA SQ_WAVE_CYCLES -d $R/gpurun_out/plan_sqw2 -o run --output-format csv -- python3 $R/tools/plan_worst.py traj3 65536 18596 1 > $R/gpurun_out/plan_sqw2.log 2>&1 || { echo "sq2 failed"; tail $R/gpurun_out/plan_sqw2.log; exit 1; }
cd $R && python3 - <<'PY'
import csv, glob, collections
for d in ('plan_sqw1', 'plan_sqw2'):
    f = glob.glob(f'gpurun_out/{d}/**/*counter_collection.csv', recursive=True)
    if not f:
        print('no csv', d); continue
    agg = collections.defaultdict(collections.Counter); disp = collections.defaultdict(set)
    for row in csv.DictReader(open(f[0])):
        if 'plan_chunk_kernel' not in row.get('Kernel_Name', ''):
            continue
        agg['chunk'][row['Counter_Name']] += float(row['Counter_Value'])
        disp['chunk'].add(row.get('Dispatch_Id'))
    for k, c in agg.items():
        n = max(1, len(disp[k]))
        print(d, k, f'{n} dispatches, per dispatch:', ' '.join(f'{a}={v / n:.4g}' for a, v in sorted(c.items())))
PY
