# SQ counter pass over the C2 bench (instruction mix and stall classes of the solver kernels)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/pmc_sq1 $R/gpurun_out/pmc_sq2
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS -d $R/gpurun_out/pmc_sq1 -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --inflight 0 > $R/gpurun_out/pmc_sq1.log 2>&1 || { echo "pmc sq1 failed"; tail $R/gpurun_out/pmc_sq1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_WAVES -d $R/gpurun_out/pmc_sq2 -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --inflight 0 > $R/gpurun_out/pmc_sq2.log 2>&1 || { echo "pmc sq2 failed"; tail $R/gpurun_out/pmc_sq2.log; exit 1; }
cd $R && python3 - <<'PY'
import csv, glob, collections
for d in ('pmc_sq1','pmc_sq2'):
    f=glob.glob(f'gpurun_out/{d}/**/*counter_collection.csv', recursive=True)
    if not f: print('no csv', d); continue
    agg=collections.defaultdict(lambda: collections.Counter()); n=collections.Counter()
    for row in csv.DictReader(open(f[0])):
        k=row.get('Kernel_Name','')
        k='XO' if ('Li1ELi20' in k or ', 1, 20>' in k) else ('IPM' if ('Li2ELi20' in k or ', 2, 20>' in k) else k[:30])
        agg[k][row['Counter_Name']]+=float(row['Counter_Value'])
    for k,c in agg.items():
        print(d, k, ' '.join(f'{a}={v:.4g}' for a,v in sorted(c.items())))
PY
