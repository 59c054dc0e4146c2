# SQ counters of the solver kernels on the slowest C2 instance alone (one wavefront)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/worst_pmc $R/gpurun_out/worst_pmc2
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS -d $R/gpurun_out/worst_pmc -o run --output-format csv -- python3 $R/tools/worst_only.py > $R/gpurun_out/worst_pmc.log 2>&1 || { echo "pmc failed"; tail -5 $R/gpurun_out/worst_pmc.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_BRANCH -d $R/gpurun_out/worst_pmc2 -o run --output-format csv -- python3 $R/tools/worst_only.py > $R/gpurun_out/worst_pmc2.log 2>&1 || { echo "pmc2 failed"; tail -5 $R/gpurun_out/worst_pmc2.log; }
python3 - <<'PY'
import csv,glob,collections
for d in ('worst_pmc','worst_pmc2'):
    fs=glob.glob(f'/root/repo/gpurun_out/{d}/**/*counter_collection.csv',recursive=True)
    if not fs: continue
    agg=collections.defaultdict(lambda: collections.defaultdict(float)); n=collections.Counter()
    for r in csv.DictReader(open(fs[0])):
        if 'mpc_solve' not in r['Kernel_Name']: continue
        k=r['Kernel_Name'].split('(')[0][-22:]
        agg[k][r['Counter_Name']]+=float(r['Counter_Value'])
    for k,v in agg.items(): print(d, k, {a:int(b) for a,b in sorted(v.items())})
PY
