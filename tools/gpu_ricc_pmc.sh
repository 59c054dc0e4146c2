# recursion micro-benchmark + SQ counters per recursion kernel (one rocprofv3 pass)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 60 ./tools/probes/ricc_probe
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/ricc_pmc
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS -d $R/gpurun_out/ricc_pmc -o run --output-format csv -- $R/tools/probes/ricc_probe > $R/gpurun_out/ricc_pmc.log 2>&1 || { echo "pmc failed"; tail -5 $R/gpurun_out/ricc_pmc.log; exit 1; }
python3 - <<'PY'
import csv,glob,collections
f=glob.glob('/root/repo/gpurun_out/ricc_pmc/**/*counter_collection.csv',recursive=True)[0]
d=collections.defaultdict(dict)
for r in csv.DictReader(open(f)):
    d[(r['Dispatch_Id'],r['Kernel_Name'][:40])][r['Counter_Name']]=float(r['Counter_Value'])
for k,v in sorted(d.items(), key=lambda kv: int(kv[0][0])):
    print(k, {a: int(b) for a,b in sorted(v.items())})
PY
