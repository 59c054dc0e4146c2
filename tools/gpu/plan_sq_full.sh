# Round 5: SQ wait classes of a full planner launch (1024 chunks at N = 16, four waves per CU) against the
# slowest chunk alone (tools/gpu/plan_sq_worst.sh): where the 2.4x per-iteration cost of a full launch goes.
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/plan_sqf1
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS -d $R/gpurun_out/plan_sqf1 -o run --output-format csv -- python3 $R/tools/plan_probe.py 16 1024 traj3 0.1 > $R/gpurun_out/plan_sqf1.log 2>&1 || { echo "sqf1 failed"; tail $R/gpurun_out/plan_sqf1.log; exit 1; }
cd $R && python3 - <<'PY'
import csv, glob, collections
f = glob.glob('gpurun_out/plan_sqf1/**/*counter_collection.csv', recursive=True)
agg = collections.Counter(); disp = set()
for row in csv.DictReader(open(f[0])):
    if 'plan_chunk_kernel' not in row.get('Kernel_Name', ''):
        continue
    agg[row['Counter_Name']] += float(row['Counter_Value']); disp.add(row.get('Dispatch_Id'))
n = len(disp)
print(f"plan_sqf1 1024 chunks N=16, {n} dispatches, per dispatch: " + " ".join(f"{k}={v / n:.4g}" for k, v in sorted(agg.items())))
w = agg['SQ_WAVE_CYCLES']
print("fractions of wave cycles: " + " ".join(f"{k}={agg[k] / w:.3f}" for k in ('SQ_WAIT_ANY', 'SQ_WAIT_INST_ANY', 'SQ_ACTIVE_INST_ANY', 'SQ_WAIT_INST_LDS')))
PY
