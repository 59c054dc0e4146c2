# Executed-work counters over the C2 bench: FP64 VALU instruction counts and VALU
# activity per solver kernel, one rocprofv3 --pmc pass (7 SQ counters), the profiled program directly after --.
# Summary: tools/pmc_f64.py -> gpurun_out/pmc_f64.csv (copy to profiles/ to keep it).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
CFG=${CFG:-C2}
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/pmc_f64_$CFG
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $R/gpurun_out/pmc_f64_$CFG -o run --output-format csv -- python3 $R/bench.py --config $CFG --steps 3 --warmup 1 --no-cpu --inflight 0 --nlp-steps 0 --closed-loop 0 --plan-chunks 0 > $R/gpurun_out/pmc_f64_$CFG.log 2>&1 || { echo "pmc f64 failed"; tail $R/gpurun_out/pmc_f64_$CFG.log; exit 1; }
tail -1 $R/gpurun_out/pmc_f64_$CFG.log
cd $R && python3 tools/pmc_f64.py $CFG
