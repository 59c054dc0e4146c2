# The round's C2 profiles of the tracker (each rocprofv3 run its own, time-limited, the program directly after --):
#   1. kernel-trace stats of the bench (20 steps)           -> gpurun_out/prof_stats/.../*kernel_stats.csv
#   2. the executed-FP64 PMC pass (7 SQ counters)           -> tools/pmc_f64.py joins it with the stats of 1
#   3. FETCH_SIZE and WRITE_SIZE, one pass each             -> tools/pmc_summary.py (HBM bytes per step)
# ROUND (e.g. r06) and COMMIT tag the summaries; copy gpurun_out/profile_<ROUND>/ into profiles/ to keep them.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
ROUND=${ROUND:-r06}
CFG=${CFG:-C2}
OUT=$R/gpurun_out/profile_$ROUND
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_stats $R/gpurun_out/pmc_f64_$CFG $R/gpurun_out/pmc_fetch $R/gpurun_out/pmc_write $OUT
mkdir -p $OUT
B="python3 $R/bench.py --config $CFG --no-cpu --inflight 0 --nlp-steps 0 --closed-loop 0 --plan-chunks 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_stats -o run --output-format csv -- $B --steps 20 --warmup 3 > $OUT/bench_under_stats.log 2>&1 || { echo "stats failed"; tail $OUT/bench_under_stats.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $R/gpurun_out/pmc_f64_$CFG -o run --output-format csv -- $B --steps 3 --warmup 1 > $OUT/pmc_f64.log 2>&1 || { echo "pmc f64 failed"; tail $OUT/pmc_f64.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch -o run --output-format csv -- $B --steps 3 --warmup 1 > $OUT/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; tail $OUT/pmc_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write -o run --output-format csv -- $B --steps 3 --warmup 1 > $OUT/pmc_write.log 2>&1 || { echo "pmc write failed"; tail $OUT/pmc_write.log; exit 1; }
cd $R
STATS=$(find gpurun_out/prof_stats -name '*kernel_stats.csv' | head -1)
cp $STATS $OUT/${ROUND}_kernel_stats.csv
python3 tools/pmc_f64.py $CFG $OUT/${ROUND}_kernel_stats.csv > $OUT/pmc_f64.json && cp gpurun_out/pmc_f64_$CFG.csv $OUT/${ROUND}_pmc_f64_$CFG.csv
python3 tools/pmc_summary.py $CFG $ROUND ${COMMIT:-unknown} > $OUT/pmc_hbm.txt && cp profiles/pmc_hbm_bytes.json $OUT/pmc_hbm_bytes.json
ls $OUT; head -3 $OUT/${ROUND}_kernel_stats.csv; cat $OUT/pmc_hbm.txt | tail -3
