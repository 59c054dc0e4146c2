# one GPU call: bench (with the closed-loop leg), kernel-trace stats, two PMC passes (HBM bytes) and the
# phase-cycle probe, each time-limited.  ROUND (e.g. r03) and COMMIT tag the PMC summary.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 500 python bench.py --steps 20 --warmup 3 --cpu-seconds 15 --closed-loop ${CL:-512} > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_stats $R/gpurun_out/pmc_fetch $R/gpurun_out/pmc_write
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_stats -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu --inflight 0 --nlp-steps 0 --closed-loop 0 --plan-chunks 0 > $R/gpurun_out/prof_stats.log 2>&1 || { echo "stats failed"; tail $R/gpurun_out/prof_stats.log; exit 1; }
tail -1 $R/gpurun_out/prof_stats.log
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --inflight 0 --nlp-steps 0 --closed-loop 0 --plan-chunks 0 > $R/gpurun_out/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; tail $R/gpurun_out/pmc_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --inflight 0 --nlp-steps 0 --closed-loop 0 --plan-chunks 0 > $R/gpurun_out/pmc_write.log 2>&1 || { echo "pmc write failed"; tail $R/gpurun_out/pmc_write.log; exit 1; }
cd $R && python tools/pmc_summary.py C2 ${ROUND:-} ${COMMIT:-}
find gpurun_out/prof_stats -name "*kernel_stats*"
: > gpurun_out/phase.log
timeout -k 10 200 python tools/phase_probe.py C2 4096 >> gpurun_out/phase.log 2>&1 && PROBE_WORST=1 timeout -k 10 200 python tools/phase_probe.py C2 1 >> gpurun_out/phase.log 2>&1 || { echo "phase probe failed"; tail gpurun_out/phase.log; exit 1; }
bash tools/gpu/configs.sh
