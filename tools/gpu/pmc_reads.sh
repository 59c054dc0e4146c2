# Round 5: where the C2 step's HBM reads come from.  rocprofv3 --pmc passes, each its own
# run and time-limited, the program directly after --: FETCH_SIZE, then TCC_HIT/TCC_MISS, then the vector L1
# (TCP) accesses and its read requests to L2, per dispatch (crossover vs interior-point kernel), over per-GPU
# batches B = 1024, 2048, 4096 (a linear fit separates per-launch from per-instance bytes) and once with the
# work-list appends off (MPC_DBG=1: the interior-point launch then has nothing to do, its waves exit at once).
# Summarise with tools/pmc_reads.py.
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/pmcr_*
B="$R/bench.py --no-cpu --inflight 0 --nlp-steps 0 --closed-loop 0 --plan-chunks 0 --steps 3 --warmup 1"
run() {   # tag, batch, counters...
  local tag=$1; local b=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d $R/gpurun_out/pmcr_$tag -o run --output-format csv -- python3 $B \
      --batch $b > $R/gpurun_out/pmcr_$tag.log 2>&1 || { echo "pass $tag failed"; tail -5 $R/gpurun_out/pmcr_$tag.log; exit 1; }
  echo "pass $tag ok"
}
for b in 1024 2048 4096; do
  run fetch_$b $b FETCH_SIZE
  run tcc_$b $b TCC_HIT_sum TCC_MISS_sum
  run tcp_$b $b TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum
done
export MPC_DBG=1
run fetch_dbg 4096 FETCH_SIZE
unset MPC_DBG
cd $R && python3 tools/pmc_reads.py > gpurun_out/pmc_reads.txt && cat gpurun_out/pmc_reads.txt
