# kernel durations of the C2 launch pair at per-GPU batches 1024, 2048, 4096 (does the crossover kernel scale with its wave count?)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for B in 1024 2048 4096; do
  rm -rf $R/gpurun_out/xs_$B
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/xs_$B -o run --output-format csv -- python3 $R/bench.py --config C2 --batch $B --no-cpu --inflight 0 --nlp-steps 0 --closed-loop 0 --plan-chunks 0 --steps 50 --warmup 3 > $R/gpurun_out/xs_$B.log 2>&1 || { echo "B=$B failed"; tail $R/gpurun_out/xs_$B.log; exit 1; }
  f=$(find $R/gpurun_out/xs_$B -name '*kernel_stats.csv' | head -1)
  echo "B=$B"; cut -d, -f1-4 $f | sed 's/(DevTable.*"/"/' | head -4
done
