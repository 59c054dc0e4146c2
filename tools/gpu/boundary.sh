# kernel-boundary cost of the C2 launch pair: the step with and without the Xpred output, each under rocprofv3
# kernel-trace stats (step - kernel averages = the two boundaries)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for m in with without; do
  rm -rf $R/gpurun_out/bnd_$m
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/bnd_$m -o run --output-format csv -- python3 $R/tools/boundary_probe.py $m > $R/gpurun_out/bnd_$m.log 2>&1 || { echo "$m failed"; tail $R/gpurun_out/bnd_$m.log; exit 1; }
  grep Xpred $R/gpurun_out/bnd_$m.log
  f=$(find $R/gpurun_out/bnd_$m -name '*kernel_stats.csv' | head -1)
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    n = r['Name']; k = 'IPM' if '2, 20>' in n else ('XO' if '1, 20>' in n else n[:24])
    print('  $m', k, r['Calls'], round(float(r['AverageNs']) / 1000, 2), 'us')"
done
