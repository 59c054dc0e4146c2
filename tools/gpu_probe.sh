cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python tools/timing_probe.py C2 4096 > gpurun_out/probe.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof1 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/prof1.log 2>&1
echo "prof rc=$?"
cat $GRAFT_REPO_ROOT/gpurun_out/probe.log
find $GRAFT_REPO_ROOT/gpurun_out/prof1 -name "*stats*" | head
