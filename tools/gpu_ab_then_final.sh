# one call: the A/B of tools/gpu_start_ab.sh (which runs the -m gpu suite first), then the profiling pass of
# tools/gpu_bench_prof.sh; the first failure ends it
cd $GRAFT_REPO_ROOT
bash tools/gpu_start_ab.sh || exit 1
bash tools/gpu_bench_prof.sh
