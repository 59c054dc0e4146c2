# one GPU call: the full -m gpu suite + bench (tools/gpu_tests.sh), then the phase_micro variants and an
# A/B of the library variants in $LIBS; stops at the first failure
cd $GRAFT_REPO_ROOT
bash tools/gpu_tests.sh || exit 1
bash tools/probes/run_micro.sh || exit 1
[ -n "$LIBS" ] && timeout -k 10 900 python tools/ab_probe.py $LIBS --configs=${CONFIGS:-C2,C3,C4,C5} --reps=20
