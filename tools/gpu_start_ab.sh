# GPU tests, then A/B of the interior-point start (libmpcqp.so = new, libmpcqp_old.so = previous) on the
# single-QP configs (both orders) and the C2 SQP leg; every step time-limited, the first failure ends it
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -q --timeout 300 --timeout-method thread -rA > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed|^E " gpurun_out/gpu_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/ab_probe.py libmpcqp.so libmpcqp_old.so --configs=C2,C3,C4,C5 --reps=30 || exit 1
timeout -k 10 600 python tools/ab_probe.py libmpcqp_old.so libmpcqp.so --configs=C2,C3,C4,C5 --reps=30 || exit 1
AB_SQP=30 timeout -k 10 600 python tools/ab_probe.py libmpcqp.so libmpcqp_old.so --configs=C2,C3 --reps=10 || exit 1
