cd $GRAFT_REPO_ROOT
( while true; do date >> gpurun_out/r06_heartbeat.log; sleep 45; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06r_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r06r_pytest.log; [ $rc -eq 0 ] || exit $rc
PROF_DIR=r06r_inc BENCH_ARGS="--workload incremental" bash scripts/gpu_prof.sh || exit $?
