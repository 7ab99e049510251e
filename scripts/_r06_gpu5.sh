cd $GRAFT_REPO_ROOT
( while true; do date >> gpurun_out/r06_heartbeat.log; sleep 45; done ) &
HB=$!
trap "kill $HB" EXIT
P=${P:-r06i}
run() { local tag=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/${P}_$tag.log 2>&1; local rc=$?; echo "$tag rc=$rc"; tail -3 gpurun_out/${P}_$tag.log; [ $rc -eq 0 ] || exit $rc; }
[ "${TESTS:-1}" = 1 ] && run tests 600 python -u -m pytest ${TESTFILES:-tests/test_parity_gpu.py tests/test_update_gpu.py tests/test_scale_gpu.py} -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "${TESTK:-topdown or diff or many or incremental or eight}"
for rep in $(seq 1 ${REPS:-2}); do
  for spec in $LIBS; do
    tag=${spec%%=*}; lib=${spec#*=}
    if [ -n "$lib" ]; then export MKV_LIB_PATH=$lib; else unset MKV_LIB_PATH; fi
    case "${WL:-diff,inc}" in *diff*) run diff_${tag}_$rep 300 python bench.py --workload diff --steps 10 --warmup 2 --no-cpu-baseline;; esac
    case "${WL:-diff,inc}" in *inc*) run inc_${tag}_$rep 300 python bench.py --workload incremental --steps 10 --warmup 3 --no-cpu-baseline;; esac
  done
done
