cd $GRAFT_REPO_ROOT
( while true; do date >> gpurun_out/r06_heartbeat.log; sleep 45; done ) &
HB=$!
trap "kill $HB" EXIT
run() { local tag=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/r06e_$tag.log 2>&1; local rc=$?; echo "$tag rc=$rc"; tail -4 gpurun_out/r06e_$tag.log; [ $rc -eq 0 ] || exit $rc; }
run scale1b 900 python -u -m pytest tests/test_shard_scale_gpu.py -x -v --timeout 400 --timeout-method thread -p no:cacheprovider --durations=0 -k "1b_diff or configs4_1b"
