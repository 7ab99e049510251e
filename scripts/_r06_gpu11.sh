cd $GRAFT_REPO_ROOT
( while true; do date >> gpurun_out/r06_heartbeat.log; sleep 45; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06aa_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r06aa_pytest.log; [ $rc -eq 0 ] || exit $rc
LIBS="prev=abl/prev/lib/libmerklekv_hip.so new=" REPS=2 TAILC=300 CMD="python tools/ab_inc.py" bash scripts/gpu_ab.sh > /dev/null || exit 1
grep -H "configs4" gpurun_out/ab/*_[12].log
LIBS="prev=abl/prev/lib/libmerklekv_hip.so new=" REPS=2 TAILC=120 CMD="python tools/ab_diff.py" bash scripts/gpu_ab.sh > /dev/null || exit 1
grep -H "vo-diff" gpurun_out/ab/*_[12].log
