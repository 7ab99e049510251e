cd $GRAFT_REPO_ROOT
( while true; do date >> gpurun_out/r06_heartbeat.log; sleep 45; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python bench.py > gpurun_out/r06f_bench.json 2> gpurun_out/r06f_bench.err; rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/r06f_bench.err; exit $rc
