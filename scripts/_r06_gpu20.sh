cd $GRAFT_REPO_ROOT
( while true; do date >> gpurun_out/r06_heartbeat.log; sleep 45; done ) &
HB=$!
trap "kill $HB" EXIT
TAG=r06z PART=tests bash scripts/gpu_evidence.sh || exit 1
TAG=r06z PART=lines bash scripts/gpu_evidence.sh || exit 1
PROF_DIR=r06z/prof_inc BENCH_ARGS="--workload incremental" bash scripts/gpu_prof.sh > /dev/null || exit 1
