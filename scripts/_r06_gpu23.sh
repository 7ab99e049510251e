cd $GRAFT_REPO_ROOT
( while true; do date >> gpurun_out/r06_heartbeat.log; sleep 45; done ) &
HB=$!
trap "kill $HB" EXIT
TAG=r06zz PART=tests bash scripts/gpu_evidence.sh || exit 1
TAG=r06zz PART=lines bash scripts/gpu_evidence.sh || exit 1
