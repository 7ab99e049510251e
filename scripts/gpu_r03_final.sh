cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/ev
timeout -k 10 600 python bench.py > gpurun_out/ev/bench.log 2> gpurun_out/ev/bench.err || exit 1
echo bench ok
EVID=2 bash scripts/gpu_r03_evidence.sh
