#!/bin/bash
# End-of-round evidence on the final tree: full -m gpu suite, smoke, default driver line, configs[4] line.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
EVID=1 bash scripts/gpu_r04n.sh || exit $?
timeout -k 10 400 python bench.py --workload incremental --steps 10 --warmup 3 > gpurun_out/ev/bench_inc.log 2>&1 || { tail -20 gpurun_out/ev/bench_inc.log; exit 1; }
tail -c 400 gpurun_out/ev/bench_inc.log
