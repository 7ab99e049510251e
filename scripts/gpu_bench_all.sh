#!/bin/bash
# All bench workloads, small sizes (functional check) unless FULL=1. Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "$FULL" ]; then
  B=""; D=""; I=""
else
  B="--records 1000000"; D="--records 1000000"; I="--records 2000000 --batch 2000"
fi
set -o pipefail
timeout -k 10 300 python bench.py --steps 3 --warmup 1 $B > gpurun_out/bench_build.json 2> gpurun_out/bench_build.err || { tail -20 gpurun_out/bench_build.err; exit 1; }
cat gpurun_out/bench_build.json
timeout -k 10 400 python bench.py --workload diff --steps 3 --warmup 1 $D > gpurun_out/bench_diff.json 2> gpurun_out/bench_diff.err || { tail -20 gpurun_out/bench_diff.err; exit 1; }
cat gpurun_out/bench_diff.json
timeout -k 10 400 python bench.py --workload incremental --steps 2 --warmup 1 $I > gpurun_out/bench_inc.json 2> gpurun_out/bench_inc.err || { tail -20 gpurun_out/bench_inc.err; exit 1; }
cat gpurun_out/bench_inc.json
