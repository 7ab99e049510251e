#!/bin/bash
# GPU tests (all) then the full-size diff bench and the default build bench. Stops on failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --workload diff --steps 10 --warmup 2 > gpurun_out/bench_diff.json 2> gpurun_out/bench_diff.err || { tail -20 gpurun_out/bench_diff.err; exit 1; }
cat gpurun_out/bench_diff.json
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 400 python bench.py --workload incremental --steps 10 --warmup 3 > gpurun_out/bench_inc.json 2> gpurun_out/bench_inc.err || { tail -20 gpurun_out/bench_inc.err; exit 1; }
cat gpurun_out/bench_inc.json
