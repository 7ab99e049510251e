#!/bin/bash
# Round-end evidence in one GPU call: build-workload kernel trace, diff-workload kernel trace + PMC
# (FETCH_SIZE / WRITE_SIZE in separate passes), incremental bench with more steps. Stops on failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PROF_DIR=prof_build bash scripts/gpu_prof.sh || exit $?
PROF_DIR=prof_diff BENCH_ARGS="--workload diff" PMC="FETCH_SIZE WRITE_SIZE" bash scripts/gpu_prof.sh || exit $?
timeout -k 10 400 python bench.py --workload incremental --steps 10 --warmup 3 > gpurun_out/bench_inc10.json 2> gpurun_out/bench_inc10.err || { tail -20 gpurun_out/bench_inc10.err; exit 1; }
cat gpurun_out/bench_inc10.json
