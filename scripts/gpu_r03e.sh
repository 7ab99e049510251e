#!/bin/bash
# Round-3 bench lines of the diff (configs[2]) and incremental (configs[4]) workloads, then the reduction
# top's SHA form A/B (kernel traces of the 10M build). Each step has its own limit; stops on failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/p3e
run() { local tag=$1 lim=$2; shift 2; echo "== $tag"; timeout -k 10 $lim "$@" > gpurun_out/p3e/$tag.json 2> gpurun_out/p3e/$tag.err; local rc=$?
  echo "$tag rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/p3e/$tag.err; exit $rc; }; tail -c 2500 gpurun_out/p3e/$tag.json; echo; }
run bench_diff 400 python bench.py --workload diff --steps 10 --warmup 2
run bench_inc 400 python bench.py --workload incremental --steps 10 --warmup 3
SPECS="build:MKV_TOP_SHA=0 build:MKV_TOP_SHA=1" bash scripts/prof_r03.sh
