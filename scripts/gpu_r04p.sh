#!/bin/bash
# Default driver line (ragged block timed like the headline loop), SQ PMC of the fixed and ragged leaf
# stages, and FETCH/WRITE PMC passes of the configs[4] incremental step (climb + walk traffic).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ev
timeout -k 10 600 python bench.py > gpurun_out/ev/bench_p.log 2> gpurun_out/ev/bench_p.err || { tail -20 gpurun_out/ev/bench_p.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/ev/bench_p.log').read().strip().splitlines()[-1]);r=d['ragged_10m'];print(d['ms_per_step'],r['ms_per_step'],r['leaf_hash_ms'],r['ratio_vs_fixed'])"
SPECS="build:X=1 ragged:X=1" bash scripts/gpu_pmc_leaf.sh > gpurun_out/ev/pmc_leaf.log 2>&1 || { tail -20 gpurun_out/ev/pmc_leaf.log; exit 1; }
cat gpurun_out/ev/pmc_leaf.log
PROF_DIR=prof_inc BENCH_ARGS="--workload incremental" PMC="FETCH_SIZE WRITE_SIZE" bash scripts/gpu_prof.sh > gpurun_out/ev/prof_inc.log 2>&1 || { tail -20 gpurun_out/ev/prof_inc.log; exit 1; }
tail -4 gpurun_out/ev/prof_inc.log
