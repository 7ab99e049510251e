#!/bin/bash
# Standalone (PMC-serialized) kernel durations of the build for each value of an environment variable:
# AB_VAR (name) x AB_VALS (values). rocprofv3 --pmc serializes the kernels, so every duration is the
# kernel alone (no co-run).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for v in $AB_VALS; do
  export $AB_VAR=$v
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc_$v -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-diff $AB_ARGS > $R/gpurun_out/pmc_$v.log 2>&1 || { echo "pmc $v failed"; tail -5 $R/gpurun_out/pmc_$v.log; exit 1; }
  python3 $R/scripts/kernel_durations.py $R/gpurun_out/pmc_$v "$AB_VAR=$v" | head -${AB_TOP:-16}
done
