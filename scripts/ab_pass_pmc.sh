#!/bin/bash
# Standalone (PMC-serialized) kernel durations of the build for the in-tree library and an A/B build
# (merklekv_amd/lib/ab_old), plus interleaved co-run build timings.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_parity_gpu.py -k "synthetic_sizes or shared_prefix or tie_runs or long_common or large_1m" > gpurun_out/pt.log 2>&1 || { tail -30 gpurun_out/pt.log; exit 1; }
tail -1 gpurun_out/pt.log
cd /tmp && export TMPDIR=/tmp
for L in new old; do
  if [ $L = old ]; then export MKV_LIB_PATH=$R/merklekv_amd/lib/ab_old/libmerklekv_hip.so; else unset MKV_LIB_PATH; fi
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc_$L -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-diff > $R/gpurun_out/pmc_$L.log 2>&1 || { echo "pmc $L failed"; tail -5 $R/gpurun_out/pmc_$L.log; exit 1; }
  python3 $R/scripts/kernel_durations.py $R/gpurun_out/pmc_$L $L
done
cd $R
unset MKV_LIB_PATH
AB_ROUNDS=3 AB_COMBOS="base MKV_LIB_PATH=$R/merklekv_amd/lib/ab_old/libmerklekv_hip.so" bash scripts/ab_combo.sh
