#!/bin/bash
# PMC-serialized kernel durations + interleaved co-run builds for the in-tree library and the A/B
# builds named in AB_LIBS (directories under merklekv_amd/lib holding libmerklekv_hip.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for L in base $AB_LIBS; do
  if [ $L = base ]; then unset MKV_LIB_PATH; else export MKV_LIB_PATH=$R/merklekv_amd/lib/$L/libmerklekv_hip.so; fi
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc_$L -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-diff > $R/gpurun_out/pmc_$L.log 2>&1 || { echo "pmc $L failed"; tail -5 $R/gpurun_out/pmc_$L.log; exit 1; }
  python3 $R/scripts/kernel_durations.py $R/gpurun_out/pmc_$L $L | grep -E "os_pass|prefix_hist|leaf|reduce_fused<false"
done
cd $R
unset MKV_LIB_PATH
combos="base"
for L in $AB_LIBS; do combos="$combos MKV_LIB_PATH=$R/merklekv_amd/lib/$L/libmerklekv_hip.so"; done
AB_ROUNDS=${AB_ROUNDS:-2} AB_COMBOS="$combos" bash scripts/ab_combo.sh
