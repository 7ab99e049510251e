#!/bin/bash
# HBM traffic of the configs[4] step (climb = k_dirty_climb + the reductions queued right after it; walk =
# the batched top-down diff), per step, from separate FETCH_SIZE / WRITE_SIZE passes, plus the calibration
# program (scripts/pmc_calib.hip: known byte counts at the climb's access widths). Output:
# gpurun_out/pmc_inc/summary.json (copied to profiles/pmc_incremental.json).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
P="$R/gpurun_out/pmc_inc"
mkdir -p "$P"
BA="--workload incremental --steps 2 --warmup 1 --no-cpu-baseline"
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c -d "$P/calib_$c" -o run --output-format csv -- "$R/scripts/pmc_calib" > "$P/calib_$c.log" 2>&1 || { echo "calib $c failed"; tail -3 "$P/calib_$c.log"; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc $c -d "$P/inc_$c" -o run --output-format csv -- python3 "$R/bench.py" $BA > "$P/inc_$c.log" 2>&1 || { echo "inc $c failed"; tail -3 "$P/inc_$c.log"; exit 1; }
done
python3 "$R/scripts/pmc_inc_summary.py" "$P" > "$P/summary.json" && cat "$P/summary.json"
