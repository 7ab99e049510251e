#!/bin/bash
# Ragged 10M build: kernel trace + SQ PMC pass (lane-refill ragged kernel).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
SPECS="ragged:X=1 build:X=1" bash scripts/prof_r03.sh || exit $?
SPECS="ragged:X=1" PMC_TOP=6 bash scripts/gpu_pmc_leaf.sh || exit $?
d=$(dirname "$(find gpurun_out/p3/ragged_X_1 -name "*kernel_trace.csv" | head -1)")
cp "$d"/*kernel_trace.csv "$d/run_kernel_trace.csv" 2>/dev/null
python3 scripts/timeline.py 3 k_leaf_direct "$d" | head -60 || true
