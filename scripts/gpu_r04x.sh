#!/bin/bash
# Current ragged and fixed build timelines (kernel trace of tools/r03_paths.py).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
SPECS="ragged:X=1 build:X=1" bash scripts/prof_r03.sh > gpurun_out/r04x_prof.log 2>&1 || { tail -20 gpurun_out/r04x_prof.log; exit 1; }
grep "ms/step" gpurun_out/r04x_prof.log
python3 scripts/timeline.py 3 k_leaf_direct gpurun_out/p3/ragged_X_1
python3 scripts/timeline.py 3 k_leaf_direct gpurun_out/p3/build_X_1
