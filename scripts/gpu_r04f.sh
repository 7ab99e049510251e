#!/bin/bash
# Ragged 10M build timeline (kernel trace, one step).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
SPECS="ragged:X=1" bash scripts/prof_r03.sh > /dev/null || exit $?
python3 scripts/timeline.py 3 k_leaf_direct gpurun_out/p3/ragged_X_1 | head -40
