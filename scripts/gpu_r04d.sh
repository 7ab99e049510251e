#!/bin/bash
# Kernel trace + one-step timeline of the fixed 10M build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
SPECS="build:X=1" bash scripts/prof_r03.sh || exit $?
d=gpurun_out/p3/build_X_1
python3 scripts/timeline.py 3 k_leaf_direct "$d" | head -40 || true
