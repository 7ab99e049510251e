#!/bin/bash
# Fixed-shape leaf hash at 2 / 3 / 4 workgroups per CU beside the 55-KiB sort tile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
REPS=3 LIBS="cur= lw3=abl/lw3/lib/libmerklekv_hip.so lw4=abl/lw4/lib/libmerklekv_hip.so" bash scripts/gpu_ab_ragged.sh || exit 1
