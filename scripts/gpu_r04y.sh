#!/bin/bash
# Sort tile 56,520 -> 56,320 B (scan scratch aliased into the key tile): ragged + fixed build A/B, sort
# tests, ragged timeline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_ragged_gpu.py tests/test_parity_gpu.py \
  > gpurun_out/r04y_t1.log 2>&1 || { tail -30 gpurun_out/r04y_t1.log; exit 1; }
tail -1 gpurun_out/r04y_t1.log
REPS=3 LIBS="cur= h2=abl/h2/lib/libmerklekv_hip.so" bash scripts/gpu_ab_ragged.sh || exit 1
SPECS="ragged:X=1" bash scripts/prof_r03.sh > gpurun_out/r04y_prof.log 2>&1 || { tail -20 gpurun_out/r04y_prof.log; exit 1; }
python3 scripts/timeline.py 3 k_leaf_direct gpurun_out/p3/ragged_X_1
