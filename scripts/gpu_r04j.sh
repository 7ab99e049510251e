#!/bin/bash
# Key ownership back in the leaf kernels (fixed: from registers; ragged: key-run dwords; edges: bytes):
# parity of the build paths, then the leaf-stage A/B and traces of the fixed and ragged builds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $PYT tests/test_ragged_gpu.py tests/test_parity_gpu.py > gpurun_out/r04j_t1.log 2>&1 \
  || { tail -40 gpurun_out/r04j_t1.log; exit 1; }
tail -1 gpurun_out/r04j_t1.log
STEPS=10 LIBS="cur=" REPS=2 bash scripts/gpu_ab_ragged.sh || exit 1
SPECS="build:X=1 ragged:X=1" bash scripts/prof_r03.sh > gpurun_out/r04j_prof.log 2>&1 || { tail -20 gpurun_out/r04j_prof.log; exit 1; }
grep -E "ms/step" gpurun_out/r04j_prof.log
python3 scripts/timeline.py 3 k_leaf_direct gpurun_out/p3/build_X_1
python3 scripts/timeline.py 3 k_leaf_direct gpurun_out/p3/ragged_X_1
