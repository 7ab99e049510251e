#!/bin/bash
# Full GPU suite on the pruned library + key copy in the sort's first pass, then the leaf-stage A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests \
  > gpurun_out/r04g_pytest.log 2>&1 || { tail -40 gpurun_out/r04g_pytest.log; exit 1; }
tail -2 gpurun_out/r04g_pytest.log
STEPS=10 LIBS="cur=" REPS=2 bash scripts/gpu_ab_ragged.sh
SPECS="ragged:X=1" bash scripts/prof_r03.sh > /dev/null || exit $?
python3 scripts/timeline.py 3 k_leaf_direct gpurun_out/p3/ragged_X_1 | head -40
