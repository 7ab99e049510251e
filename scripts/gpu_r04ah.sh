#!/bin/bash
# Leaf helper launch on the CUs the ordering stream is masked off (variant abl/helper, built from
# scripts/variants/leaf_helper.diff): ragged / parity tests on it, build A/B vs the in-tree library,
# configs[4] A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
MKV_LIB_PATH=abl/helper/lib/libmerklekv_hip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_ragged_gpu.py tests/test_parity_gpu.py \
  > gpurun_out/r04ah_t1.log 2>&1 || { tail -30 gpurun_out/r04ah_t1.log; exit 1; }
tail -1 gpurun_out/r04ah_t1.log
REPS=3 LIBS="cur= helper=abl/helper/lib/libmerklekv_hip.so" bash scripts/gpu_ab_ragged.sh || exit 1
AB_ROUNDS=2 AB_COMBOS="base MKV_LIB_PATH=abl/helper/lib/libmerklekv_hip.so" bash scripts/ab_inc.sh || exit 1
