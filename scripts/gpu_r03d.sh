#!/bin/bash
# Register-form ragged leaf kernel: parity tests under MKV_LEAF_RAGGED=2, then kernel traces of the 10M
# ragged build (LDS form vs register form) and of the 100M mixed diff (round-2 partition, base vs
# waves_per_eu(3) pass 1). Every step has its own limit; stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/p3d
MKV_LEAF_RAGGED=2 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_ragged_gpu.py tests/test_parity_gpu.py > gpurun_out/p3d/pytest_rreg.log 2>&1 || { tail -40 gpurun_out/p3d/pytest_rreg.log; exit 1; }
tail -2 gpurun_out/p3d/pytest_rreg.log
SPECS="${SPECS:-ragged:MKV_LEAF_RAGGED=2 ragged:MKV_LEAF_RAGGED=1 mixed:MKV_DIFF_PART=0 mixed:MKV_DIFF_PART=0,MKV_LIB_PATH=/root/repo/ab/w3/lib/libmerklekv_hip.so}" bash scripts/prof_r03.sh
