#!/bin/bash
# Climb variant: update / shard / scale tests, then configs[4] A/B vs HEAD (h7).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_update_gpu.py tests/test_shard_gpu.py tests/test_scale_gpu.py tests/test_antientropy_gpu.py \
  > gpurun_out/r04af_t1.log 2>&1 || { tail -30 gpurun_out/r04af_t1.log; exit 1; }
tail -1 gpurun_out/r04af_t1.log
AB_ROUNDS=3 AB_COMBOS="${AB_COMBOS:-base MKV_LIB_PATH=abl/h7/lib/libmerklekv_hip.so}" bash scripts/ab_inc.sh || exit 1
