#!/bin/bash
# Batched walk: level-4 abort test on the device (variant gate) — update / scale tests on it, configs[4] A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
MKV_LIB_PATH=abl/gate/lib/libmerklekv_hip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_update_gpu.py tests/test_scale_gpu.py tests/test_antientropy_gpu.py \
  > gpurun_out/r04aj_t1.log 2>&1 || { tail -30 gpurun_out/r04aj_t1.log; exit 1; }
tail -1 gpurun_out/r04aj_t1.log
AB_ROUNDS=3 AB_COMBOS="base MKV_LIB_PATH=abl/gate/lib/libmerklekv_hip.so" bash scripts/ab_inc.sh || exit 1
