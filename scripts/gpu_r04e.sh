#!/bin/bash
# Edge-record kernel parity, then ragged/fixed leaf-stage A/B over grid x sort-tile variants.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_ragged_gpu.py tests/test_parity_gpu.py > gpurun_out/r04e_pytest.log 2>&1 || { tail -30 gpurun_out/r04e_pytest.log; exit 1; }
tail -2 gpurun_out/r04e_pytest.log
STEPS=10 LIBS="w3s24= w2s24=abl/w2s24/lib/libmerklekv_hip.so w3s16=abl/w3s16/lib/libmerklekv_hip.so w4s24=abl/w4s24/lib/libmerklekv_hip.so w4s16=abl/w4s16/lib/libmerklekv_hip.so" REPS=2 bash scripts/gpu_ab_ragged.sh
