#!/bin/bash
# Hand-off protocol parity (ragged + parity + leaf tests), then the WGS A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_ragged_gpu.py tests/test_parity_gpu.py > gpurun_out/r04c_pytest.log 2>&1 || { tail -30 gpurun_out/r04c_pytest.log; exit 1; }
tail -2 gpurun_out/r04c_pytest.log
LIBS="w3= w2=ab/w2/lib/libmerklekv_hip.so" REPS=2 bash scripts/gpu_ab_ragged.sh
