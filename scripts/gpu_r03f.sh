#!/bin/bash
# Leaf-stage bucketing change: parity tests (default and register ragged form), interleaved build A/B
# against the committed baseline library, ragged-build kernel traces. Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/p3f
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_ragged_gpu.py tests/test_parity_gpu.py tests/test_update_gpu.py > gpurun_out/p3f/pytest.log 2>&1 || { tail -40 gpurun_out/p3f/pytest.log; exit 1; }
tail -1 gpurun_out/p3f/pytest.log
MKV_LEAF_RAGGED=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_ragged_gpu.py > gpurun_out/p3f/pytest_rreg.log 2>&1 || { tail -40 gpurun_out/p3f/pytest_rreg.log; exit 1; }
tail -1 gpurun_out/p3f/pytest_rreg.log
LIBS="cur= base=/root/repo/ab/base/lib/libmerklekv_hip.so" REPS=3 bash scripts/ab_build_libs.sh || exit 1
SPECS="ragged:MKV_LEAF_RAGGED=1 ragged:MKV_LEAF_RAGGED=2,MKV_RREG_WGS=2 build:X=1" bash scripts/prof_r03.sh
