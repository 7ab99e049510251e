#!/bin/bash
# Ragged LDS layout A/B: one front per workgroup, stride 34 (34.1 KiB, b64 reads) vs stride 33 (33.1 KiB,
# b32 reads: a 56.5-KiB sort tile fits beside three workgroups even with 1-KiB LDS granules).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_ragged_gpu.py \
  > gpurun_out/r04q_t1.log 2>&1 || { tail -30 gpurun_out/r04q_t1.log; exit 1; }
tail -1 gpurun_out/r04q_t1.log
STEPS=10 REPS=3 LIBS="cur= s33=abl/s33/lib/libmerklekv_hip.so" bash scripts/gpu_ab_ragged.sh || exit 1
MKV_LIB_PATH=abl/s33/lib/libmerklekv_hip.so SPECS="ragged:X=1" bash scripts/prof_r03.sh > gpurun_out/r04q_prof.log 2>&1 || { tail -20 gpurun_out/r04q_prof.log; exit 1; }
python3 scripts/timeline.py 3 k_leaf_direct gpurun_out/p3/ragged_X_1 | head -14
