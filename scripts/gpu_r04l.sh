#!/bin/bash
# Ragged key ownership by a chunk-span copy kernel on the leaf stream: parity, then A/B vs no copy at all.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_ragged_gpu.py \
  > gpurun_out/r04l_t1.log 2>&1 || { tail -40 gpurun_out/r04l_t1.log; exit 1; }
tail -1 gpurun_out/r04l_t1.log
STEPS=10 REPS=2 LIBS="cur= nokcp=abl/nokcp/lib/libmerklekv_hip.so i20=abl/ipt20/lib/libmerklekv_hip.so i22=abl/ipt22/lib/libmerklekv_hip.so" bash scripts/gpu_ab_ragged.sh || exit 1
SPECS="ragged:X=1" bash scripts/prof_r03.sh > gpurun_out/r04l_prof.log 2>&1 || { tail -20 gpurun_out/r04l_prof.log; exit 1; }
python3 scripts/timeline.py 3 k_leaf_direct gpurun_out/p3/ragged_X_1
