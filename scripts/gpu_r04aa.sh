#!/bin/bash
# Climb: 2 (cur) / 4 dirty entries per lane vs 1 (HEAD): update tests, configs[4] A/B, climb kernel times.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_update_gpu.py \
  > gpurun_out/r04aa_t1.log 2>&1 || { tail -30 gpurun_out/r04aa_t1.log; exit 1; }
tail -1 gpurun_out/r04aa_t1.log
MKV_LIB_PATH=abl/e4/lib/libmerklekv_hip.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_update_gpu.py \
  > gpurun_out/r04aa_t2.log 2>&1 || { tail -30 gpurun_out/r04aa_t2.log; exit 1; }
tail -1 gpurun_out/r04aa_t2.log
AB_ROUNDS=2 AB_COMBOS="base MKV_LIB_PATH=abl/e4/lib/libmerklekv_hip.so MKV_LIB_PATH=abl/h3/lib/libmerklekv_hip.so" bash scripts/ab_inc.sh || exit 1
