#!/bin/bash
# Ordering stream (st2) on a CU mask (half / half in pairs / three quarters of the CUs) instead of the
# high-priority stream over all CUs: build (fixed + ragged) A/B, then configs[4].
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
REPS=2 LIBS="cur= cu5555=abl/cu5555/lib/libmerklekv_hip.so cu3333=abl/cu3333/lib/libmerklekv_hip.so cu7777=abl/cu7777/lib/libmerklekv_hip.so" bash scripts/gpu_ab_ragged.sh || exit 1
AB_ROUNDS=1 AB_COMBOS="base MKV_LIB_PATH=abl/cu5555/lib/libmerklekv_hip.so MKV_LIB_PATH=abl/cu7777/lib/libmerklekv_hip.so" bash scripts/ab_inc.sh || exit 1
