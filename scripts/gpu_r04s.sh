#!/bin/bash
# configs[4]: update no longer waits behind the previous step's key-list copies (no event on idle
# streams); host timeline + A/B vs HEAD.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 240 python tools/inc_trace.py > gpurun_out/inc_trace.log 2>&1 || { tail -20 gpurun_out/inc_trace.log; exit 1; }
tail -9 gpurun_out/inc_trace.log
AB_ROUNDS=2 AB_COMBOS="base MKV_LIB_PATH=abl/head/lib/libmerklekv_hip.so" bash scripts/ab_inc.sh || exit 1
