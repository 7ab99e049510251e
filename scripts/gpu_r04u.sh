#!/bin/bash
# configs[4]: key-list copy beside the next update — copy workgroups 64 (cur) / 16 / 256 and SDMA.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
AB_ROUNDS=2 AB_COMBOS="base MKV_LIB_PATH=abl/cb16/lib/libmerklekv_hip.so MKV_LIB_PATH=abl/cb256/lib/libmerklekv_hip.so MKV_LIB_PATH=abl/sdma/lib/libmerklekv_hip.so" bash scripts/ab_inc.sh || exit 1
MKV_LIB_PATH=abl/sdma/lib/libmerklekv_hip.so timeout -k 10 240 python tools/inc_trace.py > gpurun_out/inc_trace_sdma.log 2>&1 || { tail -20 gpurun_out/inc_trace_sdma.log; exit 1; }
tail -6 gpurun_out/inc_trace_sdma.log
