#!/bin/bash
# Update-call outliers over 300 configs[4] steps: DMA key-list copies (cur) vs copy kernels (idle).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for v in cur idle cur idle; do
  if [ $v = cur ]; then unset MKV_LIB_PATH; else export MKV_LIB_PATH=abl/$v/lib/libmerklekv_hip.so; fi
  timeout -k 10 300 python tools/inc_trace.py 125000000 300 > gpurun_out/inc_trace_$v.log 2>&1 || { tail -20 gpurun_out/inc_trace_$v.log; exit 1; }
  echo "== $v"; tail -8 gpurun_out/inc_trace_$v.log
done
