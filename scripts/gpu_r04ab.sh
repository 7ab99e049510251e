#!/bin/bash
# Merge-join A/B: cur vs variant (VAR).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for rep in 1 2 3; do
  for v in cur h4; do
    if [ $v = cur ]; then unset MKV_LIB_PATH; else export MKV_LIB_PATH=abl/$v/lib/libmerklekv_hip.so; fi
    timeout -k 10 300 python bench.py --workload diff --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_diff.json 2> gpurun_out/ab_diff.err || { tail -5 gpurun_out/ab_diff.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab_diff.json').read().strip().splitlines()[-1])['diff']; m=d['mixed']; print('$v rep $rep mixed dev', round(m['device_ms'],3), 'ms', round(m['ms'],3), 'exact', m['exact_vs_construction'], '| value-only dev', round(d['value_only']['device_ms'],3))"
  done
done
