#!/bin/bash
# One-wait merge-join key tail: diff / shard / update tests, then mixed + value-only A/B vs HEAD (h6).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_parity_gpu.py tests/test_scale_gpu.py tests/test_shard_gpu.py tests/test_antientropy_gpu.py tests/test_reference_ports_gpu.py \
  > gpurun_out/r04ae_t1.log 2>&1 || { tail -30 gpurun_out/r04ae_t1.log; exit 1; }
tail -1 gpurun_out/r04ae_t1.log
for rep in 1 2 3; do
  for v in cur h6; do
    if [ $v = cur ]; then unset MKV_LIB_PATH; else export MKV_LIB_PATH=abl/$v/lib/libmerklekv_hip.so; fi
    timeout -k 10 300 python bench.py --workload diff --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_diff.json 2> gpurun_out/ab_diff.err || { tail -5 gpurun_out/ab_diff.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab_diff.json').read().strip().splitlines()[-1])['diff']; m=d['mixed']; v=d['value_only']; print('$v rep $rep mixed ms', round(m['ms'],3), 'dev', round(m['device_ms'],3), 'exact', m['exact_vs_construction'], '| value-only ms', round(v['ms'],3), 'exact', v['exact_vs_construction'])"
  done
done
