#!/bin/bash
# Async key-list copies on the DMA engine: update/scale tests, 200-step host timeline (outliers), the
# incremental bench line and its kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_update_gpu.py tests/test_scale_gpu.py \
  > gpurun_out/r04v_t1.log 2>&1 || { tail -30 gpurun_out/r04v_t1.log; exit 1; }
tail -1 gpurun_out/r04v_t1.log
timeout -k 10 300 python tools/inc_trace.py 125000000 200 > gpurun_out/inc_trace.log 2>&1 || { tail -20 gpurun_out/inc_trace.log; exit 1; }
tail -3 gpurun_out/inc_trace.log
timeout -k 10 400 python bench.py --workload incremental > gpurun_out/r04v_inc.json 2> gpurun_out/r04v_inc.err || { tail -20 gpurun_out/r04v_inc.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r04v_inc.json').read().strip().splitlines()[-1]);i=d['incremental'];print(d['ms_per_step'],i['update_device_ms_all_replicas'],i['keys_d2h_ms_per_pair'],i['diff_device_ms_per_pair'])"
PROF_DIR=prof_r04v BENCH_ARGS="--workload incremental" bash scripts/gpu_prof.sh > gpurun_out/r04v_prof.log 2>&1 || { tail -20 gpurun_out/r04v_prof.log; exit 1; }
python3 scripts/timeline.py 4 k_locate_multi gpurun_out/prof_r04v/trace | awk 'NR<=4 || /zero_many|span|k_diff_keys /'
