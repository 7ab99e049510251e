#!/bin/bash
# configs[4] A/B of the asynchronous key-list copy: copy kernel with 64 / 16 workgroups, SDMA copy, and the
# copy waited inside the call (no overlap).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for spec in cur= b16=abl/b16 sdma=abl/sdma syncd=abl/syncd; do
  tag=${spec%%=*}; d=${spec#*=}
  if [ -n "$d" ]; then export MKV_LIB_PATH=$d/lib/libmerklekv_hip.so; else unset MKV_LIB_PATH; fi
  timeout -k 10 300 python -u bench.py --workload incremental --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r04o_$tag.json 2> gpurun_out/r04o_$tag.err \
    || { echo "$tag failed"; tail -20 gpurun_out/r04o_$tag.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open('gpurun_out/r04o_$tag.json'));i=d['incremental'];print('$tag', round(d['ms_per_step'],3), 'upd', round(i['update_device_ms_all_replicas'],3), 'diff/pair', round(i['diff_device_ms_per_pair'],3), 'd2h/pair', round(i['keys_d2h_ms_per_pair'],3))"
done
