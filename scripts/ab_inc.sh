#!/bin/bash
# A/B of the incremental workload (configs[4]) over environment combinations: AB_COMBOS as ab_combo.sh.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in $(seq 1 ${AB_ROUNDS:-2}); do
  for c in $AB_COMBOS; do
    envs=""
    [ "$c" != "base" ] && envs=$(echo "$c" | tr ',' ' ')
    env $envs timeout -k 10 300 python bench.py --workload incremental --steps ${AB_STEPS:-8} --warmup 2 --no-cpu-baseline $AB_ARGS > gpurun_out/ab_inc.json 2>gpurun_out/ab_inc.err || { tail -5 gpurun_out/ab_inc.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab_inc.json')); i=d['incremental']; print('$c rep $rep', round(d['ms_per_step'],3), 'ms/step upd', round(i['update_device_ms_all_replicas'],3), 'diff/pair', round(i['diff_device_ms_per_pair'],3), i['diff_sizes_match_unique_updates'])"
  done
done
