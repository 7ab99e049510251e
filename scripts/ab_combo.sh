#!/bin/bash
# A/B over environment combinations: AB_COMBOS = space-separated list of "VAR=v,VAR2=w" (or "base"),
# AB_ROUNDS interleaved rounds (default 2) of the build workload.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in $(seq 1 ${AB_ROUNDS:-2}); do
  for c in $AB_COMBOS; do
    envs=""
    [ "$c" != "base" ] && envs=$(echo "$c" | tr ',' ' ')
    env $envs timeout -k 10 300 python bench.py --steps ${AB_STEPS:-30} --warmup 3 --no-cpu-baseline --no-diff $AB_ARGS > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$c rep $rep', round(d['ms_per_step'],3), 'ms/step', {k: round(x,3) for k,x in d['stage_ms_per_step'].items()}, (d.get('root') or '')[:12])"
  done
done
