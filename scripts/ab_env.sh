#!/bin/bash
# A/B over an environment variable: AB_VAR (name) x AB_VALS (values), 2 interleaved rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for v in $AB_VALS; do
    env $AB_VAR=$v timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline $AB_ARGS > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$AB_VAR=$v rep $rep', round(d['ms_per_step'],3), 'ms/step', {k: round(x,3) for k,x in d['stage_ms_per_step'].items()}, 'diff_ms', d['diff'] and round(d['diff']['ms'],3))"
  done
done
