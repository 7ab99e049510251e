#!/bin/bash
# A/B of the SHA round variants (MKV_SHA_VARIANT) with interleaved rounds in one session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for v in 0 1; do
    MKV_SHA_VARIANT=$v timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-diff > gpurun_out/ab_$v_$rep.json 2>/dev/null || exit $?
    python -c "import json,sys; d=json.load(open('gpurun_out/ab_$v_$rep.json')); print('variant $v rep $rep', round(d['ms_per_step'],3), 'ms/step', {k: round(x,3) for k,x in d['stage_ms_per_step'].items()})"
  done
done
