#!/bin/bash
# Interleaved build-workload A/B of library builds (LIBS="tag=path ..."; path "" = the in-tree library),
# REPS rounds, each run under its own limit. Prints ms/step and the stage split per run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abl
for rep in $(seq 1 ${REPS:-2}); do
  for spec in $LIBS; do
    tag=${spec%%=*}; lib=${spec#*=}
    if [ -n "$lib" ]; then export MKV_LIB_PATH=$lib; else unset MKV_LIB_PATH; fi
    timeout -k 10 300 python bench.py --steps ${STEPS:-30} --warmup 3 --no-cpu-baseline --no-diff $BENCH_ARGS > gpurun_out/abl/${tag}_$rep.json 2> gpurun_out/abl/${tag}_$rep.err || { echo "$tag rc=$?"; tail -5 gpurun_out/abl/${tag}_$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/abl/${tag}_$rep.json')); print('${tag} rep $rep', round(d['ms_per_step'],4), {k: round(x,3) for k,x in d['stage_ms_per_step'].items()})"
  done
done
unset MKV_LIB_PATH
