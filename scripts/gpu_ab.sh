#!/bin/bash
# Interleaved A/B of library builds on one box (variants from scripts/mkvariant.sh):
#   LIBS="tag=path ..." (path empty = the in-tree library), REPS rounds (default 2),
#   CMD = the measuring command (default: the leaf-stage driver tools/ab_ragged.py <tag>; any command that
#         prints its own result line works, e.g. CMD="python bench.py --steps 20 --no-cpu-baseline").
# Each run is limited to LIM seconds (default 200); the first failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for rep in $(seq 1 ${REPS:-2}); do
  for spec in $LIBS; do
    tag=${spec%%=*}; lib=${spec#*=}
    if [ -n "$lib" ]; then export MKV_LIB_PATH=$lib; else unset MKV_LIB_PATH; fi
    if [ -n "$CMD" ]; then
      timeout -k 10 ${LIM:-200} $CMD > gpurun_out/ab/${tag}_$rep.log 2>&1 || { echo "$tag rc=$?"; tail -20 gpurun_out/ab/${tag}_$rep.log; exit 1; }
      echo "$tag rep $rep: $(tail -c ${TAILC:-600} gpurun_out/ab/${tag}_$rep.log)"
    else
      timeout -k 10 ${LIM:-200} python tools/ab_ragged.py $tag || { echo "$tag rc=$?"; exit 1; }
    fi
  done
done
