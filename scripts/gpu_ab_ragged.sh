#!/bin/bash
# Interleaved leaf-stage A/B of library builds: LIBS="tag=path ..." (path "" = in-tree), REPS rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for rep in $(seq 1 ${REPS:-2}); do
  for spec in $LIBS; do
    tag=${spec%%=*}; lib=${spec#*=}
    if [ -n "$lib" ]; then export MKV_LIB_PATH=$lib; else unset MKV_LIB_PATH; fi
    timeout -k 10 200 python tools/ab_ragged.py $tag || { echo "$tag rc=$?"; exit 1; }
  done
done
