#!/bin/bash
# SQ PMC passes (serialised kernels) over the 10M fixed and ragged builds of tools/r03_paths.py; MODES and
# the env of each pass come from SPECS ("mode:ENV=..,ENV=.." as in prof_r03.sh). Output: gpurun_out/pmc/<tag>.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p "$R/gpurun_out/pmc"
cd /tmp && export TMPDIR=/tmp
SET="${PMC_SET:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE}"
for spec in $SPECS; do
  mode=${spec%%:*}; envs=${spec#*:}; tag=${mode}_${envs//[=,\/]/_}
  env ${envs//,/ } STEPS=3 timeout -s KILL 120 rocprofv3 --pmc $SET -d "$R/gpurun_out/pmc/$tag" -o run --output-format csv -- python3 "$R/tools/r03_paths.py" $mode > "$R/gpurun_out/pmc/$tag.log" 2>&1; rc=$?
  echo "== $tag rc=$rc"
  [ $rc -eq 0 ] || { tail -5 "$R/gpurun_out/pmc/$tag.log"; exit $rc; }
  python3 "$R/scripts/pmc_dispatch.py" "$R/gpurun_out/pmc/$tag" --top ${PMC_TOP:-4}
done
exit 0
