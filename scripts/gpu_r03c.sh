#!/bin/bash
# Round-3 checks after the merge-join split fix: diff parity tests, kernel traces of the 100M mixed diff
# (MKV_DIFF_PART 1 / 0), then one SQ PMC pass over the 10M ragged build. Every step has its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out/p3c
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_parity_gpu.py tests/test_scale_gpu.py -k "diff" > gpurun_out/p3c/pytest_diff.log 2>&1 || { tail -30 gpurun_out/p3c/pytest_diff.log; exit 1; }
tail -2 gpurun_out/p3c/pytest_diff.log
SPECS="mixed:MKV_DIFF_PART=1 mixed:MKV_DIFF_PART=0" bash scripts/prof_r03.sh || exit $?
cd /tmp && export TMPDIR=/tmp
SET="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
STEPS=3 timeout -s KILL 120 rocprofv3 --pmc $SET -d $R/gpurun_out/p3c/pmc_ragged -o run --output-format csv -- python3 $R/tools/r03_paths.py ragged > $R/gpurun_out/p3c/pmc_ragged.log 2>&1 || { echo "pmc failed"; tail -5 $R/gpurun_out/p3c/pmc_ragged.log; exit 1; }
python3 $R/scripts/pmc_dispatch.py $R/gpurun_out/p3c/pmc_ragged --top 8
