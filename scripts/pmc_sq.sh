#!/bin/bash
# One serialized PMC pass over a short build bench: SQ instruction / cycle counters + GRBM clock.
# PMC_SET overrides the counter list; AB_ARGS adds bench arguments. Output: gpurun_out/pmc_sq.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
SET="${PMC_SET:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE}"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc $SET -d $R/gpurun_out/pmc_sq -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-diff $AB_ARGS > $R/gpurun_out/pmc_sq.log 2>&1 || { echo "pmc failed"; tail -5 $R/gpurun_out/pmc_sq.log; exit 1; }
python3 $R/scripts/pmc_dispatch.py $R/gpurun_out/pmc_sq --top ${PMC_TOP:-14}
