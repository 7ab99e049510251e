#!/bin/bash
# Round evidence on one GPU box, in parts (PART=tests|prof|lines|all, default all), output under
# gpurun_out/${TAG:-ev}/ (copy what gets cited into profiles/<round>_*):
#   tests  the full -m gpu suite, smoke() and the default driver line (python bench.py)
#   prof   kernel trace + PMC passes of the build workload and of the diff workload (scripts/gpu_prof.sh)
#   lines  the diff workload line (configs[2]) and the incremental workload line (configs[4])
# Every GPU step runs under its own time limit; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-ev}
mkdir -p $OUT
step() { local tag=$1 lim=$2; shift 2; echo "== $tag"; timeout -k 10 $lim "$@" > $OUT/$tag.log 2>&1; local rc=$?
  echo "$tag rc=$rc"; tail -${TAILN:-3} $OUT/$tag.log; [ $rc -eq 0 ] || exit $rc; }
PART=${PART:-all}
if [ $PART = tests ] || [ $PART = all ]; then
  step pytest_gpu 1000 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
  step bench 600 python bench.py
fi
if [ $PART = prof ] || [ $PART = all ]; then
  PROF_DIR=${TAG:-ev}/prof_build PMC="FETCH_SIZE WRITE_SIZE SQ_INSTS_VALU,SQ_INSTS_SALU,GRBM_GUI_ACTIVE,SQ_WAVE_CYCLES" bash scripts/gpu_prof.sh || exit $?
  PROF_DIR=${TAG:-ev}/prof_diff BENCH_ARGS="--workload diff" PMC="FETCH_SIZE WRITE_SIZE" bash scripts/gpu_prof.sh || exit $?
fi
if [ $PART = lines ] || [ $PART = all ]; then
  step bench_diff 400 python bench.py --workload diff --steps 10 --warmup 2
  step bench_inc 400 python bench.py --workload incremental --steps 10 --warmup 3
fi
