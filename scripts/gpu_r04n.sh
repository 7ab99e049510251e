#!/bin/bash
# Round-4 evidence, part 1 (EVID=1): the full -m gpu suite, smoke and the default driver line; part 2
# (EVID=2): build / diff kernel traces + PMC passes (scripts/gpu_prof.sh) and the diff / incremental lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ev
step() { local tag=$1 lim=$2; shift 2; echo "== $tag"; timeout -k 10 $lim "$@" > gpurun_out/ev/$tag.log 2>&1; local rc=$?
  echo "$tag rc=$rc"; tail -${TAILN:-3} gpurun_out/ev/$tag.log; [ $rc -eq 0 ] || exit $rc; }
if [ "${EVID:-1}" = 1 ]; then
  step pytest_gpu 1000 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
  step bench 600 python bench.py
else
  PROF_DIR=prof_build PMC="FETCH_SIZE WRITE_SIZE SQ_INSTS_VALU,SQ_INSTS_SALU,GRBM_GUI_ACTIVE,SQ_WAVE_CYCLES" bash scripts/gpu_prof.sh || exit $?
  PROF_DIR=prof_diff BENCH_ARGS="--workload diff" PMC="FETCH_SIZE WRITE_SIZE" bash scripts/gpu_prof.sh || exit $?
  step bench_diff 400 python bench.py --workload diff --steps 10 --warmup 2
  step bench_inc 400 python bench.py --workload incremental --steps 10 --warmup 3
fi
