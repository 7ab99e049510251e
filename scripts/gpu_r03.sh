#!/bin/bash
# Round-3 GPU session: new tests first (named), full -m gpu suite, the --gpus 2 self-launch rehearsal
# (gloo, both ranks on device 0), then the default bench line. Every GPU step has its own time limit;
# the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() { local tag=$1 lim=$2; shift 2; echo "== $tag"; timeout -k 10 $lim "$@" > gpurun_out/$tag.log 2>&1; local rc=$?
  echo "$tag rc=$rc"; tail -${TAILN:-15} gpurun_out/$tag.log; [ $rc -eq 0 ] || exit $rc; }
if [ -n "$TESTS" ]; then
  step pytest_new 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider $TESTS
fi
if [ -z "$SKIP_SUITE" ]; then
  step pytest_gpu 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider
fi
if [ -z "$SKIP_MR" ]; then
  export MKV_BENCH_SAME_GPU=1 MKV_DIST_BACKEND=gloo
  step bench_gpus2 400 python bench.py --gpus 2 --records ${MR_RECORDS:-1000000} --steps 3 --warmup 1 --no-cpu-baseline --route-records 1000000
  unset MKV_BENCH_SAME_GPU MKV_DIST_BACKEND
fi
if [ -z "$SKIP_BENCH" ]; then
  step bench 600 python bench.py ${BENCH_ARGS}
fi
exit 0
