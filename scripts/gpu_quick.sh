#!/bin/bash
# Targeted GPU run: selected tests (PYTEST_K) then an optional bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "$PYTEST_K" ]; then
  timeout -k 10 600 python -m pytest tests -q -m gpu --timeout=300 -p no:cacheprovider -k "$PYTEST_K" > gpurun_out/pytest_q.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_q.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || [ $rc -eq 5 ] || exit $rc
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 600 python bench.py $BENCH > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
  echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err
fi
