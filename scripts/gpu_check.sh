#!/bin/bash
# One GPU session: smoke -> gpu tests -> short bench -> rocprofv3 kernel stats. Stops on any fault/timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
ok $rc || exit $rc
timeout -k 10 900 python -m pytest tests -q -m gpu --timeout=300 -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu.log
ok $rc || exit $rc
timeout -k 10 600 python bench.py --steps ${BENCH_STEPS:-10} --warmup 2 ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err
[ $rc -eq 0 ] || exit $rc
if [ -n "$PROFILE" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1; rc=$?
  echo "rocprof rc=$rc"; tail -3 "$GRAFT_REPO_ROOT/gpurun_out/prof.log"
fi
exit 0
