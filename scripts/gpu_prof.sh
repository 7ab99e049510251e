#!/bin/bash
# rocprofv3 kernel-trace stats of a short bench run, then separate PMC passes (no tracing domains).
# PROF_DIR (default prof) names the output directory under gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
P="$R/gpurun_out/${PROF_DIR:-prof}"
mkdir -p "$P"
BA="${BENCH_ARGS:---no-diff}"  # bench.py arguments (default: build workload, no diff section)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$P/trace" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline $BA > "$P/trace.log" 2>&1; rc=$?
echo "trace rc=$rc"; tail -2 "$P/trace.log"
[ $rc -eq 0 ] || exit $rc
if [ -n "$PMC" ]; then
  i=0
  for set in $PMC; do
    i=$((i+1))
    timeout -k 10 600 rocprofv3 --pmc ${set//,/ } -d "$P/pmc$i" -o run --output-format csv -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline $BA > "$P/pmc$i.log" 2>&1; rc=$?
    echo "pmc$i ($set) rc=$rc"; tail -1 "$P/pmc$i.log"
    [ $rc -eq 0 ] || exit $rc
  done
fi
find "$P" -name "*.csv" | head -20
