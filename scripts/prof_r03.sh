#!/bin/bash
# Kernel traces (rocprofv3 --kernel-trace --stats) of tools/r03_paths.py, one run per mode and env setting.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p "$R/gpurun_out/p3"
cd /tmp && export TMPDIR=/tmp
for spec in ${SPECS:-"build:X=1" "ragged:X=1" "mixed:MKV_DIFF_FUSED=1" "mixed:MKV_DIFF_FUSED=0"}; do
  mode=${spec%%:*}; envs=${spec#*:}; tag=${mode}_${envs//[=,\/]/_}
  env ${envs//,/ } timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/p3/$tag" -o run --output-format csv -- python3 "$R/tools/r03_paths.py" $mode > "$R/gpurun_out/p3/$tag.log" 2>&1; rc=$?
  echo "== $tag rc=$rc"; grep -E "ms/step" "$R/gpurun_out/p3/$tag.log"
  [ $rc -eq 0 ] || { tail -20 "$R/gpurun_out/p3/$tag.log"; exit $rc; }
  f=$(find "$R/gpurun_out/p3/$tag" -name "*kernel_stats.csv" | head -1)
  python3 - "$f" <<'PY'
import csv, sys
r = list(csv.DictReader(open(sys.argv[1])))
for x in r[:16]:
    print("  %-70s n=%5s avg_us=%9.1f tot_ms=%8.2f" % (x["Name"][:70], x["Calls"], float(x["AverageNs"]) / 1e3, float(x["TotalDurationNs"]) / 1e6))
PY
done
exit 0
