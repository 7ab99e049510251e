#!/bin/bash
# k_leaf_multi fixed-shape register path (plain SHA form for large batches): update/parity tests, A/B of
# the configs[4] incremental step against the HEAD library, kernel trace of the new one.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_update_gpu.py \
  > gpurun_out/r04r_t1.log 2>&1 || { tail -30 gpurun_out/r04r_t1.log; exit 1; }
tail -1 gpurun_out/r04r_t1.log
AB_ROUNDS=3 AB_COMBOS="base MKV_LIB_PATH=abl/head/lib/libmerklekv_hip.so" bash scripts/ab_inc.sh || exit 1
PROF_DIR=prof_r04r BENCH_ARGS="--workload incremental" bash scripts/gpu_prof.sh > gpurun_out/r04r_prof.log 2>&1 || { tail -20 gpurun_out/r04r_prof.log; exit 1; }
f=$(find gpurun_out/prof_r04r/trace -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
r = list(csv.DictReader(open(sys.argv[1])))
for x in r[:18]:
    print("  %-60s n=%5s avg_us=%9.1f tot_ms=%8.2f" % (x["Name"][:60], x["Calls"], float(x["AverageNs"]) / 1e3, float(x["TotalDurationNs"]) / 1e6))
PY
