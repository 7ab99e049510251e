#!/bin/bash
# Copy stream (st3) at the lowest priority: its own hardware-queue pool. configs[4] host timeline, A/B of
# the incremental step (cur / idle-only / HEAD), ragged + fixed leaf-stage A/B (the ragged key copy
# runs on st3), kernel trace of the incremental step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 240 python tools/inc_trace.py > gpurun_out/inc_trace.log 2>&1 || { tail -20 gpurun_out/inc_trace.log; exit 1; }
tail -6 gpurun_out/inc_trace.log
AB_ROUNDS=2 AB_COMBOS="base MKV_LIB_PATH=abl/idle/lib/libmerklekv_hip.so MKV_LIB_PATH=abl/head/lib/libmerklekv_hip.so" bash scripts/ab_inc.sh || exit 1
REPS=2 LIBS="cur= idle=abl/idle/lib/libmerklekv_hip.so" bash scripts/gpu_ab_ragged.sh || exit 1
PROF_DIR=prof_r04t BENCH_ARGS="--workload incremental" bash scripts/gpu_prof.sh > gpurun_out/r04t_prof.log 2>&1 || { tail -20 gpurun_out/r04t_prof.log; exit 1; }
python3 scripts/timeline.py 4 k_locate_multi gpurun_out/prof_r04t/trace | awk 'NR<=4 || /copy_to_host|zero_many|span/'
