#!/bin/bash
# Measurements of this round's tree: leaf-stage A/B (fixed + ragged builds), the default driver line, and
# kernel traces + timelines of the fixed build, the ragged build and the 100M mixed merge-join diff.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
STEPS=10 LIBS="cur=" REPS=2 bash scripts/gpu_ab_ragged.sh || exit 1
timeout -k 10 900 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r04i_bench.json 2> gpurun_out/r04i_bench.err \
  || { tail -30 gpurun_out/r04i_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r04i_bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['frac']);print(json.dumps(d.get('ragged_10m'))[:600])"
SPECS="build:X=1 ragged:X=1 mixed:X=1" bash scripts/prof_r03.sh || exit 1
python3 scripts/timeline.py 3 k_leaf_direct gpurun_out/p3/build_X_1
python3 scripts/timeline.py 3 k_leaf_direct gpurun_out/p3/ragged_X_1
