#!/bin/bash
# Ragged key copy on its own stream + asynchronous batched-diff key lists: parity of the build / update /
# anti-entropy paths, the leaf-stage A/B (sort tile sizes), and the configs[4] incremental line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $PYT tests/test_ragged_gpu.py tests/test_update_gpu.py tests/test_antientropy_gpu.py tests/test_parity_gpu.py \
  > gpurun_out/r04m_t1.log 2>&1 || { tail -40 gpurun_out/r04m_t1.log; exit 1; }
tail -1 gpurun_out/r04m_t1.log
STEPS=10 REPS=2 LIBS="cur= i20=abl/ipt20/lib/libmerklekv_hip.so i22=abl/ipt22/lib/libmerklekv_hip.so" bash scripts/gpu_ab_ragged.sh || exit 1
timeout -k 10 600 python -u bench.py --workload incremental --steps 10 --warmup 3 > gpurun_out/r04m_inc.json 2> gpurun_out/r04m_inc.err \
  || { tail -30 gpurun_out/r04m_inc.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r04m_inc.json'));print(d['value'],d['ms_per_step']);print(json.dumps(d['incremental'])[:600])"
