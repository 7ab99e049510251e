#!/bin/bash
# First run after the lost box: smoke, then the parity subsets that cover this round's new code (ragged
# hand-off / edge kernel / key copy in the first histogram pass, fused diff partition, sharded C ABI).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04h_smoke.log 2>&1 \
  || { tail -30 gpurun_out/r04h_smoke.log; exit 1; }
tail -1 gpurun_out/r04h_smoke.log
timeout -k 10 900 $PYT tests/test_ragged_gpu.py tests/test_parity_gpu.py > gpurun_out/r04h_t1.log 2>&1 \
  || { tail -40 gpurun_out/r04h_t1.log; exit 1; }
tail -1 gpurun_out/r04h_t1.log
timeout -k 10 180 tests/cpp/test_sharded > gpurun_out/r04h_cpp_sharded.log 2>&1 \
  || { tail -30 gpurun_out/r04h_cpp_sharded.log; exit 1; }
tail -3 gpurun_out/r04h_cpp_sharded.log
timeout -k 10 900 $PYT tests/test_shard_gpu.py tests/test_cpp_ports_gpu.py tests/test_update_gpu.py > gpurun_out/r04h_t2.log 2>&1 \
  || { tail -40 gpurun_out/r04h_t2.log; exit 1; }
tail -1 gpurun_out/r04h_t2.log
