#!/bin/bash
# Pass 1 writes / pass 2 reads the packed lane words only for tiles with divergent outputs: diff tests,
# then the merge-join A/B against HEAD (h4).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_parity_gpu.py tests/test_scale_gpu.py \
  > gpurun_out/r04ac_t1.log 2>&1 || { tail -30 gpurun_out/r04ac_t1.log; exit 1; }
tail -1 gpurun_out/r04ac_t1.log
bash scripts/gpu_r04ab.sh
