#!/bin/bash
# Round 4, first box: lane-refill ragged kernel parity + the default driver line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_ragged_gpu.py tests/test_parity_gpu.py > gpurun_out/r04a_pytest.log 2>&1 || { tail -30 gpurun_out/r04a_pytest.log; exit 1; }
tail -3 gpurun_out/r04a_pytest.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r04a_bench.json 2> gpurun_out/r04a_bench.err || { tail -30 gpurun_out/r04a_bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r04a_bench.json").read().strip().splitlines()[-1])
print("value", d["value"], "ms", d["ms_per_step"])
r = d.get("ragged_10m") or {}
print("ragged", {k: r.get(k) for k in ("ms_per_step", "leaf_hash_ms", "compressions_per_s", "ratio_vs_fixed")})
print("stages", d.get("stage_ms_per_step"))
PY
