"""Every A/B kernel variant the library keeps behind an environment knob stays exact: each knob setting
runs tests/ab_variant_check.py in a child process (the library reads its knobs once per process) and
that script checks ragged and fixed-shape roots, leaf digests, mixed and value-only diffs against the C
oracle (/root/reference/src/store/merkle.rs:73-121, :171-196)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

VARIANTS = [
    {"MKV_LEAF_RAGGED": "2"},                      # register-form ragged leaf kernel (k_leaf_rreg)
    {"MKV_LEAF_RAGGED": "2", "MKV_RREG_WGS": "4"},
    {"MKV_LEAF_RAGGED": "0"},                      # round-2 LDS chunk kernel for listed chunks
    {"MKV_RAGGED_WGS": "2"},                       # LDS ragged kernel at 2 workgroups per CU
    {"MKV_DIFF_PART": "1"},                        # in-pass tile splits (k_diff_pass1s)
    {"MKV_DIFF_FUSED": "1"},                       # single-pass merge-join with decoupled look-back
    {"MKV_DIFF_TOPDOWN": "0"},                     # merge-join for equal key sets too
    {"MKV_DIFF_DEFER": "0"},                       # merge-join key checks inline in pass 1
    {"MKV_DIFF_ONEWAIT": "0"},                     # top-down pair diff with the round-2 host waits
    {"MKV_DIFF_DEFER": "0", "MKV_DIFF_TOPDOWN": "0"},
    {"MKV_TOP_SHA": "1"},                          # short-chain SHA form at the reduction top
    {"MKV_TOP_REDUCE": "0"},                       # round-2 per-4-level launches up to the root
]


@pytest.mark.parametrize("env", VARIANTS, ids=lambda e: ",".join(f"{k}={v}" for k, v in e.items()))
def test_ab_variant_exact_vs_oracle(env):
    full = dict(os.environ)
    full.update(env)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "ab_variant_check.py")], env=full,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), (r.stdout[-2000:], r.stderr[-2000:])
