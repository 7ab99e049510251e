"""Diagnostic: bench.ragged_block in a fresh process, then the A/B driver's ragged run, then the block again."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import ab_ragged  # noqa: E402

ctx = bench.Ctx()
for rep in range(2):
    r = bench.ragged_block(ctx, 10_000_000, 1.29)
    print(f"ragged_block: {r['ms_per_step']:.3f} ms/step  leaf {r['leaf_hash_ms']:.3f}  ratio {r['ratio_vs_fixed']:.3f}", flush=True)
    ab_ragged.run("ab", True, 20)
