"""A/B driver for configs[4] (diagnostic): bench.configs4_measure at 125M keys, 7 x 125K updates; prints
ms/step and the device split (update, climb, walk) for the library MKV_LIB_PATH points at."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

ctx = bench.Ctx()
o = bench.configs4_measure(ctx, 125_000_000, 125_000, 8, steps=int(sys.argv[1]) if len(sys.argv) > 1 else 10, warmup=3)
r, inc = o["roofline"], o["incremental"]
print(f"configs4: step {o['ms_per_step']:.4f} ms  update {inc['update_device_ms_all_replicas']:.4f}  "
      f"climb {inc['climb_device_ms']:.4f}  walk {r['walk']['ms_per_step']:.4f}  "
      f"diff/pair {inc['diff_device_ms_per_pair']:.4f}  ok {inc['diff_sizes_match_unique_updates']}  "
      f"roots {[x[:12] for x in inc['variant_roots']]}", flush=True)
