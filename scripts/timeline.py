#!/usr/bin/env python3
"""Print the kernel timeline of one step from a rocprofv3 kernel trace (gpurun_out/prof/trace).
A step is delimited by dispatches of the marker kernel(s) (default: the leaf hash).
Usage: python scripts/timeline.py [step] [marker,marker2] [trace_dir]"""
import csv
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tdir = sys.argv[3] if len(sys.argv) > 3 else os.path.join(ROOT, "gpurun_out", "prof", "trace")
rows = list(csv.DictReader(open(os.path.join(tdir, "run_kernel_trace.csv"))))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))


def name(r):
    m = re.search(r"(k_[a-z0-9_]+)", r["Kernel_Name"])
    return m.group(1) if m else r["Kernel_Name"][:28]


markers = sys.argv[2].split(",") if len(sys.argv) > 2 else ["k_leaf_hash", "k_leaf_persist"]
starts = [i for i, r in enumerate(rows) if name(r) in markers]
step = int(sys.argv[1]) if len(sys.argv) > 1 else 3
i0 = starts[step]
i1 = starts[step + 1] if step + 1 < len(starts) else len(rows)
t0 = int(rows[i0]["Start_Timestamp"])
print(f"step {step}: {i1 - i0} dispatches")
for r in rows[i0:i1]:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print(f"  q{r['Queue_Id']:>2} {name(r):22s} {s / 1e3:9.1f} -> {e / 1e3:9.1f} us  ({(e - s) / 1e3:8.1f})  grid {r['Grid_Size_X']}")
end = max(int(r["End_Timestamp"]) for r in rows[i0:i1]) - t0
print(f"span {end / 1e3:.1f} us")
