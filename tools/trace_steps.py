"""Kernel timeline of the last calls in a rocprofv3 kernel trace (diagnostic), one block per call starting at
a marker kernel. Usage: python tools/trace_steps.py <trace_dir> [marker=k_topdown_top] [calls=2]"""
import csv
import os
import re
import sys

tdir = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "k_topdown_top"
calls = int(sys.argv[3]) if len(sys.argv) > 3 else 2
rows = list(csv.DictReader(open(os.path.join(tdir, "run_kernel_trace.csv"))))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))


def name(r):
    m = re.search(r"(k_[a-z0-9_]+)", r["Kernel_Name"])
    return m.group(1) if m else r["Kernel_Name"][:30]


st = [i for i, r in enumerate(rows) if name(r).startswith(marker)]
for s in st[-calls - 1:-1]:
    t0 = int(rows[s]["Start_Timestamp"])
    j = s
    while j < len(rows):
        r = rows[j]
        a, b = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
        print(f"  q{r['Queue_Id']:>2} {name(r):26s} {a:8.1f} -> {b:8.1f} ({b - a:6.1f}) grid {r['Grid_Size_X']}")
        j += 1
        if j < len(rows) and name(rows[j]).startswith(marker):
            break
    print()
