"""Average duration per kernel from a rocprofv3 --pmc counter_collection.csv (kernels serialized)."""
import csv
import glob
import re
import sys
from collections import defaultdict

d = sys.argv[1]
tag = sys.argv[2] if len(sys.argv) > 2 else ""
f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
dur = defaultdict(list)
seen = set()
for r in csv.DictReader(open(f)):
    key = (r.get("Dispatch_Id"), r["Kernel_Name"])
    if key in seen:
        continue
    seen.add(key)
    m = re.search(r"(k_[a-z0-9_]+)(<[^>]*>)?", r["Kernel_Name"])
    name = m.group(0) if m else r["Kernel_Name"][:40]
    dur[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(dur.items(), key=lambda x: -sum(x[1])):
    print(f"{tag} {k:40s} n={len(v):4d} avg_us={sum(v) / len(v):8.1f}")
