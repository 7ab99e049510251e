#!/usr/bin/env python3
"""Per-(kernel, grid) averages of every counter in rocprofv3 --pmc counter_collection.csv files, with
derived VALU metrics. Usage: pmc_dispatch.py <dir> [<dir> ...] [--top N]
  lane_ops/us  = SQ_INSTS_VALU x 64 / duration
  valu_frac    = SQ_INSTS_VALU x 64 / (256 CU x 128 lanes x GRBM_GUI_ACTIVE / 8) (issue share of the
                 full-rate 2-cycle wave64 peak at the measured clock)
  active_valu  = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES (quad-cycles both)
"""
import collections
import csv
import glob
import re
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
top = 20
if "--top" in sys.argv:
    top = int(sys.argv[sys.argv.index("--top") + 1])
    args = [a for a in args if a != str(top)]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(dict)
for d in args:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            m = re.search(r"(k_[a-z0-9_]+)(<[^>]*>)?", r["Kernel_Name"])
            name = (m.group(0) if m else r["Kernel_Name"][:40]) + f" g{r['Grid_Size']}"
            key = (f, r["Dispatch_Id"])
            agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur[name][key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
rows = []
for name, cs in agg.items():
    ds = list(dur[name].values())
    avg = {c: sum(v) / len(v) for c, v in cs.items()}
    rows.append((sum(ds), name, len(ds), sum(ds) / len(ds), avg))
rows.sort(reverse=True)
for tot, name, nd, us, avg in rows[:top]:
    extra = ""
    if "SQ_INSTS_VALU" in avg:
        extra += f" valu_inst={avg['SQ_INSTS_VALU']:.4g} lane_ops/us={avg['SQ_INSTS_VALU'] * 64 / us:.4g}"
        if "GRBM_GUI_ACTIVE" in avg:
            extra += f" valu_frac={avg['SQ_INSTS_VALU'] * 64 / (256 * 128 * avg['GRBM_GUI_ACTIVE'] / 8):.3f}"
            extra += f" clk_ghz={avg['GRBM_GUI_ACTIVE'] / 8 / us / 1e3:.2f}"
    if "SQ_ACTIVE_INST_VALU" in avg and "SQ_WAVE_CYCLES" in avg:
        extra += f" active_valu={avg['SQ_ACTIVE_INST_VALU'] / avg['SQ_WAVE_CYCLES']:.3f}"
    other = " ".join(f"{c}={v:.4g}" for c, v in sorted(avg.items()) if c not in ("SQ_INSTS_VALU",))
    print(f"{name[:60]:60s} n={nd:3d} avg_us={us:8.1f}{extra}\n      {other}")
