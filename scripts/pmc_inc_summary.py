#!/usr/bin/env python3
"""Summarise scripts/pmc_incremental.sh: per-step HBM bytes of the climb and of the walk (configs[4]) with
the calibration factors of scripts/pmc_calib.hip. Usage: pmc_inc_summary.py <gpurun_out/pmc_inc>"""
import csv
import glob
import json
import re
import sys

d = sys.argv[1]


def dispatches(sub):
    f = glob.glob(f"{d}/{sub}/**/*counter_collection.csv", recursive=True)[0]
    rows = {}
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_[a-z0-9_]+|rd32|rd64|wr32|rdstream)", r["Kernel_Name"])
        name = m.group(1) if m else r["Kernel_Name"][:40]
        k = int(r["Dispatch_Id"])
        rows.setdefault(k, [name, 0.0])[1] += float(r["Counter_Value"])
    return [rows[k] for k in sorted(rows)]


calib_bytes = json.loads([l for l in open(f"{d}/calib_FETCH_SIZE.log") if l.startswith("{")][-1])
cal = {}
for c, unit in (("FETCH_SIZE", 1024.0), ("WRITE_SIZE", 1024.0)):  # both counters report KiB
    per = {}
    for name, v in dispatches(f"calib_{c}"):
        per.setdefault(name, []).append(v * unit)
    cal[c] = {k: sum(v) / len(v) for k, v in per.items()}
out = {"calibration": {
    "rd32_fetch_over_bytes": cal["FETCH_SIZE"]["rd32"] / calib_bytes["rd32_bytes"],
    "rd64_fetch_over_bytes": cal["FETCH_SIZE"]["rd64"] / calib_bytes["rd64_bytes"],
    "rdstream_fetch_over_bytes": cal["FETCH_SIZE"]["rdstream"] / calib_bytes["rdstream_bytes"],
    "wr32_write_over_bytes": cal["WRITE_SIZE"]["wr32"] / calib_bytes["wr32_bytes"]}}
# Per-kernel read corrections from the calibration: the climb's reads are 32-B digests at random slots,
# each one 64-B request that FETCH_SIZE counts exactly (rd32: FETCH = 2 x the requested bytes = the 64 B
# moved), so k_dirty_climb's FETCH_SIZE is taken as is; the reductions and the walk's jumps read
# contiguous runs of digests (wide coalesced requests, counted at half: rdstream), so theirs is doubled.
# Writes: WRITE_SIZE as is (wr32: 1.06 x the bytes).
READ_FACTOR = {"k_dirty_climb": 1.0}
tot = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    climb = walk = 0.0
    steps = 0
    launches = {"climb": 0, "walk": 0}
    per = {}
    in_climb = False
    for name, v in dispatches(f"inc_{c}"):
        b = v * 1024.0
        if c == "FETCH_SIZE":
            b *= READ_FACTOR.get(name, 2.0)
        if name == "k_dirty_climb":
            steps += 1
            in_climb = True
        elif not (in_climb and name.startswith("k_reduce_")):
            in_climb = False
        if in_climb:
            climb += b
            launches["climb"] += 1
            per[name] = per.get(name, 0.0) + b
        elif name.startswith("k_topdown_") or name == "k_td_gate":
            walk += b
            launches["walk"] += 1
    tot[c] = {"climb": climb / steps, "walk": walk / steps, "steps": steps, "per": {k: v / steps for k, v in per.items()},
              "climb_launches_per_step": launches["climb"] / steps, "walk_launches_per_step": launches["walk"] / steps}
out.update({
    "tree_keys": 125_000_000, "replicas": 8, "batch": 125_000,
    "climb_read_bytes_per_step": tot["FETCH_SIZE"]["climb"], "climb_write_bytes_per_step": tot["WRITE_SIZE"]["climb"],
    "climb_read_by_kernel": tot["FETCH_SIZE"]["per"], "climb_write_by_kernel": tot["WRITE_SIZE"]["per"],
    "walk_read_bytes_per_step": tot["FETCH_SIZE"]["walk"], "walk_write_bytes_per_step": tot["WRITE_SIZE"]["walk"],
    "climb_hbm_bytes_per_step": tot["FETCH_SIZE"]["climb"] + tot["WRITE_SIZE"]["climb"],
    "walk_hbm_bytes_per_step": tot["FETCH_SIZE"]["walk"] + tot["WRITE_SIZE"]["walk"],
    "climb_launches_per_step": tot["FETCH_SIZE"]["climb_launches_per_step"],
    "walk_launches_per_step": tot["FETCH_SIZE"]["walk_launches_per_step"],
    "steps_counted": tot["FETCH_SIZE"]["steps"],
    "source": "scripts/pmc_incremental.sh (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes; calibration "
              "scripts/pmc_calib.hip)",
    "note": "reads: FETCH_SIZE x1 for k_dirty_climb (random 32-B digest reads = one 64-B request each, counted "
            "exactly: calibration rd32/rd64) and x2 for the reductions and the walk (contiguous digest runs: wide "
            "requests counted at half, calibration rdstream); writes: WRITE_SIZE"})
print(json.dumps(out, indent=1))
