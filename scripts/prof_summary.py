#!/usr/bin/env python3
"""Summarise a scripts/gpu_prof.sh run (gpurun_out/prof) into profiles/:
  <tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (copied)
  <tag>_pmc.json           per-kernel averages of every PMC counter collected + derived metrics
  pmc_leaf_hash.json       HBM bytes per leaf-hash launch (k_leaf_dma / k_leaf_persist / k_leaf_hash) (FETCH_SIZE x 2 + WRITE_SIZE, gfx950 correction)
  pmc_diff_merge.json      HBM bytes per merge-join diff (sum over its kernels), when k_diff_pass1 ran
Usage: python scripts/prof_summary.py <tag> [n_records] [prof_dir under gpurun_out/]
"""
import collections
import csv
import json
import os
import re
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, "gpurun_out", "prof")
# the kernels of one merge-join diff (k_diff.hip launch_diff_merge); key gathers excluded (output side)
MERGE_KERNELS = ("k_diff_partition", "k_diff_pass1", "k_diff_pass2")  # round 4: verify folded into pass 2
OUT = os.path.join(ROOT, "profiles")


# FETCH_SIZE corrections (calibrated by scripts/pmc_calib.hip, profiles/pmc_incremental.json
# "calibration"): a 16-B/lane streaming read is counted at half its bytes (128-B requests tallied as 64 B),
# a random read of <= 64 B is one request counted exactly. Kernels whose reads are random probes:
READ_FACTOR = {"k_diff_partition": 1.0, "k_dirty_climb": 1.0}


def kname(s):
    m = re.search(r"(k_[a-z0-9_]+)", s)
    return m.group(1) if m else s.split("(")[0][:40]


def main():
    global PROF
    tag = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 10_000_000
    if len(sys.argv) > 3:
        PROF = os.path.join(ROOT, "gpurun_out", sys.argv[3])
    os.makedirs(OUT, exist_ok=True)
    stats = os.path.join(PROF, "trace", "run_kernel_stats.csv")
    shutil.copy(stats, os.path.join(OUT, f"{tag}_kernel_stats.csv"))
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in sorted(os.listdir(PROF)):
        f = os.path.join(PROF, d, "run_counter_collection.csv")
        if d.startswith("pmc") and os.path.exists(f):
            for r in csv.DictReader(open(f)):
                dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                agg[kname(r["Kernel_Name"])][r["Counter_Name"]].append((float(r["Counter_Value"]), dur))
    summary = {}
    for k, d in agg.items():
        e = {c: sum(v for v, _ in vals) / len(vals) for c, vals in d.items()}
        for c, vals in d.items():  # launch duration of the pass that collected c (passes differ)
            e[c + "@dur_us"] = sum(t for _, t in vals) / len(vals) / 1e3
        e["avg_duration_us"] = sum(t for vals in d.values() for _, t in vals) / sum(len(v) for v in d.values()) / 1e3
        if "FETCH_SIZE" in e and "WRITE_SIZE" in e:
            e["hbm_bytes_corrected"] = (READ_FACTOR.get(k, 2.0) * e["FETCH_SIZE"] + e["WRITE_SIZE"]) * 1024
        if "GRBM_GUI_ACTIVE" in e:
            gdur = e["GRBM_GUI_ACTIVE@dur_us"]
            e["eff_clock_ghz"] = e["GRBM_GUI_ACTIVE"] / 8 / (gdur * 1e-6) / 1e9
            if "SQ_INSTS_VALU" in e:
                # VALU issue capacity: 256 CUs x 4 SIMDs, one wave64 instruction per 2 cycles per SIMD
                e["valu_busy_frac"] = e["SQ_INSTS_VALU"] * 2 / 1024 / (e["GRBM_GUI_ACTIVE"] / 8)
        if "SQ_WAIT_INST_ANY" in e and "SQ_WAVE_CYCLES" in e:
            e["issue_stall_frac"] = e["SQ_WAIT_INST_ANY"] / e["SQ_WAVE_CYCLES"]
        summary[k] = e
    json.dump(summary, open(os.path.join(OUT, f"{tag}_pmc.json"), "w"), indent=1, sort_keys=True)
    lk = next((k for k in ("k_leaf_direct", "k_leaf_dma", "k_leaf_persist", "k_leaf_hash") if k in summary), None)
    lh = summary.get(lk) if lk else None
    diff_run = "k_diff_pass1" in summary  # the diff workload also builds trees: keep the build's leaf figure
    if lh and "hbm_bytes_corrected" in lh and not diff_run:
        rec = {"n": n, "hbm_bytes_per_launch": lh["hbm_bytes_corrected"], "source": f"{tag}_pmc.json",
               "kernel": lk,
               "algorithmic_bytes_per_launch": 172 * n,
               "note": "FETCH_SIZE x2 (gfx950 wide-read under-count) + WRITE_SIZE, KB->bytes; VALU counters per "
                       "launch with the duration of the pass that collected GRBM_GUI_ACTIVE"}
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "GRBM_GUI_ACTIVE", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES"):
            if c in lh:
                rec[c] = lh[c]
        if "GRBM_GUI_ACTIVE" in lh:
            rec["avg_duration_us"] = lh["GRBM_GUI_ACTIVE@dur_us"]
        json.dump(rec, open(os.path.join(OUT, "pmc_leaf_hash.json"), "w"), indent=1)
    if all(k in summary and "hbm_bytes_corrected" in summary[k] for k in MERGE_KERNELS):
        per = {k: summary[k]["hbm_bytes_corrected"] for k in MERGE_KERNELS}
        json.dump({"union_keys": n, "hbm_bytes_per_diff": sum(per.values()), "per_kernel": per,
                   "source": f"{tag}_pmc.json", "algorithmic_bytes_per_diff": 80 * n,
                   "note": "FETCH_SIZE x2 for the streaming passes (gfx950 wide-read under-count), x1 for the "
                           "partition's random probes (calibration: scripts/pmc_calib.hip) + WRITE_SIZE, KB->bytes, "
                           "summed over the merge-join kernels of one diff"},
                  open(os.path.join(OUT, "pmc_diff_merge.json"), "w"), indent=1)
    for k in sorted(summary, key=lambda k: -summary[k].get("avg_duration_us", 0))[:8]:
        e = summary[k]
        print(f"{k:24s} {e['avg_duration_us']:9.1f} us  valu_busy={e.get('valu_busy_frac', 0):.2f} "
              f"stall={e.get('issue_stall_frac', 0):.2f} clk={e.get('eff_clock_ghz', 0):.2f} "
              f"hbm={e.get('hbm_bytes_corrected', 0) / 1e6:.0f} MB")


if __name__ == "__main__":
    main()
