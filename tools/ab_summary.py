"""Summary of interleaved A/B bench lines (scripts/_r06_gpu*.sh logs): the diff and incremental fields."""
import glob
import json
import sys

pat = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/r06g_"
for f in sorted(glob.glob(pat + "*.log")):
    try:
        line = [x for x in open(f).read().splitlines() if x.startswith("{")][-1]
    except IndexError:
        continue
    d = json.loads(line)
    tag = f[len(pat):-4]
    if d.get("metric", "").startswith("Merkle diff"):
        vo, mx = d["diff"]["value_only"], d["diff"]["mixed"]
        print(f"{tag:14s} diff: value {d['value']:.4g}  vo {vo.get('ms', 0):.3f} ms dev {vo.get('device_ms', 0):.3f}  "
              f"mixed {mx.get('ms', 0):.3f} dev {mx.get('device_ms', 0):.3f}")
    elif "incremental" in d:
        inc = d["incremental"]
        rf = d.get("roofline", {})
        print(f"{tag:14s} inc: {d['ms_per_step']:.3f} ms/step  upd {inc['update_device_ms_all_replicas']:.3f}  "
              f"climb {inc['climb_device_ms']:.3f}  walk/step {rf.get('walk', {}).get('ms_per_step', 0):.3f}  "
              f"diff/pair {inc['diff_device_ms_per_pair']:.3f}")
    else:
        print(tag, list(d.keys())[:20])
