"""Print the headline numbers of a bench JSON line (A/B helper for scripts/ab_r03.sh)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
out = {"value": d.get("value"), "ms_per_step": d.get("ms_per_step")}
st = d.get("stage_ms_per_step") or {}
out.update({k: round(v, 4) for k, v in st.items()})
for mode, v in (d.get("diff") or {}).items():
    if isinstance(v, dict) and "device_ms" in v:
        out[f"diff_{mode}_ms"] = round(v["ms"], 4)
        out[f"diff_{mode}_dev"] = round(v["device_ms"], 4)
inc = d.get("incremental") or {}
for k in ("update_device_ms_all_replicas", "diff_device_ms_per_pair", "climb_device_ms", "walk_device_ms_per_pair"):
    if k in inc:
        out[k] = inc[k]
rf = d.get("roofline") or {}
out["roofline_frac"] = rf.get("frac")
print(json.dumps(out))
