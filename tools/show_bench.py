"""One-line summary of a bench.py JSON line: python tools/show_bench.py FILE [label]."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
lab = sys.argv[2] if len(sys.argv) > 2 else ""
par = d.get("parity") or {}
match = [v for k, v in par.items() if k.endswith("_match")]
roof = d.get("roofline") or {}
out = {"label": lab, "n_gpus": d.get("n_gpus"), "value": d.get("value"), "mean_value": d.get("mean_value"), "unit": d.get("unit"),
       "median_ms": d.get("median_ms_per_step"), "parity": match, "roofline": (roof.get("kernel"), roof.get("frac")),
       "kernels": {k: v.get("ms_per_step") for k, v in (d.get("kernels") or {}).items()}}
for k in ("seal_mode_value", "sec_per_rwkv_block_8proj"):
    if d.get(k) is not None:
        out[k] = d[k]
if d.get("cpu_baseline"):
    out["cpu"] = d["cpu_baseline"].get("value")
print(json.dumps(out))
