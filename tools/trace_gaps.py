"""Summarise a rocprofv3 --kernel-trace CSV: per-step kernel sequence with durations and the idle
gaps between consecutive kernels (python tools/trace_gaps.py gpurun_out/trace/run_kernel_trace.csv)."""
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
names = [r["Kernel_Name"].split("(")[0].replace("void ", "").replace("fhs::", "") for r in rows]
idx = [i for i, n in enumerate(names) if n.startswith("k_bsgs_inner")]
a, b = idx[-2], idx[-1]
prev, gaps = None, 0.0
for i in range(a + 1, min(len(rows), b + 12)):
    s, e = int(rows[i]["Start_Timestamp"]), int(rows[i]["End_Timestamp"])
    g = (s - prev) / 1000 if prev else 0.0
    gaps += max(g, 0)
    print(f"{names[i][:36]:36s} {(e - s) / 1000:9.1f} us  gap {g:7.1f}")
    prev = e
print("total gap us", round(gaps, 1))
