"""Per-step HBM traffic per kernel from rocprofv3 --pmc runs (MI355X_MICROARCH.md "HBM"):
FETCH_SIZE is in KiB and reports half the bytes of wide streaming reads on gfx950 (x2 here);
WRITE_SIZE is in KiB.  Infinity-Cache hits are counted by these counters, so the figures are an
upper bound on true HBM bytes.

usage: python tools/pmc_traffic.py FETCH_CSV WRITE_CSV STEPS_EXECUTED OUT_JSON
STEPS_EXECUTED = number of identical BSGS steps the profiled command ran (warmup + profile + timed).
"""
import csv
import collections
import json
import sys
from pathlib import Path


def load(path, counter):
    tot = collections.defaultdict(float)
    n = collections.Counter()
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("fhs::", "").split("<")[0]
        tot[k] += float(r["Counter_Value"])
        n[k] += 1
    return tot, n


def main():
    fcsv, wcsv, steps, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    f, fn = load(fcsv, "FETCH_SIZE")
    w, wn = load(wcsv, "WRITE_SIZE")
    res = {}
    for k in sorted(set(f) | set(w)):
        rd = 2 * f.get(k, 0.0) * 1024 / steps
        wr = w.get(k, 0.0) * 1024 / steps
        res[k] = {"read_bytes_per_step": int(rd), "write_bytes_per_step": int(wr),
                  "traffic_bytes_per_step": int(rd + wr), "launches_per_step": fn.get(k, 0) / steps}
    meta = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes)",
            "correction": "FETCH_SIZE x2 (gfx950), KiB -> bytes", "steps_executed": steps}
    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    from bench import kernel_source_hash
    json.dump({"meta": meta, "kernel_source_sha256_16": kernel_source_hash(), "kernels": res}, open(out, "w"),
              indent=1)
    for k, v in res.items():
        print(f"{k:22s} read {v['read_bytes_per_step'] / 1e9:7.3f} GB  write {v['write_bytes_per_step'] / 1e9:7.3f} GB per step")


if __name__ == "__main__":
    main()
