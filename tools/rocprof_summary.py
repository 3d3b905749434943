"""Steady-state per-kernel times of a bench run from its rocprofv3 kernel trace.

usage: python tools/rocprof_summary.py TRACE_DIR BENCH_JSON OUT_JSON

TRACE_DIR holds rocprofv3 --kernel-trace --output-format csv output (*kernel_trace.csv, one row per
dispatch).  The bench ran W warmup steps, an instrumented pass and K timed steps (BENCH_JSON: the
bench line it printed); every step launches k_bsgs_inner exactly once, so the dispatches are cut into
steps at each k_bsgs_inner and the last K steps -- the timed region -- are summarised: per kernel
family (the bench's names: k_modup = k_modup / k_modup_h, k_moddown = k_special_x + k_moddown[_h], ...)
the mean device time per step and per launch, beside the all-dispatch average rocprofv3 --stats
reports (which also counts the cold warmup launches).  `longest_matvec_kernel` is the family with the
largest steady-state time per step among the kernels bench.py prices with algorithmic bytes; bench.py
reads the newest hash-matched summary to choose its `roofline` kernel.
"""
import csv
import glob
import json
import os
import re
import sys
from pathlib import Path

FAMILY = [  # (regex on the bare kernel name, bench.py family)
    (r"^k_modup", "k_modup"), (r"^k_ks_ip", "k_ks_ip"), (r"^k_bsgs_inner$", "k_bsgs_inner"),
    (r"^k_(special_x|moddown)", "k_moddown"), (r"^k_(ks_intt|centered)", "k_ks_intt"),
    (r"^k_ks_special_intt", "k_ks_special_intt"), (r"^k_giant_sum", "k_giant_sum"),
    (r"^k_giant_final", "k_giant_final"), (r"^k_rescale", "rescale"),
]
PRICED = ("k_modup", "k_ks_ip", "k_bsgs_inner")   # bench.algorithmic_bytes_per_matvec


def bare(name):
    return name.split("(")[0].replace("void ", "").replace("fhs::", "").split("<")[0].strip()


def family(name):
    b = bare(name)
    for rx, fam in FAMILY:
        if re.search(rx, b):
            return fam
    return b


def load(trace_dir):
    files = glob.glob(os.path.join(trace_dir, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no *kernel_trace.csv under {trace_dir}")
    rows = []
    for f in files:
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def summarise(rows, steps):
    cuts = [i for i, (_, _, n) in enumerate(rows) if bare(n) == "k_bsgs_inner"]
    if len(cuts) < steps + 1:
        raise SystemExit(f"only {len(cuts)} k_bsgs_inner dispatches for {steps} timed steps")
    # a step runs its baby-step key switch, then k_bsgs_inner, then its giant steps and the rescale: step k
    # spans from the dispatch after the previous rescale to the first rescale after its k_bsgs_inner
    resc = [i for i, (_, _, n) in enumerate(rows) if family(n) == "rescale"]
    bounds = []
    for c in cuts[-steps:]:
        prev_resc = max([r for r in resc if r < c], default=-1)
        next_resc = min([r for r in resc if r > c], default=len(rows) - 1)
        bounds.append((prev_resc + 1, next_resc))
    fam_t, fam_n, all_t, all_n, spans, busy = {}, {}, {}, {}, [], []
    for lo, hi in bounds:
        spans.append((rows[hi][1] - rows[lo][0]) / 1e6)
        busy.append(sum(e - s for s, e, _ in rows[lo:hi + 1]) / 1e6)
        for s, e, n in rows[lo:hi + 1]:
            f = family(n)
            fam_t[f] = fam_t.get(f, 0.0) + (e - s) / 1e6
            fam_n[f] = fam_n.get(f, 0) + 1
    for s, e, n in rows:
        f = family(n)
        all_t[f] = all_t.get(f, 0.0) + (e - s) / 1e6
        all_n[f] = all_n.get(f, 0) + 1
    kern = {}
    for f in sorted(fam_t, key=lambda k: -fam_t[k]):
        kern[f] = {"ms_per_step": round(fam_t[f] / steps, 4), "launches_per_step": fam_n[f] / steps,
                   "ms_per_launch": round(fam_t[f] / fam_n[f], 4),
                   "all_dispatch_ms_per_launch": round(all_t[f] / all_n[f], 4), "all_dispatches": all_n[f]}
    priced = [f for f in kern if f in PRICED]
    return {"steps_timed": steps, "step_span_ms_median": round(sorted(spans)[len(spans) // 2], 4),
            "step_kernel_busy_ms_median": round(sorted(busy)[len(busy) // 2], 4), "kernels": kern,
            "longest_matvec_kernel": max(priced, key=lambda f: kern[f]["ms_per_step"]) if priced else None}


def main():
    trace_dir, bench_json, out = sys.argv[1], sys.argv[2], sys.argv[3]
    b = json.loads(open(bench_json).read().strip().splitlines()[-1])
    res = summarise(load(trace_dir), int(b["steps"]))
    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    from bench import kernel_source_hash
    sus = b.get("sustained") or None
    res.update({"kernel_source_sha256_16": kernel_source_hash(), "config": b.get("config", {}).get("workload"),
                "bench_value_under_profiler": b.get("value"), "bench_kernels_events": b.get("kernels"),
                "state": (f"warm: the last {res['steps_timed']} steps of the bench's {sus.get('seconds')} s sustained "
                          "run (round 6: the same state as the line's sustained figure)") if sus else
                         "the bench's K timed steps",
                "sustained_value_under_profiler": sus.get("value") if sus else None,
                "sustained_clocks_end": sus.get("clocks_end") if sus else None,
                "source": "rocprofv3 --kernel-trace (per dispatch), last `steps` BSGS steps of the bench run"})
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v["ms_per_step"] for k, v in res["kernels"].items()}), res["longest_matvec_kernel"])


if __name__ == "__main__":
    main()
