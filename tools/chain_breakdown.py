"""Per-kernel GPU time of bench.py's cfg5 chain leg from a rocprofv3 --kernel-trace of the whole line:
python tools/chain_breakdown.py run_kernel_trace.csv bench_line.json out.json

Window: from the chain's first diagonal encode (the first k_ntt_fwd_from_dbl_sp at LOGN 15) to the end of the
trace.  The rocclr copy kernels (the host-side decrypt / correlation checks between blocks, outside the leg's
clock) and k_expand_compact (the first-BSGS parity export after the chain) are listed apart, not in the total.
Launches are bucketed by workgroup count: below 256 (fewer than the chip's CUs: latency-bound) and above."""
import collections
import csv
import json
import sys

OUTSIDE = ("__amd_rocclr_copyBuffer", "__amd_rocclr_copyBufferRectAligned", "__amd_rocclr_fillBufferAligned",
           "k_expand_compact")


def short(name):
    return name.split("(")[0].replace("void ", "").replace("fhs::", "")


def main(trace, line, out):
    tr = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    i0 = next(i for i, r in enumerate(tr) if "k_ntt_fwd_from_dbl_sp<15" in r["Kernel_Name"])
    agg = collections.defaultdict(lambda: {"launches": 0, "ms": 0.0, "small_launches": 0, "small_ms": 0.0})
    apart = collections.defaultdict(float)
    for r in tr[i0:]:
        n = short(r["Kernel_Name"])
        ms = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        if n in OUTSIDE:
            apart[n] += ms
            continue
        wg = (int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))) * \
             (int(r["Grid_Size_Y"]) // max(1, int(r["Workgroup_Size_Y"]))) * \
             (int(r["Grid_Size_Z"]) // max(1, int(r["Workgroup_Size_Z"])))
        a = agg[n]
        a["launches"] += 1
        a["ms"] += ms
        if wg < 256:
            a["small_launches"] += 1
            a["small_ms"] += ms
    busy = sum(a["ms"] for a in agg.values())
    small = sum(a["small_ms"] for a in agg.values())
    d = json.loads([x for x in open(line) if x.startswith("{")][-1]) if line.endswith(".log") else json.load(open(line))
    c = d.get("cfg5_chain") or {}
    res = {
        "source": "rocprofv3 --kernel-trace of one default bench line (tools/chain_breakdown.py)",
        "chain_total_seconds_in_line": c.get("total_seconds"),
        "chain_sec_per_block_in_line": c.get("sec_per_block"),
        "digest_matches_one_rank": (c.get("parity") or {}).get("matches_one_rank"),
        "kernel_busy_ms": round(busy, 1),
        "small_launch_ms": round(small, 1),
        "small_launch_share": round(small / busy, 3) if busy else None,
        "outside_the_leg_clock_ms": {k: round(v, 1) for k, v in apart.items()},
        "kernels": {k: {"launches": v["launches"], "ms": round(v["ms"], 2), "share": round(v["ms"] / busy, 4),
                        "us_per_launch": round(1e3 * v["ms"] / v["launches"], 1),
                        "small_launches": v["small_launches"], "small_ms": round(v["small_ms"], 2)}
                    for k, v in sorted(agg.items(), key=lambda kv: -kv[1]["ms"])},
    }
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "kernels"}))
    for k, v in list(res["kernels"].items())[:12]:
        print(f"{k[:50]:50s} {v['launches']:5d} {v['ms']:8.2f} ms {v['share']:.3f}  small {v['small_ms']:7.2f} ms")


if __name__ == "__main__":
    main(*sys.argv[1:4])
