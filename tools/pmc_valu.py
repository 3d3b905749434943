"""Per-kernel VALU issue from a rocprofv3 --pmc pass (SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE):
usage: python tools/pmc_valu.py COUNTER_CSV STEPS_EXECUTED OUT_JSON

valu_busy = SQ_ACTIVE_INST_VALU x 4 / (1024 SIMDs x GRBM_GUI_ACTIVE / 8): SQ_ACTIVE_INST_* count
quad-cycles summed over waves, GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md, PMC units
and DVFS notes) -- the fraction of SIMD cycles that issued a VALU instruction during the dispatch.
"""
import collections
import csv
import json
import sys
from pathlib import Path


def main():
    path, steps, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    disp = collections.defaultdict(dict)
    names = {}
    for r in csv.DictReader(open(path)):
        d = r["Dispatch_Id"]
        disp[d][r["Counter_Name"]] = float(r["Counter_Value"])
        names[d] = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("fhs::", "").split("<")[0]
    agg = collections.defaultdict(lambda: collections.Counter())
    for d, c in disp.items():
        k = names[d]
        agg[k]["launches"] += 1
        for n, v in c.items():
            agg[k][n] += v
    res = {}
    for k, c in sorted(agg.items()):
        cyc = c["GRBM_GUI_ACTIVE"] / 8
        res[k] = {"valu_wave_insts_per_step": c["SQ_INSTS_VALU"] / steps,
                  "valu_busy": round(c["SQ_ACTIVE_INST_VALU"] * 4 / (1024 * cyc), 3) if cyc else None,
                  "launches_per_step": c["launches"] / steps}
        print(f"{k:22s} VALU {res[k]['valu_wave_insts_per_step'] / 1e6:8.1f} M wave-insts/step  busy {res[k]['valu_busy']}")
    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    from bench import kernel_source_hash
    json.dump({"meta": {"source": "rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE",
                        "steps_executed": steps}, "kernel_source_sha256_16": kernel_source_hash(), "kernels": res},
              open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
