"""Where a kernel's wave cycles go, from rocprofv3 --pmc passes (attribute k_modup_h's
idle issue slots).  usage: python tools/pmc_stall.py OUT_JSON STEPS COUNTER_CSV [COUNTER_CSV ...]

Counters (MI355X_MICROARCH.md, rocprofv3 PMC slots): SQ_WAVE_CYCLES = SQ_WAIT_ANY (wave parked on
s_waitcnt / barrier) + SQ_WAIT_INST_ANY (ready but not issued: dependency / pipe busy; SQ_WAIT_INST_LDS its
LDS-issue part) + SQ_ACTIVE_INST_ANY (issuing), all in quad-cycles summed over waves.  Per kernel the sums
over its dispatches, per step, and the shares of SQ_WAVE_CYCLES; valu_busy = SQ_ACTIVE_INST_VALU x 4 over
the SIMD cycles (1024 SIMDs x GRBM_GUI_ACTIVE / 8, as tools/pmc_valu.py); bank-conflict cycles per LDS
instruction; instruction mix per wave-instruction of VALU.
"""
import collections
import csv
import json
import sys
from pathlib import Path


def short(name):
    return name.split("(")[0].replace("void ", "").replace("fhs::", "").split("<")[0]


def main():
    out, steps, paths = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
    agg = collections.defaultdict(collections.Counter)
    launches = collections.defaultdict(set)
    for path in paths:
        for r in csv.DictReader(open(path)):
            k = short(r["Kernel_Name"])
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            launches[k].add((path, r["Dispatch_Id"]))
    res = {}
    for k, c in sorted(agg.items()):
        n = len(launches[k]) / len(paths)
        rec = {"launches_per_step": round(n / steps, 3)}
        rec.update({name: v / steps for name, v in sorted(c.items())})
        wave = c.get("SQ_WAVE_CYCLES")
        if wave:
            for part in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS",
                         "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_MISC"):
                if part in c:
                    rec["share_" + part[3:].lower()] = round(c[part] / wave, 4)
        if c.get("GRBM_GUI_ACTIVE") and "SQ_ACTIVE_INST_VALU" in c:
            # GRBM_GUI_ACTIVE appears in several passes: average it over the passes that carry it
            passes = sum(1 for p in paths if any(True for r in csv.DictReader(open(p))
                                                 if r["Counter_Name"] == "GRBM_GUI_ACTIVE" and short(r["Kernel_Name"]) == k))
            cyc = c["GRBM_GUI_ACTIVE"] / max(passes, 1) / 8
            rec["valu_busy"] = round(c["SQ_ACTIVE_INST_VALU"] * 4 / (1024 * cyc), 3)
        if c.get("SQ_INSTS_LDS"):
            if "SQ_LDS_BANK_CONFLICT" in c:
                rec["bank_conflict_cycles_per_lds_inst"] = round(c["SQ_LDS_BANK_CONFLICT"] / c["SQ_INSTS_LDS"], 3)
        if c.get("SQ_INSTS_VALU"):
            for m in ("SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_VMEM", "SQ_INSTS_BRANCH"):
                if m in c:
                    rec[m[9:].lower() + "_per_valu"] = round(c[m] / c["SQ_INSTS_VALU"], 4)
        res[k] = rec
        shares = {x: rec[x] for x in rec if x.startswith("share_")}
        print(f"{k:22s} {shares} valu_busy={rec.get('valu_busy')}")
    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    from bench import kernel_source_hash
    json.dump({"meta": {"source": "rocprofv3 --pmc, one pass per counter set: " + ", ".join(Path(p).parent.name for p in paths),
                        "steps_executed": steps}, "kernel_source_sha256_16": kernel_source_hash(), "kernels": res},
              open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
