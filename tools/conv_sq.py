"""Reduce tools/conv_sq.sh output: per (knock-out build, shape) the conv dispatch's SQ counters
averaged over dispatches, as fractions of the wave cycles (SQ_WAVE_CYCLES / SQ_WAIT_* /
SQ_ACTIVE_INST_* count quad-cycles; SQ_VALU_MFMA_BUSY_CYCLES counts cycles summed over SIMDs)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d):
    disp = defaultdict(dict)
    ns = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "conv_mfma_kernel" in r["Kernel_Name"]:
                ns[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "conv_mfma_kernel" in r["Kernel_Name"]:
                k = r["Dispatch_Id"]
                disp[k][r["Counter_Name"]] = disp[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    keys = [k for k in disp if k in ns][3:]          # drop the 3 warm-up launches
    avg = {c: sum(disp[k][c] for k in keys) / len(keys) for c in disp[keys[0]]}
    avg["wall_us"] = sum(ns[k] for k in keys) / len(keys) / 1e3
    return avg


def main():
    out = sys.argv[1]
    res = {}
    for tag in sorted(os.listdir(out)):
        p = os.path.join(out, tag)
        if not os.path.isdir(p):
            continue
        a = {}
        for g in ("g1", "g2"):
            if os.path.isdir(os.path.join(p, g)):
                a.update(load(os.path.join(p, g)))
        clk = a["GRBM_GUI_ACTIVE"] / 8 / (a["wall_us"] * 1e3)
        wc = a.get("SQ_WAVE_CYCLES", 0.0)
        r = {"wall_us": round(a["wall_us"], 1), "clock_GHz": round(clk, 3)}
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_LDS"):
                r[c.replace("SQ_", "") + "_frac"] = round(a[c] / wc, 4)
        if "SQ_VALU_MFMA_BUSY_CYCLES" in a:
            r["mfma_busy_frac"] = round(a["SQ_VALU_MFMA_BUSY_CYCLES"] / (a["GRBM_GUI_ACTIVE"] / 8 * 1024), 4)
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_LDS_BANK_CONFLICT",
                  "SQ_LDS_IDX_ACTIVE", "SQ_WAIT_INST_LDS", "SQ_VALU_MFMA_COEXEC_CYCLES"):
            if c in a:
                r[c] = a[c]
        res[tag] = r
    json.dump(res, open(os.path.join(out, "summary.json"), "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
