"""In-network clock and MFMA-busy fraction per conv class.

Input: rocprofv3 output dirs of `bench.py --split 1` runs (tools/conv_clock.sh), one counter group
per run, each with --kernel-trace so every dispatch has its start/end timestamps:
  pass g: GRBM_GUI_ACTIVE SQ_BUSY_CYCLES
  pass m: SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
Per dispatch:
  clock_GHz  = GRBM_GUI_ACTIVE / 8 (summed over the 8 XCDs) / dispatch wall   (MI355X_MICROARCH.md
               'DVFS give-back'; reads a little high on dispatches shorter than ~0.3 ms)
  mfma_busy  = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs)
               (the counter sums MFMA-busy cycles over every SIMD; calibrated below against the
               class's known MFMA count: 16 cycles per v_mfma_f32_16x16x32_bf16)
A class is (kernel instantiation, grid): every launch of one shape at --split 1.
Writes profiles/<round>_conv_clock.json keyed by the conv source hash (bench.py reads it).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "simultaneous-diffusion-for-pointclouds_amd"))

# (label, kernel-name substring, grid threads, GFLOP per launch at B=4, MFMA passes per product)
CLASSES = [
    ("conv3x3 256->256 @32x512", "conv_mfma_kernel<1, 1, 16, 3, false, false, true, 16, 4, false>", 512 * 256,
     2 * 256 * 256 * 9 * 32 * 512 * 4, 3),
    ("conv3x3 128->128 @64x1024", "conv_mfma_kernel<1, 1, 16, 3, false, false, true, 16, 2, false>", 2048 * 128,
     2 * 128 * 128 * 9 * 64 * 1024 * 4, 3),
]


def load(d):
    """dispatch id -> {name, grid, ns, counters}"""
    disp = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            disp[r["Dispatch_Id"]] = {"name": r["Kernel_Name"], "grid": int(r["Grid_Size_X"]),
                                      "ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), "c": {}}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Dispatch_Id"]
            if k not in disp:
                disp[k] = {"name": r["Kernel_Name"], "grid": int(r["Grid_Size"]), "ns": None, "c": {}}
            disp[k]["c"][r["Counter_Name"]] = disp[k]["c"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return disp


def main():
    out, rnd = sys.argv[1], sys.argv[2]
    from sdp import _build
    res = {"conv_source_hash": _build.conv_source_hash(), "classes": [],
           "how": "rocprofv3 --kernel-trace --pmc on `bench.py --split 1` (one counter group per run); "
                  "clock = GRBM_GUI_ACTIVE / 8 / dispatch wall; mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / "
                  "(GRBM_GUI_ACTIVE / 8 * 1024 SIMDs)"}
    passes = {p: load(os.path.join(out, p)) for p in ("g", "m") if os.path.isdir(os.path.join(out, p))}
    for label, sub, grid, flop, npass in CLASSES:
        row = {"class": label, "flops_per_launch": flop}
        for p, disp in passes.items():
            sel = [v for v in disp.values() if sub in v["name"] and v["grid"] == grid and v["ns"] and v["c"]]
            if not sel:
                continue
            ns = sum(v["ns"] for v in sel) / len(sel)
            gui = sum(v["c"].get("GRBM_GUI_ACTIVE", 0.0) for v in sel) / len(sel)
            row[f"pass_{p}"] = {"dispatches": len(sel), "avg_us": round(ns / 1e3, 2),
                                "counters": {c: sum(v["c"].get(c, 0.0) for v in sel) / len(sel)
                                             for c in sel[0]["c"]}}
            if gui:
                clk = gui / 8 / ns                     # cycles per ns = GHz
                row[f"pass_{p}"]["clock_GHz"] = round(clk, 3)
            if "SQ_VALU_MFMA_BUSY_CYCLES" in sel[0]["c"] and gui:
                busy = sum(v["c"]["SQ_VALU_MFMA_BUSY_CYCLES"] for v in sel) / len(sel)
                n_mfma = npass * flop / 16384           # v_mfma_f32_16x16x32_bf16: 16384 FLOP each
                row[f"pass_{p}"]["mfma_busy_frac"] = round(busy / (gui / 8 * 1024), 4)
                row[f"pass_{p}"]["busy_cycles_per_mfma"] = round(busy / n_mfma, 3)
        clocks = [row[k]["clock_GHz"] for k in row if k.startswith("pass_") and "clock_GHz" in row[k]]
        if clocks:
            row["clock_GHz"] = round(sum(clocks) / len(clocks), 3)
            us = [row[k]["avg_us"] for k in row if k.startswith("pass_")]
            ach = flop / (sum(us) / len(us) * 1e-6) / 1e12
            peak_at_clk = 2500.0 / npass * row["clock_GHz"] / 2.4
            row["achieved_TFLOPs"] = round(ach, 1)
            row["peak_at_clock_TFLOPs"] = round(peak_at_clk, 1)
            row["frac_at_clock"] = round(ach / peak_at_clk, 4)
        for k in list(row):
            if k.startswith("pass_") and "mfma_busy_frac" in row[k]:
                row["mfma_busy_frac"] = row[k]["mfma_busy_frac"]
        res["classes"].append(row)
    dst = os.path.join(out, f"{rnd}_conv_clock.json")
    json.dump(res, open(dst, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
