"""Clock and MFMA-busy fraction of the conv classes in the network.

Input: the output dir of tools/conv_clock.sh.
  cb_<C>_b<B>.ik.log / cb_<C>_b<B>/ : isolated launches of the SDP_TIMING conv build (conv_bench_T): its
      in-kernel clock (s_memtime / s_memrealtime, per workgroup, averaged) and the GRBM_GUI_ACTIVE of
      the same command -> how far GRBM_GUI_ACTIVE / 8 / dispatch wall reads above the in-kernel clock
      at this dispatch length (MI355X_MICROARCH.md 'DVFS give-back': high below ~0.3 ms);
  g_v<V>/, m_v<V>/ : `bench.py --split 1 --views V` under --pmc: per class the dispatch wall, GRBM clock,
      SQ_VALU_MFMA_BUSY_CYCLES (cycles summed over SIMDs; 16 per v_mfma_f32_16x16x32_bf16, checked below).
Per class (the bench's 4-view launch):
  clock_GHz     = network GRBM clock x (in-kernel / GRBM) of the isolated launch of the same shape and batch
  mfma_busy     = SQ_VALU_MFMA_BUSY_CYCLES / (clock x wall x 1024 SIMDs)
  frac_at_clock = achieved TFLOP/s / (833.3 x clock / 2.4): the roofline at the clock the chip held
Writes <out>/<round>_conv_clock.json keyed by the conv source hash (bench.py reads it from profiles/).
"""
import csv
import glob
import json
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "simultaneous-diffusion-for-pointclouds_amd"))

# label, kernel-name substring, threads per view along x (grid x), grid y (Cout / 128), FLOP per view,
# MFMA passes, conv_bench C.  Both classes run conv_launch_nj2's 4-wave 128-Cout workgroups (NJ = 2):
# the 256-Cout layers as two per tile (grid y = 2)
NJ2 = "conv_mfma_kernel<1, 1, 16, 3, false, false, true, 16, 4, false, 2, false>"   # (..., NJ, IO16)
CLASSES = [
    ("conv3x3 256->256 @32x512 d1", NJ2, 256 * 256, 1, 2 * 256 * 256 * 9 * 32 * 512, 3, 256),
    ("conv3x3 128->128 @64x1024 d1", NJ2, 512 * 256, 1, 2 * 128 * 128 * 9 * 64 * 1024, 3, 128),
]


def load(d):
    """dispatch id -> {name, grid, ns, counters} over every csv under d"""
    disp = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            disp[r["Dispatch_Id"]] = {"name": r["Kernel_Name"], "grid": int(r["Grid_Size_X"]),
                                      "gy": int(r.get("Grid_Size_Y", 1) or 1),
                                      "ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), "c": {}}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            e = disp.setdefault(r["Dispatch_Id"], {"name": r["Kernel_Name"], "grid": int(r["Grid_Size"]), "gy": 1, "ns": 0,
                                                   "c": {}})
            e["c"][r["Counter_Name"]] = e["c"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return disp


def select(disp, sub, grid, gy, skip=0):
    sel = [disp[k] for k in sorted(disp, key=int) if sub in disp[k]["name"] and disp[k]["grid"] == grid
           and disp[k]["gy"] == gy and disp[k]["ns"] and disp[k]["c"]]
    return sel[skip:]


def avg(sel, f):
    return sum(f(v) for v in sel) / len(sel)


def main():
    out, rnd = sys.argv[1], sys.argv[2]
    from sdp import _build
    res = {"conv_source_hash": _build.conv_source_hash(), "calibration": [], "classes": [],
           "how": __doc__.split("Writes")[0].strip()}
    # 1. GRBM vs in-kernel clock on isolated launches (conv_bench_T dispatches the library's kernel)
    cal = {}
    for label, sub, gpv, gy, flop, npass, C in CLASSES:
        for B in (4, 32):
            tag = f"cb_{C}_b{B}"
            ik = re.search(r"in-kernel clock ([0-9.]+) GHz", open(os.path.join(out, tag + ".ik.log")).read())
            sel = select(load(os.path.join(out, tag)), "conv_mfma_kernel", gpv * B, gy, skip=3)
            if not ik or not sel:
                continue
            ns = avg(sel, lambda v: v["ns"])
            grbm = avg(sel, lambda v: v["c"]["GRBM_GUI_ACTIVE"]) / 8 / ns
            busy = avg(sel, lambda v: v["c"]["SQ_VALU_MFMA_BUSY_CYCLES"])
            n_mfma = npass * flop * B / 16384
            cal[(C, B)] = float(ik.group(1)) / grbm
            res["calibration"].append({"class": label, "batch": B, "wall_us": round(ns / 1e3, 1),
                                       "in_kernel_clock_GHz": float(ik.group(1)), "grbm_clock_GHz": round(grbm, 3),
                                       "in_kernel_over_grbm": round(cal[(C, B)], 4),
                                       "mfma_busy_cycles_per_mfma": round(busy / n_mfma, 3),
                                       "mfma_busy_frac": round(busy / (float(ik.group(1)) * ns * 1024), 4)})
    # 2. the network
    for label, sub, gpv, gy, flop, npass, C in CLASSES:
        row = {"class": label}
        for V in (4, 16):
            g = select(load(os.path.join(out, f"g_v{V}")), sub, gpv * V, gy)
            m = select(load(os.path.join(out, f"m_v{V}")), sub, gpv * V, gy)
            if not g or not m:
                continue
            ns = (avg(g, lambda v: v["ns"]) + avg(m, lambda v: v["ns"])) / 2
            grbm = (avg(g, lambda v: v["c"]["GRBM_GUI_ACTIVE"]) + avg(m, lambda v: v["c"]["GRBM_GUI_ACTIVE"])) / 2 / 8 / ns
            busy = avg(m, lambda v: v["c"]["SQ_VALU_MFMA_BUSY_CYCLES"])
            k = cal.get((C, 4 if V == 4 else 32), 1.0)
            clk = grbm * k
            ach = flop * V / (ns * 1e-9) / 1e12
            peak = 2500.0 / npass * clk / 2.4
            row[f"views{V}"] = {"dispatches": len(g) + len(m), "wall_us": round(ns / 1e3, 2),
                                "grbm_clock_GHz": round(grbm, 3), "clock_GHz": round(clk, 3),
                                "mfma_busy_frac": round(busy / (clk * ns * 1024), 4),
                                "achieved_TFLOPs": round(ach, 1), "peak_at_clock_TFLOPs": round(peak, 1),
                                "frac_at_clock": round(ach / peak, 4), "frac_at_2.4GHz": round(ach / (2500.0 / npass), 4)}
        if "views4" in row:
            for key in ("clock_GHz", "mfma_busy_frac", "frac_at_clock"):
                row[key] = row["views4"][key]
        res["classes"].append(row)
    dst = os.path.join(out, f"{rnd}_conv_clock.json")
    json.dump(res, open(dst, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
