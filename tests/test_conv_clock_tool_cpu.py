"""tools/conv_clock.py: the reduction of the in-kernel-clock calibration and the
network PMC passes into profiles/rNN_conv_clock.json, on synthetic rocprofv3 CSVs with known answers."""
import csv
import json
import os
import subprocess
import sys

from conftest import REPO

NJ2 = "conv_mfma_kernel<1, 1, 16, 3, false, false, true, 16, 4, false, 2, false>"   # (..., NJ, IO16)
CLASSES = [("256", 256 * 256, 2 * 256 * 256 * 9 * 32 * 512), ("128", 512 * 256, 2 * 128 * 128 * 9 * 64 * 1024)]


def _write(d, rows):
    """rows: (dispatch id, kernel, grid x, ns, {counter: value})"""
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "run_kernel_trace.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Dispatch_Id", "Kernel_Name", "Grid_Size_X", "Grid_Size_Y", "Start_Timestamp", "End_Timestamp"])
        for i, name, gx, ns, _ in rows:
            w.writerow([i, name, gx, 1, 1000, 1000 + ns])
    with open(os.path.join(d, "run_counter_collection.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Dispatch_Id", "Kernel_Name", "Grid_Size", "Counter_Name", "Counter_Value"])
        for i, name, gx, _, cs in rows:
            for k, v in cs.items():
                w.writerow([i, name, gx, k, v])


def test_clock_and_mfma_busy_reduction(tmp_path):
    out = str(tmp_path)
    clk_ik, clk_grbm, wall = 1.6, 2.0, 200_000   # in-kernel 1.6 GHz, GRBM reads 2.0 over 200 us
    for C, gx, flop in CLASSES:
        for B in (4, 32):
            with open(os.path.join(out, f"cb_{C}_b{B}.ik.log"), "w") as f:
                f.write(f"in-kernel clock {clk_ik} GHz\n")
            n_mfma = 3 * flop * B / 16384
            rows = [(k, NJ2, gx * B, wall, {"GRBM_GUI_ACTIVE": clk_grbm * wall * 8, "SQ_VALU_MFMA_BUSY_CYCLES": 16 * n_mfma})
                    for k in range(6)]
            _write(os.path.join(out, f"cb_{C}_b{B}"), rows)
    busy = 0.5   # network: GRBM 2.0 GHz -> calibrated 1.6; MFMA busy half of the SIMD-cycles
    for V in (4, 16):
        for tag in ("g", "m"):
            rows = []
            for j, (C, gx, flop) in enumerate(CLASSES):
                cs = {"GRBM_GUI_ACTIVE": clk_grbm * wall * 8}
                cs["SQ_BUSY_CYCLES" if tag == "g" else "SQ_VALU_MFMA_BUSY_CYCLES"] = busy * clk_ik * wall * 1024
                rows.append((10 + j, NJ2, gx * V, wall, cs))
            _write(os.path.join(out, f"{tag}_v{V}"), rows)
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "conv_clock.py"), out, "rtest"], capture_output=True,
                       text=True, timeout=120, cwd=REPO)
    assert r.returncode == 0, r.stderr[-2000:]
    doc = json.load(open(os.path.join(out, "rtest_conv_clock.json")))
    assert len(doc["calibration"]) == 4 and len(doc["classes"]) == 2
    for c in doc["calibration"]:
        assert abs(c["in_kernel_over_grbm"] - 0.8) < 1e-3 and abs(c["mfma_busy_cycles_per_mfma"] - 16) < 1e-6
    for row in doc["classes"]:
        assert abs(row["clock_GHz"] - 1.6) < 1e-3
        assert abs(row["mfma_busy_frac"] - busy) < 1e-3
        v4 = row["views4"]
        assert abs(v4["frac_at_clock"] - v4["achieved_TFLOPs"] / (833.3 * 1.6 / 2.4)) < 2e-3
