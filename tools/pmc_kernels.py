"""Print per-(kernel, grid) averages of every PMC counter found under a rocprofv3 output dir."""
import sys
from collections import defaultdict

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_traffic import load  # noqa: E402

per = load(sys.argv[1])
filt = sys.argv[2] if len(sys.argv) > 2 else ""
rows = []
for (name, grid, wg), cs in per.items():
    if filt not in name:
        continue
    rows.append((name, grid, {c: sum(v) / len(v) for c, v in cs.items()}, max(len(v) for v in cs.values())))
rows.sort(key=lambda r: -r[2].get("SQ_WAVE_CYCLES", r[2].get("GRBM_GUI_ACTIVE", 0)) * r[3])
for name, grid, avg, n in rows[:12]:
    print(f"== {name[:90]} grid={grid} n={n}")
    for c in sorted(avg):
        print(f"   {c:32s} {avg[c]:16.1f}")
