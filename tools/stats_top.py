"""Print the top kernels of a rocprofv3 kernel_stats.csv, per bench step: stats_top.py CSV STEPS [N]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2])
rows.sort(key=lambda x: -float(x["TotalDurationNs"]))
tot = sum(float(x["TotalDurationNs"]) for x in rows)
print(f"total {tot / 1e6 / steps:.2f} ms/step")
for x in rows[: int(sys.argv[3]) if len(sys.argv) > 3 else 16]:
    print(f"{float(x['TotalDurationNs']) / 1e6 / steps:8.2f} ms/step {float(x['AverageNs']) / 1e3:8.1f} us "
          f"{x['Calls']:>5}  {x['Name'][:100]}")
