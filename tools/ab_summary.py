"""Summarise tools/gpu_ab.sh logs: per-class conv averages and the line value of each arm."""
import glob
import json
import re
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
for f in sorted(glob.glob(f"{d}/ab_[AB]*.log")):
    cls = {}
    val = None
    for line in open(f):
        m = re.match(r"\[\w+\] (conv\S* .*?)\s+launches\s+\d+ avg\s+([\d.]+) us", line)
        if m:
            cls[m.group(1).strip()] = float(m.group(2))
        if line.startswith("{"):
            j = json.loads(line)
            val = (j["value"], j["ms_per_step"], (j.get("sustained") or {}).get("value"))
    short = {k.split(" @")[0].replace("conv3x3 ", "") + "@" + k.split("@")[1]: v for k, v in cls.items()}
    print(f.split("/")[-1], val, " ".join(f"{k}={v:.1f}" for k, v in sorted(short.items())))
