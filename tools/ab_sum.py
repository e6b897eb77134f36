"""Summarise bench.py JSON lines of A/B logs: ab_sum.py LOG... -> value, ms/step, dominant conv, merge, memory-bound us."""
import json
import os
import sys

for f in sys.argv[1:]:
    ls = [x for x in open(f) if x.startswith("{")]
    if not ls:
        print(f"{os.path.basename(f):24s} (no result line)")
        continue
    d = json.loads(ls[-1])
    mb = {m["kernel"].split(" (")[0]: m["avg_launch_us"] for m in d["roofline"].get("memory_bound", [])}
    su = (d.get("sustained") or {}).get("value", 0)
    print(f"{os.path.basename(f):24s} {d['value']:8.2f} {d['ms_per_step']:7.3f} ms  sust {su:7.2f}  conv {d['roofline']['avg_launch_us']:6.1f} us"
          f"  merge {mb.get('consistency_merge', 0):6.1f} us")
