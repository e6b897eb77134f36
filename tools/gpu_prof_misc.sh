#!/bin/bash
# Kernel stats of the 32-view-megabatch line step (one config-4 rank) and of the bf16 train step.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pm_mb32 -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-fp32-line --sustained-s 0 --megabatch-views 32 > gpurun_out/pm_mb32.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pm_train -o run --output-format csv -- python bench.py --workload train --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/pm_train.log 2>&1 || exit $?
for d in pm_mb32 pm_train; do
python3 - gpurun_out/$d/run_kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:40]:
    if any(k in r["Name"] for k in ("merge", "inpp", "maxpool5_bwd", "wgrad_reduce")):
        print(f"{float(r['TotalDurationNs'])/1e6:9.2f} ms {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:9.1f}us {r['Name'][:70]}")
PY
done
