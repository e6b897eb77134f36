#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6g; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_train -o run --output-format csv -- python bench.py --workload train --steps 5 --warmup 1 --no-cpu-baseline > $O/train.log 2>&1 || { echo "train prof failed"; tail -5 $O/train.log; exit 1; }
f=$(find $O/prof_train -name "run_kernel_stats.csv" | head -1); python3 tools/stats_top.py $f 11 25
