#!/bin/bash
# Kernel stats of a short training bench: gpurun_out/train_stats.csv
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/tp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tp -o run --output-format csv -- \
  python3 bench.py --workload train --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/tp.log 2>&1
cp "$(find gpurun_out/tp -name '*kernel_stats.csv' | head -1)" gpurun_out/train_stats.csv
tail -1 gpurun_out/tp.log | cut -c1-200
