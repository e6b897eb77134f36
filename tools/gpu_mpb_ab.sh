#!/bin/bash
# CRP maxpool backward grid (SDP_MPB_BLOCKS = block count aimed for when splitting rows): training
# parity at the extremes, then rocprofv3 kernel stats of the train workload per setting.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/mpb
mkdir -p $O
for t in 1024 8192; do
  SDP_MPB_BLOCKS=$t timeout -k 10 300 python -u -m pytest tests/test_gpu_training.py -x -q --timeout 200 --timeout-method thread > $O/parity_$t.log 2>&1
  rc=$?; echo "parity $t rc=$rc $(tail -1 $O/parity_$t.log)"; [ $rc -ne 0 ] && exit $rc
done
for t in 2048 1024 4096 8192; do
  SDP_MPB_BLOCKS=$t timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p$t -o run --output-format csv -- python bench.py --workload train --steps 5 --warmup 1 --no-cpu-baseline > $O/p$t.log 2>&1 || exit $?
  echo "$t: $(grep -h maxpool5_bwd $O/p$t/run_kernel_stats.csv | cut -d, -f2-4)"
done
