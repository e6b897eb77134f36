#!/bin/bash
# round-6 session A: merge aggregation parity + per-kernel profile at 32 views; begin-conv occupancy A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6a; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_config4.py -x -q --timeout 200 --timeout-method thread -k "merge or config4 or kitti or allforone" > $O/parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 $O/parity.log; [ $rc -ne 0 ] && exit $rc
for arm in agg0 agg1; do
  if [ $arm = agg0 ]; then export SDP_LIB=tools/_var/agg0/libsdp.so; else unset SDP_LIB; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$arm -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --megabatch-views 32 --no-cpu-baseline --no-fp32-line --split 1 --sustained-s 0 > $O/mb32_$arm.log 2>&1 || { echo "prof $arm failed"; exit 1; }
  f=$(find $O/prof_$arm -name "run_kernel_stats.csv" | head -1); echo "== $arm"; python3 tools/stats_top.py $f 17 40 | grep -i "merge\|total"
done
unset SDP_LIB
ARMS="base||;bm4|SDP_LIB=tools/_var/bm4/libsdp.so|;bmd2|SDP_LIB=tools/_var/bmd2/libsdp.so|" bash tools/ab_line.sh
