#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6d; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_config4.py tests/test_gpu_runner_pinned.py -x -q --timeout 200 --timeout-method thread > $O/parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -1 $O/parity.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --megabatch-views 32 --no-cpu-baseline --no-fp32-line --split 1 --sustained-s 0 > $O/mb32_prof.log 2>&1 || { echo "prof failed"; exit 1; }
f=$(find $O/prof -name "run_kernel_stats.csv" | head -1); python3 tools/stats_top.py $f 17 40 | grep -i "merge\|total"
ROUNDS="1 2 3" ARMS="old32|SDP_LIB=tools/_var/tile0/libsdp.so|--megabatch-views 32 --sustained-s 0;new32||--megabatch-views 32 --sustained-s 0;old4|SDP_LIB=tools/_var/tile0/libsdp.so|--sustained-s 0;new4||--sustained-s 0" bash tools/ab_line.sh | grep -v "^      "
