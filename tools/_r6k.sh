#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6k; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_config4.py tests/test_gpu_runner_pinned.py -x -q --timeout 200 --timeout-method thread > $O/parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -1 $O/parity.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/merge_dump.py /tmp/new.npz > /dev/null && SDP_LIB=tools/_var/prevw/libsdp.so timeout -k 10 200 python tools/merge_dump.py /tmp/old.npz > /dev/null || exit 1
echo "== fused world vs world array"; python3 tools/merge_cmp.py /tmp/new.npz /tmp/old.npz | tail -1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --megabatch-views 32 --no-cpu-baseline --no-fp32-line --split 1 --sustained-s 0 > $O/mb32_prof.log 2>&1 || { echo "prof failed"; exit 1; }
f=$(find $O/prof -name "run_kernel_stats.csv" | head -1); python3 tools/stats_top.py $f 17 40 | grep -i "merge"
ROUNDS="1 2 3" ARMS="prev32|SDP_LIB=tools/_var/prevw/libsdp.so|--megabatch-views 32 --sustained-s 0;new32||--megabatch-views 32 --sustained-s 0;prev4|SDP_LIB=tools/_var/prevw/libsdp.so|--sustained-s 0;new4||--sustained-s 0" bash tools/ab_line.sh > $O/ab.log 2>&1
python3 tools/ab_sum.py gpurun_out/ab/prev32_?.log gpurun_out/ab/new32_?.log gpurun_out/ab/prev4_?.log gpurun_out/ab/new4_?.log
