#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6h; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_config4.py tests/test_gpu_runner_pinned.py -x -q --timeout 200 --timeout-method thread > $O/parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -1 $O/parity.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/merge_dump.py /tmp/new.npz && SDP_LIB=tools/_var/f64ang/libsdp.so timeout -k 10 200 python tools/merge_dump.py /tmp/f64a.npz && SDP_LIB=tools/_var/f64ang/libsdp.so timeout -k 10 200 python tools/merge_dump.py /tmp/f64b.npz || exit 1
echo "== control (f64 vs f64)"; python3 tools/merge_cmp.py /tmp/f64a.npz /tmp/f64b.npz | tail -1
echo "== f32 angles vs f64"; python3 tools/merge_cmp.py /tmp/new.npz /tmp/f64a.npz > $O/cmp.log; tail -1 $O/cmp.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --megabatch-views 32 --no-cpu-baseline --no-fp32-line --split 1 --sustained-s 0 > $O/mb32_prof.log 2>&1 || { echo "prof failed"; exit 1; }
f=$(find $O/prof -name "run_kernel_stats.csv" | head -1); python3 tools/stats_top.py $f 17 40 | grep -i "merge"
ROUNDS="1 2 3" ARMS="f64_32|SDP_LIB=tools/_var/f64ang/libsdp.so|--megabatch-views 32 --sustained-s 0;f32_32||--megabatch-views 32 --sustained-s 0;f64_4|SDP_LIB=tools/_var/f64ang/libsdp.so|--sustained-s 0;f32_4||--sustained-s 0" bash tools/ab_line.sh > $O/ab.log 2>&1
python3 tools/ab_sum.py gpurun_out/ab/f64_32_?.log gpurun_out/ab/f32_32_?.log gpurun_out/ab/f64_4_?.log gpurun_out/ab/f32_4_?.log
