#!/bin/bash
# Weight-gradient accumulator split A/B (A: SDP_WGRAD_SPLIT=0 variant library, B: the tree) on the
# bf16 train step, after the tree's training parity (fp32x3 gradients vs the oracle, bf16 cosine).
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_training.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ws_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -1 gpurun_out/ws_parity.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2 3; do
SDP_LIB=tools/_var/nosplit/libsdp.so timeout -k 10 200 python bench.py --workload train --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ws_A$r.log 2>&1 || exit $?
echo "nosplit run $r: $(grep -o '"value": [0-9.]*' gpurun_out/ws_A$r.log | head -1)"
timeout -k 10 200 python bench.py --workload train --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ws_B$r.log 2>&1 || exit $?
echo "split run $r: $(grep -o '"value": [0-9.]*' gpurun_out/ws_B$r.log | head -1)"
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ws_prof -o run --output-format csv -- python bench.py --workload train --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/ws_rocprof.log 2>&1 || exit $?
grep wgrad_kernel gpurun_out/ws_prof/run_kernel_stats.csv | cut -c1-150
