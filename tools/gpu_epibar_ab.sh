#!/bin/bash
# Transposed-epilogue scheduling A/B on the bf16 train step: A = per-channel-block sched_barrier
# (variant library tools/_var/epibar), B = the tree (no barrier); training parity of the tree first.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_training.py -x -q --timeout 200 --timeout-method thread > gpurun_out/eb_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -1 gpurun_out/eb_parity.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2 3; do
SDP_LIB=tools/_var/epibar/libsdp.so timeout -k 10 200 python bench.py --workload train --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/eb_A$r.log 2>&1 || exit $?
echo "barrier run $r: $(grep -o '"value": [0-9.]*' gpurun_out/eb_A$r.log | head -1)"
timeout -k 10 200 python bench.py --workload train --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/eb_B$r.log 2>&1 || exit $?
echo "no barrier run $r: $(grep -o '"value": [0-9.]*' gpurun_out/eb_B$r.log | head -1)"
done
