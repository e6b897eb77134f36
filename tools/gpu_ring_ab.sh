#!/bin/bash
# bf16 weight-ring depth A/B (A: SDP_BF16_RING=3 variant library, B: the tree's 9-slot ring) on the
# train bench, after the training parity tests of the tree.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_training.py -x -q --timeout 200 --timeout-method thread > gpurun_out/rg_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -1 gpurun_out/rg_parity.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
SDP_LIB=tools/_var/ring3/libsdp.so timeout -k 10 200 python bench.py --workload train --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/rg_A$r.log 2>&1 || exit $?
echo "ring3 run $r: $(grep -o '"value": [0-9.]*' gpurun_out/rg_A$r.log | head -1)"
timeout -k 10 200 python bench.py --workload train --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/rg_B$r.log 2>&1 || exit $?
echo "ring9 run $r: $(grep -o '"value": [0-9.]*' gpurun_out/rg_B$r.log | head -1)"
done
