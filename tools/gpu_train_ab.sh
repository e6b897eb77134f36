#!/bin/bash
# Training A/Bs on one box: training parity (tree, and SDP_WGRAD_OCC=3), then the train bench with
# the SDP_BF16_RING=3 variant library (ring3) and the tree (ring 9) under SDP_WGRAD_OCC = 2 | 3 | 1.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_training.py -x -q --timeout 200 --timeout-method thread > gpurun_out/tr_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -1 gpurun_out/tr_parity.log; [ $rc -ne 0 ] && exit $rc
SDP_WGRAD_OCC=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_training.py -x -q --timeout 200 --timeout-method thread > gpurun_out/tr_parity3.log 2>&1
rc=$?; echo "parity(occ3) rc=$rc"; tail -1 gpurun_out/tr_parity3.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
SDP_LIB=tools/_var/ring3/libsdp.so timeout -k 10 200 python bench.py --workload train --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/tr_ring3_$r.log 2>&1 || exit $?
echo "ring3 occ2 run $r: $(grep -o '"value": [0-9.]*' gpurun_out/tr_ring3_$r.log | head -1)"
for o in 2 3 1; do
SDP_WGRAD_OCC=$o timeout -k 10 200 python bench.py --workload train --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/tr_occ${o}_$r.log 2>&1 || exit $?
echo "ring9 occ$o run $r: $(grep -o '"value": [0-9.]*' gpurun_out/tr_occ${o}_$r.log | head -1)"
done
done
