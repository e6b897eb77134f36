#!/bin/bash
# bf16 weight-gradient staging A/B (SDP_WGRAD_OCC = 2 default | 3 | 1) on the train bench, after the
# training parity tests under OCC 3 and the default.
set -u
mkdir -p gpurun_out
SDP_WGRAD_OCC=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_training.py -x -q --timeout 200 --timeout-method thread > gpurun_out/wg_parity3.log 2>&1
rc=$?; echo "parity(occ3) rc=$rc"; tail -1 gpurun_out/wg_parity3.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_training.py -x -q --timeout 200 --timeout-method thread > gpurun_out/wg_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -1 gpurun_out/wg_parity.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
for o in 2 3 1; do
SDP_WGRAD_OCC=$o SDP_PROFILE_TRAIN=1 timeout -k 10 200 python bench.py --workload train --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/wg_occ${o}_$r.log 2>&1 || exit $?
echo "occ $o run $r: $(grep -o '"value": [0-9.]*' gpurun_out/wg_occ${o}_$r.log | head -1)"
done
done
