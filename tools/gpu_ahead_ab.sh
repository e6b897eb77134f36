#!/bin/bash
# bf16 A-fragment prefetch A/B (SDP_BF16_AHEAD 0 = variant, 1 = tree): conv_bench full and KO=3
# (no DMA, no transform) at B=8 in bf16, then the bf16 train step, after the tree's training parity.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_training.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ah_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -1 gpurun_out/ah_parity.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
for k in 0 3; do
echo "ahead0 KO=$k"; timeout -k 5 60 tools/_cb/ahead0_$k 256 256 32 512 8 1 20 2 || exit $?; timeout -k 5 60 tools/_cb/ahead0_$k 128 128 64 1024 8 1 20 2 || exit $?
echo "ahead1 KO=$k"; timeout -k 5 60 tools/_cb/conv_bench_$k 256 256 32 512 8 1 20 2 || exit $?; timeout -k 5 60 tools/_cb/conv_bench_$k 128 128 64 1024 8 1 20 2 || exit $?
done
SDP_LIB=tools/_var/ahead0/libsdp.so timeout -k 10 200 python bench.py --workload train --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ah_A$r.log 2>&1 || exit $?
echo "train ahead0 run $r: $(grep -o '"value": [0-9.]*' gpurun_out/ah_A$r.log | head -1)"
timeout -k 10 200 python bench.py --workload train --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ah_B$r.log 2>&1 || exit $?
echo "train ahead1 run $r: $(grep -o '"value": [0-9.]*' gpurun_out/ah_B$r.log | head -1)"
done
