#!/bin/bash
# Winograd A/B on one box: microbench (knock-outs, in-kernel clock), score-net parity with the
# Winograd path on (goldens), then the line bench with SDP_WINO=0 (direct) and SDP_WINO=3.
set -u
mkdir -p gpurun_out
RUN=1 KOS="${KOS:-0 2 4 16 32 39}" timeout -k 10 200 bash tools/wino_bench.sh > gpurun_out/w_micro.log 2>&1 || exit $?
timeout -k 10 100 bash tools/wino_clock.sh > gpurun_out/w_clock.log 2>&1 || exit $?
SDP_WINO=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "scorenet or split or fused" > gpurun_out/w_parity.log 2>&1
echo "parity rc=$?"
SDP_WINO=0 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32-line --sustained-s 3 > gpurun_out/w_bench0.log 2>&1 || exit $?
SDP_WINO=3 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32-line --sustained-s 3 > gpurun_out/w_bench3.log 2>&1 || exit $?
