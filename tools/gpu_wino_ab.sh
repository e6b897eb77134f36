#!/bin/bash
# Winograd A/B on one box: score-net parity (goldens), then the line bench with SDP_WINO=0 (direct) and default.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k "scorenet or split or fused" > gpurun_out/w_parity.log 2>&1
echo "parity rc=$?"
SDP_WINO=0 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32-line --sustained-s 3 > gpurun_out/w_bench0.log 2>&1 && echo "bench0 ok"
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32-line --sustained-s 3 > gpurun_out/w_bench3.log 2>&1 && echo "bench3 ok"
