#!/bin/bash
# Generic env A/B on one box: parity subset with B's env, then the line bench under A's and B's env.
# usage: A="SDP_X=0" B="SDP_X=1" bash tools/gpu_ab.sh
set -u
mkdir -p gpurun_out
env $B timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "scorenet or split or fused" > gpurun_out/ab_parity.log 2>&1
echo "parity rc=$?"
for r in 1 2; do
env $A timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32-line --sustained-s 3 > gpurun_out/ab_A$r.log 2>&1 || exit $?
env $B timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32-line --sustained-s 3 > gpurun_out/ab_B$r.log 2>&1 || exit $?
done
