#!/bin/bash
# Env A/B of the training workload on one box (training parity tests with B's env first).
# usage: A="SDP_X=0" B="SDP_X=1" bash tools/gpu_ab_train.sh
set -u
mkdir -p gpurun_out
env $B timeout -k 10 400 python -u -m pytest tests/test_gpu_training.py -x -q --timeout 300 --timeout-method thread > gpurun_out/abt_parity.log 2>&1
echo "training parity rc=$?"
for r in 1 2; do
env $A timeout -k 10 200 python bench.py --workload train --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/abt_A$r.log 2>&1 || exit $?
env $B timeout -k 10 200 python bench.py --workload train --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/abt_B$r.log 2>&1 || exit $?
done
