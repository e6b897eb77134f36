#!/bin/bash
# bf16 training step vs MFMA shape: default (16x16 everywhere), SDP_MFMA_SHAPE=32 (forward convs on
# 32x32x16), and 32x32 for the data gradient too (SDP_DGRAD16=0 SDP_DGRAD_SHAPE=32); 2 rounds.
set -u
mkdir -p gpurun_out
for r in 1 2; do
for arm in "SDP_X=0" "SDP_MFMA_SHAPE=32" "SDP_MFMA_SHAPE=32 SDP_DGRAD16=0 SDP_DGRAD_SHAPE=32"; do
env $arm timeout -k 10 200 python bench.py --workload train --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/sh_tmp.log 2>&1 || exit $?
echo "$arm run $r: $(grep -o '"value": [0-9.]*' gpurun_out/sh_tmp.log | head -1)"
done
done
