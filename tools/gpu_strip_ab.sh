#!/bin/bash
# Tile-order A/B on one box: PMC traffic of the 256- and 128-channel classes with SDP_STRIP=0/1, then the line bench.
set -u
export TMPDIR=/tmp
O=gpurun_out/strip; mkdir -p $O
for s in 0 1; do
  for cfg in "256 256 32 512" "128 128 64 1024"; do
    SDP_STRIP=$s timeout -s KILL 60 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum \
      -d $O/s${s}_${cfg%% *} -o run --output-format csv -- tools/_cb/conv_bench_0 $cfg 4 1 20 1 > $O/s${s}_${cfg%% *}.log 2>&1 || exit 1
  done
done
A="SDP_STRIP=0" B="SDP_STRIP=1" bash tools/gpu_ab.sh
