#!/bin/bash
# bf16-mode knock-outs of the forward conv (tools/conv_bench, B=8 as in the training step):
# 0 full, 1 no patch DMA, 2 no transform, 3 neither, 4 no weight loads, 16 no epilogue stores.
set -u
for ko in 0 1 2 3 4 16; do
  echo "KO=$ko"
  timeout -k 5 60 tools/_cb/conv_bench_$ko 256 256 32 512 8 1 20 2 || exit $?
  timeout -k 5 60 tools/_cb/conv_bench_$ko 128 128 64 1024 8 1 20 2 || exit $?
done
