#!/bin/bash
# Knock-out timing of the forward conv (SH=16): 0 full, 1 no patch DMA, 4 no weight loads, 16 no
# epilogue, 31 = bare MFMA loop (no DMA, transform, weights, chunk barrier, epilogue).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for round in 1 2; do
  for ko in 0 1 4 16 31; do
    for shape in "256 256 32 512" "128 128 64 1024"; do
      echo -n "round $round KO=$ko: "
      timeout -k 5 60 tools/_cb/conv_bench_$ko $shape 4 1 40 1 || exit 1
    done
  done
done
