#!/bin/bash
# MFMA shape A/B (conv_kernel.h SH): interleaved rounds of the same binary with SDP_MFMA_SHAPE=32|16.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for round in 1 2 3; do
  for sh in 32 16; do
    for shape in "256 256 32 512" "128 128 64 1024"; do
      echo -n "round $round SH=$sh: "
      SDP_MFMA_SHAPE=$sh timeout -k 5 60 tools/_cb/conv_bench_0 $shape 4 1 40 ${MODE:-1} || exit 1
    done
  done
done
