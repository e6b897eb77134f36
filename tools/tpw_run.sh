#!/bin/bash
# Tiles-per-workgroup A/B (conv_kernel.h multi-tile pipeline): interleaved rounds, SDP_TPW=1|2|4.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for round in 1 2 3; do
  for tpw in 1 2 4; do
    for shape in "256 256 32 512" "128 128 64 1024"; do
      echo -n "round $round TPW=$tpw: "
      SDP_TPW=$tpw timeout -k 5 60 tools/_cb/conv_bench_0 $shape 4 1 40 1 || exit 1
    done
  done
done
