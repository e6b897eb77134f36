#!/bin/bash
# Conv diagnostics on one box (binaries from tools/conv_bench.sh + a -DSDP_TIMING build conv_bench_T):
# knock-outs 0 full, 1 no patch DMA, 2 no transform, 4 no weight loads, 16 no epilogue, 31 bare MFMA
# loop; then the per-workgroup phase clocks.  Shapes: 256->256 @32x512 and 128->128 @64x1024, B=4.
# DG=1: the data gradient (conv_dgrad, dact 3 + residual) instead of the forward.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for round in 1 2; do
  for ko in ${KOS:-0 1 2 4 16 31}; do
    for shape in "256 256 32 512" "128 128 64 1024"; do
      echo -n "round $round KO=$ko: "
      timeout -k 5 60 tools/_cb/conv_bench_$ko $shape ${BATCH:-4} 1 40 ${MODE:-1} ${DG:+dgrad} || exit 1
    done
  done
done
for shape in "256 256 32 512" "128 128 64 1024"; do
  timeout -k 5 60 tools/_cb/conv_bench_T $shape ${BATCH:-4} 1 40 ${MODE:-1} ${DG:+dgrad} || exit 1
done
