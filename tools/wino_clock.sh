#!/bin/bash
# In-kernel clock of the Winograd conv (SDP_TIMING builds of tools/wino_bench): full kernel vs bare MFMA loop.
cd "$(dirname "$0")/.."
for k in t0 t39; do
  echo "== $k"
  timeout -k 5 60 tools/_wb/wino_bench_$k 256 256 32 512 4 1 50
  timeout -k 5 60 tools/_wb/wino_bench_$k 128 128 64 1024 4 1 50
done
echo "== direct (conv_bench KO=0), for comparison"
timeout -k 5 60 tools/_cb/conv_bench_0 256 256 32 512 4 1 50 1
