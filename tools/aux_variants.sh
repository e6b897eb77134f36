#!/bin/bash
# Build conv_bench variants that differ only in cache-policy bits (SDP_DMA_AUX / SDP_STORE_AUX).
set -eu
cd "$(dirname "$0")/.."
mkdir -p tools/_cb
SRC=simultaneous-diffusion-for-pointclouds_amd/csrc
for v in "0 0" "0 2" "2 2" "2 0"; do
  set -- $v
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -DSDP_CONV_BENCH_ONLY -DSDP_DMA_AUX=$1 \
    -DSDP_STORE_AUX=$2 -c $SRC/conv.hip -o tools/_cb/conv_aux_$1_$2.o &
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -DSDP_CONV_BENCH_ONLY -DSDP_DMA_AUX=$1 \
    -DSDP_STORE_AUX=$2 -c $SRC/conv_inst.hip -o tools/_cb/conv_inst_aux_$1_$2.o &
done
wait
[ -f tools/_cb/main.o ] || /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -c tools/conv_bench.cpp -o tools/_cb/main.o
for v in "0 0" "0 2" "2 2" "2 0"; do
  set -- $v
  /opt/rocm/bin/hipcc --offload-arch=gfx950 tools/_cb/main.o tools/_cb/conv_aux_$1_$2.o tools/_cb/conv_inst_aux_$1_$2.o -o tools/_cb/conv_bench_aux_$1_$2
done
