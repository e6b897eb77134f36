#!/bin/bash
# Build conv_bench variants (knock-out masks) here; run them on the GPU with RUN=1.
# TAG=<name>: name the (single) build conv_bench_<name> instead of by its mask (e.g. EXTRA=-DSDP_TIMING TAG=T)
set -eu
cd "$(dirname "$0")/.."
mkdir -p tools/_cb
SRC=simultaneous-diffusion-for-pointclouds_amd/csrc
if [ "${RUN:-0}" = 0 ]; then
  for ko in ${KOS:-0 1 2 4 8 16}; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -DSDP_CONV_BENCH_ONLY -DSDP_KO=$ko ${EXTRA:-} \
      -c $SRC/conv.hip -o tools/_cb/conv_${TAG:-$ko}.o &
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -DSDP_CONV_BENCH_ONLY -DSDP_KO=$ko ${EXTRA:-} \
      -c $SRC/conv_inst.hip -o tools/_cb/conv_inst_${TAG:-$ko}.o &
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -DSDP_CONV_BENCH_ONLY -DSDP_KO=$ko ${EXTRA:-} \
      -c $SRC/conv_bwd.hip -o tools/_cb/conv_bwd_${TAG:-$ko}.o &
    for code in 1015 1016 1025 1026; do   # the 8 x 16 data-gradient launchers (conv_inst.hip codes)
      /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -DSDP_INST=$code -DSDP_KO=$ko ${EXTRA:-} \
        -c $SRC/conv_inst.hip -o tools/_cb/dg_${code}_${TAG:-$ko}.o &
    done
  done
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 ${EXTRA:-} -c tools/conv_bench.cpp -o tools/_cb/main.o
  H=$(python3 -c "import sys; sys.path.insert(0, 'simultaneous-diffusion-for-pointclouds_amd'); from sdp import _build; print(_build.conv_source_hash())")
  for ko in ${KOS:-0 1 2 4 8 16}; do
    t=${TAG:-$ko}
    /opt/rocm/bin/hipcc --offload-arch=gfx950 tools/_cb/main.o tools/_cb/conv_$t.o tools/_cb/conv_inst_$t.o tools/_cb/conv_bwd_$t.o \
      tools/_cb/dg_10[12][56]_$t.o -o tools/_cb/conv_bench_$t
    echo "$H ${EXTRA:-}" > tools/_cb/conv_bench_$t.hash     # the conv sources (and extra flags) it was built from
  done
else
  for ko in ${KOS:-0 1 2 4 8 16}; do
    echo "KO=$ko"
    timeout -k 5 60 tools/_cb/conv_bench_$ko 256 256 32 512 ${B:-4} 1 20 ${MODE:-1}
    timeout -k 5 60 tools/_cb/conv_bench_$ko 128 128 64 1024 ${B:-4} 1 20 ${MODE:-1}
  done
fi
