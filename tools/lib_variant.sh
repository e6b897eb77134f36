#!/bin/bash
# Build a libsdp.so variant that differs only in compile-time defines, for in-network A/B runs:
#   tools/lib_variant.sh NAME "-DSDP_DMA_AUX=2 ..."  ->  tools/_var/NAME/libsdp.so
# Run it with SDP_LIB=tools/_var/NAME/libsdp.so (sdp/_lib.py loads that file as is).
set -eu
cd "$(dirname "$0")/.."
NAME=$1; DEFS=$2
D=tools/_var/$NAME
mkdir -p $D
make -C simultaneous-diffusion-for-pointclouds_amd/csrc -j${JOBS:-8} OBJDIR=$PWD/$D/obj OUT=$PWD/$D/libsdp.so EXTRA="$DEFS" > $D/build.log 2>&1 \
  || { tail -30 $D/build.log; exit 1; }
rm -rf $D/obj
echo "built $D/libsdp.so ($DEFS)"
