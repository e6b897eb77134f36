#!/bin/bash
# timing-only knock-outs of the line: every IN++ finalize launch / every 5x5 max-pool left out (numerics void)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ROUNDS="1 2" ARMS="base||--sustained-s 0;koinpp|SDP_LIB=tools/_var/koinpp/libsdp.so|--sustained-s 0;kopool|SDP_LIB=tools/_var/kopool/libsdp.so|--sustained-s 0;koboth|SDP_LIB=tools/_var/koboth/libsdp.so|--sustained-s 0" bash tools/ab_line.sh > gpurun_out/ko_ab.log 2>&1
python3 tools/ab_sum.py gpurun_out/ab/base_?.log gpurun_out/ab/koinpp_?.log gpurun_out/ab/kopool_?.log gpurun_out/ab/koboth_?.log
