#!/bin/bash
# Edit-build loop: incremental make of libsdp.so in csrc/, then mark it current (sdp/_build.py stamp).
set -eu
cd "$(dirname "$0")/.."
make -j${JOBS:-8} -C simultaneous-diffusion-for-pointclouds_amd/csrc "$@"
python3 -c "import sys; sys.path.insert(0, 'simultaneous-diffusion-for-pointclouds_amd'); from sdp import _build; _build.write_stamp()"
