#!/bin/bash
# forward stream split re-measured on the round-6 kernels
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ROUNDS="1 2" ARMS="s1||--split 1;s2||--split 2;s3||--split 3;s4||--split 4" bash tools/ab_line.sh > gpurun_out/split_ab.log 2>&1
python3 tools/ab_sum.py gpurun_out/ab/s1_?.log gpurun_out/ab/s2_?.log gpurun_out/ab/s3_?.log gpurun_out/ab/s4_?.log
ROUNDS="1" ARMS="v8s2||--views 8 --split 2;v8s3||--views 8 --split 3;v8s4||--views 8 --split 4" bash tools/ab_line.sh > gpurun_out/split8_ab.log 2>&1
python3 tools/ab_sum.py gpurun_out/ab/v8s?_1.log
