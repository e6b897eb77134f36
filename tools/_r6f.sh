#!/bin/bash
# conv records at the final conv source: PMC traffic + in-network clock (ROUND=r06)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/round
timeout -k 10 200 env ROUND=r06 bash tools/class_traffic.sh > gpurun_out/round/traffic.log 2>&1; rc=$?; echo "traffic rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/round/traffic.log; exit $rc; }
timeout -k 10 500 env ROUND=r06 bash tools/conv_clock.sh > gpurun_out/round/clock.log 2>&1; rc=$?; echo "clock rc=$rc"; tail -3 gpurun_out/round/clock.log
