#!/bin/bash
# final tree: smoke + GPU suite; the NaN merge test against the pre-fix build (must fail)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/round; mkdir -p $O
timeout -k 10 300 python __graft_entry__.py smoke > $O/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 850 python -u -m pytest tests -m gpu -q -rA --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
SDP_LIB=tools/_var/nanbug/libsdp.so timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread -k nan_points > $O/nanbug.log 2>&1; echo "pre-fix build on the NaN test: rc=$? (1 = the test catches it)"; tail -1 $O/nanbug.log
