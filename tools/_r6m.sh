#!/bin/bash
# final tree: smoke + GPU suite + the bench workloads (round_profiles PART=2)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/round; mkdir -p $O
timeout -k 10 300 python __graft_entry__.py smoke > $O/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 850 python -u -m pytest tests -m gpu -q -rA --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
PART=2 ROUND=r06 bash tools/round_profiles.sh
