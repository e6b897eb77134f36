#!/bin/bash
# provenance: the library compiled on the box from the tree's sources, then smoke + GPU suite + a 14-s sustained line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/fresh; mkdir -p $O
rm -rf simultaneous-diffusion-for-pointclouds_amd/sdp/_lib simultaneous-diffusion-for-pointclouds_amd/build
timeout -k 10 600 python -c "import sys; sys.path.insert(0, 'simultaneous-diffusion-for-pointclouds_amd'); from sdp import _build; _build.ensure_built()" > $O/build.log 2>&1; rc=$?; echo "on-box build rc=$rc"; tail -1 $O/build.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python __graft_entry__.py smoke > $O/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 850 python -u -m pytest tests -m gpu -q -rA --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32-line --sustained-s 14 > $O/bench_sustained14s.log 2>&1; rc=$?; echo "sustained rc=$rc"; grep "^{" $O/bench_sustained14s.log | cut -c1-200
