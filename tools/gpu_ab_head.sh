#!/bin/bash
# GPU tests on the current library, the HBM write ceiling (tools/write_bw), then an A/B of the
# head kernels: current library vs the listed variants (tools/_var/<name>/libsdp.so).
#   VARIANTS="headdirect mfma_v1" bash tools/gpu_ab_head.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/ab
mkdir -p $O
if [ "${SKIP_TESTS:-0}" = 0 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
  [ $rc -ne 0 ] && exit $rc
fi
if [ "${SKIP_TESTS:-0}" = 0 ] && [ -x tools/_cb/write_bw ]; then timeout -k 10 120 tools/_cb/write_bw 20 > $O/write_bw.log 2>&1; echo "write_bw rc=$?"; cat $O/write_bw.log; fi
for rep in $(seq ${REPS:-2}); do
  for v in new ${VARIANTS:-}; do
    if [ $v = new ]; then L=; else L=SDP_LIB=tools/_var/$v/libsdp.so; fi
    env $L timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-fp32-line > $O/bench_${v}_$rep.log 2>&1 || { echo "bench $v failed"; tail -5 $O/bench_${v}_$rep.log; exit 1; }
    echo "== $v rep $rep: $(grep -o '"value": [0-9.]*' $O/bench_${v}_$rep.log | head -1)"
    grep -o '"kernel": "\(begin\|end\)[^}]*' $O/bench_${v}_$rep.log | sed 's/"algorithmic_bytes.*frac"/ frac/' | head -2
  done
done
exit 0
