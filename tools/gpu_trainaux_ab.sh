#!/bin/bash
# A/B of the training-side memory kernels (maxpool5 backward residual prefetch, batched weight re-pack
# gathers): training parity on the tree, then the train bench alternating HEAD~ (tools/_var/base) and
# the tree, then rocprofv3 kernel stats of both.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/trainaux
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_training.py -x -q --timeout 200 --timeout-method thread > $O/parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -1 $O/parity.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  SDP_LIB=tools/_var/base/libsdp.so timeout -k 10 200 python bench.py --workload train --steps 20 --warmup 3 --no-cpu-baseline > $O/base_$r.log 2>&1 || exit $?
  echo "base run $r: $(grep -o '"value": [0-9.]*' $O/base_$r.log | head -1)"
  timeout -k 10 200 python bench.py --workload train --steps 20 --warmup 3 --no-cpu-baseline > $O/tree_$r.log 2>&1 || exit $?
  echo "tree run $r: $(grep -o '"value": [0-9.]*' $O/tree_$r.log | head -1)"
done
SDP_LIB=tools/_var/base/libsdp.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_base -o run --output-format csv -- python bench.py --workload train --steps 5 --warmup 1 --no-cpu-baseline > $O/prof_base.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_tree -o run --output-format csv -- python bench.py --workload train --steps 5 --warmup 1 --no-cpu-baseline > $O/prof_tree.log 2>&1 || exit $?
echo done
