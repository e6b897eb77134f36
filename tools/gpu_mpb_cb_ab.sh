#!/bin/bash
# CRP maxpool backward channels per block (tools/_var/mpb64 = SDP_MPB_CB=64: 256-B pieces of every
# pixel's channel row per fetch, vs 128 B at the default 32): training parity with the variant, then
# rocprofv3 kernel stats of the train workload for the tree and the variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/mpbcb
mkdir -p $O
SDP_LIB=tools/_var/mpb64/libsdp.so timeout -k 10 300 python -u -m pytest tests/test_gpu_training.py -x -q --timeout 200 --timeout-method thread > $O/parity.log 2>&1
rc=$?; echo "parity mpb64 rc=$rc $(tail -1 $O/parity.log)"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tree -o run --output-format csv -- python bench.py --workload train --steps 5 --warmup 1 --no-cpu-baseline > $O/tree.log 2>&1 || exit $?
SDP_LIB=tools/_var/mpb64/libsdp.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/mpb64 -o run --output-format csv -- python bench.py --workload train --steps 5 --warmup 1 --no-cpu-baseline > $O/mpb64.log 2>&1 || exit $?
echo done
