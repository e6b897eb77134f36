#!/bin/bash
# Knock-out variants of the dominant conv class: time + L2->EA traffic (what the excess reads are)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/ko
mkdir -p $O
for ko in ${KOS:-0 1 4 16}; do
  timeout -k 5 60 tools/_cb/conv_bench_$ko 256 256 32 512 4 1 20 1 || exit 1
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum \
    -d $O/ko$ko -o run --output-format csv -- tools/_cb/conv_bench_$ko 256 256 32 512 4 1 20 1 > $O/ko$ko.log 2>&1 || exit 1
  python tools/pmc_simple.py $O/ko$ko
done
