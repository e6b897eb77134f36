#!/bin/bash
# Interleaved timing rounds of the cache-policy variants + one PMC pass each (EA read/write bytes).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/aux
mkdir -p $O
for round in 1 2 3; do
  for v in 0_0 0_2 2_2 2_0; do
    echo -n "round $round aux $v: "
    timeout -k 5 60 tools/_cb/conv_bench_aux_$v 256 256 32 512 4 1 40 1 || exit 1
  done
done
for v in 0_0 0_2 2_2 2_0; do
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum \
    -d $O/v$v -o run --output-format csv -- tools/_cb/conv_bench_aux_$v 256 256 32 512 4 1 20 1 > $O/v$v.log 2>&1 || exit 1
  python tools/pmc_simple.py $O/v$v
done
