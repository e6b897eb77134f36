#!/bin/bash
# Conv tile-shape experiment on the GPU: time + L2->HBM traffic of one conv class per tile width.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/tile
mkdir -p $O
for tc in 64 32; do
  for dil in 1 2 4; do
    for mode in 1 0; do
      SDP_TC=$tc timeout -k 5 60 tools/_cb/conv_bench_0 256 256 32 512 4 $dil 20 $mode || exit 1
    done
  done
  SDP_TC=$tc timeout -s KILL 60 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum \
    -d $O/pmc_tc$tc -o run --output-format csv -- tools/_cb/conv_bench_0 256 256 32 512 4 1 20 1 > $O/pmc_tc$tc.log 2>&1 || exit 1
  python - $O/pmc_tc$tc <<'PY'
import csv, glob, sys, collections
d = collections.defaultdict(dict)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        d[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
rd = [v["TCC_EA0_RDREQ_sum"] * 128 for v in d.values()]
wr = [64 * v["TCC_EA0_WRREQ_64B_sum"] + 32 * (v["TCC_EA0_WRREQ_sum"] - v["TCC_EA0_WRREQ_64B_sum"]) for v in d.values()]
n = len(rd)
print(f"{sys.argv[1]}: {n} dispatches, read {sum(rd)/n/1e6:.1f} MB, write {sum(wr)/n/1e6:.1f} MB per launch")
PY
done
