#!/bin/bash
# Workgroup-shape experiment for the 256-channel class: WM=1 (128 px x 256 Cout) vs WM=2 (256 px x 128 Cout)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/wm
mkdir -p $O
for wm in 1 2; do
  for dil in 1 2 4; do
    SDP_WM=$wm timeout -k 5 60 tools/_cb/conv_bench_0 256 256 32 512 4 $dil 20 1 || exit 1
  done
  SDP_WM=$wm timeout -s KILL 60 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum \
    -d $O/wm$wm -o run --output-format csv -- tools/_cb/conv_bench_0 256 256 32 512 4 1 20 1 > $O/wm$wm.log 2>&1 || exit 1
  python tools/pmc_simple.py $O/wm$wm
  SDP_WM=$wm timeout -s KILL 60 rocprofv3 --kernel-trace --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum \
    -d $O/l2_wm$wm -o run --output-format csv -- tools/_cb/conv_bench_0 256 256 32 512 4 1 20 1 > $O/l2_wm$wm.log 2>&1 || exit 1
  python - $O/l2_wm$wm <<'PY'
import collections, csv, glob, sys
d = collections.defaultdict(dict)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        d[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
for c in ("TCP_TCC_READ_REQ_sum", "TCP_TOTAL_CACHE_ACCESSES_sum"):
    v = [x[c] for x in d.values() if c in x]
    print(sys.argv[1], c, sum(v) / max(len(v), 1))
PY
done
