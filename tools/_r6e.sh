#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6e; mkdir -p $O
for t in 0 s2; do
  for cls in "256 256 32 512" "128 128 64 1024"; do
    n=${t}_$(echo $cls | cut -d' ' -f1)
    timeout -s KILL 60 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum \
      -d $O/$n -o run --output-format csv -- tools/_cb/conv_bench_$t $cls 4 1 20 1 > $O/$n.log 2>&1 || { echo "pmc $n failed"; exit 1; }
    timeout -k 5 60 tools/_cb/conv_bench_$t $cls 4 1 20 1 | tail -1
  done
done
python3 - $O <<'PY'
import collections, csv, glob, sys
for f0 in sorted(glob.glob(sys.argv[1] + "/*/")):
    d = collections.defaultdict(dict)
    for f in glob.glob(f"{f0}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            d[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
    rd = [v["TCC_EA0_RDREQ_sum"] * 128 for v in d.values()]
    print(f0, "reads MB/launch", round(sum(rd) / len(rd) / 1e6, 1), "dispatches", len(rd))
PY
ROUNDS="1 2 3" ARMS="base||;strip1|SDP_LIB=tools/_var/strip1/libsdp.so|;strip2|SDP_LIB=tools/_var/strip2/libsdp.so|" bash tools/ab_line.sh > $O/ab.log 2>&1
python3 tools/ab_sum.py gpurun_out/ab/base_?.log gpurun_out/ab/strip?_?.log
