#!/bin/bash
# HBM traffic of the fp32x3 256->256 @32x512 class (4 views) with and without the Cout-block pairing
# of conv_launch_nj2 (ConvArgs::cpair: the two 128-Cout workgroups of a tile dealt as adjacent blocks of
# the XCD-ordered index, so the second patch read hits that XCD's L2), as DESIGN.md section 4 quotes it:
# tools/_cb/conv_bench_0 (the library's dispatch) against tools/_cb/conv_bench_nocpair (built with
# EXTRA=-DSDP_CONV_CPAIR=0 TAG=nocpair KOS=0 tools/conv_bench.sh).  One --pmc group per run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ROUND=${ROUND:-r06}
O=gpurun_out/pair_traffic
mkdir -p $O
for b in 0 nocpair; do
  timeout -k 5 60 tools/_cb/conv_bench_$b 256 256 32 512 4 1 20 1 > $O/time_$b.log 2>&1 || exit 1
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum \
    -d $O/$b -o run --output-format csv -- tools/_cb/conv_bench_$b 256 256 32 512 4 1 20 1 > $O/$b.log 2>&1 || exit 1
done
python3 - $O $ROUND <<'PY'
import collections, csv, glob, json, re, sys
out, rnd = sys.argv[1], sys.argv[2]
rows = []
for b in ("0", "nocpair"):
    d = collections.defaultdict(dict)
    for f in glob.glob(f"{out}/{b}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            d[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
    rd = [v["TCC_EA0_RDREQ_sum"] * 128 for v in d.values()]           # x64 B x2: gfx950 wide-read correction
    wr = [64 * v["TCC_EA0_WRREQ_64B_sum"] + 32 * (v["TCC_EA0_WRREQ_sum"] - v["TCC_EA0_WRREQ_64B_sum"]) for v in d.values()]
    t = re.findall(r"mode 1: ([0-9.]+) us", open(f"{out}/time_{b}.log").read())
    rows.append({"build": "cpair (library)" if b == "0" else "no cpair (grid.y Cout blocks)",
                 "hash_and_flags": open(f"tools/_cb/conv_bench_{b}.hash").read().strip(), "dispatches": len(rd),
                 "read_bytes": sum(rd) / len(rd), "write_bytes": sum(wr) / len(wr), "isolated_us": float(t[0]) if t else None})
doc = {"class": "conv3x3 256->256 @32x512 d1, fp32x3, 4 views", "rows": rows}
json.dump(doc, open(f"{out}/{rnd}_pair_traffic.json", "w"), indent=1)
print(json.dumps(doc, indent=1))
PY
