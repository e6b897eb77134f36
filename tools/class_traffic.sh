#!/bin/bash
# HBM traffic per launch of the dominant conv class (conv3x3 256->256 @32x512 d1, 4 views), measured
# by PMC on isolated launches of the library's own kernel (tools/conv_bench, built from csrc/conv.hip)
# for fp32x3 and fp32, written as profiles/<ROUND>_traffic.json tagged with the hash of the conv sources
# the binary was built from (tools/_cb/conv_bench_0.hash), which bench.py checks before printing
# roofline.traffic.  Passes: one --pmc group per run, --kernel-trace only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ROUND=${ROUND:-r04}
O=gpurun_out/class_traffic
mkdir -p $O
for mode in 1 0; do
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum \
    -d $O/m$mode -o run --output-format csv -- tools/_cb/conv_bench_0 256 256 32 512 4 1 20 $mode > $O/m$mode.log 2>&1 || exit 1
done
# the 128-channel class (2-wave workgroups in fp32x3, as the library dispatches it)
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum \
  -d $O/c128 -o run --output-format csv -- tools/_cb/conv_bench_0 128 128 64 1024 4 1 20 1 > $O/c128.log 2>&1 || exit 1
python - $O $ROUND <<'PY'
import collections, csv, glob, json, os, sys
sys.path.insert(0, "simultaneous-diffusion-for-pointclouds_amd")
from sdp import _build
out, rnd = sys.argv[1], sys.argv[2]
rows = []
for sub, prec, cls, alg in (("m1", "fp32x3", "conv3x3 256->256 @32x512 d1", 2 * 4 * 32 * 512 * 256 * 4 + 256 * 256 * 9 * 4),
                            ("m0", "fp32", "conv3x3 256->256 @32x512 d1", 2 * 4 * 32 * 512 * 256 * 4 + 256 * 256 * 9 * 4),
                            ("c128", "fp32x3", "conv3x3 128->128 @64x1024 d1", 2 * 4 * 64 * 1024 * 128 * 4 + 128 * 128 * 9 * 4)):
    d = collections.defaultdict(dict)
    for f in glob.glob(f"{out}/{sub}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            d[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
    rd = [v["TCC_EA0_RDREQ_sum"] * 128 for v in d.values()]           # x64 B x2: gfx950 wide-read correction
    wr = [64 * v["TCC_EA0_WRREQ_64B_sum"] + 32 * (v["TCC_EA0_WRREQ_sum"] - v["TCC_EA0_WRREQ_64B_sum"]) for v in d.values()]
    n = len(rd)
    rows.append({"precision": prec, "views": 4, "class": cls, "dispatches": n,
                 "read_bytes": sum(rd) / n, "write_bytes": sum(wr) / n, "hbm_bytes": (sum(rd) + sum(wr)) / n,
                 "algorithmic_bytes": alg,
                 "how": "rocprofv3 --pmc TCC_EA0_RDREQ/WRREQ on isolated launches (tools/conv_bench, affine+ELU "
                        "prologue, circular, 4 views)"})
built = open("tools/_cb/conv_bench_0.hash").read().split()
if built[0] != _build.conv_source_hash() or len(built) > 1:
    sys.exit(f"tools/_cb/conv_bench_0 was built from other conv sources/flags ({built}): rebuild it (KOS=0 tools/conv_bench.sh)")
doc = {"conv_source_hash": built[0], "rows": rows}
dst = f"{out}/{rnd}_traffic.json"   # merged back under gpurun_out/; copied into profiles/ by hand
json.dump(doc, open(dst, "w"), indent=1)
print(json.dumps(doc, indent=1))
PY
