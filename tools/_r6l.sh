#!/bin/bash
# maxpool5 DMA lead (SDP_MP_D) A/B: score-net goldens on each variant, then the line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6l; mkdir -p $O
for v in d3 d4 d6; do
  SDP_LIB=tools/_var/$v/libsdp.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "scorenet" > $O/parity_$v.log 2>&1
  rc=$?; echo "parity $v rc=$rc"; tail -1 $O/parity_$v.log; [ $rc -ne 0 ] && exit $rc
done
ROUNDS="1 2" ARMS="base||--sustained-s 0;d3|SDP_LIB=tools/_var/d3/libsdp.so|--sustained-s 0;d4|SDP_LIB=tools/_var/d4/libsdp.so|--sustained-s 0;d6|SDP_LIB=tools/_var/d6/libsdp.so|--sustained-s 0" bash tools/ab_line.sh > $O/ab.log 2>&1
grep -v "^ *[a-z0-9]* r[12]:" $O/ab.log | head -0
python3 - <<'PY'
import json, glob
for arm in ("base", "d3", "d4", "d6"):
    for r in (1, 2):
        f = f"gpurun_out/ab/{arm}_{r}.log"
        d = json.loads([x for x in open(f) if x.startswith("{")][-1])
        mb = {m["kernel"]: m["avg_launch_us"] for m in d["roofline"]["memory_bound"] if m["kernel"].startswith("maxpool")}
        print(arm, r, d["value"], {k[9:]: v for k, v in mb.items()})
PY
